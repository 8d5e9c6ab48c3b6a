// jmme_epzs_g1h1.hip -- the EPZS kernels for the quarter-pel grid (EPZSSubPelGrid = 1),
// 16-bit samples (jmme_epzs_impl.inc)
#define JMME_EPZS_GRID 1
#define JMME_EPZS_HBD 1
#include "jmme_epzs_impl.inc"
