// jmme_epzs_g1h0.hip -- the EPZS kernels for the quarter-pel grid (EPZSSubPelGrid = 1),
// 8-bit samples (jmme_epzs_impl.inc)
#define JMME_EPZS_GRID 1
#define JMME_EPZS_HBD 0
#include "jmme_epzs_impl.inc"
