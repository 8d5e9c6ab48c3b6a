// jmme_epzs_g0h1.hip -- the EPZS kernels for the integer grid,
// 16-bit samples (jmme_epzs_impl.inc)
#define JMME_EPZS_GRID 0
#define JMME_EPZS_HBD 1
#include "jmme_epzs_impl.inc"
