// jmme_epzs_g0h0.hip -- the EPZS kernels for the integer grid,
// 8-bit samples (jmme_epzs_impl.inc)
#define JMME_EPZS_GRID 0
#define JMME_EPZS_HBD 0
#include "jmme_epzs_impl.inc"
