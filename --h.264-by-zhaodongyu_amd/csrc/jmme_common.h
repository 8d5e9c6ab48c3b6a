// jmme_common.h -- host+device helpers shared by the HIP kernels and the C-ABI.
//
// Restates (not copies) the JM 18.5 tables the integer-pel search uses
// (JM = /root/reference/4.对比程序/jm18.5/JM):
//   spiral_search order      JM/lencod/src/mv_search.c:406-442
//   mvbits[]                 JM/lencod/src/mv_search.c:366-374
//   block_size[] / BlockSAD  JM/lencod/inc/macroblock.h:58, me_fullfast.c:196-260
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define JMME_HD __host__ __device__ __forceinline__
#else
#define JMME_HD static inline
#endif

namespace jmme {

// Index of integer offset (ox, oy) in JM's spiral order.  Ring l = max(|ox|,|oy|)
// starts at (2l-1)^2; inside a ring JM first walks i = -l+1..l-1 emitting
// (i,-l),(i,+l), then i = -l..l emitting (-l,i),(+l,i).
JMME_HD int spiral_index(int ox, int oy) {
  int ax = ox < 0 ? -ox : ox;
  int ay = oy < 0 ? -oy : oy;
  int l = ax > ay ? ax : ay;
  if (l == 0) return 0;
  int base = (2 * l - 1) * (2 * l - 1);
  if (ay == l && ax < l) return base + 2 * (ox + l - 1) + (oy > 0 ? 1 : 0);
  return base + 2 * (2 * l - 1) + 2 * (oy + l) + (ox > 0 ? 1 : 0);
}

JMME_HD void spiral_offset(int idx, int *ox, int *oy) {
  if (idx <= 0) { *ox = 0; *oy = 0; return; }
  int l = 1;
  while ((2 * l + 1) * (2 * l + 1) <= idx) l++;
  int r = idx - (2 * l - 1) * (2 * l - 1);
  if (r < 2 * (2 * l - 1)) {
    *ox = r / 2 - l + 1;
    *oy = (r & 1) ? l : -l;
  } else {
    r -= 2 * (2 * l - 1);
    *oy = r / 2 - l;
    *ox = (r & 1) ? l : -l;
  }
}

// mvbits[v]: 1 for 0, 2*floor(log2|v|)+3 otherwise.  With w = 2|v|+1 this is
// 2*floor(log2 w)+1 = 63 - 2*clz(w), valid for v = 0 too (no branch).
JMME_HD int mvbits(int v) {
  unsigned a = (unsigned)(v < 0 ? -v : v);
  unsigned w = 2u * a + 1u;
  return 63 - 2 * __builtin_clz(w);
}

// Partition slots.  Slot order: 0 16x16 | 1-2 16x8 | 3-4 8x16 | 5-8 8x8 |
// 9-16 8x4 | 17-24 4x8 | 25-40 4x4.  Geometry in 4x4-block units.
struct SlotGeom { int8_t bt, bx, by, w, h; };

JMME_HD int slot_of(int bt, int bx, int by) {
  switch (bt) {
    case 1: return (bx == 0 && by == 0) ? 0 : -1;
    case 2: return (bx == 0 && (by == 0 || by == 2)) ? 1 + by / 2 : -1;
    case 3: return (by == 0 && (bx == 0 || bx == 2)) ? 3 + bx / 2 : -1;
    case 4: return ((bx == 0 || bx == 2) && (by == 0 || by == 2)) ? 5 + (by / 2) * 2 + bx / 2 : -1;
    case 5: return ((bx == 0 || bx == 2) && by >= 0 && by < 4) ? 9 + by * 2 + bx / 2 : -1;
    case 6: return (bx >= 0 && bx < 4 && (by == 0 || by == 2)) ? 17 + (by / 2) * 4 + bx : -1;
    case 7: return (bx >= 0 && bx < 4 && by >= 0 && by < 4) ? 25 + by * 4 + bx : -1;
    default: return -1;
  }
}

JMME_HD constexpr SlotGeom slot_geom(int s) {
  SlotGeom g{};
  if (s == 0) { g.bt = 1; g.bx = 0; g.by = 0; g.w = 4; g.h = 4; }
  else if (s <= 2) { g.bt = 2; g.bx = 0; g.by = (int8_t)(2 * (s - 1)); g.w = 4; g.h = 2; }
  else if (s <= 4) { g.bt = 3; g.bx = (int8_t)(2 * (s - 3)); g.by = 0; g.w = 2; g.h = 4; }
  else if (s <= 8) { g.bt = 4; g.bx = (int8_t)(2 * ((s - 5) & 1)); g.by = (int8_t)(2 * ((s - 5) >> 1)); g.w = 2; g.h = 2; }
  else if (s <= 16) { g.bt = 5; g.bx = (int8_t)(2 * ((s - 9) & 1)); g.by = (int8_t)((s - 9) >> 1); g.w = 2; g.h = 1; }
  else if (s <= 24) { g.bt = 6; g.bx = (int8_t)((s - 17) & 3); g.by = (int8_t)(2 * ((s - 17) >> 2)); g.w = 1; g.h = 2; }
  else { g.bt = 7; g.bx = (int8_t)((s - 25) & 3); g.by = (int8_t)((s - 25) >> 2); g.w = 1; g.h = 1; }
  return g;
}

}  // namespace jmme
