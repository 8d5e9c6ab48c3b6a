// jmme_subpel_dev.h -- device helpers of JM's sub-pel refinement shared by the
// refinement kernels (jmme_subpel.hip) and the chained searches' in-chain
// refinement (jmme_search.hip chain_kernel): the spiral table, mv_cost,
// the per-block distortion sums and dist().  JM = /root/reference/4.对比程序/jm18.5/JM.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jmme.h"
#include "jmme_common.h"
#include "jmme_subpel_internal.h"

namespace jmme {
namespace spd {
namespace {

constexpr int64_t kDistMax = ((int64_t)0x7fffffff) << 5;   // DISTBLK_MAX, JM/lencod/inc/defines.h:135
constexpr int kPadY = JMME_SUBPEL_PAD_Y, kPadX = JMME_SUBPEL_PAD_X;

// spiral_search[0..8] (mv_search.c:406-442) as (x, y); spiral_hpel_search = 2x.
// Small position tables are read as packed bit fields (value + 1, two bits an
// entry), not from a __constant__ array: indexed by a lane's own position, such
// an array is a vector-memory round trip per lookup inside the refinement's folds.
constexpr int8_t kSpiral9Tab[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {1, 1}};
template <int N>
constexpr uint32_t pack_axis2(const int8_t (&t)[N][2], int a) {
  uint32_t v = 0;
  for (int i = 0; i < N; ++i) v |= (uint32_t)(t[i][a] + 1) << (2 * i);
  return v;
}
constexpr uint32_t kSpiralX = pack_axis2(kSpiral9Tab, 0), kSpiralY = pack_axis2(kSpiral9Tab, 1);
__device__ __forceinline__ int spiral_x(int i) { return (int)((kSpiralX >> (2 * i)) & 3u) - 1; }
__device__ __forceinline__ int spiral_y(int i) { return (int)((kSpiralY >> (2 * i)) & 3u) - 1; }

__device__ __forceinline__ int64_t mv_cost(int lambda, int cx, int cy, int px, int py) {   // mv_search.h:100-104
  return (int64_t)lambda * (int64_t)(mvbits(cx - px) + mvbits(cy - py));
}

// 4 reference bytes of one sub-image at padded row `y`, column `x` (any alignment)
__device__ __forceinline__ uint32_t ref4(const uint8_t *plane, int sp, int y, int x) {
  const uint8_t *a = plane + (size_t)(y + kPadY) * sp + (x + kPadX);
  const uintptr_t u = reinterpret_cast<uintptr_t>(a);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(u & ~(uintptr_t)3);
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(u & 3));
}

// 4 samples of a row as ints: v[k] = p[k] (8-bit: one dword, any alignment)
__device__ __forceinline__ void row4(const uint8_t *p, int (&v)[4]) {
  const uintptr_t u = reinterpret_cast<uintptr_t>(p);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(u & ~(uintptr_t)3);
  const uint32_t d = __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(u & 3));
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = (int)((d >> (8 * k)) & 255);
}
__device__ __forceinline__ void row4(const uint16_t *p, int (&v)[4]) {   // 16-bit samples, 2-byte aligned
  const uintptr_t u = reinterpret_cast<uintptr_t>(p);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(u & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(u & 2);
  const uint32_t d0 = __builtin_amdgcn_alignbyte(w[1], w[0], sh), d1 = __builtin_amdgcn_alignbyte(w[2], w[1], sh);
  v[0] = (int)(d0 & 0xffff); v[1] = (int)(d0 >> 16); v[2] = (int)(d1 & 0xffff); v[3] = (int)(d1 >> 16);
}

__device__ __forceinline__ int had4_sum(const int *d) {   // HadamardSAD4x4 before its (s+1)>>1
  int m[16], e[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {   // vertical pairs (rows 0/3, 1/2)
    m[i] = d[i] + d[12 + i];
    m[4 + i] = d[4 + i] + d[8 + i];
    m[8 + i] = d[4 + i] - d[8 + i];
    m[12 + i] = d[i] - d[12 + i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    e[i] = m[i] + m[4 + i];
    e[4 + i] = m[8 + i] + m[12 + i];
    e[8 + i] = m[i] - m[4 + i];
    e[12 + i] = m[12 + i] - m[8 + i];
  }
  int s = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int a0 = e[4 * r] + e[4 * r + 3], a1 = e[4 * r + 1] + e[4 * r + 2];
    const int a2 = e[4 * r + 1] - e[4 * r + 2], a3 = e[4 * r] - e[4 * r + 3];
    s += abs(a0 + a1) + abs(a0 - a1) + abs(a2 + a3) + abs(a3 - a2);
  }
  return s;
}

// 8x8 Walsh-Hadamard sum of magnitudes: every output of JM's HadamardSAD8x8
// is a distinct-sign +-1 combination of the 64 inputs, so the order of the
// butterflies does not change the sum
__device__ __forceinline__ int had8_sum(int (&d)[64]) {
#pragma unroll
  for (int r = 0; r < 8; ++r) {
#pragma unroll
    for (int h = 1; h < 8; h <<= 1)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (!(i & h)) {
          const int a = d[8 * r + i], b = d[8 * r + i + h];
          d[8 * r + i] = a + b;
          d[8 * r + i + h] = a - b;
        }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
#pragma unroll
    for (int h = 1; h < 8; h <<= 1)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (!(i & h)) {
          const int a = d[8 * i + c], b = d[8 * (i + h) + c];
          d[8 * i + c] = a + b;
          d[8 * (i + h) + c] = a - b;
        }
  }
  int s = 0;
#pragma unroll
  for (int k = 0; k < 64; ++k) s += abs(d[k]);
  return s;
}

// computePred*'s return value for bound T (> 0): JM stops once the partial sum
// exceeds T >> 5 and then returns T (dist_scale_f, mv_search.h:19-20)
__device__ __forceinline__ int64_t dist(int sum, int64_t T) { return (int64_t)sum > (T >> 5) ? T : (int64_t)sum << 5; }

__device__ __forceinline__ void blk_size(int bt, int &bsx, int &bsy) {   // block_size[], macroblock.h:58-68
  bsx = (bt == 1 || bt == 2) ? 16 : (bt == 3 || bt == 4 || bt == 5) ? 8 : 4;
  bsy = (bt == 1 || bt == 3) ? 16 : (bt == 2 || bt == 4 || bt == 6) ? 8 : 4;
}

// The distortion sum of one transform / 4x4 block of one candidate
// (computeSAD / computeSSE / computeSATD restated per block; their per-row or
// per-block early exits are reproduced by dist() in the fold).
// 8-bit samples: v_sad_u8 for SAD, bytes unpacked for SSE / SATD.  16-bit
// samples (job_sum below): the same sums over unpacked samples.
__device__ __forceinline__ int job_sum(const uint8_t *sub, size_t ps, int sp, const uint8_t *org, int cp, int ymax,
                                       int xmax, int metric, bool big, int cx, int cy, int bxo, int byo) {
  const int pl = ((cy & 3) << 2) | (cx & 3);
  const uint8_t *plane = sub + (size_t)pl * ps;
  int yy, xx;
  if (metric == 2) {   // computeSATD: UMVLine4X per transform block
    yy = min(max((cy + (byo << 2)) >> 2, -kPadY), ymax);
    xx = min(max((cx + (bxo << 2)) >> 2, -kPadX), xmax);
  } else {             // computeSAD / computeSSE: UMVLine4X of the block origin
    yy = min(max(cy >> 2, -kPadY), ymax) + byo;
    xx = min(max(cx >> 2, -kPadX), xmax) + bxo;
  }
  org += (size_t)byo * cp + bxo;
  int s = 0;
  if (metric == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      s = __builtin_amdgcn_sad_u8(ref4(plane, sp, yy + r, xx), *reinterpret_cast<const uint32_t *>(org + r * cp), s);
  } else if (metric == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t a = *reinterpret_cast<const uint32_t *>(org + r * cp), w = ref4(plane, sp, yy + r, xx);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int d = (int)((a >> (8 * k)) & 255) - (int)((w >> (8 * k)) & 255);
        s += d * d;
      }
    }
  } else if (!big) {
    int d[16];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t a = *reinterpret_cast<const uint32_t *>(org + r * cp), w = ref4(plane, sp, yy + r, xx);
#pragma unroll
      for (int k = 0; k < 4; ++k) d[4 * r + k] = (int)((a >> (8 * k)) & 255) - (int)((w >> (8 * k)) & 255);
    }
    s = (had4_sum(d) + 1) >> 1;
  } else {
    int d[64];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t a = *reinterpret_cast<const uint32_t *>(org + r * cp + 4 * h);
        const uint32_t w = ref4(plane, sp, yy + r, xx + 4 * h);
#pragma unroll
        for (int k = 0; k < 4; ++k) d[8 * r + 4 * h + k] = (int)((a >> (8 * k)) & 255) - (int)((w >> (8 * k)) & 255);
      }
    }
    s = (had8_sum(d) + 2) >> 2;
  }
  return s;
}

__device__ __forceinline__ int job_sum(const uint16_t *sub, size_t ps, int sp, const uint16_t *org, int cp, int ymax,
                                       int xmax, int metric, bool big, int cx, int cy, int bxo, int byo) {
  const int pl = ((cy & 3) << 2) | (cx & 3);
  const uint16_t *plane = sub + (size_t)pl * ps;
  int yy, xx;
  if (metric == 2) {
    yy = min(max((cy + (byo << 2)) >> 2, -kPadY), ymax);
    xx = min(max((cx + (bxo << 2)) >> 2, -kPadX), xmax);
  } else {
    yy = min(max(cy >> 2, -kPadY), ymax) + byo;
    xx = min(max(cx >> 2, -kPadX), xmax) + bxo;
  }
  org += (size_t)byo * cp + bxo;
  auto ref = [&](int r, int c, int (&v)[4]) { row4(plane + (size_t)(yy + r + kPadY) * sp + (xx + c + kPadX), v); };
  int s = 0;
  if (metric <= 1) {   // computeSAD / computeSSE (int sums, as JM's mcost)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int a[4], w[4];
      row4(org + r * cp, a);
      ref(r, 0, w);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int d = a[k] - w[k];
        s += metric == 0 ? abs(d) : d * d;
      }
    }
  } else if (!big) {
    int d[16];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int a[4], w[4];
      row4(org + r * cp, a);
      ref(r, 0, w);
#pragma unroll
      for (int k = 0; k < 4; ++k) d[4 * r + k] = a[k] - w[k];
    }
    s = (had4_sum(d) + 1) >> 1;
  } else {
    int d[64];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        int a[4], w[4];
        row4(org + r * cp + 4 * h, a);
        ref(r, 4 * h, w);
#pragma unroll
        for (int k = 0; k < 4; ++k) d[8 * r + 4 * h + k] = a[k] - w[k];
      }
    }
    s = (had8_sum(d) + 2) >> 2;
  }
  return s;
}

}  // namespace
}  // namespace spd
}  // namespace jmme
