// jmme_tq.hip -- gfx950 kernels for JM 18.5's block transforms, 4x4
// quantisation and Hadamard SATD, batched over n
// independent blocks.
//
//   forward4x4 / inverse4x4 / hadamard4x4 / ihadamard4x4 /
//   hadamard4x2 / ihadamard4x2 / hadamard2x2 / ihadamard2x2 /
//   forward8x8 / inverse8x8           JM/lcommon/src/transform.c:20-528
//   HadamardSAD4x4 / HadamardSAD8x8   JM/lencod/src/me_distortion.c:175-341
//   quant_4x4_normal                  JM/lencod/src/quant4x4_normal.c:39-110
//
// These are streaming kernels (tens of integer ops per 32-256 B block): the
// bound is HBM.  A wave owns 64 consecutive blocks (one per lane): it streams
// their bytes with lane-contiguous 16-B loads/stores (fully coalesced) and
// transposes through a padded LDS slab so each lane gets its own block.
// Butterflies are the same integer operations in the same order as JM (the
// >> steps make the order significant), so results are bit-exact.
#include <hip/hip_runtime.h>
#include "jmme.h"
#include "jmme_tq_internal.h"

namespace jmme {

namespace {

constexpr int kTB = 64;   // one wave per workgroup: the LDS slab is per wave

// ---- 1-D butterflies: x[k*s] -> y[k*t] ------------------------------------
__device__ __forceinline__ void fwd4(const int *x, int s, int *y, int t) {       // transform.c:32-44
  const int a = x[0] + x[3 * s], b = x[s] + x[2 * s], c = x[s] - x[2 * s], d = x[0] - x[3 * s];
  y[0] = a + b; y[t] = 2 * d + c; y[2 * t] = a - b; y[3 * t] = d - 2 * c;
}
__device__ __forceinline__ void inv4(const int *x, int s, int *y, int t) {       // transform.c:82-94
  const int e = x[0] + x[2 * s], f = x[0] - x[2 * s];
  const int g = (x[s] >> 1) - x[3 * s], h = x[s] + (x[3 * s] >> 1);
  y[0] = e + h; y[t] = f + g; y[2 * t] = f - g; y[3 * t] = e - h;
}
__device__ __forceinline__ void had4(const int *x, int s, int *y, int t) {       // transform.c:133-145
  const int a = x[0] + x[3 * s], b = x[s] + x[2 * s], c = x[s] - x[2 * s], d = x[0] - x[3 * s];
  y[0] = a + b; y[t] = d + c; y[2 * t] = a - b; y[3 * t] = d - c;
}
__device__ __forceinline__ void ihad4(const int *x, int s, int *y, int t) {      // transform.c:183-195
  const int e = x[0] + x[2 * s], f = x[0] - x[2 * s], g = x[s] - x[3 * s], h = x[s] + x[3 * s];
  y[0] = e + h; y[t] = f + g; y[2 * t] = f - g; y[3 * t] = e - h;
}
__device__ __forceinline__ void fwd8(const int *x, int s, int *y, int t) {       // transform.c:365-402
  const int s07 = x[0] + x[7 * s], s16 = x[s] + x[6 * s], s25 = x[2 * s] + x[5 * s], s34 = x[3 * s] + x[4 * s];
  const int d07 = x[0] - x[7 * s], d16 = x[s] - x[6 * s], d25 = x[2 * s] - x[5 * s], d34 = x[3 * s] - x[4 * s];
  const int e0 = s07 + s34, e1 = s16 + s25, e2 = s07 - s34, e3 = s16 - s25;
  const int o4 = d16 + d25 + ((d07 >> 1) + d07), o5 = d07 - d34 - ((d25 >> 1) + d25);
  const int o6 = d07 + d34 - ((d16 >> 1) + d16), o7 = d16 - d25 + ((d34 >> 1) + d34);
  y[0] = e0 + e1; y[t] = o4 + (o7 >> 2); y[2 * t] = e2 + (e3 >> 1); y[3 * t] = o5 + (o6 >> 2);
  y[4 * t] = e0 - e1; y[5 * t] = o6 - (o5 >> 2); y[6 * t] = (e2 >> 1) - e3; y[7 * t] = (o4 >> 2) - o7;
}
__device__ __forceinline__ void inv8(const int *x, int s, int *y, int t) {       // transform.c:474-506
  const int p0 = x[0], p1 = x[s], p2 = x[2 * s], p3 = x[3 * s], p4 = x[4 * s], p5 = x[5 * s], p6 = x[6 * s],
            p7 = x[7 * s];
  const int a0 = p0 + p4, a1 = p0 - p4, a2 = p6 - (p2 >> 1), a3 = p2 + (p6 >> 1);
  const int b0 = a0 + a3, b2 = a1 - a2, b4 = a1 + a2, b6 = a0 - a3;
  const int c0 = -p3 + p5 - p7 - (p7 >> 1), c1 = p1 + p7 - p3 - (p3 >> 1);
  const int c2 = -p1 + p7 + p5 + (p5 >> 1), c3 = p3 + p5 + p1 + (p1 >> 1);
  const int b1 = c0 + (c3 >> 2), b3 = c1 + (c2 >> 2), b5 = c2 - (c1 >> 2), b7 = c3 - (c0 >> 2);
  y[0] = b0 + b7; y[t] = b2 - b5; y[2 * t] = b4 + b3; y[3 * t] = b6 + b1;
  y[4 * t] = b6 - b1; y[5 * t] = b4 - b3; y[6 * t] = b2 + b5; y[7 * t] = b0 - b7;
}

typedef int v4i __attribute__((ext_vector_type(4)));

// LDS slab stride (dwords) for D-dword blocks: +4 (16-B rows) / +1 keeps the
// per-lane block reads and writes conflict-free
template <int D>
__host__ __device__ constexpr int slab_stride() { return D + ((D % 4 == 0) ? 4 : 1); }

// Wave-cooperative load of nb (<= 64) consecutive D-dword blocks at src: the
// wave reads them as lane-contiguous chunks, parks them in the slab, and lane
// l picks up block l.
template <int D>
__device__ __forceinline__ void wave_load(const int32_t *src, int nb, int32_t *slab, int lane, int *v) {
  constexpr int S = slab_stride<D>();
  if (D % 4 == 0) {
    constexpr int C = D / 4;   // 16-B chunks per block
#pragma unroll
    for (int k = 0; k < C; ++k) {
      const int ch = k * 64 + lane, blk = ch / C, part = ch - blk * C;
      if (blk < nb) {
        const v4i q = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(src) + ch);
        *reinterpret_cast<v4i *>(slab + blk * S + 4 * part) = q;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int dw = k * 64 + lane, blk = dw / D;
      if (blk < nb) slab[blk * S + dw - blk * D] = __builtin_nontemporal_load(src + dw);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < D; ++k) v[k] = slab[lane * S + k];
  __syncthreads();   // the slab is free again
}

// the reverse: lane l's block v goes to dst + l*D as lane-contiguous chunks
template <int D>
__device__ __forceinline__ void wave_store(int32_t *dst, int nb, int32_t *slab, int lane, const int *v) {
  constexpr int S = slab_stride<D>();
#pragma unroll
  for (int k = 0; k < D; ++k) slab[lane * S + k] = v[k];
  __syncthreads();
  if (D % 4 == 0) {
    constexpr int C = D / 4;
#pragma unroll
    for (int k = 0; k < C; ++k) {
      const int ch = k * 64 + lane, blk = ch / C, part = ch - blk * C;
      if (blk < nb)
        __builtin_nontemporal_store(*reinterpret_cast<const v4i *>(slab + blk * S + 4 * part),
                                    reinterpret_cast<v4i *>(dst) + ch);
    }
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int dw = k * 64 + lane, blk = dw / D;
      if (blk < nb) __builtin_nontemporal_store(slab[blk * S + dw - blk * D], dst + dw);
    }
  }
  __syncthreads();
}

// one block through op OP (a jmme_transform_op)
template <int OP>
__device__ __forceinline__ void transform_one(const int *in, int *out) {
  int tmp[64];
  if (OP == JMME_TF_FORWARD4x4 || OP == JMME_TF_INVERSE4x4 || OP == JMME_TF_IHADAMARD4x4) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (OP == JMME_TF_FORWARD4x4) fwd4(in + 4 * r, 1, tmp + 4 * r, 1);
      if (OP == JMME_TF_INVERSE4x4) inv4(in + 4 * r, 1, tmp + 4 * r, 1);
      if (OP == JMME_TF_IHADAMARD4x4) ihad4(in + 4 * r, 1, tmp + 4 * r, 1);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (OP == JMME_TF_FORWARD4x4) fwd4(tmp + c, 4, out + c, 4);
      if (OP == JMME_TF_INVERSE4x4) inv4(tmp + c, 4, out + c, 4);
      if (OP == JMME_TF_IHADAMARD4x4) ihad4(tmp + c, 4, out + c, 4);
    }
  } else if (OP == JMME_TF_HADAMARD4x4) {          // vertical pass halves, transform.c:160-166
#pragma unroll
    for (int r = 0; r < 4; ++r) had4(in + 4 * r, 1, tmp + 4 * r, 1);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      int y[4];
      had4(tmp + c, 4, y, 1);
#pragma unroll
      for (int k = 0; k < 4; ++k) out[4 * k + c] = y[k] >> 1;
    }
  } else if (OP == JMME_TF_HADAMARD4x2 || OP == JMME_TF_IHADAMARD4x2) {   // transform.c:220-300
#pragma unroll
    for (int c = 0; c < 4; ++c) { tmp[c] = in[c] + in[4 + c]; tmp[4 + c] = in[c] - in[4 + c]; }
    if (OP == JMME_TF_HADAMARD4x2) {
      had4(tmp, 1, out, 1);
      had4(tmp + 4, 1, out + 4, 1);
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) ihad4(tmp + 4 * i, 1, out + i, 2);   // 4 rows x 2 columns out
    }
  } else if (OP == JMME_TF_HADAMARD2x2 || OP == JMME_TF_IHADAMARD2x2) {   // transform.c:302-331
    const int p0 = in[0] + in[1], p1 = in[0] - in[1], p2 = in[2] + in[3], p3 = in[2] - in[3];
    out[0] = p0 + p2; out[1] = p1 + p3; out[2] = p0 - p2; out[3] = p1 - p3;
  } else {                                          // 8x8
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (OP == JMME_TF_FORWARD8x8) fwd8(in + 8 * r, 1, tmp + 8 * r, 1);
      else inv8(in + 8 * r, 1, tmp + 8 * r, 1);
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      if (OP == JMME_TF_FORWARD8x8) fwd8(tmp + c, 8, out + c, 8);
      else inv8(tmp + c, 8, out + c, 8);
    }
  }
}

__host__ __device__ constexpr int tf_elems(int op) {
  return (op == JMME_TF_FORWARD8x8 || op == JMME_TF_INVERSE8x8) ? 64
         : (op == JMME_TF_HADAMARD4x2 || op == JMME_TF_IHADAMARD4x2) ? 8
         : (op == JMME_TF_HADAMARD2x2 || op == JMME_TF_IHADAMARD2x2) ? 4 : 16;
}

template <int OP>
__global__ __launch_bounds__(kTB) void transform_kernel(const int32_t *__restrict__ in, int32_t *__restrict__ out,
                                                        int n) {
  constexpr int E = tf_elems(OP);
  __shared__ __attribute__((aligned(16))) int32_t slab[64 * slab_stride<E>()];
  const int lane = threadIdx.x;
  for (int base = blockIdx.x * 64; base < n; base += gridDim.x * 64) {
    const int nb = min(64, n - base);
    int v[E], w[E];
    wave_load<E>(in + (size_t)base * E, nb, slab, lane, v);
    transform_one<OP>(v, w);
    wave_store<E>(out + (size_t)base * E, nb, slab, lane, w);
  }
}

// ---- 8x8 blocks: a row per lane ----------------------------------------------
// A lane per row keeps a lane's state at one row (8 values) instead of a whole
// block (64 + 64 + 64: 170 VGPRs, 2 waves/SIMD -- 57-59 % of HBM): the 8 lanes
// of a block load its 256 B as two lane-contiguous 16-B chunks each (fully
// coalesced, no staging), run JM's row butterflies, transpose through a padded
// per-wave LDS tile, run the column butterflies and transpose back.  Same
// integer operations in the same order as transform.c:365-506.
constexpr int kT8 = 9;     // LDS row stride (dwords) of the 8x8 tiles
constexpr int kWG8 = 256;  // 4 waves per workgroup: one-wave workgroups left too few waves per CU
#ifndef JMME_T8_U
#define JMME_T8_U 4
#endif
constexpr int kU8 = JMME_T8_U;   // 8x8 transforms: block groups per loop iteration (loads in flight)
#ifndef JMME_QUANT_UQ
#define JMME_QUANT_UQ 16   // (4: 0.251 ms, 8: 0.244-0.245 ms, 16: 0.240 ms per 4M blocks)
#endif
constexpr int kUQ = JMME_QUANT_UQ;   // quant: blocks per 16-lane group per loop iteration

template <int OP>
__global__ __launch_bounds__(kWG8) void transform8_kernel(const int32_t *__restrict__ in, int32_t *__restrict__ out,
                                                          int n) {
  // kU8 groups of 32 blocks per iteration: all their loads are issued before
  // the first is used (HBM wants ~100+ KB in flight per CU)
  __shared__ int32_t tile[kWG8 / 8 * 8 * kT8];
  const int b = threadIdx.x >> 3, r = threadIdx.x & 7;   // block of a group of 32, row
  int32_t *t = tile + b * 8 * kT8;
  constexpr int kG = kWG8 / 8;
  for (int base = blockIdx.x * kG * kU8; base < n; base += gridDim.x * kG * kU8) {
    v4i q[kU8][2];
#pragma unroll
    for (int u = 0; u < kU8; ++u) {
      const int blk = base + u * kG + b;
      if (blk < n) {
        const v4i *src = reinterpret_cast<const v4i *>(in + ((size_t)blk * 64 + r * 8));
        q[u][0] = __builtin_nontemporal_load(src);
        q[u][1] = __builtin_nontemporal_load(src + 1);
      } else {
        q[u][0] = q[u][1] = v4i{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int u = 0; u < kU8; ++u) {
      const int blk = base + u * kG + b;
      int x[8] = {q[u][0].x, q[u][0].y, q[u][0].z, q[u][0].w, q[u][1].x, q[u][1].y, q[u][1].z, q[u][1].w}, y[8];
      if (OP == JMME_TF_FORWARD8x8) fwd8(x, 1, y, 1); else inv8(x, 1, y, 1);   // rows
#pragma unroll
      for (int k = 0; k < 8; ++k) t[r * kT8 + k] = y[k];
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = t[k * kT8 + r];                      // column r
      if (OP == JMME_TF_FORWARD8x8) fwd8(x, 1, y, 1); else inv8(x, 1, y, 1);   // columns
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k * kT8 + r] = y[k];
      __syncthreads();
      if (blk < n) {
        // store j writes 16-B chunk 8j + r of the block: the 8 lanes of a block
        // cover one whole 128-B line per store instruction (rows 4j .. 4j+3)
        v4i *dst = reinterpret_cast<v4i *>(out + (size_t)blk * 64);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int *src = t + (4 * j + (r >> 1)) * kT8 + 4 * (r & 1);
          __builtin_nontemporal_store(v4i{src[0], src[1], src[2], src[3]}, dst + 8 * j + r);
        }
      }
      __syncthreads();
    }
  }
}

// 8-point Walsh-Hadamard butterflies in place (the order of wht_abs_sum)
__device__ __forceinline__ void wht8(int *v) {
#pragma unroll
  for (int len = 1; len < 8; len <<= 1)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (!(j & len)) {
        const int a = v[j], c = v[j + len];
        v[j] = a + c;
        v[j + len] = a - c;
      }
}

// HadamardSAD8x8 (me_distortion.c:261-341) a row per lane: one 16-B load of 8
// int16 differences, row WHT, transpose, column WHT, |.| summed over the 8
// lanes of the block by cross-lane adds
__global__ __launch_bounds__(kWG8) void satd8_kernel(const int16_t *__restrict__ diff, int32_t *__restrict__ out, int n) {
  __shared__ int32_t tile[kWG8 / 8 * 8 * kT8];
  const int b = threadIdx.x >> 3, r = threadIdx.x & 7;
  int32_t *t = tile + b * 8 * kT8;
  constexpr int kG = kWG8 / 8;
  for (int base = blockIdx.x * kG * kU8; base < n; base += gridDim.x * kG * kU8) {
    v4i q[kU8];
#pragma unroll
    for (int u = 0; u < kU8; ++u) {   // every group's row loaded before the first is used
      const int blk = base + u * kG + b;
      q[u] = blk < n ? __builtin_nontemporal_load(reinterpret_cast<const v4i *>(diff + ((size_t)blk * 64 + r * 8)))
                     : v4i{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < kU8; ++u) {
      const int blk = base + u * kG + b;
      const int w[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
      int v[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) { v[2 * k] = (int)(int16_t)(w[k] & 0xffff); v[2 * k + 1] = w[k] >> 16; }
      wht8(v);
#pragma unroll
      for (int k = 0; k < 8; ++k) t[r * kT8 + k] = v[k];
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = t[k * kT8 + r];
      __syncthreads();
      wht8(v);
      int sum = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) sum += abs(v[k]);
      sum += __shfl_xor(sum, 1, 64);
      sum += __shfl_xor(sum, 2, 64);
      sum += __shfl_xor(sum, 4, 64);
      if (blk < n && r == 0) out[blk] = (sum + 2) >> 2;   // me_distortion.c:339
    }
  }
}

// ---- SATD ------------------------------------------------------------------
// Sum of |Walsh-Hadamard(d)|: every output of JM's HadamardSAD4x4/8x8 is a +-1
// combination of the inputs with a distinct sign pattern, so the sum of
// magnitudes does not depend on JM's output order.
template <int N>
__device__ __forceinline__ int wht_abs_sum(int *v) {
#pragma unroll
  for (int r = 0; r < N; ++r)
#pragma unroll
    for (int len = 1; len < N; len <<= 1)
#pragma unroll
      for (int j = 0; j < N; ++j)
        if (!(j & len)) {
          const int a = v[r * N + j], b = v[r * N + j + len];
          v[r * N + j] = a + b;
          v[r * N + j + len] = a - b;
        }
#pragma unroll
  for (int c = 0; c < N; ++c)
#pragma unroll
    for (int len = 1; len < N; len <<= 1)
#pragma unroll
      for (int j = 0; j < N; ++j)
        if (!(j & len)) {
          const int a = v[j * N + c], b = v[(j + len) * N + c];
          v[j * N + c] = a + b;
          v[(j + len) * N + c] = a - b;
        }
  int s = 0;
#pragma unroll
  for (int k = 0; k < N * N; ++k) s += abs(v[k]);
  return s;
}

template <int N>
__global__ __launch_bounds__(kTB) void satd_kernel(const int16_t *__restrict__ diff, int32_t *__restrict__ out,
                                                   int n) {
  constexpr int D = N * N / 2;   // int16 pairs
  __shared__ __attribute__((aligned(16))) int32_t slab[64 * slab_stride<D>()];
  const int lane = threadIdx.x;
  for (int base = blockIdx.x * 64; base < n; base += gridDim.x * 64) {
    const int nb = min(64, n - base);
    int w[D], v[N * N];
    wave_load<D>(reinterpret_cast<const int32_t *>(diff) + (size_t)base * D, nb, slab, lane, w);
#pragma unroll
    for (int k = 0; k < D; ++k) {
      v[2 * k] = (int)(int16_t)(w[k] & 0xffff);
      v[2 * k + 1] = w[k] >> 16;
    }
    const int s = wht_abs_sum<N>(v);
    if (lane < nb) out[base + lane] = N == 4 ? (s + 1) >> 1 : (s + 2) >> 2;   // me_distortion.c:256, :339
  }
}

// ---- quant_4x4_normal --------------------------------------------------------
// A lane per scan position, 16 lanes per block, 4 blocks per wave; every wave
// works alone (no workgroup barrier, no LDS arrays).  JM's loop
// (quant4x4_normal.c:59-104) is sequential only through `run` and the output
// index; both are functions of which earlier scan positions quantise to a
// nonzero level, i.e. of the block's 16-bit slice of one ballot: the output
// index is the popcount of the nonzero positions below, the run the distance
// to the highest one.  The (level, run) lists are compacted with one
// ds_permute each (a push: nonzero lane k to slot idx, the zero lanes behind
// them in order -- a bijection), the 4 blocks' 17-dword level lists are then
// pulled (ds_bpermute) into one lane-contiguous run of 68 dwords, and the cost
// is a 16-lane DPP reduction.  kUQ rounds' loads are issued before the first
// round's arithmetic.  With one parameter set (param_idx NULL) the lane's
// scale / offset / inverse scale and the cost table are loaded once per wave.
// (Round 3's form, with LDS compaction tables and three workgroup barriers per
// round, measured 33 % of HBM: 64 % of its wave cycles parked on waits --
// rocprofv3 SQ_WAIT_ANY -- for the barriers and a three-deep dependent load
// chain per round.)
template <bool UNI>   // UNI: one parameter set (param_idx NULL)
__global__ __launch_bounds__(kWG8) void quant4x4_kernel(const jmme_quant4x4_params *__restrict__ params,
                                                        const int32_t *__restrict__ param_idx,
                                                        int32_t *__restrict__ coef, int32_t *__restrict__ levels,
                                                        int32_t *__restrict__ runs,
                                                        int32_t *__restrict__ coeff_cost,
                                                        int32_t *__restrict__ nonzero, int n) {
  const int lane = threadIdx.x & 63, gw = lane >> 4, k = lane & 15;
  const int wave = (blockIdx.x * kWG8 + threadIdx.x) >> 6, nwaves = gridDim.x * (kWG8 / 64);
  constexpr bool uni = UNI;
  constexpr int U = UNI ? kUQ : kUQ / 2;   // rounds in flight (the per-block parameters cost registers)
  // one parameter set: this lane's scan position and factors, once
  // (lane k of a block also holds c_cost[k]: a level-1 lane pulls c_cost[run] from lane run of its block)
  int pq0 = 0, sc0 = 0, of0 = 0, iv0 = 0, qper0 = 0, cavlc0 = 0, ck0 = 0;
  if (uni) {
    const jmme_quant4x4_params &q = params[0];
    pq0 = q.scan[k][1] * 4 + q.scan[k][0];   // (horizontal, vertical)
    sc0 = q.scale[pq0]; of0 = q.offset[pq0]; iv0 = q.inv_scale[pq0];
    qper0 = q.qp_per; cavlc0 = q.is_cavlc; ck0 = q.c_cost[k];
  }
  // this lane's dword of the wave's 68-dword level run: block j, entry pos (16: the 0 terminator)
  const int lj = lane / 17, lpos = lane - 17 * lj;
  const int tj = 3, tpos = 13 + (lane & 3);   // lanes 0-3: dwords 64-67 (block 3, entries 13-16)
  for (int b4 = wave * 4 * U; b4 < n; b4 += nwaves * 4 * U) {
    int x[U], cc[U], pq[U], sc[U], of[U], iv[U], qper[U], cavlc[U], ck[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = b4 + 4 * u + gw;
      const bool live = b < n;
      if (uni) {
        pq[u] = pq0; sc[u] = sc0; of[u] = of0; iv[u] = iv0; qper[u] = qper0; cavlc[u] = cavlc0; ck[u] = ck0;
      } else {
        const jmme_quant4x4_params &q = params[live ? param_idx[b] : 0];
        pq[u] = q.scan[k][1] * 4 + q.scan[k][0];
        sc[u] = q.scale[pq[u]]; of[u] = q.offset[pq[u]]; iv[u] = q.inv_scale[pq[u]];
        qper[u] = q.qp_per; cavlc[u] = q.is_cavlc; ck[u] = q.c_cost[k];
      }
      x[u] = live ? coef[(size_t)b * 16 + pq[u]] : 0;
      cc[u] = (k == 0 && live) ? coeff_cost[b] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = b4 + 4 * u + gw;
      const bool live = b < n;
      const int q_bits = 15 + qper[u];                  // Q_BITS, defines.h:311
      const int xv = x[u];
      int level = xv == 0 ? 0 : (abs(xv) * sc[u] + of[u]) >> q_bits;
      if (cavlc[u] && level > 2063) level = 2063;       // CAVLC_LEVEL_LIMIT, defines.h:99
      const unsigned mg = (unsigned)(__builtin_amdgcn_ballot_w64(level != 0) >> (16 * gw)) & 0xffffu;
      const unsigned below = mg & ((1u << k) - 1u);
      const int idx = __builtin_popcount(below), nnz = __builtin_popcount(mg);
      const int run = below ? k - (32 - __builtin_clz(below)) : k;   // positions since the previous nonzero
      const int sl = xv < 0 ? -level : level;
      const int crun = __builtin_amdgcn_ds_bpermute(4 * (16 * gw + run), ck[u]);   // c_cost[run]
      int term = 0, deq = 0;
      if (level) {
        term = level > 1 ? 999999 : crun;                     // MAX_VALUE, defines.h:123
        deq = ((sl * iv[u] << qper[u]) + 8) >> 4;             // rshift_rnd_sf(., 4)
      }
      // compaction: nonzero lanes to slots 0..nnz-1 in scan order, zero lanes behind
      const int dst = 16 * gw + (level ? idx : nnz + (k - idx));
      const int lv = __builtin_amdgcn_ds_permute(4 * dst, level ? sl : 0);
      const int rv = __builtin_amdgcn_ds_permute(4 * dst, level ? run : 0);
      term += __shfl_xor(term, 8, 64);
      term += __shfl_xor(term, 4, 64);
      term += __shfl_xor(term, 2, 64);
      term += __shfl_xor(term, 1, 64);
      // the 4 blocks' level lists (17 dwords each, the entry past the last level 0) as one run
      const int v0 = __builtin_amdgcn_ds_bpermute(4 * (16 * lj + (lpos & 15)), lv);
      const int v1 = __builtin_amdgcn_ds_bpermute(4 * (16 * tj + (tpos & 15)), lv);
      if (live) {
        coef[(size_t)b * 16 + pq[u]] = deq;   // (0 where x was 0: every lane stores, whole lines)
        runs[(size_t)b * 16 + k] = rv;
        if (k == 0) {
          coeff_cost[b] = cc[u] + term;
          nonzero[b] = mg != 0;
        }
      }
      const int w0 = b4 + 4 * u;   // the wave's first block this round
      if (w0 + lj < n) levels[(size_t)w0 * 17 + lane] = lpos == 16 ? 0 : v0;
      if (lane < 4 && w0 + tj < n) levels[(size_t)w0 * 17 + 64 + lane] = tpos == 16 ? 0 : v1;
    }
  }
}

// residual_transform_quant_luma_4x4 (JM/lencod/src/block.c:660-724) of inter
// blocks, whole: check_zero, forward4x4, quant_4x4_normal, and -- when a level
// survives -- inverse4x4 and sample_reconstruct (lcommon/src/blk_prediction.c:48-62,
// dq_bits = DQ_BITS = 6), else the prediction copied.  One lane per block: the
// drop-in hands over the four 4x4 blocks of an 8x8 prediction at a time, so this
// is a latency path (a handful of blocks per launch), and the quantisation walks
// the scan in JM's order with JM's run counting.
__global__ __launch_bounds__(64) void residual4x4_kernel(const jmme_quant4x4_params *__restrict__ params,
                                                         const jmme_resid4x4_req *__restrict__ req,
                                                         jmme_resid4x4_res *__restrict__ res, int n) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= n) return;
  const jmme_resid4x4_req &q = req[b];
  jmme_resid4x4_res &o = res[b];
  int ores[16], coef[16];
  int any = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) { ores[k] = q.ores[k]; any |= ores[k]; }
  o.zero = any == 0;
  o.nonzero = 0;
  o.cost = 0;
  if (!any) {   // check_zero: no coefficients; JM stores ACLevel[0] = 0 and copies the prediction
    o.levels[0] = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) o.recon[k] = q.pred[k];
    return;
  }
  const jmme_quant4x4_params &P = params[q.param];
  transform_one<JMME_TF_FORWARD4x4>(ores, coef);
  const int qp_per = P.qp_per, q_bits = 15 + qp_per;   // Q_BITS, defines.h:311
  int run = 0, nl = 0, cost = 0, nonzero = 0;
  for (int c = 0; c < 16; ++c) {   // quant_4x4_normal, quant4x4_normal.c:68-106
    const int i = P.scan[c][0], j = P.scan[c][1], pos = 4 * j + i;
    const int v = coef[pos];
    if (v != 0) {
      int level = (abs(v) * P.scale[pos] + P.offset[pos]) >> q_bits;
      if (level != 0) {
        if (P.is_cavlc) level = min(level, 2063);   // CAVLC_LEVEL_LIMIT, defines.h:99
        cost += level > 1 ? 999999 : P.c_cost[run];   // MAX_VALUE, defines.h:123
        level = v < 0 ? -level : level;
        coef[pos] = ((level * P.inv_scale[pos] << qp_per) + 8) >> 4;   // rshift_rnd_sf(., 4)
        o.levels[nl] = level;
        o.runs[nl] = run;
        ++nl;
        run = 0;
        nonzero = 1;
      } else {
        coef[pos] = 0;
        ++run;
      }
    } else {
      ++run;
    }
  }
  o.levels[nl] = 0;
  o.cost = cost;
  o.nonzero = nonzero;
#pragma unroll
  for (int k = 0; k < 16; ++k) o.coef[k] = coef[k];
  if (nonzero) {
    int rres[16];
    transform_one<JMME_TF_INVERSE4x4>(coef, rres);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      o.rres[k] = rres[k];
      o.recon[k] = (jmme_imgpel)min(max(((rres[k] + 32) >> 6) + (int)q.pred[k], 0), q.max_pel);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) o.recon[k] = q.pred[k];
  }
}

int grid_for(int n, int per_wg = 64) {
  const int g = (n + per_wg - 1) / per_wg;
  return g < 1 ? 1 : (g > 8192 ? 8192 : g);
}

}  // namespace

hipError_t launch_transform(int op, const int32_t *in, int32_t *out, int n, hipStream_t s) {
  const int g = grid_for(n);
  if (op == JMME_TF_FORWARD8x8 || op == JMME_TF_INVERSE8x8) {
    const int g8 = grid_for(n, kWG8 / 8 * kU8);
    if (op == JMME_TF_FORWARD8x8) hipLaunchKernelGGL(transform8_kernel<JMME_TF_FORWARD8x8>, dim3(g8), dim3(kWG8), 0, s, in, out, n);
    else hipLaunchKernelGGL(transform8_kernel<JMME_TF_INVERSE8x8>, dim3(g8), dim3(kWG8), 0, s, in, out, n);
    return hipGetLastError();
  }
  switch (op) {
#define JMME_TF(OP) case OP: hipLaunchKernelGGL(transform_kernel<OP>, dim3(g), dim3(kTB), 0, s, in, out, n); break;
    JMME_TF(JMME_TF_FORWARD4x4) JMME_TF(JMME_TF_INVERSE4x4) JMME_TF(JMME_TF_HADAMARD4x4)
    JMME_TF(JMME_TF_IHADAMARD4x4) JMME_TF(JMME_TF_HADAMARD4x2) JMME_TF(JMME_TF_IHADAMARD4x2)
    JMME_TF(JMME_TF_HADAMARD2x2) JMME_TF(JMME_TF_IHADAMARD2x2)
#undef JMME_TF
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

int transform_elems(int op) { return (op < 0 || op > JMME_TF_INVERSE8x8) ? 0 : tf_elems(op); }

hipError_t launch_satd(int size, const int16_t *diff, int32_t *out, int n, hipStream_t s) {
  const int g = grid_for(n);
  if (size == 4) hipLaunchKernelGGL(satd_kernel<4>, dim3(g), dim3(kTB), 0, s, diff, out, n);
  else if (size == 8) hipLaunchKernelGGL(satd8_kernel, dim3(grid_for(n, kWG8 / 8 * kU8)), dim3(kWG8), 0, s, diff, out, n);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_quant4x4(const jmme_quant4x4_params *params, const int32_t *param_idx, int32_t *coef, int32_t *levels,
                           int32_t *runs, int32_t *coeff_cost, int32_t *nonzero, int n, hipStream_t s) {
  const int per_wg = kWG8 / 16 * (param_idx ? kUQ / 2 : kUQ), g = (n + per_wg - 1) / per_wg;
  const dim3 grid(g < 1 ? 1 : (g > 65536 ? 65536 : g));
  if (param_idx)
    hipLaunchKernelGGL(quant4x4_kernel<false>, grid, dim3(kWG8), 0, s, params, param_idx, coef, levels, runs,
                       coeff_cost, nonzero, n);
  else
    hipLaunchKernelGGL(quant4x4_kernel<true>, grid, dim3(kWG8), 0, s, params, param_idx, coef, levels, runs,
                       coeff_cost, nonzero, n);
  return hipGetLastError();
}

hipError_t launch_residual4x4(const jmme_quant4x4_params *params, const jmme_resid4x4_req *req,
                              jmme_resid4x4_res *res, int n, hipStream_t s) {
  hipLaunchKernelGGL(residual4x4_kernel, dim3((n + 63) / 64), dim3(64), 0, s, params, req, res, n);
  return hipGetLastError();
}

}  // namespace jmme
