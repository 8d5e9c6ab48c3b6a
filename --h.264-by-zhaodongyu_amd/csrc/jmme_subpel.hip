// jmme_subpel.hip -- gfx950 kernels for JM 18.5's quarter-pel reference
// interpolation and sub-pel motion refinement,
// JM = /root/reference/4.对比程序/jm18.5/JM:
//
//   getSubImagesLuma               JM/lencod/src/img_luma.c:611-680 (six-tap :151-431,
//                                  bilinear :448-600, taps img_luma.h:21)
//   sub_pel_motion_estimation      JM/lencod/src/me_fullsearch.c:186-289
//   EPZS_sub_pel_motion_estimation JM/lencod/src/me_epzs_sub.c:30-222 (tables me_epzs.h:23-42)
//   computeSAD / computeSSE / computeSATD, HadamardSAD4x4 / 8x8
//                                  JM/lencod/src/me_distortion.c:175-426, 745-825, 1189-1240
//   UMVLine4X                      JM/lencod/inc/refbuf.h:22-26
//
// Interpolation.  Every JM sub-image, including its padding, equals the
// filter evaluated on the edge-replicated picture (JM clamps each tap into
// the padded plane, whose border is itself a replica), so an 8 x 256 output
// tile needs only a 14 x 262 integer tile with clamped reads.  One thread
// makes 4 columns of two rows for all 16 sub-images: 28 horizontal six-tap
// sums shared by the two rows, 5 vertical ones and the (+512)>>10 centre
// sample per row, then the 12 bilinear averages, written as one dword (8-bit)
// or two (16-bit) per sub-image.  The kernel is a one-pass stream: 1 sample
// read, 16 written per padded sample (HBM roofline).
//
// Refinement.  One wave per 16 refinements; lane k < 16 owns refinement k and
// runs JM's control flow for it.  Each phase of JM's loop (the half-pel ring,
// the quarter-pel ring; EPZS: first ring, the next_start_pos..next_end_pos
// follow-up, for both levels) is costed for all 16 at once: the (candidate,
// 4x4 or 8x8 block) jobs of the 16 are dealt over the 64 lanes, pass after
// pass, and block sums are added into a per-(refinement, candidate) LDS
// slot; the owners then walk their candidates in JM's order with JM's
// comparisons.  JM's distortion functions stop early and return their bound
// T once the partial sum exceeds T >> 5; sums only grow, so that happens
// exactly when the full sum does, and the fold computes the same value:
// d = (sum > T >> 5) ? T : sum << 5.
#include <hip/hip_runtime.h>

#include "jmme.h"
#include "jmme_common.h"
#include "jmme_subpel_internal.h"
#include "jmme_refine_dev.h"

// Cache policy of the sub-image stores: sc0 | sc1 (system scope, written through
// rather than left dirty in L2).  A/B on the 1080p reference (tools/ab_interp.sh,
// two interleaved rounds, sub-image parity green in each, profiles/round5/interp/):
// default policy 9.9-10.0 us (47.5 % of 8 TB/s), nt 9.2 (51.5 %), sc1 8.9 (53 %),
// sc1 | nt 9.3-9.9, sc0 | nt 9.3, sc0 | sc1 8.8 us (53.7 %); the refinement that
// reads the sub-images after them is unchanged (0.200-0.202 ms per frame either way).
#ifndef JMME_INTERP_AUX
#define JMME_INTERP_AUX 17
#endif
#ifndef JMME_INTERP_ROWS
#define JMME_INTERP_ROWS 3   // (2: 13.7-14.2 us, 3: 11.6, 4: 12.8-13.0, 5: 12.0, 6: 13.0, 8: 15.2 us per 1080p reference)
#endif

namespace jmme {

namespace {

using namespace spd;   // kDistMax, kPad*, spiral_x/y, mv_cost, job_sum, dist, blk_size (jmme_subpel_dev.h)

__device__ __forceinline__ int clipv(int v, int maxv) { return min(max(v, 0), maxv); }   // iClip1(max_imgpel_value)
__device__ __forceinline__ int avg2(int a, int b) { return (a + b + 1) >> 1; }   // rshift_rnd_sf(a + b, 1)
__device__ __forceinline__ int six(int c, int d, int b, int e, int a, int f) {   // ONE_FOURTH_TAP {20, -5, 1}
  return 20 * (c + d) - 5 * (b + e) + (a + f);
}
__device__ __forceinline__ uint32_t pack4(int a, int b, int c, int d) {
  return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16) | ((uint32_t)d << 24);
}

// ------------------------------------------------------------ sub-images --
// A workgroup makes a 256 x 12 tile of every sub-image; a thread makes 4 columns
// of three consecutive rows, sharing the 8 rows of horizontal six-tap sums the three
// need (2.67 six-tap rows per output row; two rows needed 3.5, one row 6).  Four rows
// (2.25) issue fewer six-taps but leave 560 workgroups for 256 CUs against 746.
constexpr int kRowsT = JMME_INTERP_ROWS;   // output rows per thread
constexpr int kTileW = 256, kTileH = 4 * kRowsT, kSW = kTileW + 16, kSH = kTileH + 6;

// four samples of one row as written to a sub-image: one dword (8-bit) or two
// (16-bit samples, SourceBitDepthLuma 9..14)
template <typename T> struct Pack4;
template <> struct Pack4<uint8_t> {
  using V = uint32_t;
  __device__ static V make(int a, int b, int c, int d) { return pack4(a, b, c, d); }
};
template <> struct Pack4<uint16_t> {
  using V = uint2;
  __device__ static V make(int a, int b, int c, int d) {
    return make_uint2((uint32_t)a | ((uint32_t)b << 16), (uint32_t)c | ((uint32_t)d << 16));
  }
};

// ---- 8-bit: the six-taps two columns at a time in packed 16-bit lanes ------
// Every six-tap of 8-bit samples lies in [-2550, 10710] and fits an int16 lane,
// so the horizontal sums of columns (0, 1) and (2, 3), the vertical sums of
// raw samples and the (+16) >> 5 clips run as v_pk_* on pairs; only the centre
// plane's second pass (six-tap of the horizontal sums, up to ~4.3e5) needs 32
// bits.  The same values as the scalar form below, in the same order of the
// same integer operations (img_luma.c:151-431 getHor/Ver/VerTmp six-taps).
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2 as_s16x2(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
__device__ __forceinline__ uint32_t as_u32(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ s16x2 six2(s16x2 a, s16x2 b, s16x2 c, s16x2 d, s16x2 e, s16x2 f) {
  // 20 (c + d) - 5 (b + e) + (a + f), per 16-bit lane
  const s16x2 k20 = {20, 20}, k5 = {5, 5};
  return (c + d) * k20 - (b + e) * k5 + (a + f);
}
__device__ __forceinline__ s16x2 clip5(s16x2 x) {   // iClip1(255, (x + 16) >> 5) per lane
  const s16x2 k16 = {16, 16}, k0 = {0, 0}, k255 = {255, 255};
  const s16x2 y = (x + k16) >> 5;
  return __builtin_elementwise_min(__builtin_elementwise_max(y, k0), k255);
}
// bytes 0 and 2 of two packed pairs -> 4 samples (lo pair first)
__device__ __forceinline__ uint32_t pack_pairs(s16x2 lo, s16x2 hi) {
  return __builtin_amdgcn_perm(as_u32(hi), as_u32(lo), 0x06040200u);
}

// rows: the thread's staged rows (row 0 = picture row row0 - 2), pitch in bytes;
// a thread makes 4 columns of kRowsT output rows
// (8-bit rows are staged from the dword boundary 2 bytes below the tile's first
// sample: X0 - kPadX - 2 is 2 mod 4 for every tile)
static_assert(kTileW % 4 == 0 && ((-(kPadX + 2)) & 3) == 2, "8-bit staging offset");
__device__ __forceinline__ void interp_rows8(const uint8_t *rows, int pitch, int tx, int row0, int ph, uint8_t *dst,
                                             int dst_pitch, size_t plane_stride, int col) {
  constexpr int NR = kRowsT + 5;
  // the 12 bytes at the thread's dword: sample I[c] of the scalar form is byte c + 2
  uint32_t D1[NR], D2[NR];
  s16x2 h01[NR], h23[NR], r23[NR], r45[NR], r67[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(rows + (size_t)r * pitch) + tx;
    const uint32_t d0 = q[0], d1 = q[1], d2 = q[2];
    D1[r] = d1;
    D2[r] = d2;
    // P_j = (I_j, I_j+1) as two 16-bit lanes, I_j = byte j + 2 of d0:d1:d2
    const s16x2 P0 = as_s16x2(__builtin_amdgcn_perm(d1, d0, 0x0c030c02u));
    const s16x2 P1 = as_s16x2(__builtin_amdgcn_perm(d1, d0, 0x0c040c03u));
    const s16x2 P2 = as_s16x2(__builtin_amdgcn_perm(d1, d0, 0x0c050c04u));
    const s16x2 P3 = as_s16x2(__builtin_amdgcn_perm(d1, d0, 0x0c060c05u));
    const s16x2 P4 = as_s16x2(__builtin_amdgcn_perm(d1, d0, 0x0c070c06u));
    const s16x2 P5 = as_s16x2(__builtin_amdgcn_perm(d2, d1, 0x0c040c03u));
    const s16x2 P6 = as_s16x2(__builtin_amdgcn_perm(d2, d1, 0x0c050c04u));
    const s16x2 P7 = as_s16x2(__builtin_amdgcn_perm(d2, d1, 0x0c060c05u));
    h01[r] = six2(P0, P1, P2, P3, P4, P5);   // getHorSubImageSixTap, columns 0, 1 (imgY_sub_tmp)
    h23[r] = six2(P2, P3, P4, P5, P6, P7);   // columns 2, 3
    r23[r] = P2;                             // raw samples of columns 0..5 for the vertical taps
    r45[r] = P4;
    r67[r] = P6;
  }
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, -1, 0x00020000);
  const uint32_t off0 = (uint32_t)row0 * (uint32_t)dst_pitch + (uint32_t)col;
#pragma unroll
  for (int m = 0; m < kRowsT; ++m) {   // output row row0 + m: staged rows m .. m + 5
    if (row0 + m >= ph) break;
    auto sixv = [&](const s16x2 (&v)[NR]) { return six2(v[m], v[m + 1], v[m + 2], v[m + 3], v[m + 4], v[m + 5]); };
    const s16x2 v23 = clip5(sixv(r23)), v45 = clip5(sixv(r45)), v67 = clip5(sixv(r67));   // getVerSubImageSixTap
    const uint32_t P20 = pack_pairs(v23, v45);                                              // columns 0..3
    // columns 1..4: (v23.y, v45.x, v45.y) then v67.x
    const uint32_t P20n = __builtin_amdgcn_perm(as_u32(v67), __builtin_amdgcn_perm(as_u32(v45), as_u32(v23),
                                                                                  0x0c060402u), 0x04020100u);
    const uint32_t P02 = pack_pairs(clip5(h01[m + 2]), clip5(h23[m + 2]));                  // getHorSubImageSixTap, rounded
    const uint32_t Q02 = pack_pairs(clip5(h01[m + 3]), clip5(h23[m + 3]));
    // getVerSubImageSixTapTmp: the six-tap of the horizontal sums, 32-bit
    int s22[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int t[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const s16x2 hv = k < 2 ? h01[m + j] : h23[m + j];
        t[j] = (k & 1) ? (int)hv.y : (int)hv.x;
      }
      s22[k] = clipv((six(t[2], t[3], t[1], t[4], t[0], t[5]) + 512) >> 10, 255);
      // (kept out of a fused v_ashr_pk_u8_i32: packed with the next column's value
      // by that instruction, the upper half of its destination came out wrong --
      // sub-images 6, 9, 10, 11 and 14 differed from JM's)
      asm volatile("" : "+v"(s22[k]));
    }
    const uint32_t P00 = D1[m + 2];                                           // integer samples, columns 0..3
    const uint32_t P00n = __builtin_amdgcn_alignbyte(D2[m + 2], D1[m + 2], 1);   // columns 1..4
    const uint32_t Q00 = D1[m + 3];
    const uint32_t P22 = pack4(s22[0], s22[1], s22[2], s22[3]);
    auto L = [](uint32_t a, uint32_t b) { return __builtin_amdgcn_lerp(a, b, 0x01010101u); };
    uint32_t o[16];
    o[0] = P00; o[2] = P02; o[8] = P20; o[10] = P22;
    o[1] = L(P00, P02);     // [0][1] getSubImageBiLinear
    o[4] = L(P00, P20);     // [1][0]
    o[5] = L(P02, P20);     // [1][1]
    o[6] = L(P02, P22);     // [1][2]
    o[9] = L(P20, P22);     // [2][1]
    o[3] = L(P02, P00n);    // [0][3] getHorSubImageBiLinear
    o[7] = L(P02, P20n);    // [1][3]
    o[11] = L(P22, P20n);   // [2][3]
    o[12] = L(P20, Q00);    // [3][0] getVerSubImageBiLinear
    o[13] = L(P20, Q02);    // [3][1]
    o[14] = L(P22, Q02);    // [3][2]
    o[15] = L(Q02, P20n);   // [3][3] getDiagSubImageBiLinear
    const int vo = (int)(off0 + (uint32_t)m * (uint32_t)dst_pitch);
#pragma unroll
    for (int k = 0; k < 16; ++k)
      __builtin_amdgcn_raw_buffer_store_b32(o[k], rsrc, vo, (int)((uint32_t)k * (uint32_t)plane_stride), JMME_INTERP_AUX);
  }
}

// T = sample type; pitches and the plane stride in samples; maxv = max_imgpel_value
template <typename T>
__global__ __launch_bounds__(256) void sub_images_kernel(const T *__restrict__ src, int src_pitch, int W, int H,
                                                         T *__restrict__ dst, int dst_pitch, size_t plane_stride,
                                                         int pw, int ph, int maxv, int aligned) {
  // 8-bit: each row is staged from the dword boundary below its first sample
  // (sh = 2 bytes: X0 is a multiple of 256, kPadX + 2 = 34), so whole rows move as
  // aligned dwords when they lie inside the picture
  constexpr int kRowW = sizeof(T) == 1 ? kSW + 4 : kSW, kRowD = kRowW / 4;
  __shared__ __attribute__((aligned(16))) T S[kSH][kRowW];
  const int X0 = blockIdx.x * kTileW, Y0 = blockIdx.y * kTileH;   // padded output coordinates
  const int xs = X0 - kPadX - 2, sh = sizeof(T) == 1 ? xs & 3 : 0, xa = xs - sh;
  // S[r][c + sh] = picture sample (Y0 - kPadY - 2 + r, X0 - kPadX - 2 + c), clamped
  if (sizeof(T) == 1 && aligned && xa >= 0 && xa + 4 * kRowD <= W) {
    for (int k = threadIdx.x; k < kSH * kRowD; k += 256) {
      const int r = k / kRowD, q = k - r * kRowD;
      const int y = min(max(Y0 - kPadY - 2 + r, 0), H - 1);
      reinterpret_cast<uint32_t *>(S[r])[q] = *reinterpret_cast<const uint32_t *>(src + (size_t)y * src_pitch + xa + 4 * q);
    }
  } else {
    for (int k = threadIdx.x; k < kSH * kSW; k += 256) {
      const int r = k / kSW, c = k - r * kSW;
      const int y = min(max(Y0 - kPadY - 2 + r, 0), H - 1), x = min(max(xs + c, 0), W - 1);
      S[r][c + sh] = src[(size_t)y * src_pitch + x];
    }
  }
  __syncthreads();
  const int ty = threadIdx.x >> 6, tx = threadIdx.x & 63;   // a wave writes 256 contiguous samples per sub-image
  const int row0 = Y0 + kRowsT * ty, col = X0 + 4 * tx;
  if (row0 >= ph || col >= pw) return;
  if constexpr (sizeof(T) == 1) {
    interp_rows8(&S[kRowsT * ty][0], kRowW, tx, row0, ph, dst, dst_pitch, plane_stride, col);
    return;
  }
  int I[kRowsT + 5][9];   // I[dr + 2][dc + 2] = sample at (row0 + dr, col + dc)
#pragma unroll
  for (int r = 0; r < kRowsT + 5; ++r)
#pragma unroll
    for (int c = 0; c < 9; ++c) I[r][c] = S[kRowsT * ty + r][4 * tx + c + sh];
  // horizontal six-tap (getHorSubImageSixTap) at rows -2..4, columns 0..3: the
  // unrounded sums are p_Vid->imgY_sub_tmp
  int h[kRowsT + 5][4];
#pragma unroll
  for (int r = 0; r < kRowsT + 5; ++r)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      h[r][k] = six(I[r][k + 2], I[r][k + 3], I[r][k + 1], I[r][k + 4], I[r][k], I[r][k + 5]);
  using PK = Pack4<T>;
  // stores: a wave-uniform plane base (SGPRs) plus a 32-bit per-lane offset, so
  // each of the 16 stores per row is one global_store with a scalar base instead
  // of 64-bit address arithmetic per plane (a plane is < 4 GiB)
  // (a raw buffer over the 16 planes: the plane is the scalar soffset, the sample
  // the per-lane voffset; the 16 planes of one reference span < 4 GiB)
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, -1, 0x00020000);
  const uint32_t off0 = ((uint32_t)row0 * (uint32_t)dst_pitch + (uint32_t)col) * (uint32_t)sizeof(T);
  auto store = [&](int k, int m, typename Pack4<T>::V v) {
    const int vo = (int)(off0 + (uint32_t)m * (uint32_t)dst_pitch * (uint32_t)sizeof(T));
    const int so = (int)((uint32_t)k * (uint32_t)plane_stride * (uint32_t)sizeof(T));
    if constexpr (sizeof(T) == 1) __builtin_amdgcn_raw_buffer_store_b32(v, rsrc, vo, so, JMME_INTERP_AUX);
    else {
      typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
      __builtin_amdgcn_raw_buffer_store_b64(u32x2v{v.x, v.y}, rsrc, vo, so, JMME_INTERP_AUX);
    }
  };
#pragma unroll
  for (int m = 0; m < kRowsT; ++m) {   // output row row0 + m: input rows m .. m + 5
    if (row0 + m >= ph) break;
    int s00[2][5], s02[2][4], s20[5], s22[4];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      s00[0][k] = I[m + 2][k + 2];
      s00[1][k] = I[m + 3][k + 2];
      // getVerSubImageSixTap
      s20[k] = clipv((six(I[m + 2][k + 2], I[m + 3][k + 2], I[m + 1][k + 2], I[m + 4][k + 2], I[m][k + 2],
                          I[m + 5][k + 2]) + 16) >> 5, maxv);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s02[0][k] = clipv((h[m + 2][k] + 16) >> 5, maxv);
      s02[1][k] = clipv((h[m + 3][k] + 16) >> 5, maxv);
      // getVerSubImageSixTapTmp
      s22[k] = clipv((six(h[m + 2][k], h[m + 3][k], h[m + 1][k], h[m + 4][k], h[m][k], h[m + 5][k]) + 512) >> 10, maxv);
    }
    typename PK::V o[16];
    o[0] = PK::make(s00[0][0], s00[0][1], s00[0][2], s00[0][3]);
    o[2] = PK::make(s02[0][0], s02[0][1], s02[0][2], s02[0][3]);
    o[8] = PK::make(s20[0], s20[1], s20[2], s20[3]);
    o[10] = PK::make(s22[0], s22[1], s22[2], s22[3]);
    if constexpr (sizeof(T) == 1) {
      // 8-bit: the twelve bilinear planes straight from the packed ones, four
      // samples per v_lerp_u8 (per byte (a + b + 1) >> 1 = rshift_rnd_sf(a + b, 1))
      const uint32_t P00n = pack4(s00[0][1], s00[0][2], s00[0][3], s00[0][4]);
      const uint32_t Q00 = pack4(s00[1][0], s00[1][1], s00[1][2], s00[1][3]);
      const uint32_t Q02 = pack4(s02[1][0], s02[1][1], s02[1][2], s02[1][3]);
      const uint32_t P20n = pack4(s20[1], s20[2], s20[3], s20[4]);
      const uint32_t P00 = o[0], P02 = o[2], P20 = o[8], P22 = o[10];
      auto L = [](uint32_t a, uint32_t b) { return __builtin_amdgcn_lerp(a, b, 0x01010101u); };
      o[1] = L(P00, P02);     // [0][1] getSubImageBiLinear
      o[4] = L(P00, P20);     // [1][0]
      o[5] = L(P02, P20);     // [1][1]
      o[6] = L(P02, P22);     // [1][2]
      o[9] = L(P20, P22);     // [2][1]
      o[3] = L(P02, P00n);    // [0][3] getHorSubImageBiLinear
      o[7] = L(P02, P20n);    // [1][3]
      o[11] = L(P22, P20n);   // [2][3]
      o[12] = L(P20, Q00);    // [3][0] getVerSubImageBiLinear
      o[13] = L(P20, Q02);    // [3][1]
      o[14] = L(P22, Q02);    // [3][2]
      o[15] = L(Q02, P20n);   // [3][3] getDiagSubImageBiLinear
#pragma unroll
      for (int k = 0; k < 16; ++k) store(k, m, o[k]);
      continue;
    }
    int q[12][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      q[0][k] = avg2(s00[0][k], s02[0][k]);       // [0][1] getSubImageBiLinear
      q[1][k] = avg2(s00[0][k], s20[k]);          // [1][0]
      q[2][k] = avg2(s02[0][k], s20[k]);          // [1][1]
      q[3][k] = avg2(s02[0][k], s22[k]);          // [1][2]
      q[4][k] = avg2(s20[k], s22[k]);             // [2][1]
      q[5][k] = avg2(s02[0][k], s00[0][k + 1]);   // [0][3] getHorSubImageBiLinear
      q[6][k] = avg2(s02[0][k], s20[k + 1]);      // [1][3]
      q[7][k] = avg2(s22[k], s20[k + 1]);         // [2][3]
      q[8][k] = avg2(s20[k], s00[1][k]);          // [3][0] getVerSubImageBiLinear
      q[9][k] = avg2(s20[k], s02[1][k]);          // [3][1]
      q[10][k] = avg2(s22[k], s02[1][k]);         // [3][2]
      q[11][k] = avg2(s02[1][k], s20[k + 1]);     // [3][3] getDiagSubImageBiLinear
    }
    const int qi[12] = {1, 4, 5, 6, 9, 3, 7, 11, 12, 13, 14, 15};
#pragma unroll
    for (int j = 0; j < 12; ++j) o[qi[j]] = PK::make(q[j][0], q[j][1], q[j][2], q[j][3]);
#pragma unroll
    for (int k = 0; k < 16; ++k) store(k, m, o[k]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void subpel_kernel(SubpelParams p) {
  __shared__ WaveLds<T> lds[kWaves];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i0 = __builtin_amdgcn_readfirstlane((blockIdx.x * kWaves + wv) * p.per_wave);
  if (i0 >= p.n) return;
  refine_wave<T>(p, lds[wv], lane, i0);
}

}  // namespace

hipError_t launch_sub_images(const uint8_t *src, int src_pitch, int w, int h, uint8_t *dst, int dst_pitch,
                             size_t plane_stride, hipStream_t s, int bits) {
  const int pw = w + 2 * kPadX, ph = h + 2 * kPadY;
  // the stores address the 16 planes through one buffer resource with a 32-bit
  // voffset + soffset: the last plane's last row must lie below 4 GiB
  if ((15 * plane_stride + (size_t)ph * dst_pitch) * (bits > 8 ? 2 : 1) >= ((size_t)1 << 32))
    return hipErrorInvalidValue;
  dim3 grid((pw + kTileW - 1) / kTileW, (ph + kTileH - 1) / kTileH);
  if (bits > 8)
    hipLaunchKernelGGL(sub_images_kernel<uint16_t>, grid, dim3(256), 0, s, reinterpret_cast<const uint16_t *>(src),
                       src_pitch, w, h, reinterpret_cast<uint16_t *>(dst), dst_pitch, plane_stride, pw, ph,
                       (1 << bits) - 1, 0);
  else
    hipLaunchKernelGGL(sub_images_kernel<uint8_t>, grid, dim3(256), 0, s, src, src_pitch, w, h, dst, dst_pitch,
                       plane_stride, pw, ph, 255, (int)(((reinterpret_cast<uintptr_t>(src) | (uintptr_t)src_pitch) & 3) == 0));
  return hipGetLastError();
}

hipError_t launch_subpel(const SubpelParams &p, hipStream_t s) {
  if (p.n <= 0) return hipSuccess;
  // small batches (the drop-in's speculative ones) spread over more waves: the
  // wave's passes over its (candidate, block) jobs are the latency, so with
  // fewer owners per wave the chip finishes them sooner; full frames keep 16
  SubpelParams q = p;
  const int waves_wanted = 256 * 4 * 2;   // two waves per SIMD over 256 CUs
  q.per_wave = std::min(kK, std::max(1, (p.n + waves_wanted - 1) / waves_wanted));
  const int per_wg = kWaves * q.per_wave;
  if (p.hbd)
    hipLaunchKernelGGL(subpel_kernel<uint16_t>, dim3((p.n + per_wg - 1) / per_wg), dim3(256), 0, s, q);
  else
    hipLaunchKernelGGL(subpel_kernel<uint8_t>, dim3((p.n + per_wg - 1) / per_wg), dim3(256), 0, s, q);
  return hipGetLastError();
}

}  // namespace jmme
