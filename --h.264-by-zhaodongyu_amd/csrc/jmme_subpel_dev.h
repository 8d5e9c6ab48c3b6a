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

// spiral_search[0..8] (mv_search.c:406-442) as (x, y); spiral_hpel_search = 2x
__constant__ int8_t kSpiral9[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {1, 1}};

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

// ------------------------------------------------------------- refinement --
// EPZS search_point_qp[0..9] (me_epzs.h:42; search_point_hp = 2x), as (x, y)
__constant__ int8_t kEpzsPt[10][2] = {{0, 0}, {-1, 0}, {0, 1}, {1, 0}, {0, -1}, {-1, 1}, {1, 1}, {1, -1}, {-1, -1}, {-1, 1}};
// next_start_pos / next_end_pos (me_epzs.h:23-39), row-major
__constant__ int8_t kNextStart[25] = {0, 8, 5, 6, 7, 8, 0, 5, 8, 8, 5, 5, 0, 6, 5, 6, 6, 6, 0, 7, 7, 8, 7, 7, 0};
__constant__ int8_t kNextEnd[25] = {0, 10, 7, 8, 9, 10, 0, 6, 10, 9, 7, 6, 0, 7, 7, 8, 8, 7, 0, 8, 9, 9, 9, 8, 0};

__device__ __forceinline__ void wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

constexpr int kK = 16;        // refinements per wave (lanes 0..15 own one each)
constexpr int kWaves = 4;
constexpr int kMaxCand = 10;  // candidates of one phase (search_point tables: 10 entries)

// One phase's job description of request k, as the cooperating lanes read it.
// code: p0 [0,4) | lg_nb [4,7) | lg_nbx [8,10) | metric [12,14) | big 14 | sc [15,17) | tab 17
template <typename T>
struct WaveLds {
  int sums[kK][kMaxCand];
  int4 job[kK];                  // (mx, my, code, pos_x | pos_y << 16)
  const T *sub[kK];
};

// Per-request geometry the owner lane keeps.
template <typename T>
struct Own {
  int bsy, lg_nbx, pos_x, pos_y;
  const T *sub;
};

// One phase for the whole wave: owner lane k asks for the candidates at table
// positions [p0, p1) of table `tab` scaled by `sc` around padded (mx, my) with
// its metric; all 64 lanes share the (candidate, block) jobs of the 16
// requests, pass after pass, and add the block sums into sums[k][c].
template <typename T>
__device__ void run_phase(const SubpelParams &p, WaveLds<T> &L, int lane, const Own<T> &o, int p0, int p1, int metric,
                          bool t8, int sc, int tab, int mx, int my) {
  const bool big = metric == 2 && t8;
  const int lg_nbx = big ? o.lg_nbx - 1 : o.lg_nbx;
  const int lg_nb = lg_nbx + (big ? (o.bsy == 16 ? 1 : 0) : (o.bsy == 16 ? 2 : o.bsy == 8 ? 1 : 0));
  const int nc = (lane < kK && p1 > p0) ? p1 - p0 : 0;
  const int jobs = nc << lg_nb;
  if (lane < kK) {
    L.job[lane] = make_int4(mx, my, p0 | (lg_nb << 4) | (lg_nbx << 8) | (metric << 12) | ((int)big << 14) |
                                        (sc << 15) | (tab << 17),
                            o.pos_x | (o.pos_y << 16));
    L.sub[lane] = o.sub;
#pragma unroll
    for (int c = 0; c < kMaxCand; ++c) L.sums[lane][c] = 0;
  }
  // inclusive scan of the job counts over lanes 0..15
  int incl = jobs;
#pragma unroll
  for (int off = 1; off < kK; off <<= 1) {
    const int t = __shfl_up(incl, off, 64);
    if (lane >= off) incl += t;
  }
  const int total = __builtin_amdgcn_readlane(incl, kK - 1);
  int pre[kK];   // exclusive prefix (uniform)
#pragma unroll
  for (int m = 0; m < kK; ++m) pre[m] = __builtin_amdgcn_readlane(incl, m) - __builtin_amdgcn_readlane(jobs, m);
  wave_sync();
  const int ymax = p.height + 2 * kPadY - 1 - 16 - kPadY, xmax = p.width + 2 * kPadX - 1 - 16 - kPadX;
  for (int base = 0; base < total; base += 64) {
    const int j = base + lane;
    if (j < total) {
      int k = 0;
#pragma unroll
      for (int m = 1; m < kK; ++m) k += j >= pre[m];
      const int4 jb = L.job[k];
      const int e = j - pre[k];
      const int jl_nb = (jb.z >> 4) & 7, jl_nbx = (jb.z >> 8) & 3;
      const int c = e >> jl_nb, b = e & ((1 << jl_nb) - 1);
      const int jm = (jb.z >> 12) & 3;
      const bool jbig = (jb.z >> 14) & 1;
      const int jsc = (jb.z >> 15) & 3, pos = (jb.z & 15) + c;
      const int ox = ((jb.z >> 17) & 1) ? kEpzsPt[pos][0] : kSpiral9[pos][0];
      const int oy = ((jb.z >> 17) & 1) ? kEpzsPt[pos][1] : kSpiral9[pos][1];
      const int bs = jbig ? 8 : 4;
      const int bxo = (b & ((1 << jl_nbx) - 1)) * bs, byo = (b >> jl_nbx) * bs;
      const T *org = reinterpret_cast<const T *>(p.cur) + (size_t)(jb.w >> 16) * p.cur_pitch + (jb.w & 0xffff);
      const int s = job_sum(L.sub[k], p.plane_stride, p.sub_pitch, org, p.cur_pitch, ymax, xmax, jm, jbig,
                            jb.x + jsc * ox, jb.y + jsc * oy, bxo, byo);
      atomicAdd(&L.sums[k][c], s);
    }
  }
  wave_sync();
}

// One wave's refinements: lane k < p.per_wave owns request i0 + k (the body of
// subpel_kernel; the EPZS kernel's fused single-search path calls it with
// per_wave = 1, its own answer as ir_one and its request staged in LDS as req_one).
template <typename T>
__device__ __forceinline__ void refine_wave(const SubpelParams &p, WaveLds<T> &L, int lane, int i0,
                                            const jmme_block_res *ir_one = nullptr,
                                            const jmme_subpel_req *req_one = nullptr) {
  const int i = i0 + lane;
  // owner lanes: lane k < 16 holds request i0 + k; inactive owners ask for nothing
  jmme_subpel_req q{};
  bool act = false;
  if (lane < p.per_wave && i < p.n) {
    q = req_one ? *req_one : p.req[i];
    act = q.blocktype >= 1 && q.blocktype <= 7;
  }
  int mvx = q.mv_x, mvy = q.mv_y;
  int64_t min_mcost = q.min_mcost;
  if (act && (ir_one || p.int_res)) {
    const jmme_block_res ir = ir_one ? *ir_one : p.int_res[i];
    mvx = ir.mv_x;
    mvy = ir.mv_y;
    min_mcost = q.start_hp ? (int64_t)ir.cost : kDistMax;
  }
  Own<T> o;
  int bsx = 4;
  o.bsy = 4;
  if (act) blk_size(q.blocktype, bsx, o.bsy);
  o.lg_nbx = bsx == 16 ? 2 : bsx == 8 ? 1 : 0;
  o.pos_x = q.pos_x;
  o.pos_y = q.pos_y;
  o.sub = reinterpret_cast<const T *>(act ? p.subs[q.ref_slot] : p.subs[0]);
  const bool t8 = q.flags & JMME_SP_TEST8x8;
  const int pxp = q.pos_x << 2, pyp = q.pos_y << 2;   // pos_x_padded (mv_search.c:685-686)
  const int px = q.pred_x, py = q.pred_y;
  const bool epzs = q.variant == 1;
  const int *sums = L.sums[lane < kK ? lane : 0];
  int best_pos = 0, second_pos = 0;
  int64_t second_mcost = kDistMax;
  int lambda = q.lambda_h;
  // EPZS bookkeeping (me_epzs_sub.c:43-57)
  const int max_pos2 = epzs ? ((!q.start_hp || !q.start_qp) ? max(1, (int)q.search_pos2) : (int)q.search_pos2)
                            : (!q.start_hp ? max(1, (int)q.search_pos2) : (int)q.search_pos2);
  const int64_t sub_threshold = q.subthres + (int64_t)q.lambda_h * 2;
  bool early = false;
  const bool chk0 = (q.flags & JMME_SP_CHECK0) && (q.ref_slot & 31) == 0 && q.blocktype == 1 && mvx == 0 && mvy == 0;

  // ---- phase A: half-pel ring (me_fullsearch.c:221-250 | me_epzs_sub.c:66-88)
  {
    const int p1 = epzs ? min(5, max_pos2) : max_pos2;
    run_phase(p, L, lane, o, q.start_hp, act ? p1 : 0, q.metric_h, t8, 2, epzs, mvx + pxp, mvy + pyp);
    if (act) {
      for (int pos = q.start_hp; pos < p1; ++pos) {
        const int ox = epzs ? kEpzsPt[pos][0] : kSpiral9[pos][0], oy = epzs ? kEpzsPt[pos][1] : kSpiral9[pos][1];
        const int cx = mvx + 2 * ox, cy = mvy + 2 * oy;
        int64_t mcost = mv_cost(lambda, cx, cy, px, py);
        const int sm = sums[pos - q.start_hp];
        if (!epzs) {
          if (mcost >= min_mcost) continue;
          mcost += dist(sm, min_mcost - mcost);
          if (pos == 0 && chk0) mcost -= (int64_t)lambda * 16;   // weighted_cost(lambda_factor, 16)
          if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
        } else if (mcost < second_mcost) {
          mcost += dist(sm, second_mcost - mcost);
          if (mcost < min_mcost) {
            second_mcost = min_mcost; second_pos = best_pos; min_mcost = mcost; best_pos = pos;
          } else if (mcost < second_mcost) {
            second_mcost = mcost; second_pos = pos;
          }
        }
      }
      if (!epzs) {
        if (best_pos) { mvx += 2 * kSpiral9[best_pos][0]; mvy += 2 * kSpiral9[best_pos][1]; }
      } else {
        early = best_pos == 0 && px == mvx && py == mvy && min_mcost < sub_threshold;   // :90-93
      }
    }
  }
  // ---- phase B: EPZS half-pel follow-up (me_epzs_sub.c:96-127)
  {
    int s0 = 0, s1 = 0;
    if (act && epzs && !early && q.search_pos2 >= 9 && (best_pos != 0 || (abs(px - mvx) + abs(py - mvy)))) {
      s0 = kNextStart[best_pos * 5 + second_pos];
      s1 = kNextEnd[best_pos * 5 + second_pos];
    }
    run_phase(p, L, lane, o, s0, s1, q.metric_h, t8, 2, 1, mvx + pxp, mvy + pyp);
    if (act && epzs && !early) {
      for (int pos = s0; pos < s1; ++pos) {
        const int cx = mvx + 2 * kEpzsPt[pos][0], cy = mvy + 2 * kEpzsPt[pos][1];
        int64_t mcost = mv_cost(lambda, cx, cy, px, py);
        if (mcost < min_mcost) {
          mcost += dist(sums[pos - s0], min_mcost - mcost);
          if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
        }
      }
      if (best_pos) { mvx += 2 * kEpzsPt[best_pos][0]; mvy += 2 * kEpzsPt[best_pos][1]; }
    }
  }
  // ---- phase C: quarter-pel ring (me_fullsearch.c:252-282 | me_epzs_sub.c:135-172)
  lambda = q.lambda_q;
  {
    int p1 = 0;
    if (act && !early) {
      if (!epzs) {
        if (!q.start_qp) min_mcost = kDistMax;
        best_pos = 0;
        p1 = q.search_pos4;
      } else {
        p1 = (min_mcost < sub_threshold) ? 1 : 5;
        second_mcost = kDistMax;
        if (!q.start_qp) { best_pos = -1; min_mcost = kDistMax; } else best_pos = 0;
      }
    }
    run_phase(p, L, lane, o, q.start_qp, p1, q.metric_q, t8, 1, epzs, mvx + pxp, mvy + pyp);
    if (act && !early) {
      for (int pos = q.start_qp; pos < p1; ++pos) {
        const int ox = epzs ? kEpzsPt[pos][0] : kSpiral9[pos][0], oy = epzs ? kEpzsPt[pos][1] : kSpiral9[pos][1];
        const int cx = mvx + ox, cy = mvy + oy;
        int64_t mcost = mv_cost(lambda, cx, cy, px, py);
        const int sm = sums[pos - q.start_qp];
        if (!epzs) {
          if (mcost >= min_mcost) continue;
          mcost += dist(sm, min_mcost - mcost);
          if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
        } else if (mcost < second_mcost) {
          mcost += dist(sm, second_mcost - mcost);
          if (mcost < min_mcost) {
            second_mcost = min_mcost; second_pos = best_pos; min_mcost = mcost; best_pos = pos;
          } else if (mcost < second_mcost) {
            second_mcost = mcost; second_pos = pos;
          }
        }
      }
      if (!epzs && best_pos) { mvx += kSpiral9[best_pos][0]; mvy += kSpiral9[best_pos][1]; }
    }
  }
  // ---- phase D: EPZS quarter-pel follow-up (me_epzs_sub.c:175-210)
  {
    int s0 = 0, s1 = 0;
    const bool go = act && epzs && !early && min_mcost > sub_threshold &&
                    (best_pos != 0 || (abs(px - mvx) + abs(py - mvy)));
    if (go) {
      // JM reads next_start_pos[best][second] with second possibly -1 (start_qp 0):
      // row-major [best-1][4], or, for best 0, the zero padding before the
      // tables in JM's build (see oracle/subpel_oracle.c) -> an empty loop
      const int k = best_pos * 5 + second_pos;
      s0 = k >= 0 ? kNextStart[k] : 0;
      s1 = k >= 0 ? kNextEnd[k] : 0;
    }
    run_phase(p, L, lane, o, s0, s1, q.metric_q, t8, 1, 1, mvx + pxp, mvy + pyp);
    if (go) {
      for (int pos = s0; pos < s1; ++pos) {
        const int cx = mvx + kEpzsPt[pos][0], cy = mvy + kEpzsPt[pos][1];
        int64_t mcost = mv_cost(lambda, cx, cy, px, py);
        if (mcost < min_mcost) {
          mcost += dist(sums[pos - s0], min_mcost - mcost);
          if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
        }
      }
    }
    if (act && epzs && !early && best_pos > 0) { mvx += kEpzsPt[best_pos][0]; mvy += kEpzsPt[best_pos][1]; }
  }
  if (act) {
    jmme_block_res r;
    r.mv_x = (int16_t)mvx;
    r.mv_y = (int16_t)mvy;
    r.reserved = 0;
    r.cost = min_mcost;
    p.out[i] = r;
  }
}

}  // namespace
}  // namespace spd
}  // namespace jmme
