// jmme_refine_dev.h -- JM's sub-pel refinement as device code, shared by the
// batched refinement kernel (jmme_subpel.hip subpel_kernel, 16 requests a
// wave) and the EPZS kernels' refinement of their own answer (jmme_epzs*.hip):
// sub_pel_motion_estimation (JM/lencod/src/me_fullsearch.c:186-289) and
// EPZS_sub_pel_motion_estimation (JM/lencod/src/me_epzs_sub.c:30-222).
// (Kept out of jmme_subpel_dev.h, which the item kernels include too.)
#pragma once
#include "jmme_subpel_dev.h"

namespace jmme {
namespace spd {
namespace {

// ------------------------------------------------------------- refinement --
// EPZS search_point_qp[0..9] (me_epzs.h:42; search_point_hp = 2x), as (x, y)
constexpr int8_t kEpzsPtTab[10][2] = {{0, 0}, {-1, 0}, {0, 1}, {1, 0}, {0, -1}, {-1, 1}, {1, 1}, {1, -1}, {-1, -1}, {-1, 1}};
constexpr uint32_t kEpzsX = pack_axis2(kEpzsPtTab, 0), kEpzsY = pack_axis2(kEpzsPtTab, 1);
__device__ __forceinline__ int ept_x(int i) { return (int)((kEpzsX >> (2 * i)) & 3u) - 1; }
__device__ __forceinline__ int ept_y(int i) { return (int)((kEpzsY >> (2 * i)) & 3u) - 1; }
// search point i of table `tab` (1: EPZS search_point_qp, 0: the spiral)
__device__ __forceinline__ int tab_x(int tab, int i) { return tab ? ept_x(i) : spiral_x(i); }
__device__ __forceinline__ int tab_y(int tab, int i) { return tab ? ept_y(i) : spiral_y(i); }
// next_start_pos / next_end_pos (me_epzs.h:23-39), row-major
constexpr int8_t kNextStartTab[25] = {0, 8, 5, 6, 7, 8, 0, 5, 8, 8, 5, 5, 0, 6, 5, 6, 6, 6, 0, 7, 7, 8, 7, 7, 0};
constexpr int8_t kNextEndTab[25] = {0, 10, 7, 8, 9, 10, 0, 6, 10, 9, 7, 6, 0, 7, 7, 8, 8, 7, 0, 8, 9, 9, 9, 8, 0};
// four bits an entry: entries 0..15 in the first word, 16..24 in the second
constexpr uint64_t pack_nib(const int8_t (&t)[25], int lo) {
  uint64_t v = 0;
  for (int i = lo; i < 25 && i < lo + 16; ++i) v |= (uint64_t)t[i] << (4 * (i - lo));
  return v;
}
constexpr uint64_t kNS0 = pack_nib(kNextStartTab, 0), kNS1 = pack_nib(kNextStartTab, 16);
constexpr uint64_t kNE0 = pack_nib(kNextEndTab, 0), kNE1 = pack_nib(kNextEndTab, 16);
__device__ __forceinline__ int next_start(int k) { return (int)(((k < 16 ? kNS0 >> (4 * k) : kNS1 >> (4 * (k - 16)))) & 15u); }
__device__ __forceinline__ int next_end(int k) { return (int)(((k < 16 ? kNE0 >> (4 * k) : kNE1 >> (4 * (k - 16)))) & 15u); }

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
      const int ox = tab_x((jb.z >> 17) & 1, pos), oy = tab_y((jb.z >> 17) & 1, pos);
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

// ---------------------------------------------- one refinement from LDS --
// A refinement alone (the EPZS server's searches alone) is a chain of four
// dependent phases; read from the sub-images each is a memory round trip.
// Every candidate of the four phases lies within +-3 qpel of the integer
// answer (half-pel ring and follow-up +-2, quarter-pel ring and follow-up +-1
// around the half-pel winner), so the samples any of them reads -- through
// UMVLine4X's clamp of a block origin, or of each transform block's origin for
// SATD -- lie in a window of (bsy + 2) rows x (bsx + 2) samples of each of the
// 16 sub-images, starting at the clamped position of (mv - 3 qpel): clamping
// is monotone, so every clamped origin is at or after that one, and at most
// 2 + bs - 4 past it.  That window (and the current block) is loaded once into
// LDS, one round trip, and the four phases read LDS.
template <typename T>
struct TileLds {
  static constexpr int kND = sizeof(T) == 1 ? 6 : 10;   // dwords of a window row (any alignment)
  uint32_t t[16][18][kND];                               // [sub-image][row][dword]
  uint32_t org[16][8];                                   // the current block, bsx * sizeof(T) / 4 dwords a row
  int sums[kMaxCand];
  int ylo, d0, th;                                       // window origin: clamped row, first dword; rows
};

// 4 samples at padded column X of tile row `row` (the window's first dword d0)
__device__ __forceinline__ uint32_t tile4(const uint32_t *row, int d0, int X) {
  const int off = X - 4 * d0;
  return __builtin_amdgcn_alignbyte(row[(off >> 2) + 1], row[off >> 2], (uint32_t)(off & 3));
}
__device__ __forceinline__ void tile4(const uint32_t *row, int d0, int X, int (&v)[4]) {   // 16-bit samples
  const int off = 2 * X - 4 * d0;
  const int dw = off >> 2;
  const uint32_t sh = (uint32_t)(off & 2);
  const uint32_t a = __builtin_amdgcn_alignbyte(row[dw + 1], row[dw], sh), b = __builtin_amdgcn_alignbyte(row[dw + 2], row[dw + 1], sh);
  v[0] = (int)(a & 0xffff); v[1] = (int)(a >> 16); v[2] = (int)(b & 0xffff); v[3] = (int)(b >> 16);
}

// job_sum with the reference and the current block from the window
template <typename T>
__device__ __forceinline__ int tile_sum(const TileLds<T> &W, int ymax, int xmax, int metric, bool big, int cx, int cy,
                                        int bxo, int byo) {
  const int pl = ((cy & 3) << 2) | (cx & 3);
  int yy, xx;
  if (metric == 2) {
    yy = min(max((cy + (byo << 2)) >> 2, -kPadY), ymax);
    xx = min(max((cx + (bxo << 2)) >> 2, -kPadX), xmax);
  } else {
    yy = min(max(cy >> 2, -kPadY), ymax) + byo;
    xx = min(max(cx >> 2, -kPadX), xmax) + bxo;
  }
  const int ty = yy - W.ylo, X = xx + kPadX;
  constexpr int kS = sizeof(T) == 1 ? 4 : 2;   // samples per org dword
  auto org4 = [&](int r, int c, int (&a)[4]) {   // current block samples (r, c..c+3)
    if constexpr (sizeof(T) == 1) {
      const uint32_t d = W.org[byo + r][(bxo + c) / kS];
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] = (int)((d >> (8 * k)) & 255);
    } else {
      const uint32_t d0 = W.org[byo + r][(bxo + c) / kS], d1 = W.org[byo + r][(bxo + c) / kS + 1];
      a[0] = (int)(d0 & 0xffff); a[1] = (int)(d0 >> 16); a[2] = (int)(d1 & 0xffff); a[3] = (int)(d1 >> 16);
    }
  };
  auto ref4t = [&](int r, int c, int (&w)[4]) {
    const uint32_t *row = W.t[pl][ty + r];
    if constexpr (sizeof(T) == 1) {
      const uint32_t d = tile4(row, W.d0, X + c);
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = (int)((d >> (8 * k)) & 255);
    } else {
      tile4(row, W.d0, X + c, w);
    }
  };
  int s = 0;
  if (metric == 0 && sizeof(T) == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      s = __builtin_amdgcn_sad_u8(tile4(W.t[pl][ty + r], W.d0, X), W.org[byo + r][bxo / 4], s);
  } else if (metric <= 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int a[4], w[4];
      org4(r, 0, a);
      ref4t(r, 0, w);
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
      org4(r, 0, a);
      ref4t(r, 0, w);
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
        org4(r, 4 * h, a);
        ref4t(r, 4 * h, w);
#pragma unroll
        for (int k = 0; k < 4; ++k) d[8 * r + 4 * h + k] = a[k] - w[k];
      }
    }
    s = (had8_sum(d) + 2) >> 2;
  }
  return s;
}

// the window of a refinement alone (wave-uniform arguments): sub-images `sub`,
// block (pos_x, pos_y) bsx x bsy, integer answer (mvx, mvy) qpel, and the
// current block as the search staged it in LDS (cur: bsx * sizeof(T) / 4 dwords
// a row).  Always 18 rows of every sub-image (clamped into the padded plane),
// so the lane -> (sub-image, row, dword) map has constant divisors and every
// load of the window is issued before the first is waited for.
template <typename T>
__device__ __forceinline__ void tile_load(const SubpelParams &p, TileLds<T> &W, int lane, const T *sub,
                                          const uint32_t *cur, int pos_x, int pos_y, int bsx, int bsy, int mvx,
                                          int mvy) {
  constexpr int kND = TileLds<T>::kND, kPer = 18 * kND, kIt = 16 * kPer / 64;
  static_assert(16 * kPer % 64 == 0, "whole wave passes");
  const int ymax = p.height + 2 * kPadY - 1 - 16 - kPadY, xmax = p.width + 2 * kPadX - 1 - 16 - kPadX;
  const int ylo = min(max(((pos_y << 2) + mvy - 3) >> 2, -kPadY), ymax);
  const int xlo = min(max(((pos_x << 2) + mvx - 3) >> 2, -kPadX), xmax);
  const int PC0 = xlo + kPadX;
  const int d0 = sizeof(T) == 1 ? PC0 >> 2 : PC0 >> 1;
  const int last_row = p.height + 2 * kPadY - 1;                       // padded rows of a sub-image
  const int last_dw = (int)((size_t)p.sub_pitch * sizeof(T) / 4) - 1;   // dwords of a padded row
  const uint32_t *base = reinterpret_cast<const uint32_t *>(sub);
  const uint32_t ps_dw = (uint32_t)(p.plane_stride * sizeof(T) / 4), sp_dw = (uint32_t)(p.sub_pitch * sizeof(T) / 4);
  uint32_t v[kIt];
#pragma unroll
  for (int k = 0; k < kIt; ++k) {
    const int i = lane + 64 * k, pl = i / kPer, rem = i - pl * kPer, r = rem / kND, d = rem - r * kND;
    const int row = min(ylo + kPadY + r, last_row), dw = min(d0 + d, last_dw);
    v[k] = base[(size_t)pl * ps_dw + (uint32_t)row * sp_dw + (uint32_t)dw];
  }
  const int nd = bsx * (int)sizeof(T) / 4;   // the current block, from the search's copy
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = lane + 64 * k;
    if (i < nd * bsy) {
      const int r = i / nd, c = i - r * nd;
      W.org[r][c] = cur[i];
    }
  }
  uint32_t *t = &W.t[0][0][0];
#pragma unroll
  for (int k = 0; k < kIt; ++k) t[lane + 64 * k] = v[k];
  if (lane == 0) {
    W.ylo = ylo;
    W.d0 = d0;
    W.th = bsy + 2;
  }
  wave_sync();
}

// The 8x8 SATD jobs of a phase (computeSATD with test8x8, HadamardSAD8x8),
// eight lanes to a job: lane r of a group takes row r of the difference, its
// 8-point Hadamard in the lane, then the column transform across the group's
// lanes by DPP -- the mirror partner 7 - lane first (low half: a + b, high
// half: b - a), then lane ^ 1 and lane ^ 2: that column map is, row for row,
// +-1 times a distinct row of the 8x8 Hadamard (checked exhaustively on its
// matrix; with the mirror last it is not), so the sum of magnitudes is
// HadamardSAD8x8's -- and the group's sum.
// A job in one lane is ~700 VALU on 20 of 64 lanes; this is ~130 on all of them.
__device__ __forceinline__ int dpp_xor1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, true); }
__device__ __forceinline__ int dpp_xor2(int v) { return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, true); }
__device__ __forceinline__ int dpp_mirror8(int v) { return __builtin_amdgcn_mov_dpp(v, 0x141, 0xf, 0xf, true); }
template <typename T>
__device__ __forceinline__ void tile_satd8(TileLds<T> &W, int lane, int ymax, int xmax, int jobs, int lg_nb, int lg_nbx,
                                           int p0, int tab, int sc, int mx, int my) {
  const int g = lane >> 3, r = lane & 7;
  for (int base = 0; base < jobs; base += 8) {
    const int j = min(base + g, jobs - 1);   // (a group past the last job redoes it and adds nothing)
    const int c = j >> lg_nb, b = j & ((1 << lg_nb) - 1), pos = p0 + c;
    const int ox = tab_x(tab, pos), oy = tab_y(tab, pos);
    const int bxo = (b & ((1 << lg_nbx) - 1)) * 8, byo = (b >> lg_nbx) * 8;
    const int cx = mx + sc * ox, cy = my + sc * oy;
    const int pl = ((cy & 3) << 2) | (cx & 3);
    const int yy = min(max((cy + (byo << 2)) >> 2, -kPadY), ymax), xx = min(max((cx + (bxo << 2)) >> 2, -kPadX), xmax);
    const uint32_t *row = W.t[pl][yy - W.ylo + r];
    const int X = xx + kPadX;
    int d[8];
    if constexpr (sizeof(T) == 1) {
      const uint32_t w0 = tile4(row, W.d0, X), w1 = tile4(row, W.d0, X + 4);
      const uint32_t a0 = W.org[byo + r][bxo / 4], a1 = W.org[byo + r][bxo / 4 + 1];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        d[k] = (int)((a0 >> (8 * k)) & 255) - (int)((w0 >> (8 * k)) & 255);
        d[4 + k] = (int)((a1 >> (8 * k)) & 255) - (int)((w1 >> (8 * k)) & 255);
      }
    } else {
      int w[8];
      tile4(row, W.d0, X, *reinterpret_cast<int(*)[4]>(&w[0]));
      tile4(row, W.d0, X + 4, *reinterpret_cast<int(*)[4]>(&w[4]));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t a = W.org[byo + r][bxo / 2 + k];
        d[2 * k] = (int)(a & 0xffff) - w[2 * k];
        d[2 * k + 1] = (int)(a >> 16) - w[2 * k + 1];
      }
    }
#pragma unroll
    for (int h = 1; h < 8; h <<= 1)   // the row
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (!(i & h)) {
          const int u = d[i], v = d[i + h];
          d[i] = u + v;
          d[i + h] = u - v;
        }
    const bool lo1 = !(r & 1), lo2 = !(r & 2), lo4 = r < 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {   // the column, across the group: the mirror first (see above)
      int v = d[i], pv = dpp_mirror8(v);
      v = lo4 ? v + pv : pv - v;
      pv = dpp_xor1(v);
      v = lo1 ? v + pv : pv - v;
      pv = dpp_xor2(v);
      d[i] = lo2 ? v + pv : pv - v;
    }
    int s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += abs(d[i]);
    s += dpp_xor1(s);
    s += dpp_xor2(s);
    s += dpp_mirror8(s);
    if (r == 0 && base + g < jobs) atomicAdd(&W.sums[c], (s + 2) >> 2);
  }
  wave_sync();
}

// one phase of lane 0's request from the window: candidates [p0, p1) of table
// `tab` scaled by sc around padded (mx, my), all 64 lanes on its (candidate,
// block) jobs; sums[c] as run_phase leaves them
template <typename T>
__device__ void tile_phase(const SubpelParams &p, TileLds<T> &W, int lane, int bsx, int bsy, int p0, int p1,
                           int metric, bool t8, int sc, int tab, int mx, int my) {
  const bool big = metric == 2 && t8;
  const int lg_nbx = big ? (bsx == 16 ? 1 : 0) : (bsx == 16 ? 2 : bsx == 8 ? 1 : 0);
  const int lg_nb = lg_nbx + (big ? (bsy == 16 ? 1 : 0) : (bsy == 16 ? 2 : bsy == 8 ? 1 : 0));
  const int nc = p1 > p0 ? p1 - p0 : 0, jobs = nc << lg_nb;
  if (lane < kMaxCand) W.sums[lane] = 0;
  wave_sync();
  const int ymax = p.height + 2 * kPadY - 1 - 16 - kPadY, xmax = p.width + 2 * kPadX - 1 - 16 - kPadX;
  const int bs = big ? 8 : 4;
  if (big) {   // 8x8 SATD: eight lanes a job, one row each
    tile_satd8(W, lane, ymax, xmax, jobs, lg_nb, lg_nbx, p0, tab, sc, mx, my);
    return;
  }
  for (int j = lane; j < jobs; j += 64) {
    const int c = j >> lg_nb, b = j & ((1 << lg_nb) - 1), pos = p0 + c;
    const int ox = tab_x(tab, pos), oy = tab_y(tab, pos);
    const int bxo = (b & ((1 << lg_nbx) - 1)) * bs, byo = (b >> lg_nbx) * bs;
    atomicAdd(&W.sums[c], tile_sum(W, ymax, xmax, metric, big, mx + sc * ox, my + sc * oy, bxo, byo));
  }
  wave_sync();
}

// The first (cost, lane) minimum over lanes 0..15 of the wave (lanes >= n, and
// lanes whose `live` is false, hold no candidate): every lane gets the cost and
// the lane.  A fold of JM's refinement walks its candidates in order with strict
// `<` and an early-exit distortion that returns the running bound exactly when the
// full cost exceeds it (dist(), jmme_subpel_dev.h), so its minimum is this
// lexicographic one over the full costs (me_epzs_sub.c:66-88, 96-127, 150-172,
// 175-210).  Four butterfly steps instead of a dependent compare per candidate.
template <int CTRL>
__device__ __forceinline__ void argmin_step(int64_t &v, int &k) {
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)((uint64_t)v >> 32), CTRL, 0xf, 0xf, true);
  const int ok = __builtin_amdgcn_mov_dpp(k, CTRL, 0xf, 0xf, true);
  const int64_t ov = (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  const bool take = ov < v || (ov == v && ok < k);
  v = take ? ov : v;
  k = take ? ok : k;
}

__device__ __forceinline__ void wave_argmin16(int64_t c, bool live, int lane, int64_t &cmin, int &kmin) {
  int64_t v = live ? c : INT64_MAX;
  int k = live ? lane : 64;
  // DPP within each row of 16 lanes: lane ^ 1, lane ^ 2 (quad_perm), then the
  // half-row mirror (i <-> 7 - i) and the row mirror (i <-> 15 - i) pair the
  // quads and the halves: after the four steps every lane of row 0 holds its minimum
  argmin_step<0xB1>(v, k);
  argmin_step<0x4E>(v, k);
  argmin_step<0x141>(v, k);
  argmin_step<0x140>(v, k);
  cmin = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32)) << 32) |
                   (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v));
  kmin = __builtin_amdgcn_readfirstlane(k);
}

// a wave-uniform copy of v (lane 0's), dword by dword into SGPRs
template <typename S>
__device__ __forceinline__ S uni(const S &v) {
  static_assert(sizeof(S) % 4 == 0, "whole dwords");
  uint32_t w[sizeof(S) / 4];
  __builtin_memcpy(w, &v, sizeof(S));
#pragma unroll
  for (int k = 0; k < (int)(sizeof(S) / 4); ++k) w[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)w[k]);
  S r;
  __builtin_memcpy(&r, w, sizeof(S));
  return r;
}

// One wave's refinements: lane k < p.per_wave owns request i0 + k (the body of
// subpel_kernel; the EPZS kernel's fused single-search path calls it with
// per_wave = 1, its own answer as ir_one and its request staged in LDS as req_one).
// With a window W (per_wave = 1 only), the phases read the window above, which
// the caller has loaded (tile_load) for this request's integer answer.
template <typename T, bool TILE = false>
__device__ __forceinline__ void refine_wave(const SubpelParams &p, WaveLds<T> &L, int lane, int i0,
                                            const jmme_block_res *ir_one = nullptr,
                                            const jmme_subpel_req *req_one = nullptr, TileLds<T> *W = nullptr,
                                            unsigned long long *stamps = nullptr) {
  const int i = i0 + lane;
  // owner lanes: lane k < 16 holds request i0 + k; inactive owners ask for nothing.
  // With a window (one request), every lane holds it, read into SGPRs: the folds
  // below are then scalar code with scalar branches, not one lane's VALU chain
  jmme_subpel_req q{};
  bool act = false;
  if constexpr (TILE) {
    q = uni(*req_one);
    act = i0 < p.n && q.blocktype >= 1 && q.blocktype <= 7;
  } else if (lane < p.per_wave && i < p.n) {
    q = req_one ? *req_one : p.req[i];
    act = q.blocktype >= 1 && q.blocktype <= 7;
  }
  int mvx = q.mv_x, mvy = q.mv_y;
  int64_t min_mcost = q.min_mcost;
  if (act && (ir_one || p.int_res)) {
    const jmme_block_res ir = TILE ? uni(*ir_one) : ir_one ? *ir_one : p.int_res[i];
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
  if constexpr (!TILE) o.sub = reinterpret_cast<const T *>(act ? p.subs[q.ref_slot] : p.subs[0]);
  const bool t8 = q.flags & JMME_SP_TEST8x8;
  const int pxp = q.pos_x << 2, pyp = q.pos_y << 2;   // pos_x_padded (mv_search.c:685-686)
  const int px = q.pred_x, py = q.pred_y;
  const bool epzs = q.variant == 1;
  const int *sums_p = TILE ? W->sums : L.sums[lane < kK ? lane : 0];
  int sums_off = 0;   // (window: where this phase's candidates start in the sums computed)
  int sv = 0;         // (window: lane k holds the pass's sum of position c_p0 + k, read once per pass)
  auto sums = [&](int k) -> int {   // a phase's sum of candidate k (a scalar with a window)
    if constexpr (TILE) return __builtin_amdgcn_readlane(sv, k + sums_off);
    else return sums_p[k];
  };
  // what the window's sums hold: positions [c_p0, kMaxCand) of table 1 around (c_mx, c_my) with metric
  // c_metric and scale c_sc (c_p0 < 0: nothing kept)
  int c_p0 = -1, c_metric = -1, c_sc = -1, c_mx = 0, c_my = 0, npass = 0;
  // a phase: the 16-per-wave form, or the request from its window.  With a window,
  // a phase on EPZS's search_point table costs every later position of the table
  // too (the same centre, metric and scale), so the follow-up phase after it
  // (me_epzs_sub.c:96-127, 175-210: positions next_start..next_end around the
  // same centre) reads sums already made: two passes instead of four
  auto phase = [&](int a0, int a1, int metric, bool t8v, int sc, int tab, int mx, int my) {
    if constexpr (TILE) {
      if (a1 <= a0) return;   // (no candidates: the fold below reads nothing)
      if (tab == 1 && c_p0 >= 0 && a0 >= c_p0 && a1 <= kMaxCand && metric == c_metric && sc == c_sc && mx == c_mx &&
          my == c_my) {
        sums_off = a0 - c_p0;
        return;
      }
      const int e1 = tab == 1 ? kMaxCand : a1;
      tile_phase(p, *W, lane, bsx, o.bsy, a0, e1, metric, t8v, sc, tab, mx, my);
      sv = sums_p[lane < kMaxCand ? lane : 0];   // (the fold reads them by readlane, not one LDS trip each)
      if (stamps) {   // (pass ends; constant indices: a computed one puts the array in scratch)
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        if (npass == 0) stamps[4] = t;
        else stamps[5] = t;
      }
      ++npass;
      sums_off = 0;
      c_p0 = tab == 1 ? a0 : -1;
      c_metric = metric;
      c_sc = sc;
      c_mx = mx;
      c_my = my;
    } else {
      run_phase(p, L, lane, o, a0, a1, metric, t8v, sc, tab, mx, my);
    }
  };
  int best_pos = 0, second_pos = 0;
  int64_t second_mcost = kDistMax;
  int lambda = q.lambda_h;
  // EPZS bookkeeping (me_epzs_sub.c:43-57)
  const int max_pos2 = epzs ? ((!q.start_hp || !q.start_qp) ? max(1, (int)q.search_pos2) : (int)q.search_pos2)
                            : (!q.start_hp ? max(1, (int)q.search_pos2) : (int)q.search_pos2);
  const int64_t sub_threshold = q.subthres + (int64_t)q.lambda_h * 2;
  bool early = false;
  const bool chk0 = (q.flags & JMME_SP_CHECK0) && (q.ref_slot & 31) == 0 && q.blocktype == 1 && mvx == 0 && mvy == 0;
  // (window, EPZS) a phase's candidates pos in [a0, a1) of the search_point table, lane k = pos - a0:
  // their full costs, mv cost + sum << 5, with the vectors at scale sc around (mvx, mvy)
  auto cand_cost = [&](int a0, int a1, int sc, int lam, bool &live) -> int64_t {
    const int pos = a0 + lane;
    live = lane < 16 && pos < a1;
    const int sm = __shfl(sv, (lane + sums_off) & 63, 64);   // the pass's sum of candidate lane
    const int cx = mvx + sc * ept_x(live ? pos : 0), cy = mvy + sc * ept_y(live ? pos : 0);
    return mv_cost(lam, cx, cy, px, py) + ((int64_t)sm << 5);
  };
  // JM's top-2 fold (strict <, best / second tracking): the first minimum over the running best
  // (its cost and position, ahead of every candidate) and the candidates; the second is the first
  // minimum over the rest, with the running best ahead when a candidate took its place, else the
  // running second (cost DISTBLK_MAX) ahead.  (sc, lamsc unused here: scale of the vectors; kept
  // explicit at the call sites.)
  auto top2 = [&](int a0, int a1, int sc, int, int lam, int64_t &mn, int &bp, int64_t &sec, int &sp) {
    if (a1 <= a0) return;
    bool live;
    const int64_t c = cand_cost(a0, a1, sc, lam, live);
    int64_t c1;
    int k1;
    wave_argmin16(c, live, lane, c1, k1);
    if (k1 >= 64 || mn <= c1) {        // the running best stays
      if (k1 < 64 && c1 < sec) { sec = c1; sp = a0 + k1; }
      return;
    }
    int64_t c2;
    int k2;
    wave_argmin16(c, live && lane != k1, lane, c2, k2);
    // the running best becomes the second unless a later candidate is strictly below it
    if (k2 < 64 && c2 < mn) { sec = c2; sp = a0 + k2; } else { sec = mn; sp = bp; }
    mn = c1;
    bp = a0 + k1;
  };
  // JM's follow-up fold (strict <, minimum only)
  auto min1 = [&](int a0, int a1, int sc, int lam, int64_t &mn, int &bp) {
    if (a1 <= a0) return;
    bool live;
    const int64_t c = cand_cost(a0, a1, sc, lam, live);
    int64_t c1;
    int k1;
    wave_argmin16(c, live, lane, c1, k1);
    if (k1 < 64 && c1 < mn) { mn = c1; bp = a0 + k1; }
  };

  // ---- phase A: half-pel ring (me_fullsearch.c:221-250 | me_epzs_sub.c:66-88)
  {
    const int p1 = epzs ? min(5, max_pos2) : max_pos2;
    phase(q.start_hp, act ? p1 : 0, q.metric_h, t8, 2, epzs, mvx + pxp, mvy + pyp);
    if (TILE && act && epzs) {   // the top-2 fold as two wave minima (wave_argmin16)
      top2(q.start_hp, p1, 2, 2, lambda, min_mcost, best_pos, second_mcost, second_pos);
      early = best_pos == 0 && px == mvx && py == mvy && min_mcost < sub_threshold;   // :90-93
    } else if (act) {
      for (int pos = q.start_hp; pos < p1; ++pos) {
        const int ox = tab_x(epzs, pos), oy = tab_y(epzs, pos);
        const int cx = mvx + 2 * ox, cy = mvy + 2 * oy;
        int64_t mcost = mv_cost(lambda, cx, cy, px, py);
        const int sm = sums(pos - q.start_hp);
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
        if (best_pos) { mvx += 2 * spiral_x(best_pos); mvy += 2 * spiral_y(best_pos); }
      } else {
        early = best_pos == 0 && px == mvx && py == mvy && min_mcost < sub_threshold;   // :90-93
      }
    }
  }
  if (TILE && stamps) stamps[0] = __builtin_amdgcn_s_memrealtime();   // (server clocks: phase ends)
  // ---- phase B: EPZS half-pel follow-up (me_epzs_sub.c:96-127)
  {
    int s0 = 0, s1 = 0;
    if (act && epzs && !early && q.search_pos2 >= 9 && (best_pos != 0 || (abs(px - mvx) + abs(py - mvy)))) {
      s0 = next_start(best_pos * 5 + second_pos);
      s1 = next_end(best_pos * 5 + second_pos);
    }
    phase(s0, s1, q.metric_h, t8, 2, 1, mvx + pxp, mvy + pyp);
    if (TILE && act && epzs && !early) {
      min1(s0, s1, 2, lambda, min_mcost, best_pos);
      if (best_pos) { mvx += 2 * ept_x(best_pos); mvy += 2 * ept_y(best_pos); }
    } else if (act && epzs && !early) {
      for (int pos = s0; pos < s1; ++pos) {
        const int cx = mvx + 2 * ept_x(pos), cy = mvy + 2 * ept_y(pos);
        int64_t mcost = mv_cost(lambda, cx, cy, px, py);
        if (mcost < min_mcost) {
          mcost += dist(sums(pos - s0), min_mcost - mcost);
          if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
        }
      }
      if (best_pos) { mvx += 2 * ept_x(best_pos); mvy += 2 * ept_y(best_pos); }
    }
  }
  if (TILE && stamps) stamps[1] = __builtin_amdgcn_s_memrealtime();   // (server clocks: phase ends)
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
    phase(q.start_qp, p1, q.metric_q, t8, 1, epzs, mvx + pxp, mvy + pyp);
    if (TILE && act && !early && epzs) {
      top2(q.start_qp, p1, 1, 1, lambda, min_mcost, best_pos, second_mcost, second_pos);
    } else if (act && !early) {
      for (int pos = q.start_qp; pos < p1; ++pos) {
        const int ox = tab_x(epzs, pos), oy = tab_y(epzs, pos);
        const int cx = mvx + ox, cy = mvy + oy;
        int64_t mcost = mv_cost(lambda, cx, cy, px, py);
        const int sm = sums(pos - q.start_qp);
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
      if (!epzs && best_pos) { mvx += spiral_x(best_pos); mvy += spiral_y(best_pos); }
    }
  }
  if (TILE && stamps) stamps[2] = __builtin_amdgcn_s_memrealtime();   // (server clocks: phase ends)
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
      s0 = k >= 0 ? next_start(k) : 0;
      s1 = k >= 0 ? next_end(k) : 0;
    }
    phase(s0, s1, q.metric_q, t8, 1, 1, mvx + pxp, mvy + pyp);
    if (TILE && go) {
      min1(s0, s1, 1, lambda, min_mcost, best_pos);
    } else if (go) {
      for (int pos = s0; pos < s1; ++pos) {
        const int cx = mvx + ept_x(pos), cy = mvy + ept_y(pos);
        int64_t mcost = mv_cost(lambda, cx, cy, px, py);
        if (mcost < min_mcost) {
          mcost += dist(sums(pos - s0), min_mcost - mcost);
          if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
        }
      }
    }
    if (act && epzs && !early && best_pos > 0) { mvx += ept_x(best_pos); mvy += ept_y(best_pos); }
  }
  if (TILE && stamps) stamps[3] = __builtin_amdgcn_s_memrealtime();   // (server clocks: phase ends)
  if (act && (!TILE || lane == 0)) {
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
