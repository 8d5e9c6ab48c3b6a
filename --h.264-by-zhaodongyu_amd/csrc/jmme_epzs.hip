// jmme_epzs.hip -- gfx950 kernel for JM 18.5's EPZS integer-pel search
// (SURVEY.md §8 row a11), JM = /root/reference/4.对比程序/jm18.5/JM:
//
//   EPZS_motion_estimation        JM/lencod/src/me_epzs.c:54-407   (variant 0)
//   EPZS_subMB_motion_estimation  JM/lencod/src/me_epzs.c:417-780  (variant 1)
//   refinement patterns           JM/lencod/src/me_epzs_common.c:46-80, 176-230, 530-565
//   computeSAD / UMVLine4X        JM/lencod/src/me_distortion.c:349-426, inc/refbuf.h:22-26
//
// One wave per search.  The control flow (median check, early exits,
// predictor scan, pattern walk, dual refinement) is wave-uniform scalar code;
// the candidate evaluations it needs at each step -- a chunk of up to 64
// predictors, or one round of up to 12 pattern points -- are costed in
// parallel, one candidate per lane, and then folded in JM's order with
// readlanes, so every `<` comparison sees the values JM's sequential loop
// sees.  JM's early-terminating SAD (computeSAD stops a row after exceeding
// the bound) only ever stops on candidates that lose, so full SADs give the
// same decisions.  The EPZSMap becomes a per-wave LDS bitmap of visited
// integer offsets from the centre, seeded with the cells JM's never-cleared
// uint16 map already holds at this search's BlkCount.
#include <hip/hip_runtime.h>

#include "jmme.h"
#include "jmme_common.h"
#include "jmme_epzs_internal.h"
#include "jmme_subpel_dev.h"

#include <type_traits>

namespace jmme {

namespace {

constexpr int kWG = 256;
constexpr int kWaves = kWG / 64;
constexpr int64_t kDistMax = ((int64_t)0x7fffffff) << 5;   // DISTBLK_MAX, JM/lencod/inc/defines.h:135

// (dx, dy, start_nmbr, next_points) in qpel; me_epzs_common.c:46-80 data and
// the stopSearch / nextLast / nextpattern wiring of EPZSInit (:176-230)
struct Pat {
  int8_t n, stop, next_last, next;
  int8_t pt[12][4];
};
enum { P_SDIAMOND, P_SQUARE, P_EDIAMOND, P_LDIAMOND, P_SBDIAMOND, P_PMVFAST };
__constant__ Pat kPats[6] = {
    {4, 1, 1, P_SDIAMOND, {{0, 4, 3, 3}, {4, 0, 0, 3}, {0, -4, 1, 3}, {-4, 0, 2, 3}}},
    {8, 1, 1, P_SQUARE,
     {{0, 4, 7, 3}, {4, 4, 7, 5}, {4, 0, 1, 3}, {4, -4, 1, 5}, {0, -4, 3, 3}, {-4, -4, 3, 5}, {-4, 0, 5, 3},
      {-4, 4, 5, 5}}},
    {12, 1, 1, P_EDIAMOND,
     {{-4, 4, 10, 5}, {0, 8, 10, 8}, {0, 4, 10, 7}, {4, 4, 1, 5}, {8, 0, 1, 8}, {4, 0, 1, 7}, {4, -4, 4, 5},
      {0, -8, 4, 8}, {0, -4, 4, 7}, {-4, -4, 7, 5}, {-8, 0, 7, 8}, {-4, 0, 7, 7}}},
    {8, 1, 1, P_LDIAMOND,
     {{0, 8, 6, 5}, {4, 4, 0, 3}, {8, 0, 0, 5}, {4, -4, 2, 3}, {0, -8, 2, 5}, {-4, -4, 4, 3}, {-8, 0, 4, 5},
      {-4, 4, 6, 3}}},
    {12, 0, 1, P_SDIAMOND,        // SBP large diamond: half-pel points, EPZSSubPelGrid = 1 only
     {{0, 8, 6, 12}, {4, 4, 0, 12}, {8, 0, 0, 12}, {4, -4, 2, 12}, {0, -8, 2, 12}, {-4, -4, 4, 12}, {-8, 0, 4, 12},
      {-4, 4, 6, 12}, {0, 2, 6, 12}, {2, 0, 0, 12}, {0, -2, 2, 12}, {-2, 0, 4, 12}}},
    {8, 0, 1, P_SDIAMOND,
     {{0, 8, 6, 5}, {4, 4, 0, 3}, {8, 0, 0, 5}, {4, -4, 2, 3}, {0, -8, 2, 5}, {-4, -4, 4, 3}, {-8, 0, 4, 5},
      {-4, 4, 6, 3}}},
};

__device__ __forceinline__ int primary_pattern(int v) {
  return v == 5 ? P_PMVFAST : v == 4 ? P_SBDIAMOND : v == 3 ? P_LDIAMOND : v == 2 ? P_EDIAMOND
                                                                        : v == 1 ? P_SQUARE : P_SDIAMOND;
}
__device__ __forceinline__ int dual_pattern(int v) {
  return v == 6 ? P_PMVFAST : v == 5 ? P_SBDIAMOND : v == 4 ? P_LDIAMOND : v == 3 ? P_EDIAMOND
                                                                        : v == 2 ? P_SQUARE : P_SDIAMOND;
}

// LDS writes and reads of one wave stay in order; this keeps the compiler
// from moving them across each other and waits for the outstanding ones
__device__ __forceinline__ void wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

struct WaveLds {
  uint32_t cur[128];      // the current block: 4 (8-bit) or 2 (16-bit) samples per dword
  int pk[64][3];          // compacted candidates (x, y, source index)
};
// the visited-position bitmap (EPZSMap) lives in dynamic LDS, map_words per wave:
// integer-pel cells on the integer grid, quarter-pel cells on the sub-pel grid

struct Search {
  const uint8_t *ref;    // integer grid: the reference plane; sub-pel grid: its 16 sub-images
  int pitch, W, H;       // pitch: of the plane, or of the sub-images
  size_t ps;             // sub-pel grid: samples per sub-image (pitch too: in samples)
  int pos_x, pos_y, bsx, bsy;
  int pred_x, pred_y, cx, cy, max_x, max_y, side_x;
  int lambda;
  const uint32_t *cur;   // LDS, bsx/4 (16-bit: bsx/2) dwords per row
  uint32_t *map;
  uint32_t *flags;       // one bit per map word this search stamped (after the bitmap)
};

// SAD of row r of the block at (ox, oy) against the current block's row r
// (LDS).  UMVLine4X semantics: the row index and, off the picture's sides,
// every sample are clamped into the picture.
template <int NQ, bool HBD>
__device__ __forceinline__ unsigned row_sad(const Search &s, int ox, int oy, int r);
// 8-bit samples: NQ dwords of 4 samples, v_sad_u8
template <int NQ>
__device__ __forceinline__ unsigned row_sad8(const Search &s, int ox, int oy, int r) {
  const uint8_t *row = s.ref + (size_t)min(max(oy + r, 0), s.H - 1) * s.pitch;
  const uint32_t *cur = s.cur + r * NQ;
  unsigned sad = 0;
  if (ox >= 0 && ox + 4 * NQ <= s.W) {
    const int xa = ox & ~3, sh = ox & 3;
    const uint8_t *base = row + xa;
    uint32_t w[NQ + 1];
#pragma unroll
    for (int q = 0; q < NQ; ++q) w[q] = *reinterpret_cast<const uint32_t *>(base + 4 * q);
    w[NQ] = *reinterpret_cast<const uint32_t *>(base + (sh ? 4 * NQ : 4 * NQ - 4));   // stays inside the row
#pragma unroll
    for (int q = 0; q < NQ; ++q) sad = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w[q + 1], w[q], sh), cur[q], sad);
  } else {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      uint32_t d = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) d |= (uint32_t)row[min(max(ox + 4 * q + k, 0), s.W - 1)] << (8 * k);
      sad = __builtin_amdgcn_sad_u8(d, cur[q], sad);
    }
  }
  return sad;
}
// 16-bit samples (SourceBitDepthLuma 9..14): NQ dwords of 2 samples, v_sad_u16
template <int NQ>
__device__ __forceinline__ unsigned row_sad16(const Search &s, int ox, int oy, int r) {
  const uint16_t *row = reinterpret_cast<const uint16_t *>(s.ref) + (size_t)min(max(oy + r, 0), s.H - 1) * s.pitch;
  const uint32_t *cur = s.cur + r * NQ;
  unsigned sad = 0;
  if (ox >= 0 && ox + 2 * NQ <= s.W) {
    const uint32_t *base = reinterpret_cast<const uint32_t *>(row + (ox & ~1));
    const uint32_t sh = (uint32_t)(ox & 1) * 2;
    uint32_t w[NQ + 1];
#pragma unroll
    for (int q = 0; q < NQ; ++q) w[q] = base[q];
    w[NQ] = base[sh ? NQ : NQ - 1];   // stays inside the row
#pragma unroll
    for (int q = 0; q < NQ; ++q) sad = __builtin_amdgcn_sad_u16(__builtin_amdgcn_alignbyte(w[q + 1], w[q], sh), cur[q], sad);
  } else {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t d = (uint32_t)row[min(max(ox + 2 * q, 0), s.W - 1)] |
                         ((uint32_t)row[min(max(ox + 2 * q + 1, 0), s.W - 1)] << 16);
      sad = __builtin_amdgcn_sad_u16(d, cur[q], sad);
    }
  }
  return sad;
}
template <int NQ, bool HBD>
__device__ __forceinline__ unsigned row_sad(const Search &s, int ox, int oy, int r) {
  if constexpr (HBD) return row_sad16<NQ>(s, ox, oy, r);
  else return row_sad8<NQ>(s, ox, oy, r);
}

// Sub-pel grid: SAD of row r of the block at padded quarter-pel position
// (cx, cy): UMVLine4X picks sub-image (cy & 3, cx & 3) and clamps the origin
// to [-20, H+3] x [-32, W+15] (refbuf.h:22-26, mbuffer.c:549-550); the padded
// sub-image holds every sample the block then reads.
template <int NQ, bool HBD>
__device__ __forceinline__ unsigned row_sad_grid(const Search &s, int cx, int cy, int r) {
  const int pl = ((cy & 3) << 2) | (cx & 3);
  const int yy = min(max(cy >> 2, -20), s.H + 3), xx = min(max(cx >> 2, -32), s.W + 15);
  const size_t off = (size_t)pl * s.ps + (size_t)(yy + 20 + r) * s.pitch + (xx + 32);
  const uintptr_t u = reinterpret_cast<uintptr_t>(HBD ? s.ref + 2 * off : s.ref + off);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(u & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(u & 3);
  const uint32_t *cur = s.cur + r * NQ;
  uint32_t v[NQ + 1];
#pragma unroll
  for (int q = 0; q <= NQ; ++q) v[q] = w[q];
  unsigned sad = 0;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint32_t d = __builtin_amdgcn_alignbyte(v[q + 1], v[q], sh);
    sad = HBD ? __builtin_amdgcn_sad_u16(d, cur[q], sad) : __builtin_amdgcn_sad_u8(d, cur[q], sad);
  }
  return sad;
}

// Costs (mv_cost + SAD << 5) of the candidates held by lanes 0..K-1 (qpel
// (mx, my)), returned in the same lanes.  One lane per (candidate, row):
// 64/bsy candidates per pass, row sums reduced inside aligned lane groups.
// Passes of C candidates go B at a time (the sub-pel grid's clamped reads have
// no branch, so the B passes' loads issue back to back and their latencies
// overlap: a search is a chain of such rounds, one wave, latency-bound).
template <int NQ, int LOGR, bool GRID, bool HBD>
__device__ __forceinline__ int64_t eval_t(const Search &s, int lane, int K, int mx, int my) {
  constexpr int R = 1 << LOGR, C = 64 >> LOGR;
  constexpr int B = GRID ? (C >= 16 ? 1 : 16 / C) : 1;   // up to 16 candidates in flight
  const int grp = lane >> LOGR, r = lane & (R - 1);
  unsigned mine = 0;
  for (int base = 0; base < K; base += B * C) {
    unsigned sad[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int c = base + b * C + grp;
      const int cmx = __shfl(mx, c & 63, 64), cmy = __shfl(my, c & 63, 64);
      sad[b] = 0u;
      if (c < K)
        sad[b] = GRID ? row_sad_grid<NQ, HBD>(s, (s.pos_x << 2) + cmx, (s.pos_y << 2) + cmy, r)
                      : row_sad<NQ, HBD>(s, s.pos_x + (cmx >> 2), s.pos_y + (cmy >> 2), r);
    }
#pragma unroll
    for (int b = 0; b < B; ++b) {
#pragma unroll
      for (int m = 1; m < R; m <<= 1) sad[b] += __shfl_xor(sad[b], m, 64);
      const int j = lane - base - b * C;
      const unsigned v = __shfl(sad[b], (j & (C - 1)) << LOGR, 64);
      if (j >= 0 && j < C) mine = v;
    }
  }
  const int64_t mvc = (int64_t)s.lambda * (mvbits(mx - s.pred_x) + mvbits(my - s.pred_y));
  return mvc + ((int64_t)mine << 5);
}

template <bool GRID, bool HBD>
__device__ __noinline__ int64_t eval_costs_v(const uint8_t *ref, int pitch, size_t ps, int W, int H, const uint32_t *cur,
                                              int pos_x, int pos_y, int bsx, int bsy, int pred_x, int pred_y,
                                              int lambda, int lane, int K, int mx, int my) {
  Search s;
  s.ref = ref;
  s.pitch = pitch;
  s.ps = ps;
  s.W = W;
  s.H = H;
  s.cur = cur;
  s.pos_x = pos_x;
  s.pos_y = pos_y;
  s.bsx = bsx;
  s.bsy = bsy;
  s.pred_x = pred_x;
  s.pred_y = pred_y;
  s.lambda = lambda;
  constexpr int M = HBD ? 2 : 1;   // dwords per 4 samples
  switch ((bsx << 8) | bsy) {
    case (16 << 8) | 16: return eval_t<4 * M, 4, GRID, HBD>(s, lane, K, mx, my);
    case (16 << 8) | 8: return eval_t<4 * M, 3, GRID, HBD>(s, lane, K, mx, my);
    case (8 << 8) | 16: return eval_t<2 * M, 4, GRID, HBD>(s, lane, K, mx, my);
    case (8 << 8) | 8: return eval_t<2 * M, 3, GRID, HBD>(s, lane, K, mx, my);
    case (8 << 8) | 4: return eval_t<2 * M, 2, GRID, HBD>(s, lane, K, mx, my);
    case (4 << 8) | 8: return eval_t<1 * M, 3, GRID, HBD>(s, lane, K, mx, my);
    default: return eval_t<1 * M, 2, GRID, HBD>(s, lane, K, mx, my);
  }
}

// scalar arguments keep the out-of-line call's context in registers
template <bool GRID, bool HBD>
__device__ __forceinline__ int64_t eval_costs(const Search &s, int lane, int K, int mx, int my) {
  return eval_costs_v<GRID, HBD>(s.ref, s.pitch, s.ps, s.W, s.H, s.cur, s.pos_x, s.pos_y, s.bsx, s.bsy, s.pred_x, s.pred_y,
                            s.lambda, lane, K, mx, my);
}

// order-preserving compaction of the lanes with `pred` set: returns the
// packed position of this lane (valid where pred) and the count
__device__ __forceinline__ int pack_index(bool pred, int &count) {
  const unsigned long long m = __ballot(pred);
  count = __popcll(m);
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

__device__ __forceinline__ bool in_range(const Search &s, int mx, int my) {
  return abs(mx - s.cx) <= s.max_x && abs(my - s.cy) <= s.max_y;
}
// EPZSMap[max_y - mv.y + my][max_x - mv.x + mx] (me_epzs.c:223, me_epzs_int.c:214): on the integer
// grid only every 4th cell is used, so cells are numbered per integer offset there
template <bool GRID>
__device__ __forceinline__ int cell_of(const Search &s, int mx, int my) {
  return GRID ? (my - s.cy + s.max_y) * s.side_x + (mx - s.cx + s.max_x)
              : ((my - s.cy + s.max_y) >> 2) * s.side_x + ((mx - s.cx + s.max_x) >> 2);
}
__device__ __forceinline__ bool test_cell(const Search &s, int c) { return (s.map[c >> 5] >> (c & 31)) & 1u; }
__device__ __forceinline__ void set_cell(const Search &s, int c) {
  atomicOr(&s.map[c >> 5], 1u << (c & 31));
  atomicOr(&s.flags[c >> 10], 1u << ((c >> 5) & 31));
}
// a wave's map area at the start of a kernel (garbage LDS): all zero, so that
// each search need clear only the words the previous one flagged
__device__ __forceinline__ void map_init(uint32_t *area, int map_words, int lane) {
  for (int i = lane; i < (map_words >> 2); i += 64) reinterpret_cast<uint4 *>(area)[i] = make_uint4(0u, 0u, 0u, 0u);
}

// value of lane j (j wave-uniform) as a scalar
__device__ __forceinline__ int rl(int v, int j) { return __builtin_amdgcn_readlane(v, j); }
__device__ __forceinline__ int64_t rl64(int64_t v, int j) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, j), hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), j);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int16_t int_mv(int v) { return (int16_t)(v & 0xFFFC); }   // set_integer_mv

// Validity intervals (the drop-in's speculative searches, jmme_epzs_bounds):
// every comparison with the stop criterion S or the prevSad value P is monotone
// in it and reads "x >= t"; ge() returns the outcome and narrows [lo, hi] to the
// values that give the same one (restated in oracle/epzs_oracle.c).  The values
// are wave-uniform, so this is scalar bookkeeping.
struct Iv {
  int64_t lo, hi;
};
__device__ __forceinline__ bool ge(int64_t x, int64_t t, Iv &v) {
  if (x >= t) {
    v.lo = t > v.lo ? t : v.lo;
    return true;
  }
  v.hi = t - 1 < v.hi ? t - 1 : v.hi;
  return false;
}
__device__ __forceinline__ int64_t fdiv(int64_t a, int64_t b) { return a / b - ((a % b) != 0 && a < 0); }
__device__ __forceinline__ int64_t cdiv(int64_t a, int64_t b) { return -fdiv(-a, b); }
// P <= S with both inputs: pinned on the given P so each interval stands alone
__device__ __forceinline__ bool le2(int64_t pr, int64_t st, Iv &pv, Iv &sv) {
  if (pr <= st) {
    pv.hi = pr < pv.hi ? pr : pv.hi;
    sv.lo = pr > sv.lo ? pr : sv.lo;
    return true;
  }
  pv.lo = pr > pv.lo ? pr : pv.lo;
  sv.hi = pr - 1 < sv.hi ? pr - 1 : sv.hi;
  return false;
}

// stamps (the server's JMME_PHASES clocks, else null): s_memrealtime after the
// set-up, the centre, the predictors, the pattern walk and the visited cells
template <bool GRID, bool HBD>
__device__ jmme_block_res search_one(const EpzsParams &p, const jmme_epzs_req &q, WaveLds &w, uint32_t *map, int lane,
                                     jmme_epzs_res *out, unsigned long long *stamps = nullptr) {
  Search s;
  s.ref = GRID ? p.subs[q.ref_slot] : p.refs[q.ref_slot];
  s.pitch = GRID ? p.sub_pitch : p.pitch;
  s.ps = p.plane_stride;
  s.W = p.width;
  s.H = p.height;
  s.pos_x = q.pos_x;
  s.pos_y = q.pos_y;
  s.bsx = q.bsx;
  s.bsy = q.bsy;
  s.pred_x = q.pred_x;
  s.pred_y = q.pred_y;
  s.cx = q.center_x;
  s.cy = q.center_y;
  s.max_x = q.max_x;
  s.max_y = q.max_y;
  s.side_x = GRID ? 2 * q.max_x + 1 : (2 * q.max_x >> 2) + 1;
  s.lambda = q.lambda;
  s.cur = w.cur;
  s.map = map;
  const int bw = epzs_bitmap_words(GRID, p.max_qpel), nfl = (bw + 31) >> 5;
  s.flags = map + bw;
  const int side_y = GRID ? 2 * q.max_y + 1 : (2 * q.max_y >> 2) + 1;
  const int nq = q.bsx >> 2;

  if constexpr (HBD) {   // 16-bit: bsx/2 dwords a row, up to 128
    const int nd = q.bsx >> 1;
    const uint16_t *cur16 = reinterpret_cast<const uint16_t *>(p.cur);
    for (int i = lane; i < nd * q.bsy; i += 64) {
      const int r = i / nd, c = i - r * nd;
      w.cur[i] = *reinterpret_cast<const uint32_t *>(cur16 + (size_t)(q.pos_y + r) * p.pitch + q.pos_x + 2 * c);
    }
  } else if (lane < nq * q.bsy) {
    const int r = lane / nq, c = lane - r * nq;
    w.cur[lane] = *reinterpret_cast<const uint32_t *>(p.cur + (size_t)(q.pos_y + r) * p.pitch + q.pos_x + 4 * c);
  }
  (void)side_y;
  // the words the previous search on this map stamped (the rest is zero)
  for (int i = lane; i < nfl; i += 64) {
    uint32_t f = s.flags[i];
    while (f) {
      const int b = __builtin_ctz(f);
      f &= f - 1;
      map[32 * i + b] = 0u;
    }
    s.flags[i] = 0u;
  }
  wave_sync();
  for (int i = lane; i < q.n_stale; i += 64) {   // cells already holding this BlkCount
    const int dx = p.stale[2 * (q.stale_off + i)], dy = p.stale[2 * (q.stale_off + i) + 1];
    if ((GRID || (!(dx & 3) && !(dy & 3))) && in_range(s, s.cx + dx, s.cy + dy))
      set_cell(s, cell_of<GRID>(s, s.cx + dx, s.cy + dy));
  }
  if (lane == 0) set_cell(s, cell_of<GRID>(s, s.cx, s.cy));
  wave_sync();

  const bool frame = q.flags & JMME_EPZS_FRAME, pslice = q.flags & JMME_EPZS_PSLICE;
  // variant: the subMB form (EPZS_subMB_motion_estimation / EPZS_integer_subMB_motion_estimation)
  const int bt = q.blocktype, refi = q.ref_idx, variant = GRID ? q.variant == 3 : q.variant;
  const int64_t lambda_dist = (int64_t)q.lambda * (variant ? 3 : 2);
  const int mv_range = variant ? 12 : 10;
  int64_t stop = q.medthres + lambda_dist, prev = q.prev_sad;
  if (stamps) stamps[0] = __builtin_amdgcn_s_memrealtime();
  int64_t best = rl64(eval_costs<GRID, HBD>(s, lane, 1, s.cx, s.cy), 0);
  if (stamps) stamps[1] = stamps[2] = __builtin_amdgcn_s_memrealtime();   // ([2]: no predictor round)
  int tmpx = s.cx, tmpy = s.cy, path = 5;
  bool update = true;
  Iv sv{INT64_MIN, INT64_MAX}, pv{INT64_MIN, INT64_MAX};

  // me_epzs_int.c:67-80 / 496-507 add prevSad * 8 (subMB: 6) < min to the ref > 0 early exit
  if (refi > 0 && frame &&
      (!ge(prev, stop < best ? stop : best, pv) || (GRID && !ge(prev, fdiv(best - 1, variant ? 6 : 8) + 1, pv)))) {
    path = 1;
    update = false;
  } else if (best > stop) {
    int64_t second = kDistMax;
    bool check_median = false, done = false, first_seen = false;
    int tmp2x = 0, tmp2y = 0;
    stop = q.stop_crit;
    // the predictor list is JM's as generated with min_mcost = the centre's
    // cost: conditional entries (temporal neighbours, window, block-type
    // predictors, me_epzs_common.c:1528, 1654, 1224) join on that value
    const int64_t gen_min = best;
    bool cok[4] = {true, true, true, true};
    if (ge(stop, 2 * best + 2, sv)) {   // best < (stop >> 1)
      path = 2;
      update = GRID && !variant;   // EPZS_integer_motion_estimation keeps the value (me_epzs_int.c:118-120)
      done = true;
    } else if (p.pred_cond) {
      // which conditions the list holds: each is one comparison with S
      unsigned present = 0;
      for (int base = 0; base < q.n_pred; base += 64) {
        const int i = base + lane;
        const int c = i < q.n_pred ? p.pred_cond[q.pred_off + i] : 0;
        present |= (__ballot(c == 1) ? 2u : 0u) | (__ballot(c == 2) ? 4u : 0u) | (__ballot(c == 3) ? 8u : 0u);
      }
      if (present & 2u) cok[1] = !ge(stop, gen_min, sv);                    // gen_min > S
      if (present & 4u) cok[2] = !ge(stop, fdiv(gen_min - 1, 2) + 1, sv);   // gen_min > 2 S
      if (present & 8u) cok[3] = !ge(stop, fdiv(gen_min - 1, 3) + 1, sv);   // gen_min > 3 S
    }
    // predictors, 64 at a time; JM's order is restored in the fold
    for (int base = 0; !done && base < q.n_pred; base += 64) {
      const int i = base + lane;
      bool valid = i < q.n_pred;
      if (valid && p.pred_cond) valid = cok[p.pred_cond[q.pred_off + i] & 3];
      int mx = 0, my = 0;
      if (valid) {
        mx = p.preds[2 * (q.pred_off + i)];
        my = p.preds[2 * (q.pred_off + i) + 1];
        if (!GRID) {   // set_integer_mv (me_epzs.c:165)
          mx = int_mv(mx);
          my = int_mv(my);
        }
      }
      const bool inr = valid && in_range(s, mx, my);
      const int cell = inr ? cell_of<GRID>(s, mx, my) : -1 - lane;
      bool dup = inr && test_cell(s, cell);
      const int cnt = min(64, q.n_pred - base);
      for (int j = 0; j < cnt - 1; ++j) {   // an earlier predictor of this chunk on the same cell
        const int cj = __builtin_amdgcn_readlane(cell, j);   // (j is uniform: a scalar read, no LDS round trip)
        dup |= j < lane && cj == cell;
      }
      const bool eval = inr && !dup;
      if (eval) set_cell(s, cell);
      int ke;
      const int k = pack_index(eval, ke);
      if (eval) {
        w.pk[k][0] = mx;
        w.pk[k][1] = my;
      }
      wave_sync();
      const int px = lane < ke ? w.pk[lane][0] : 0, py = lane < ke ? w.pk[lane][1] : 0;
      wave_sync();
      const int64_t cost = eval_costs<GRID, HBD>(s, lane, ke, px, py);
      // sub-pel grid subMB: before the 3/4 check, the ref > 0 prevSad exit that
      // returns without touching *mv (me_epzs_int.c:590-600)
      const bool pexit = GRID && variant && refi > 0 && frame;
      // me_epzs.c:583-596 checks after every entry of JM's list; between updates
      // the minimum is unchanged, so checking after its first entry and after
      // each evaluated one is the same.  JM's first entry is the first valid
      // one (the entries whose condition failed are not in JM's list).
      const unsigned long long vm = __ballot(valid);
      int jexit = ke;   // an exit after packed entry jexit: JM never reaches (or stamps) the ones after it
      if (variant && !first_seen && vm) {
        first_seen = true;
        if (!((__ballot(eval) >> __builtin_ctzll(vm)) & 1ull)) {
          jexit = -1;
          if (pexit && !ge(prev, fdiv(best - 1, 3) + 1, pv)) {          // prev * 3 < best
            path = 6;
            update = false;
            done = true;
          } else if (ge(stop, cdiv(4 * best + 4, 3), sv)) {           // best < (3 stop) >> 2
            path = 3;
            update = false;
            done = true;
          }
        }
      }
      if (!done) jexit = ke;
      for (int j = 0; !done && j < ke; ++j) {
        const int64_t c = rl64(cost, j);
        jexit = j;
        const int jx = rl(px, j), jy = rl(py, j);
        if (c < best) {
          tmp2x = tmpx;
          tmp2y = tmpy;
          tmpx = jx;
          tmpy = jy;
          second = best;
          best = c;
          check_median = true;
        } else if (c < second) {
          tmp2x = jx;
          tmp2y = jy;
          second = c;
          check_median = true;
        }
        if (variant && pexit && !ge(prev, fdiv(best - 1, 3) + 1, pv)) {   // prev * 3 < best
          path = 6;
          update = false;
          done = true;
        } else if (variant && ge(stop, cdiv(4 * best + 4, 3), sv)) {       // best < (3 stop) >> 2
          path = 3;
          update = false;
          done = true;
        }
      }
      if (done && jexit < ke - 1) {   // un-stamp the chunk's entries past the exit
        if (eval && k > jexit) atomicAnd(&s.map[cell >> 5], ~(1u << (cell & 31)));
        wave_sync();
      }
    }
    if (stamps) stamps[2] = __builtin_amdgcn_s_memrealtime();
    // me_epzs_int.c:249-265: prev * 3 < best
    if (GRID && !done && !variant && refi > 0 && frame && !ge(prev, fdiv(best - 1, 3) + 1, pv)) {
      path = 7;
      update = false;
      done = true;
    }
    if (!done && !ge(stop, best, sv)) {   // best > stop
      int P = primary_pattern(q.pattern);
      if (q.pattern != 0) {
        if (ge(stop, best - ((3 * q.medthres) >> 1) + 1, sv)) {   // best < stop + 3 medthres / 2
          P = ((GRID && variant && bt == 7) || (tmpx == 0 && tmpy == 0) ||
               (abs(tmpx - s.cx) < mv_range && abs(tmpy - s.cy) < mv_range))
                  ? P_SDIAMOND : P_SQUARE;
        } else if (variant || (!GRID && bt > 4) || (refi > 0 && bt != 1)) {   // me_epzs_int.c:282 drops bt > 4
          P = P_SQUARE;
        }
      }
      int cenx = tmpx, ceny = tmpy, point = 0, pstop = 0, next_last = 0, dir = 0;
      for (;;) {
        int total = kPats[P].n;
        do {
          const int n = kPats[P].n;
          int idx = point + lane;
          if (idx >= n) idx -= n;
          const bool active = lane < total;
          const int mx = cenx + kPats[P].pt[active ? idx : 0][0], my = ceny + kPats[P].pt[active ? idx : 0][1];
          const bool inr = active && in_range(s, mx, my);
          const int cell = inr ? cell_of<GRID>(s, mx, my) : 0;
          const bool eval = inr && !test_cell(s, cell);
          if (eval) set_cell(s, cell);
          int ke;
          const int k = pack_index(eval, ke);
          if (eval) {
            w.pk[k][0] = mx;
            w.pk[k][1] = my;
            w.pk[k][2] = idx;
          }
          wave_sync();
          const int px = lane < ke ? w.pk[lane][0] : 0, py = lane < ke ? w.pk[lane][1] : 0;
          const int pi = lane < ke ? w.pk[lane][2] : 0;
          wave_sync();
          const int64_t cost = eval_costs<GRID, HBD>(s, lane, ke, px, py);
          for (int j = 0; j < ke; ++j) {
            const int64_t c = rl64(cost, j);
            if (c < best) {
              best = c;
              tmpx = rl(px, j);
              tmpy = rl(py, j);
              dir = rl(pi, j);
            }
          }
          if (next_last || (tmpx == cenx && tmpy == ceny)) {
            pstop = kPats[P].stop;
            P = kPats[P].next;
            total = kPats[P].n;
            next_last = kPats[P].next_last;
            dir = 0;
            point = 0;
          } else {
            total = kPats[P].pt[dir][3];
            point = kPats[P].pt[dir][2];
            cenx = tmpx;
            ceny = tmpy;
          }
        } while (pstop != 1);

        // 4 prev < best || (3 prev < best && prev <= stop)
        if (refi > 0 && frame &&
            (!ge(prev, fdiv(best - 1, 4) + 1, pv) || (!ge(prev, fdiv(best - 1, 3) + 1, pv) && le2(prev, stop, pv, sv)))) {
          path = 4;
          update = false;
          break;
        }
        // me_epzs_int.c:337-340 / 298-301: best < 2 prev; best > (3 stop) >> 1 (integer grid: best > stop)
        const bool dual_ok =
            GRID ? check_median && !(variant && bt == 7) && (refi == 0 || ge(prev, cdiv(best + 1, 2), pv)) &&
                       (!variant || pslice) && !ge(stop, fdiv(2 * best - 1, 3) + 1, sv) && q.dual > 0
                 : check_median && (pslice || (!variant && bt < 5)) && !ge(stop, best, sv) && q.dual > 0;
        if (!dual_ok) break;
        point = 0;
        pstop = 0;
        dir = 0;
        next_last = 0;
        if ((tmpx == 0 && tmpy == 0) || (tmpx == s.cx && tmpy == s.cy))
          P = ((GRID && variant && bt == 7) || (abs(tmpx - s.cx) < mv_range && abs(tmpy - s.cy) < mv_range))
                  ? P_SDIAMOND : P_SQUARE;
        else
          P = dual_pattern(q.dual);
        cenx = tmp2x;
        ceny = tmp2y;
        check_median = false;
      }
    }
  }
  if (stamps) stamps[3] = __builtin_amdgcn_s_memrealtime();
  bool written = false;
  if (update && (refi == 0 || ge(prev, best + 1, pv))) {   // prev > best
    prev = best;
    written = true;
  }
  const int motx = tmpx, moty = tmpy;   // JM's tmp: what every return path stores to p_motion
  if (path <= 2 || path == 6) {   // returned before touching *mv
    tmpx = s.cx;
    tmpy = s.cy;
  }
  // the drop-in keeps JM's never-cleared EPZSMap: every cell this search
  // stamped (the centre, evaluated predictors and pattern points, and the
  // cells that already held its BlkCount), as (dx, dy) qpel from the centre
  int nv = 0;
  if (p.visited) {
    // each lane takes a contiguous run of flag words, i.e. the stamped map words
    // in order: one popcount pass, one wave prefix sum, then every lane writes
    // its cells (row-major order kept)
    int16_t *const vout = p.visited + 2 * (size_t)p.max_visited * (size_t)(out - p.out);
    const int per = (nfl + 63) >> 6, f0 = min(lane * per, nfl), f1 = min(f0 + per, nfl);
    int cnt = 0;
    for (int fi = f0; fi < f1; ++fi) {
      uint32_t f = s.flags[fi];
      while (f) {
        const int b = __builtin_ctz(f);
        f &= f - 1;
        cnt += __popc(s.map[32 * fi + b]);
      }
    }
    int pre = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {   // inclusive prefix sum over the wave
      const int v = __shfl_up(pre, o, 64);
      if (lane >= o) pre += v;
    }
    int at = pre - cnt;
    for (int fi = f0; fi < f1 && at < p.max_visited; ++fi) {
      uint32_t f = s.flags[fi];
      while (f) {
        const int fb = __builtin_ctz(f);
        f &= f - 1;
        const int wi = 32 * fi + fb;
        uint32_t bits = s.map[wi];
        while (bits) {
          const int b = __builtin_ctz(bits);
          bits &= bits - 1;
          const int c = wi * 32 + b, cyi = c / s.side_x, cxi = c - cyi * s.side_x;
          if (at < p.max_visited) {
            vout[2 * at] = (int16_t)(GRID ? cxi - s.max_x : 4 * cxi - s.max_x);
            vout[2 * at + 1] = (int16_t)(GRID ? cyi - s.max_y : 4 * cyi - s.max_y);
          }
          ++at;
        }
      }
    }
    nv = __shfl(pre, 63, 64);
  }
  if (stamps) stamps[4] = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    jmme_epzs_res r;
    r.mv_x = (int16_t)tmpx;
    r.mv_y = (int16_t)tmpy;
    r.path = path;
    r.cost = best;
    r.prev_sad = prev;
    r.motion_x = (int16_t)motx;
    r.motion_y = (int16_t)moty;
    r.n_visited = nv;
    *out = r;
    const size_t t = (size_t)(out - p.out);
    if (p.bounds) {
      jmme_epzs_bounds b;
      b.stop_lo = sv.lo;
      b.stop_hi = sv.hi;
      b.prev_lo = pv.lo;
      b.prev_hi = pv.hi;
      b.prev_written = written ? 1 : 0;
      b.n_visited = nv;
      p.bounds[t] = b;
    }
    if (p.int_out) {   // the integer result as jmme_subpel_refine_async's d_int reads it
      jmme_block_res br;
      br.mv_x = (int16_t)tmpx;
      br.mv_y = (int16_t)tmpy;
      br.reserved = 0;
      br.cost = best;
      p.int_out[t] = br;
    }
  }
  wave_sync();
  jmme_block_res br;   // (wave-uniform) the answer as the refinement takes it
  br.mv_x = (int16_t)tmpx;
  br.mv_y = (int16_t)tmpy;
  br.reserved = 0;
  br.cost = best;
  return br;
}

// the fused path: this wave refines its own answer (a separate kernel
// instance, so the batch kernel's register allocation is not touched)
template <typename T>
__device__ __forceinline__ void refine_fused(const SubpelParams &sp, spd::WaveLds<T> &L, int lane, int t,
                                          jmme_block_res br, const jmme_subpel_req *req) {
  spd::refine_wave<T>(sp, L, lane, t, &br, req);
}


#ifndef JMME_EPZS_WAVES_PER_EU
#define JMME_EPZS_WAVES_PER_EU 4
#endif
// the search is latency-bound (a few dependent cache-resident fetch rounds
// per search): waves in flight matter more than a few spilled registers
template <bool GRID, bool HBD, bool FUSED>
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(JMME_EPZS_WAVES_PER_EU))) void epzs_kernel(
    EpzsParams p) {
  using SpT = std::conditional_t<HBD, uint16_t, uint8_t>;
  __shared__ WaveLds s_w[kWaves];
  __shared__ spd::WaveLds<SpT> s_sp[FUSED ? kWaves : 1];
  extern __shared__ __attribute__((aligned(16))) uint32_t s_map[];   // quads: map_words is a multiple of 4
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t *map = s_map + (size_t)wave * p.map_words;
  map_init(map, p.map_words, lane);
  wave_sync();
  for (int t = blockIdx.x * kWaves + wave; t < p.n; t += gridDim.x * kWaves) {
    const jmme_epzs_req q = FUSED ? p.one.q : p.req[t];
    // requests of the other grid, or with a window the map was not sized for, are refused
    const bool ok = (GRID ? q.variant >= 2 : q.variant <= 1) && q.max_x <= p.max_qpel && q.max_y <= p.max_qpel &&
                    (!FUSED || (t == 0 && q.n_pred <= kEpzsStageP && q.n_stale <= kEpzsStageS));
    if (ok) {
      EpzsParams pl = p;
      jmme_epzs_req ql = q;
      if constexpr (FUSED) {   // the lists from the kernel arguments (the host fuses only lists that fit)
        pl.preds = reinterpret_cast<const int16_t *>(p.one.preds);
        pl.stale = reinterpret_cast<const int16_t *>(p.one.stale);
        pl.pred_cond = p.pred_cond ? p.one.cond : nullptr;
      }
      const jmme_block_res br = search_one<GRID, HBD>(pl, ql, s_w[wave], map, lane, p.out + t);
      if constexpr (FUSED) {
        if (p.one.spq.blocktype) refine_fused<SpT>(p.fused_sp, s_sp[wave], lane, 0, br, &p.one.spq);
      }
      (void)br;
    } else if (lane == 0) {
      jmme_epzs_res r{};
      r.path = -1;
      p.out[t] = r;
      // a refused request leaves nothing a caller could take for a search that
      // ran: empty intervals (stop_lo > stop_hi) and a zeroed integer result
      if (p.bounds) {
        jmme_epzs_bounds b{};
        b.stop_lo = 1;
        b.stop_hi = 0;
        b.prev_lo = 1;
        b.prev_hi = 0;
        p.bounds[t] = b;
      }
      if (p.int_out) p.int_out[t] = jmme_block_res{};
    }
  }
  if constexpr (FUSED) {   // the host polls this word instead of synchronising the stream
    if (p.done && blockIdx.x == 0 && wave == 0) {
      __threadfence_system();
      if (lane == 0) __hip_atomic_store(p.done, p.done_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// A resident server for the searches alone (JMME_SINGLE_MODE 3): one wave
// polls the request number in mapped host memory, copies each request (the
// EpzsParams of a fused search, lists included) into LDS and serves it as the
// fused kernel does, then stores the number it served after a system-scope
// fence.  No launch per search.  Every exit is reached by the one wave: the
// host's quit word, idle_ticks without a request, or life_ticks in all
// (s_memrealtime, 100 MHz); its last store clears `alive`.  The data the
// searches read (planes, sub-images, tables) must not change while it runs:
// the host stops it before any such write (a kernel boundary is what makes
// another launch's writes visible to this one's caches).
template <bool GRID, bool HBD>
__global__ __launch_bounds__(64) void epzs_server_kernel(EpzsBox *box, uint32_t last, uint32_t idle_ticks,
                                                          unsigned long long life_ticks) {
  using SpT = std::conditional_t<HBD, uint16_t, uint8_t>;
  __shared__ WaveLds s_w;
  __shared__ spd::WaveLds<SpT> s_sp;
  __shared__ __attribute__((aligned(16))) EpzsParams s_p;
  extern __shared__ __attribute__((aligned(16))) uint32_t s_map[];
  static_assert(sizeof(EpzsParams) % 16 == 0, "the request is copied as uint4s");
  const int lane = threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t_idle = t0;
  int map_area = -1;   // (the map area's layout the flags describe; -1: not initialised)
  for (;;) {
    const uint32_t s = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)__hip_atomic_load(&box->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM));
    if (s == last) {
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      const uint32_t quit = (uint32_t)__builtin_amdgcn_readfirstlane(
          (int)__hip_atomic_load(&box->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
      if (quit || now - t_idle > idle_ticks || now - t0 > life_ticks) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    last = s;
    const unsigned long long t_seen = __builtin_amdgcn_s_memrealtime();
    {   // the request, behind the acquire of its number
      const uint4 *src = reinterpret_cast<const uint4 *>(&box->p);
      uint4 *dst = reinterpret_cast<uint4 *>(&s_p);
      for (int i = lane; i < (int)(sizeof(EpzsParams) / 16); i += 64) dst[i] = src[i];
    }
    __syncthreads();
    if (lane == 0) {   // the lists from the LDS copy
      s_p.preds = reinterpret_cast<const int16_t *>(s_p.one.preds);
      s_p.stale = reinterpret_cast<const int16_t *>(s_p.one.stale);
      s_p.pred_cond = s_p.pred_cond ? s_p.one.cond : nullptr;
    }
    __syncthreads();
    const unsigned long long t_copy = __builtin_amdgcn_s_memrealtime();
    const EpzsParams &p = s_p;
    const jmme_epzs_req &q = p.one.q;
    if (map_area != p.max_qpel) {   // first request, or another window size: the whole area once
      map_init(s_map, p.map_words, lane);
      wave_sync();
      map_area = p.max_qpel;
    }
    const bool ok = (GRID ? q.variant >= 2 : q.variant <= 1) && q.max_x <= p.max_qpel && q.max_y <= p.max_qpel &&
                    q.n_pred <= kEpzsStageP && q.n_stale <= kEpzsStageS;
    if (ok) {
      unsigned long long st[5] = {t_copy, t_copy, t_copy, t_copy, t_copy};
      const jmme_block_res br = search_one<GRID, HBD>(p, q, s_w, s_map, lane, p.out, st);
      if (lane == 0) {
        box->search = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_seen);
        box->ph[0] = (uint32_t)(st[0] - t_copy);   // set-up: current block, map, stale cells
        box->ph[1] = (uint32_t)(st[1] - st[0]);    // the centre
        box->ph[2] = (uint32_t)(st[2] - st[1]);    // predictors (0 on the early exits)
        box->ph[3] = (uint32_t)(st[3] - st[2]);    // pattern walk and dual refinement
        box->ph[4] = (uint32_t)(st[4] - st[3]);    // visited cells
      }
      if (p.one.spq.blocktype) refine_fused<SpT>(p.fused_sp, s_sp, lane, 0, br, &p.one.spq);
    } else if (lane == 0) {   // as the batch kernel refuses one
      jmme_epzs_res r{};
      r.path = -1;
      p.out[0] = r;
      if (p.bounds) {
        jmme_epzs_bounds b{};
        b.stop_lo = 1;
        b.stop_hi = 0;
        b.prev_lo = 1;
        b.prev_hi = 0;
        p.bounds[0] = b;
      }
      if (p.int_out) p.int_out[0] = jmme_block_res{};
    }
    if (lane == 0) {
      box->service = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_seen);
      box->copy = (uint32_t)(t_copy - t_seen);
    }
    __threadfence_system();
    if (lane == 0) __hip_atomic_store(&box->done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    t_idle = __builtin_amdgcn_s_memrealtime();
  }
  __threadfence_system();
  if (lane == 0) __hip_atomic_store(&box->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

hipError_t launch_epzs_server(EpzsBox *d_box, bool grid, bool hbd, int map_words, uint32_t last, uint32_t idle_ticks,
                              unsigned long long life_ticks, hipStream_t s) {
  auto k = grid ? (hbd ? epzs_server_kernel<true, true> : epzs_server_kernel<true, false>)
                : (hbd ? epzs_server_kernel<false, true> : epzs_server_kernel<false, false>);
  const size_t lds = (size_t)map_words * sizeof(uint32_t);
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(1), dim3(64), lds, s, d_box, last, idle_ticks, life_ticks);
  return hipGetLastError();
}

size_t epzs_map_words(bool grid, int max_qpel) {   // bitmap + flags, whole quads
  const int bw = epzs_bitmap_words(grid, max_qpel);
  return (size_t)bw + (size_t)epzs_flag_words(bw);
}

hipError_t launch_epzs(const EpzsParams &p, hipStream_t s) {
  int grid = (p.n + kWaves - 1) / kWaves;
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  const size_t lds = (size_t)kWaves * p.map_words * sizeof(uint32_t);
  auto k = p.fused ? (p.grid ? (p.hbd ? epzs_kernel<true, true, true> : epzs_kernel<true, false, true>)
                             : (p.hbd ? epzs_kernel<false, true, true> : epzs_kernel<false, false, true>))
                   : (p.grid ? (p.hbd ? epzs_kernel<true, true, false> : epzs_kernel<true, false, false>)
                             : (p.hbd ? epzs_kernel<false, true, false> : epzs_kernel<false, false, false>));
  if (lds > 65536) {   // sub-pel grid beyond R = 45: one workgroup may take up to 160 KiB
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(kWG), lds, s, p);
  return hipGetLastError();
}

}  // namespace jmme
