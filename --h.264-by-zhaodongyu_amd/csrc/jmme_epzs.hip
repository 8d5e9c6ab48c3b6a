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

namespace jmme {

namespace {

constexpr int kWG = 256;
constexpr int kWaves = kWG / 64;
constexpr int kMaxSide = 2 * (kEpzsMaxQpel >> 2) + 1;
constexpr int kMapWords = (kMaxSide * kMaxSide + 31) / 32;
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
    {12, 0, 1, P_SDIAMOND, {}},   // SBP large diamond: half-pel points, rejected on the host
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
  uint32_t map[kMapWords];
  uint32_t cur[64];
};

struct Search {
  const uint8_t *ref;
  int pitch, W, H;
  int pos_x, pos_y, bsx, bsy;
  int pred_x, pred_y, cx, cy, max_x, max_y, side_x;
  int lambda;
  const uint32_t *cur;   // LDS, bsx/4 dwords per row
  uint32_t *map;
};

// SAD of the block at (ox, oy) of the reference against the current block
// (LDS); arguments by value so the out-of-line call keeps them in registers
template <int BSX, int BSY>
__device__ __forceinline__ unsigned sad_t(const uint8_t *ref, int pitch, int W, int H, const uint32_t *cur, int ox,
                                          int oy) {
  constexpr int NQ = BSX / 4;
  unsigned sad = 0;
  if (ox >= 0 && oy >= 0 && ox + BSX <= W && oy + BSY <= H) {
    const int xa = ox & ~3, sh = ox & 3;
    const uint8_t *base = ref + (size_t)oy * pitch + xa;
    const int last = sh ? 4 * NQ : 4 * NQ - 4;   // the extra dword stays inside the row
#pragma unroll
    for (int r = 0; r < BSY; ++r) {
      const uint8_t *row = base + (size_t)r * pitch;
      uint32_t w[NQ + 1];
#pragma unroll
      for (int q = 0; q < NQ; ++q) w[q] = *reinterpret_cast<const uint32_t *>(row + 4 * q);
      w[NQ] = *reinterpret_cast<const uint32_t *>(row + last);
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        sad = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w[q + 1], w[q], sh), cur[r * NQ + q], sad);
    }
  } else {
    // UMVLine4X: every sample clamped into the picture
#pragma unroll
    for (int r = 0; r < BSY; ++r) {
      const uint8_t *row = ref + (size_t)min(max(oy + r, 0), H - 1) * pitch;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        uint32_t d = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) d |= (uint32_t)row[min(max(ox + 4 * q + k, 0), W - 1)] << (8 * k);
        sad = __builtin_amdgcn_sad_u8(d, cur[r * NQ + q], sad);
      }
    }
  }
  return sad;
}

__device__ __noinline__ unsigned block_sad(const uint8_t *ref, int pitch, int W, int H, const uint32_t *cur, int bs,
                                           int ox, int oy) {
  switch (bs) {
    case (16 << 8) | 16: return sad_t<16, 16>(ref, pitch, W, H, cur, ox, oy);
    case (16 << 8) | 8: return sad_t<16, 8>(ref, pitch, W, H, cur, ox, oy);
    case (8 << 8) | 16: return sad_t<8, 16>(ref, pitch, W, H, cur, ox, oy);
    case (8 << 8) | 8: return sad_t<8, 8>(ref, pitch, W, H, cur, ox, oy);
    case (8 << 8) | 4: return sad_t<8, 4>(ref, pitch, W, H, cur, ox, oy);
    case (4 << 8) | 8: return sad_t<4, 8>(ref, pitch, W, H, cur, ox, oy);
    default: return sad_t<4, 4>(ref, pitch, W, H, cur, ox, oy);
  }
}

// mv_cost + (computeSAD << 5) of an integer qpel vector
__device__ __forceinline__ int64_t cand_cost(const Search &s, int mx, int my) {
  const int64_t mvc = (int64_t)s.lambda * (mvbits(mx - s.pred_x) + mvbits(my - s.pred_y));
  const unsigned sad =
      block_sad(s.ref, s.pitch, s.W, s.H, s.cur, (s.bsx << 8) | s.bsy, s.pos_x + (mx >> 2), s.pos_y + (my >> 2));
  return mvc + ((int64_t)sad << 5);
}

__device__ __forceinline__ bool in_range(const Search &s, int mx, int my) {
  return abs(mx - s.cx) <= s.max_x && abs(my - s.cy) <= s.max_y;
}
__device__ __forceinline__ int cell_of(const Search &s, int mx, int my) {
  return ((my - s.cy + s.max_y) >> 2) * s.side_x + ((mx - s.cx + s.max_x) >> 2);
}
__device__ __forceinline__ bool test_cell(const Search &s, int c) { return (s.map[c >> 5] >> (c & 31)) & 1u; }
__device__ __forceinline__ void set_cell(const Search &s, int c) { atomicOr(&s.map[c >> 5], 1u << (c & 31)); }

__device__ __forceinline__ int16_t int_mv(int v) { return (int16_t)(v & 0xFFFC); }   // set_integer_mv

__device__ void search_one(const EpzsParams &p, const jmme_epzs_req &q, WaveLds &w, int lane, jmme_epzs_res *out) {
  Search s;
  s.ref = p.refs[q.ref_slot];
  s.pitch = p.pitch;
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
  s.side_x = (2 * q.max_x >> 2) + 1;
  s.lambda = q.lambda;
  s.cur = w.cur;
  s.map = w.map;
  const int side_y = (2 * q.max_y >> 2) + 1;
  const int nq = q.bsx >> 2;

  if (lane < nq * q.bsy) {
    const int r = lane / nq, c = lane - r * nq;
    w.cur[lane] = *reinterpret_cast<const uint32_t *>(p.cur + (size_t)(q.pos_y + r) * p.pitch + q.pos_x + 4 * c);
  }
  const int words = (s.side_x * side_y + 31) >> 5;
  for (int i = lane; i < words; i += 64) w.map[i] = 0;
  wave_sync();
  for (int i = lane; i < q.n_stale; i += 64) {   // cells already holding this BlkCount
    const int dx = p.stale[2 * (q.stale_off + i)], dy = p.stale[2 * (q.stale_off + i) + 1];
    if (!(dx & 3) && !(dy & 3) && in_range(s, s.cx + dx, s.cy + dy)) set_cell(s, cell_of(s, s.cx + dx, s.cy + dy));
  }
  if (lane == 0) set_cell(s, cell_of(s, s.cx, s.cy));
  wave_sync();

  const bool frame = q.flags & JMME_EPZS_FRAME, pslice = q.flags & JMME_EPZS_PSLICE;
  const int bt = q.blocktype, refi = q.ref_idx, variant = q.variant;
  const int64_t lambda_dist = (int64_t)q.lambda * (variant ? 3 : 2);
  const int mv_range = variant ? 12 : 10;
  int64_t stop = q.medthres + lambda_dist, prev = q.prev_sad;
  int64_t best = cand_cost(s, s.cx, s.cy);   // every lane, same addresses
  int tmpx = s.cx, tmpy = s.cy, path = 5;
  bool update = true;

  if (refi > 0 && frame && prev < (stop < best ? stop : best)) {
    path = 1;
    update = false;
  } else if (best > stop) {
    int64_t second = kDistMax;
    bool check_median = false, done = false;
    int tmp2x = 0, tmp2y = 0;
    stop = q.stop_crit;
    if (best < (stop >> 1)) {
      path = 2;
      update = false;
      done = true;
    }
    // predictors, 64 at a time; JM's order is restored in the fold
    for (int base = 0; !done && base < q.n_pred; base += 64) {
      const int i = base + lane;
      const bool valid = i < q.n_pred;
      int mx = 0, my = 0;
      if (valid) {
        mx = int_mv(p.preds[2 * (q.pred_off + i)]);
        my = int_mv(p.preds[2 * (q.pred_off + i) + 1]);
      }
      const bool inr = valid && in_range(s, mx, my);
      const int cell = inr ? cell_of(s, mx, my) : -1 - lane;
      bool dup = inr && test_cell(s, cell);
      for (int j = 0; j < 63; ++j) {   // an earlier predictor of this chunk on the same cell
        const int cj = __shfl(cell, j, 64);
        dup |= j < lane && cj == cell;
      }
      const bool eval = inr && !dup;
      const int64_t cost = eval ? cand_cost(s, mx, my) : 0;
      if (eval) set_cell(s, cell);
      wave_sync();
      const unsigned long long emask = __ballot(eval);
      const int cnt = min(64, q.n_pred - base);
      for (int j = 0; j < cnt; ++j) {
        if ((emask >> j) & 1ull) {
          const int64_t c = __shfl(cost, j, 64);
          const int jx = __shfl(mx, j, 64), jy = __shfl(my, j, 64);
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
        }
        if (variant && best < ((3 * stop) >> 2)) {   // me_epzs.c:583-596
          path = 3;
          update = false;
          done = true;
          break;
        }
      }
    }
    if (!done && best > stop) {
      int P = primary_pattern(q.pattern);
      if (q.pattern != 0) {
        if (best < stop + ((3 * q.medthres) >> 1)) {
          P = ((tmpx == 0 && tmpy == 0) || (abs(tmpx - s.cx) < mv_range && abs(tmpy - s.cy) < mv_range))
                  ? P_SDIAMOND : P_SQUARE;
        } else if (variant || bt > 4 || (refi > 0 && bt != 1)) {
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
          const int cell = inr ? cell_of(s, mx, my) : 0;
          const bool eval = inr && !test_cell(s, cell);
          const int64_t cost = eval ? cand_cost(s, mx, my) : 0;
          if (eval) set_cell(s, cell);
          wave_sync();
          const unsigned long long emask = __ballot(eval);
          for (int j = 0; j < total; ++j) {
            if ((emask >> j) & 1ull) {
              const int64_t c = __shfl(cost, j, 64);
              if (c < best) {
                best = c;
                tmpx = __shfl(mx, j, 64);
                tmpy = __shfl(my, j, 64);
                dir = __shfl(idx, j, 64);
              }
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

        if (refi > 0 && frame && (4 * prev < best || (3 * prev < best && prev <= stop))) {
          path = 4;
          update = false;
          break;
        }
        if (!(check_median && (pslice || (!variant && bt < 5)) && best > stop && q.dual > 0)) break;
        point = 0;
        pstop = 0;
        dir = 0;
        next_last = 0;
        if ((tmpx == 0 && tmpy == 0) || (tmpx == s.cx && tmpy == s.cy))
          P = (abs(tmpx - s.cx) < mv_range && abs(tmpy - s.cy) < mv_range) ? P_SDIAMOND : P_SQUARE;
        else
          P = dual_pattern(q.dual);
        cenx = tmp2x;
        ceny = tmp2y;
        check_median = false;
      }
    }
  }
  if (update && (refi == 0 || prev > best)) prev = best;
  if (path <= 2) {   // returned before touching *mv
    tmpx = s.cx;
    tmpy = s.cy;
  }
  if (lane == 0) {
    jmme_epzs_res r;
    r.mv_x = (int16_t)tmpx;
    r.mv_y = (int16_t)tmpy;
    r.path = path;
    r.cost = best;
    r.prev_sad = prev;
    *out = r;
  }
  wave_sync();
}

__global__ __launch_bounds__(kWG) void epzs_kernel(EpzsParams p) {
  __shared__ WaveLds s_w[kWaves];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int t = blockIdx.x * kWaves + wave; t < p.n; t += gridDim.x * kWaves) {
    const jmme_epzs_req q = p.req[t];
    search_one(p, q, s_w[wave], lane, p.out + t);
  }
}

}  // namespace

hipError_t launch_epzs(const EpzsParams &p, hipStream_t s) {
  int grid = (p.n + kWaves - 1) / kWaves;
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(epzs_kernel, dim3(grid), dim3(kWG), 0, s, p);
  return hipGetLastError();
}

}  // namespace jmme
