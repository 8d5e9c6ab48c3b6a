// jmme_search.hip -- gfx950 kernels for JM 18.5 integer-pel full search (FS)
// and fast full search (FFS), one workgroup per macroblock x reference unit.
//
// Semantics restated from JM 18.5 (JM = /root/reference/4.对比程序/jm18.5/JM):
//   FS   full_search_motion_estimation   JM/lencod/src/me_fullsearch.c:39-103
//        computeSAD (luma)               JM/lencod/src/me_distortion.c:349-426
//   FFS  setup_fast_full_search          JM/lencod/src/me_fullfast.c:269-608
//        update_full_search_large_blocks JM/lencod/src/me_fullfast.c:196-260
//        fast_full_search_motion_est.    JM/lencod/src/me_fullfast.c:618-689
//   mv_cost (JCOST_CALC_SCALEUP)         JM/lencod/inc/mv_search.h:100-104
//   UMVLine4X reference clamp            JM/lencod/inc/refbuf.h:22-26
//
// Exactness argument.  JM walks the spiral with strict '<' and an early-exit
// SAD that returns the threshold when it exits (me_distortion.c:384-385), so
// the result is the lexicographic minimum of (cost, spiral rank) over all
// eligible candidates.  We evaluate every candidate exhaustively and reduce
// that key; no early exit, same answer.
//
// Work mapping (one workgroup = one MB x ref unit, 256 threads = 4 waves):
//   * partitions are grouped by identical search window and predictor (FS:
//     centre + range + predictor; FFS: the MB's surface + predictor); each
//     group stages its reference window (2R+16)^2 pels from HBM into LDS once,
//     as "word[y][x] = pels x..x+3" so every SAD row read is an aligned
//     ds_read_b32;
//   * a thread takes a vertical PAIR of search positions: the 17 reference
//     rows they need are read once, the 2 x 16 4x4 SADs formed with v_sad_u8
//     (the current MB row is a broadcast ds_read_b128), summed to the 41
//     partition SADs, and a running minimum per partition kept in registers;
//   * key (fast path): 32 bits = cost << 10 | rank >> 3.  cost < 2^22 holds for
//     every partition while lambda <= kMaxLambda32, so one v_lshl_add_u32 and
//     one v_min_u32 update a partition.  The 3 dropped rank bits are recovered
//     exactly afterwards: the winner's rank lies in [8c, 8c+8), and those <= 8
//     positions are re-evaluated per partition (refine pass);
//   * key (exact fallback): 64 bits = cost << 32 | rank, for ranges > 44 or
//     huge lambdas (deferred pass).
#include <hip/hip_runtime.h>
#include <type_traits>
#include "jmme.h"
#include "jmme_common.h"
#include "jmme_internal.h"

namespace jmme {

namespace {

constexpr int kNS = JMME_NSLOT;
constexpr int kWaves = kWG / 64;
constexpr unsigned long long kAll = (1ull << kNS) - 1;
constexpr uint32_t kMaxLambda32 = 28450;   // 32*65280 + lambda*74 < 2^22: 22-bit cost field exact
constexpr int kCostShift = 10;             // key32 = cost << 10 | rank >> 3
constexpr int kRankDrop = 3;
constexpr int kCand = 1 << kRankDrop;      // refine candidates per partition
#ifndef JMME_WAVES_PER_EU
#define JMME_WAVES_PER_EU 4
#endif

struct Lds {
  int wp;        // words per window row
  int rawp;      // bytes per raw row
  uint32_t *words;
  uint8_t *raw;
  uint32_t *cur;            // 64 words: MB row r, column group c at [r*4+c]
  int4 *slot;               // 41 x jmme_block_req
  unsigned long long *grp;  // per slot: mask of slots sharing window AND predictor
  unsigned long long *red;  // kWaves x 41 reduction scratch
  uint32_t *match;          // 41 x kCand refine flags
  int *flag;                // unit must be redone with 64-bit keys
};

__host__ __device__ inline int lds_rawp(int R) { return 4 * ((3 + 2 * R + 13 + 2) / 4 + 2); }

__device__ __forceinline__ Lds carve(unsigned char *smem, int R) {
  Lds L;
  const int rows = 2 * R + 16;
  L.wp = (2 * R + 13) | 1;
  L.rawp = lds_rawp(R);
  size_t off = 0;
  L.words = reinterpret_cast<uint32_t *>(smem + off); off += (size_t)rows * L.wp * 4;
  off = (off + 15) & ~(size_t)15;
  L.raw = smem + off;                                    off += (size_t)rows * L.rawp;
  off = (off + 15) & ~(size_t)15;
  L.cur = reinterpret_cast<uint32_t *>(smem + off);      off += 64 * 4;
  L.slot = reinterpret_cast<int4 *>(smem + off);         off += kNS * 16;
  L.grp = reinterpret_cast<unsigned long long *>(smem + off); off += kNS * 8;
  L.red = reinterpret_cast<unsigned long long *>(smem + off); off += kWaves * kNS * 8;
  L.match = reinterpret_cast<uint32_t *>(smem + off);    off += kNS * kCand * 4;
  L.flag = reinterpret_cast<int *>(smem + off);          off += 16;
  return L;
}

// Diagnostic phase clocks (build with -DJMME_STAMPS; never in the shipped
// library): s_memtime at phase boundaries, summed per unit, written by lane 0.
#ifdef JMME_STAMPS
#define STAMP(acc) do { __builtin_amdgcn_sched_barrier(0); unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
                        acc += t_ - t_last; t_last = t_; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define STAMP(acc) do { } while (0)
#endif

__device__ __forceinline__ int ufl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ unsigned long long ufl64(unsigned long long v) {
  unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// slot request fields from the int4 image of jmme_block_req
__device__ __forceinline__ int rq_pred_x(int4 q) { return (int)(short)(q.x & 0xffff); }
__device__ __forceinline__ int rq_pred_y(int4 q) { return (int)(short)((unsigned)q.x >> 16); }
__device__ __forceinline__ int rq_cen_x(int4 q) { return (int)(short)(q.y & 0xffff); }
__device__ __forceinline__ int rq_cen_y(int4 q) { return (int)(short)((unsigned)q.y >> 16); }
__device__ __forceinline__ int rq_range(int4 q) { return (int)(short)(q.z & 0xffff); }
__device__ __forceinline__ int rq_flags(int4 q) { return (int)(short)((unsigned)q.z >> 16); }
__device__ __forceinline__ int rq_lambda(int4 q) { return q.w; }

// bijective XCD-aware remap: blocks are dealt round-robin to the 8 XCDs, so
// give each XCD a contiguous run of units (neighbouring macroblocks read
// overlapping reference windows, which then hit that XCD's L2).
__device__ __forceinline__ int xcd_unit(int b, int nb) {
  const int nx = 8;
  int q = nb / nx, r = nb % nx, x = b % nx;
  return x * q + (x < r ? x : r) + b / nx;
}

// the 41 partition SADs from the 16 4x4 SADs (JM sums them in
// update_full_search_large_blocks, me_fullfast.c:196-260 -- integer sums)
__device__ __forceinline__ void partition_sads(const uint32_t *a, uint32_t *ps) {
#pragma unroll
  for (int k = 0; k < 16; ++k) ps[25 + k] = a[k];                                           // 4x4
#pragma unroll
  for (int by = 0; by < 4; ++by)
#pragma unroll
    for (int h = 0; h < 2; ++h) ps[9 + by * 2 + h] = a[by * 4 + 2 * h] + a[by * 4 + 2 * h + 1];   // 8x4
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int bx = 0; bx < 4; ++bx) ps[17 + v * 4 + bx] = a[(2 * v) * 4 + bx] + a[(2 * v + 1) * 4 + bx];  // 4x8
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int h = 0; h < 2; ++h) ps[5 + v * 2 + h] = ps[9 + (2 * v) * 2 + h] + ps[9 + (2 * v + 1) * 2 + h];  // 8x8
  ps[3] = ps[5] + ps[7];
  ps[4] = ps[6] + ps[8];   // 8x16
  ps[1] = ps[5] + ps[6];
  ps[2] = ps[7] + ps[8];   // 16x8
  ps[0] = ps[1] + ps[2];   // 16x16
}

// branch-free spiral_index (jmme_common.h) for the sweep
__device__ __forceinline__ int spiral_index_bl(int ox, int oy) {
  const int ax = abs(ox), ay = abs(oy);
  const int l = max(ax, ay);
  const int base = (2 * l - 1) * (2 * l - 1);
  const int top = base + 2 * (ox + l - 1) + (oy > 0);
  const int side = base + 2 * (2 * l - 1) + 2 * (oy + l) + (ox > 0);
  const int v = (ay == l && ax < l) ? top : side;
  return l == 0 ? 0 : v;
}

// mv cost lambda*(mvbits[dx]+mvbits[dy]) of candidate (candx, candy) against
// predictor (px, py), mv_search.h:100-104; GetMaxMVD gate for FFS.
struct MvCost { uint32_t mvc; bool ok; };
template <bool FFS>
__device__ __forceinline__ MvCost mv_cost(int candx, int candy, int px, int py, int lam, int max_mvd) {
  const int dx = candx - px, dy = candy - py;
  MvCost r;
  r.mvc = (uint32_t)lam * (uint32_t)(mvbits(dx) + mvbits(dy));
  r.ok = FFS ? (max(abs(dx), abs(dy)) < max_mvd - 1) : true;   // me_fullfast.c:663
  return r;
}

// check_for_00 (me_fullsearch.c:61,78-82): at the (0,0) vector subtract
// weighted_cost(lambda,16), floored at 0.
__device__ __forceinline__ uint32_t check00_adjust(uint32_t mvc, int lam, bool is00) {
  const uint32_t t = 16u * (uint32_t)lam;
  return is00 ? (mvc > t ? mvc - t : 0u) : mvc;
}

// what a position contributes, shared by all partitions of the group
struct PosCtx {
  uint32_t mvc, mvc0, rank;   // mvc0: slot 0's cost after check_for_00
  int lring;
  bool is00, ok;
};

struct GroupCtx {
  int R, cqx, cqy, px, py, lam, chk00, max_mvd;
  bool preseed;
  unsigned long long gmask, rlim;
  const int4 *slot;
};

// FFS partition searched over a smaller range than the surface (me_fullfast.c:627)
template <bool FFS>
__device__ __forceinline__ bool slot_eligible(const GroupCtx &g, const PosCtx &c, int s) {
  if (!FFS) return true;
  bool oks = c.ok;
  if ((g.rlim >> s) & 1) {
    const int rs = ufl(rq_range(g.slot[s]));
    oks = oks && (c.lring <= rs || (g.preseed && c.is00));
  }
  return oks;
}

template <bool KEY32, bool FFS, bool ALL, typename Best>
__device__ __forceinline__ void update_slots(const uint32_t (&ps)[kNS], const GroupCtx &g, const PosCtx &c,
                                             Best (&best)[kNS]) {
  if (KEY32) {
    const uint32_t k32 = (c.mvc << kCostShift) | (c.rank >> kRankDrop);
    const uint32_t k32_0 = (c.mvc0 << kCostShift) | (c.rank >> kRankDrop);
#pragma unroll
    for (int s = 0; s < kNS; ++s) {
      if (!ALL && !((g.gmask >> s) & 1)) continue;
      // cost<<10 | rank>>3  ==  (SAD << 15) + ((mvc << 10) | rank >> 3)
      const uint32_t k = (ps[s] << (5 + kCostShift)) + (s == 0 ? k32_0 : k32);
      const uint32_t kk = FFS ? (slot_eligible<FFS>(g, c, s) ? k : ~0u) : k;
      best[s] = min((uint32_t)best[s], kk);
    }
  } else {
#pragma unroll
    for (int s = 0; s < kNS; ++s) {
      if (!ALL && !((g.gmask >> s) & 1)) continue;
      const uint32_t hi = (ps[s] << 5) + (s == 0 ? c.mvc0 : c.mvc);
      const unsigned long long k = ((unsigned long long)hi << 32) | c.rank;
      const unsigned long long kk = FFS ? (slot_eligible<FFS>(g, c, s) ? k : ~0ull) : k;
      best[s] = best[s] < kk ? best[s] : kk;
    }
  }
}

// exact SAD of partition s at window offset (oxw, oyw), for the refine pass
__device__ __forceinline__ uint32_t partition_sad_at(const Lds &L, int s, int oxw, int oyw) {
  const SlotGeom gm = slot_geom(s);
  uint32_t sad = 0;
  for (int r = 0; r < 4 * gm.h; ++r) {
    const int row = gm.by * 4 + r;
    const uint32_t *w = L.words + (oyw + row) * L.wp + oxw + gm.bx * 4;
    for (int c = 0; c < gm.w; ++c) sad = __builtin_amdgcn_sad_u8(w[4 * c], L.cur[row * 4 + gm.bx + c], sad);
  }
  return sad;
}

template <bool KEY32, bool FFS>
__device__ __forceinline__ void unit_body(const KParams &p, int u, unsigned char *smem) {
  using Best = typename std::conditional<KEY32, uint32_t, unsigned long long>::type;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;

  const jmme_mb_req *rq = p.req + u;
  const int mb_x = ufl(rq->mb_x);
  const int mb_y = ufl(rq->mb_y);
  const int list = ufl(rq->list);
  const int ref_idx = ufl(rq->ref_idx);
  const unsigned long long slot_mask = ufl64(rq->slot_mask) & kAll;
  const int ffs_cx = ufl(rq->ffs_center_x);
  const int ffs_cy = ufl(rq->ffs_center_y);
  const int ffs_range = ufl(rq->ffs_range);
  const bool preseed = FFS && ufl(rq->ffs_pos00_valid) != 0;
  const uint8_t *ref = p.refs[list * kMaxRefs + ref_idx];

  Lds L = carve(smem, p.lds_range);
#ifdef JMME_STAMPS
  unsigned long long t_last = __builtin_amdgcn_s_memtime();
  unsigned long long st_setup = 0, st_stage = 0, st_sweep = 0, st_reduce = 0, st_refine = 0, st_out = 0;
#endif

  // ---- unit setup: slot requests, groups, current MB
  if (tid < kNS) {
    const int4 *src = reinterpret_cast<const int4 *>(&rq->blk[0]);
    L.slot[tid] = src[tid];
  }
  if (tid == 255) L.flag[0] = 0;
  if (tid >= 64 && tid < 128) {
    int t = tid - 64, r = t >> 2, c = t & 3;
    L.cur[t] = *reinterpret_cast<const uint32_t *>(p.cur + (size_t)(mb_y + r) * p.pitch + mb_x + 4 * c);
  }
  __syncthreads();
  if (tid < kNS) {
    const int4 me = L.slot[tid];
    unsigned long long g = 0;
    if ((slot_mask >> tid) & 1) {
      for (int t = 0; t < kNS; ++t) {
        if (!((slot_mask >> t) & 1)) continue;
        const int4 o = L.slot[t];
        // a group = partitions with the same search window AND the same
        // predictor/lambda: one SAD sweep and one mv-cost per position serve
        // the whole group (a window with several predictors is swept once per
        // predictor -- straight-line code, no per-partition predictor loads)
        const bool same_win = FFS || (o.y == me.y && rq_range(o) == rq_range(me));
        g |= (unsigned long long)(same_win && o.x == me.x && o.w == me.w) << t;
      }
      if (KEY32 && (uint32_t)rq_lambda(me) > kMaxLambda32) L.flag[0] = 1;
    }
    L.grp[tid] = g;
  }
  __syncthreads();
  if (KEY32 && ufl(L.flag[0])) {
    // the 22-bit cost field could overflow: redo the whole unit with 64-bit keys
    if (tid == 0) p.defer_list[atomicAdd(p.defer_count, 1u)] = u;
    return;
  }

  STAMP(st_setup);
  // One pass per group: stage the window, sweep it, reduce, (refine), write.
  // Nothing is carried from one group to the next.
  unsigned long long remaining = slot_mask;
  while (remaining) {
    const int lead = __builtin_ctzll(remaining);
    const unsigned long long gmask = ufl64(L.grp[lead]) & remaining;
    remaining &= ~gmask;
    const int4 lq = L.slot[lead];
    GroupCtx g;
    g.cqx = ufl(FFS ? ffs_cx : rq_cen_x(lq));   // window centre, qpel (multiple of 4)
    g.cqy = ufl(FFS ? ffs_cy : rq_cen_y(lq));
    g.R = ufl(FFS ? ffs_range : rq_range(lq));
    g.px = ufl(rq_pred_x(lq));
    g.py = ufl(rq_pred_y(lq));
    g.lam = ufl(rq_lambda(lq));
    g.max_mvd = p.max_mvd;
    g.preseed = preseed;
    g.gmask = gmask;
    g.slot = L.slot;
    const int R = g.R;
    if (R < 0 || R > p.lds_range || ((g.cqx | g.cqy) & 3)) {
      // outside what this launch was sized for (or a sub-pel-grid centre):
      // refuse loudly instead of overrunning LDS; the host reports it
      if (tid == 0) atomicOr(p.status, (R < 0 || R > p.lds_range) ? 1u : 2u);
      continue;
    }
    g.rlim = 0;
    if (FFS) {
      for (int t = 0; t < kNS; ++t)
        if ((gmask >> t) & 1) g.rlim |= (unsigned long long)(rq_range(L.slot[t]) < R) << t;
      g.rlim = ufl64(g.rlim);
    }
    g.chk00 = ufl((!FFS && (gmask & 1)) ? (rq_flags(L.slot[0]) & JMME_BLK_CHECK00) : 0);

    // ---- stage the (2R+16)^2 reference window, clamped like UMVLine4X.
    // Rows are clamped into the picture; when the window's columns lie inside
    // the picture each row is fetched as aligned dwords (one round trip, all
    // loads in flight), else byte by byte with column clamping.
    const int x0 = mb_x + (g.cqx >> 2) - R;
    const int y0 = mb_y + (g.cqy >> 2) - R;
    const int wrows = 2 * R + 16;
    const int wpr = 2 * R + 13;                 // words per window row
    const int xa = x0 & ~3;                     // dword-aligned start (floor)
    const int sh = x0 - xa;                     // 0..3
    const int nd = (sh + wpr + 2) / 4 + 2;      // dwords per row the words read (incl. alignbyte hi)
    const int rdw = L.rawp >> 2;
    uint32_t *raw32 = reinterpret_cast<uint32_t *>(L.raw);
    __syncthreads();   // previous group's readers are done with the window
#ifdef JMME_ABL_NOSTAGE  // timing ablation only: skip fetching the window
    constexpr bool kFetch = false;
#else
    constexpr bool kFetch = true;
#endif
    if (!kFetch) {
    } else if (xa >= 0 && xa + 4 * nd <= p.width) {
      const int total = wrows * nd;
#pragma unroll 4
      for (int i = tid; i < total; i += kWG) {
        const int r = i / nd, d = i - r * nd;
        const int gy = clampi(y0 + r, 0, p.height - 1);
        raw32[r * rdw + d] = *reinterpret_cast<const uint32_t *>(ref + (size_t)gy * p.pitch + xa + 4 * d);
      }
    } else {
      const int rb = 4 * nd;
      const int total = wrows * rb;
#pragma unroll 8
      for (int i = tid; i < total; i += kWG) {
        const int r = i / rb, c = i - r * rb;
        const int gy = clampi(y0 + r, 0, p.height - 1);
        const int gx = clampi(xa + c, 0, p.width - 1);
        L.raw[r * L.rawp + c] = ref[(size_t)gy * p.pitch + gx];
      }
    }
    __syncthreads();
    for (int i = tid; i < wrows * wpr; i += kWG) {
      const int r = i / wpr, c = i - r * wpr + sh;
      const uint32_t *rw = raw32 + r * rdw;
      L.words[r * L.wp + (c - sh)] = __builtin_amdgcn_alignbyte(rw[(c >> 2) + 1], rw[c >> 2], c & 3);
    }
    __syncthreads();
    if (p.debug_words && u == 0 && gmask == (slot_mask & ufl64(L.grp[__builtin_ctzll(slot_mask)]))) {
      for (int i = tid; i < wrows * L.wp; i += kWG) p.debug_words[i] = L.words[i];
    }

    STAMP(st_stage);
    // per-thread running minima of the keys
    Best best[kNS];
#pragma unroll
    for (int s = 0; s < kNS; ++s) best[s] = (Best)~0ull;

    // ---- sweep all (2R+1)^2 positions of the window.  A task is a vertical
    // pair of positions (x, y), (x, y+1): the 17 reference rows they need are
    // read from LDS once and feed both.  Specialised for a group that is all
    // 41 partitions (no per-partition mask tests) or a subset.
    auto sweep = [&](auto all_tag) {
      const int D = 2 * R + 1;
      const int DP = (D + 1) >> 1;          // position pairs per column
      const int ntask = D * DP;
      const int qstep = kWG / D, rstep = kWG - (kWG / D) * D;
      int tx = tid % D, ty = tid / D;       // task column, pair row
      for (int t = tid; t < ntask; t += kWG) {
        uint32_t a0[16], a1[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) { a0[k] = 0; a1[k] = 0; }
        {
          // opaque zero: keeps the broadcast reads of the current MB inside the
          // loop instead of letting LICM pin 64 VGPRs for them
          int zero;
          asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
          const uint4 *cur4 = reinterpret_cast<const uint4 *>(L.cur) + zero;
          const uint32_t *wrow = L.words + (2 * ty) * L.wp + tx;
          // software pipeline, one row ahead: row r+1's reference words and MB
          // row are requested before row r's v_sad_u8s, so each LDS round trip
          // hides behind a row of arithmetic (and the other waves of the SIMD)
          uint32_t n0, n1, n2, n3;
          uint4 cn;
#ifdef JMME_ABL_NOLDS    // timing ablation only: no window reads
          n0 = tx; n1 = n0 ^ 1; n2 = n0 ^ 2; n3 = n0 ^ 3;
#else
          n0 = wrow[0]; n1 = wrow[4]; n2 = wrow[8]; n3 = wrow[12];
#endif
          cn = cur4[0];
          uint4 cprev = make_uint4(0, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 17; ++r) {
            const uint32_t w0 = n0, w1 = n1, w2 = n2, w3 = n3;
            const uint4 c = cn;
            if (r < 16) {
              const uint32_t *w = wrow + (r + 1) * L.wp;
#ifdef JMME_ABL_NOLDS
              n0 = (r + 1) * 0x01010101u + tx; n1 = n0 ^ 1; n2 = n0 ^ 2; n3 = n0 ^ 3;
              (void)w;
#else
              n0 = w[0]; n1 = w[4]; n2 = w[8]; n3 = w[12];
#endif
              if (r < 15) cn = cur4[r + 1];
            }
            __builtin_amdgcn_sched_barrier(0);
            if (r < 16) {   // row r of the MB against position y
              const int b = (r >> 2) * 4;
              a0[b + 0] = __builtin_amdgcn_sad_u8(w0, c.x, a0[b + 0]);
              a0[b + 1] = __builtin_amdgcn_sad_u8(w1, c.y, a0[b + 1]);
              a0[b + 2] = __builtin_amdgcn_sad_u8(w2, c.z, a0[b + 2]);
              a0[b + 3] = __builtin_amdgcn_sad_u8(w3, c.w, a0[b + 3]);
            }
            if (r > 0) {    // row r-1 of the MB against position y+1
              const int b = ((r - 1) >> 2) * 4;
              a1[b + 0] = __builtin_amdgcn_sad_u8(w0, cprev.x, a1[b + 0]);
              a1[b + 1] = __builtin_amdgcn_sad_u8(w1, cprev.y, a1[b + 1]);
              a1[b + 2] = __builtin_amdgcn_sad_u8(w2, cprev.z, a1[b + 2]);
              a1[b + 3] = __builtin_amdgcn_sad_u8(w3, cprev.w, a1[b + 3]);
            }
            cprev = c;
            __builtin_amdgcn_sched_barrier(0);
          }
          // pin the accumulators here: otherwise the SADs are sunk into the
          // (branchy) cost code and all 17 rows of loads stay live
#pragma unroll
          for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(a0[k]), "+v"(a1[k]));
        }
        const int ox = tx - R;
        const int candx = g.cqx + 4 * ox;     // candidate MV (qpel, relative to the block)
        auto eval_position = [&](const uint32_t (&acc)[16], int oyw) {
          const int oy = oyw - R;
          uint32_t ps[kNS];
          partition_sads(acc, ps);
          PosCtx c;
          c.lring = max(abs(ox), abs(oy));
          const int sidx = spiral_index_bl(ox, oy);
          const int candy = g.cqy + 4 * oy;
          c.is00 = (candx == 0) && (candy == 0);
          c.rank = FFS ? ((g.preseed && c.is00) ? 0u : (uint32_t)sidx + 1u) : (uint32_t)sidx;
          const MvCost mc = mv_cost<FFS>(candx, candy, g.px, g.py, g.lam, g.max_mvd);
          c.mvc = mc.mvc;
          c.ok = mc.ok;
          c.mvc0 = g.chk00 ? check00_adjust(mc.mvc, g.lam, c.is00) : mc.mvc;
          update_slots<KEY32, FFS, decltype(all_tag)::value>(ps, g, c, best);
        };
#ifdef JMME_ABL_NOCOST   // timing ablation only: keep the SADs live, skip the cost/minimum work
#pragma unroll
        for (int k = 0; k < 16; ++k) asm volatile("" :: "v"(a0[k]), "v"(a1[k]));
        (void)eval_position;
#else
        eval_position(a0, 2 * ty);
        if (2 * ty + 1 < D) eval_position(a1, 2 * ty + 1);   // odd D: last pair has one position
#endif
        tx += rstep;
        ty += qstep;
        if (tx >= D) { tx -= D; ++ty; }
      }
    };
    if (gmask == kAll) sweep(std::integral_constant<bool, true>{});
    else sweep(std::integral_constant<bool, false>{});
    STAMP(st_sweep);

    // ---- workgroup reduction of this group's per-thread minima
#pragma unroll
    for (int s = 0; s < kNS; ++s) {
      if (!((gmask >> s) & 1)) continue;
      Best k = best[s];
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        if (KEY32) {
          const uint32_t o = __shfl_xor((uint32_t)k, off, 64);
          k = min((uint32_t)k, o);
        } else {
          const unsigned lo = __shfl_xor((unsigned)k, off, 64);
          const unsigned hi = __shfl_xor((unsigned)((unsigned long long)k >> 32), off, 64);
          const unsigned long long o = ((unsigned long long)hi << 32) | lo;
          k = o < (unsigned long long)k ? o : k;
        }
      }
      if (lane == 0) L.red[wave * kNS + s] = (unsigned long long)k;
    }
    __syncthreads();
    if (tid < kNS) {
      unsigned long long k = L.red[tid];
#pragma unroll
      for (int w = 1; w < kWaves; ++w) { const unsigned long long o = L.red[w * kNS + tid]; k = o < k ? o : k; }
      L.red[tid] = k;   // wave 0's row now holds the group result
    }
    __syncthreads();
    STAMP(st_reduce);

    // ---- refine (32-bit keys): recover the 3 rank bits the key dropped.
    // The winner has cost == key>>10 and rank in [8c, 8c+8), c = key & 1023;
    // re-evaluate those positions exactly and take the smallest matching rank.
    if (KEY32) {
      const int D = 2 * R + 1;
      for (int item = tid; item < kNS * kCand; item += kWG) {
        const int s = item / kCand, j = item - s * kCand;
        uint32_t m = 0;
        const uint32_t key = (uint32_t)L.red[s];
        if (((gmask >> s) & 1) && key != ~0u) {
          const uint32_t mincost = key >> kCostShift;
          const int rk = (int)(((key & ((1u << kCostShift) - 1)) << kRankDrop) + j);
          int ox = 0, oy = 0;
          bool valid;
          if (FFS && rk == 0) {          // the pre-seeded (0,0) vector
            ox = -(g.cqx >> 2); oy = -(g.cqy >> 2);
            valid = g.preseed && abs(ox) <= R && abs(oy) <= R;
          } else {
            const int sidx = FFS ? rk - 1 : rk;
            valid = sidx < D * D;
            if (valid) spiral_offset(sidx, &ox, &oy);
          }
          if (valid) {
            const int candx = g.cqx + 4 * ox, candy = g.cqy + 4 * oy;
            PosCtx c;
            c.is00 = (candx == 0) && (candy == 0);
            c.lring = max(abs(ox), abs(oy));
            const int sidx = spiral_index(ox, oy);
            c.rank = FFS ? ((g.preseed && c.is00) ? 0u : (uint32_t)sidx + 1u) : (uint32_t)sidx;
            const MvCost mc = mv_cost<FFS>(candx, candy, g.px, g.py, g.lam, g.max_mvd);
            c.ok = mc.ok;
            const uint32_t mv = (s == 0 && g.chk00) ? check00_adjust(mc.mvc, g.lam, c.is00) : mc.mvc;
            const uint32_t cost = (partition_sad_at(L, s, ox + R, oy + R) << 5) + mv;
            m = (c.rank == (uint32_t)rk) && cost == mincost && slot_eligible<FFS>(g, c, s);
          }
        }
        L.match[item] = m;
      }
      __syncthreads();
    }
    STAMP(st_refine);

    // ---- results of this group
    if (tid < kNS && ((gmask >> tid) & 1)) {
      const unsigned long long k = L.red[tid];
      jmme_block_res res;
      res.reserved = 0;
      uint32_t rank = 0, cost = 0;
      bool found = false;
      if (KEY32) {
        const uint32_t key = (uint32_t)k;
        if (key != ~0u) {
          for (int j = 0; j < kCand && !found; ++j)
            if (L.match[tid * kCand + j]) {
              found = true;
              rank = ((key & ((1u << kCostShift) - 1)) << kRankDrop) + j;
            }
          cost = key >> kCostShift;
          if (!found) atomicOr(p.status, 4u);   // cannot happen: refine lost the winner
        }
      } else if (k != ~0ull) {
        found = true;
        rank = (uint32_t)(k & 0x7fffffffu);
        cost = (uint32_t)(k >> 32);
      }
      if (!found) {
        // nothing eligible: JM leaves best_pos = 0 and returns the incoming min_mcost
        res.mv_x = (int16_t)g.cqx; res.mv_y = (int16_t)g.cqy; res.cost = JMME_DISTBLK_MAX;
      } else {
        int ox, oy;
        if (FFS && rank == 0) { ox = -(g.cqx >> 2); oy = -(g.cqy >> 2); }   // the pre-seeded (0,0)
        else spiral_offset(FFS ? (int)rank - 1 : (int)rank, &ox, &oy);
        res.mv_x = (int16_t)(g.cqx + 4 * ox);
        res.mv_y = (int16_t)(g.cqy + 4 * oy);
        res.cost = (int64_t)cost;
      }
      p.out[(size_t)u * kNS + tid] = res;
    }
    STAMP(st_out);
  }
#ifdef JMME_STAMPS
  if (p.stamps && tid == 0) {
    unsigned long long *o = p.stamps + (size_t)u * 8;
    o[0] = st_setup; o[1] = st_stage; o[2] = st_sweep; o[3] = st_reduce; o[4] = st_refine; o[5] = st_out;
    o[6] = __builtin_popcountll(slot_mask); o[7] = 1;
  }
#endif
}

// direct pass: one workgroup per unit (XCD-aware order)
template <bool KEY32, bool FFS>
__global__ __launch_bounds__(kWG, KEY32 ? JMME_WAVES_PER_EU : 2) void me_units_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int u = xcd_unit(blockIdx.x, gridDim.x);
  if (u >= p.n) return;
  unit_body<KEY32, FFS>(p, u, smem);
}

// deferred pass (64-bit keys): a small grid drains the device-side list of
// units the 32-bit pass could not take; every workgroup exits when the list ends
template <bool FFS>
__global__ __launch_bounds__(kWG, 1) void me_units_deferred_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const unsigned cnt = *p.unit_count;
  for (unsigned i = blockIdx.x; i < cnt; i += gridDim.x) {
    unit_body<false, FFS>(p, p.unit_list[i], smem);
    __syncthreads();
  }
}

}  // namespace

size_t units_lds_bytes(int R) {
  const int rows = 2 * R + 16;
  const int wp = (2 * R + 13) | 1;
  size_t off = (size_t)rows * wp * 4;
  off = (off + 15) & ~(size_t)15;
  off += (size_t)rows * lds_rawp(R);
  off = (off + 15) & ~(size_t)15;
  off += 64 * 4 + kNS * 16 + kNS * 8 + kWaves * kNS * 8 + kNS * kCand * 4 + 16;
  return off;
}

hipError_t launch_units(const KParams &p, bool key32, int grid, hipStream_t s) {
  const size_t lds = units_lds_bytes(p.lds_range);
  const bool ffs = p.mode == JMME_FAST_FULL_SEARCH;
  if (p.unit_list) {
    if (ffs) hipLaunchKernelGGL(me_units_deferred_kernel<true>, dim3(grid), dim3(kWG), lds, s, p);
    else hipLaunchKernelGGL(me_units_deferred_kernel<false>, dim3(grid), dim3(kWG), lds, s, p);
  } else if (key32) {
    if (ffs) hipLaunchKernelGGL((me_units_kernel<true, true>), dim3(grid), dim3(kWG), lds, s, p);
    else hipLaunchKernelGGL((me_units_kernel<true, false>), dim3(grid), dim3(kWG), lds, s, p);
  } else {
    if (ffs) hipLaunchKernelGGL((me_units_kernel<false, true>), dim3(grid), dim3(kWG), lds, s, p);
    else hipLaunchKernelGGL((me_units_kernel<false, false>), dim3(grid), dim3(kWG), lds, s, p);
  }
  return hipGetLastError();
}

}  // namespace jmme
