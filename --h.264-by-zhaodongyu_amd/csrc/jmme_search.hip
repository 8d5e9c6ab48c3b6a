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
// the result is the lexicographic minimum of (cost, spiral index) over all
// eligible candidates.  We evaluate every candidate exhaustively and reduce
// that key; no early exit, same answer.
//
// Work mapping (one workgroup = one MB x ref unit, 256 threads):
//   * partitions are grouped by identical search window (FS: centre + range;
//     FFS: the MB's single surface); each group stages its reference window
//     (2R+16)^2 pels from HBM into LDS once, as "word[y][x] = pels x..x+3" so
//     every SAD row read is an aligned ds_read_b32;
//   * each thread takes search positions; for one position it forms the 16
//     4x4 SADs with v_sad_u8 (4 abs-diffs per lane-op; the current MB row is a
//     broadcast ds_read_b128), sums them to the 41 partition SADs and updates
//     a running (cost, rank) minimum per partition in registers;
//   * partitions that share a predictor share the mv-cost arithmetic;
//   * at the end a wave shuffle + LDS reduction produces the 41 results.
#include <hip/hip_runtime.h>
#include <type_traits>
#include "jmme.h"
#include "jmme_common.h"
#include "jmme_internal.h"

namespace jmme {

namespace {

constexpr int kNS = JMME_NSLOT;
constexpr int kWaves = kWG / 64;
constexpr int kKey32First = 9;
#ifndef JMME_WAVES_PER_EU
#define JMME_WAVES_PER_EU 2
#endif                 // slots 9..40 (8x4, 4x8, 4x4) use 32-bit keys

struct Lds {
  int wp;        // words per window row
  int rawp;      // bytes per raw row
  int rows;      // window rows
  uint32_t *words;
  uint8_t *raw;
  uint32_t *cur;          // 64 words: row r, column group c at [r*4+c]
  int4 *slot;             // 41 x jmme_block_req
  unsigned long long *grp;  // per slot: mask of slots sharing its window
  unsigned long long *cls;  // per slot: mask of slots sharing its predictor/lambda
  unsigned long long *red;  // kWaves x 41 reduction scratch
  int *flag;                // unit must be redone with 64-bit keys
};

__device__ __forceinline__ Lds carve(unsigned char *smem, int R) {
  Lds L;
  L.rows = 2 * R + 16;
  L.wp = (2 * R + 13) | 1;
  L.rawp = 4 * ((3 + 2 * R + 13 + 2) / 4 + 2);
  size_t off = 0;
  L.words = reinterpret_cast<uint32_t *>(smem + off); off += (size_t)L.rows * L.wp * 4;
  off = (off + 15) & ~(size_t)15;
  L.raw = smem + off;                                    off += (size_t)L.rows * L.rawp;
  off = (off + 15) & ~(size_t)15;
  L.cur = reinterpret_cast<uint32_t *>(smem + off);      off += 64 * 4;
  L.slot = reinterpret_cast<int4 *>(smem + off);         off += kNS * 16;
  L.grp = reinterpret_cast<unsigned long long *>(smem + off); off += kNS * 8;
  L.cls = reinterpret_cast<unsigned long long *>(smem + off); off += kNS * 8;
  L.red = reinterpret_cast<unsigned long long *>(smem + off); off += kWaves * kNS * 8;
  L.flag = reinterpret_cast<int *>(smem + off);            off += 16;
  return L;
}

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

constexpr unsigned long long kAll = (1ull << kNS) - 1;
constexpr uint32_t kKey32MaxLambda = 3556;   // lambda*74 + 8x4 SAD<<5 < 2^19: 32-bit keys exact

// the 41 partition SADs from the 16 4x4 SADs; JM sums them in
// update_full_search_large_blocks (me_fullfast.c:196-260) -- integer sums, any order
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

struct SlotCtx {
  uint32_t mvc, rank;
  int lring;
  bool is00, ok;
  int chk00, lam;
  bool preseed;
  unsigned long long rlim;
  const int4 *slot;
  int candx, candy, max_mvd;
};

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

// Per-slot minimum update.  ps[] holds UNSCALED partition SADs.
//  * 32-bit key (slots 9..40 when KEY32): (cost << 13) | rank with
//    cost = SAD<<5 + mvc  ==  (SAD << 18) + K32,  K32 = (mvc << 13) | rank
//    (exact: the lambda guard keeps cost < 2^19), i.e. ONE v_lshl_add_u32
//    and one v_min_u32 per partition;
//  * 64-bit key otherwise: hi = SAD<<5 + mvc (one v_lshl_add_u32), lo = rank.
template <bool KEY32, bool FFS, bool ALL, int NB64, int NB32>
__device__ __forceinline__ void update_slots(const uint32_t (&ps)[kNS], unsigned long long cmask,
                                             const SlotCtx &c, unsigned long long (&best64)[NB64],
                                             uint32_t (&best32)[NB32]) {
  const uint32_t k32 = (c.mvc << 13) | c.rank;
#pragma unroll
  for (int s = 0; s < kNS; ++s) {
    if (!ALL && !((cmask >> s) & 1)) continue;
    bool oks = c.ok;
    if (FFS && ((c.rlim >> s) & 1)) {
      // FFS partition searched over a smaller range than the surface (me_fullfast.c:627)
      const int rs = ufl(rq_range(c.slot[s]));
      oks = oks && (c.lring <= rs || (c.preseed && c.is00));
    }
    if (KEY32 && s >= kKey32First) {
      const uint32_t k = (ps[s] << 18) + k32;
      best32[s - kKey32First] = min(best32[s - kKey32First], FFS ? (oks ? k : ~0u) : k);
    } else {
      uint32_t m = c.mvc;
      if (!FFS && s == 0 && c.chk00) {
        const uint32_t t = 16u * (uint32_t)c.lam;           // weighted_cost(lambda,16), me_fullsearch.c:80
        if (c.is00) m = m > t ? m - t : 0u;
      }
      const uint32_t hi = (ps[s] << 5) + m;
      const unsigned long long k = ((unsigned long long)hi << 32) | c.rank;
      const unsigned long long kk = FFS ? (oks ? k : ~0ull) : k;
      best64[s] = best64[s] < kk ? best64[s] : kk;
    }
  }
}

template <bool KEY32, bool FFS>
__device__ __forceinline__ void unit_body(const KParams &p, int u, unsigned char *smem) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  constexpr bool ffs = FFS;

  const jmme_mb_req *rq = p.req + u;
  const int mb_x = ufl(rq->mb_x);
  const int mb_y = ufl(rq->mb_y);
  const int list = ufl(rq->list);
  const int ref_idx = ufl(rq->ref_idx);
  const unsigned long long slot_mask = ufl64(rq->slot_mask) & ((1ull << kNS) - 1);
  const int ffs_cx = ufl(rq->ffs_center_x);
  const int ffs_cy = ufl(rq->ffs_center_y);
  const int ffs_range = ufl(rq->ffs_range);
  const bool preseed = ffs && ufl(rq->ffs_pos00_valid) != 0;
  const uint8_t *ref = p.refs[list * kMaxRefs + ref_idx];

  Lds L = carve(smem, p.lds_range);

  // ---- unit setup: slot requests, window groups, predictor classes, current MB
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
    int4 me = L.slot[tid];
    unsigned long long g = 0, c = 0;
    if ((slot_mask >> tid) & 1) {
      for (int t = 0; t < kNS; ++t) {
        if (!((slot_mask >> t) & 1)) continue;
        int4 o = L.slot[t];
        // a group = partitions with the same search window AND the same
        // predictor/lambda: one SAD sweep and one mv-cost per position serve
        // the whole group (a window with several predictors is swept once per
        // predictor -- straight-line code, no per-partition predictor loads)
        bool same_win = ffs || (o.y == me.y && rq_range(o) == rq_range(me));
        bool same_cls = same_win && o.x == me.x && o.w == me.w;
        g |= (unsigned long long)same_cls << t;
        c |= (unsigned long long)same_win << t;
      }
    }
    L.grp[tid] = g;
    L.cls[tid] = c;
    // 32-bit keys are exact only while lambda*74 + SAD<<5 < 2^19 (kKey32MaxLambda)
    if (KEY32 && ((slot_mask >> tid) & 1) && (uint32_t)rq_lambda(me) > kKey32MaxLambda) L.flag[0] = 1;
  }
  __syncthreads();
  if (KEY32 && ufl(L.flag[0])) {
    // redo the whole unit with 64-bit keys in the deferred pass
    if (tid == 0) p.defer_list[atomicAdd(p.defer_count, 1u)] = u;
    return;
  }

  // One pass per search window (group of partitions sharing it): stage the
  // window, sweep it, reduce and write that group's results.  Nothing is
  // carried from one group to the next.
  unsigned long long remaining = slot_mask;
  while (remaining) {
    const int lead = __builtin_ctzll(remaining);
    const unsigned long long gmask = ufl64(L.grp[lead]) & remaining;
    remaining &= ~gmask;
    // per-thread running minima of the (cost, rank) keys
    unsigned long long best64[KEY32 ? kKey32First : kNS];
    uint32_t best32[KEY32 ? kNS - kKey32First : 1];
#pragma unroll
    for (int s = 0; s < (KEY32 ? kKey32First : kNS); ++s) best64[s] = ~0ull;
#pragma unroll
    for (int s = 0; s < (KEY32 ? kNS - kKey32First : 1); ++s) best32[s] = ~0u;
    const int4 lq = L.slot[lead];
    const int cqx = ufl(ffs ? ffs_cx : rq_cen_x(lq));   // window centre, qpel (multiple of 4)
    const int cqy = ufl(ffs ? ffs_cy : rq_cen_y(lq));
    const int R = ufl(ffs ? ffs_range : rq_range(lq));
    if (R < 0 || R > p.lds_range || ((cqx | cqy) & 3)) {
      // outside what this launch was sized for (or a sub-pel-grid centre):
      // refuse loudly instead of overrunning LDS; the host reports it
      if (tid == 0) atomicOr(p.status, (R < 0 || R > p.lds_range) ? 1u : 2u);
      continue;
    }
    // FFS: partitions searched over a smaller range than the surface (me_fullfast.c:627)
    unsigned long long rlim = 0;
    if (ffs) {
      for (int t = 0; t < kNS; ++t)
        if ((gmask >> t) & 1) rlim |= (unsigned long long)(rq_range(L.slot[t]) < R) << t;
      rlim = ufl64(rlim);
    }
    const int chk00 = ufl((!ffs && (gmask & 1)) ? (rq_flags(L.slot[0]) & JMME_BLK_CHECK00) : 0);
    const int cls_px = ufl(rq_pred_x(lq));
    const int cls_py = ufl(rq_pred_y(lq));
    const int cls_lam = ufl(rq_lambda(lq));

    // ---- stage the (2R+16)^2 reference window, clamped like UMVLine4X.
    // Rows are clamped into the picture; when the window's columns lie
    // inside the picture each row is fetched as aligned dwords (one round
    // trip, all loads in flight), else byte by byte with column clamping.
    const int x0 = mb_x + (cqx >> 2) - R;
    const int y0 = mb_y + (cqy >> 2) - R;
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

    // ---- sweep all (2R+1)^2 positions of the window.  A task is a vertical
    // pair of positions (x, y), (x, y+1): the 17 reference rows they need are
    // read from LDS once and feed both (halves the LDS traffic per position).
    // the sweep, specialised for a window that serves all 41 partitions (no
    // per-partition mask tests) or a subset
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
          uint4 cprev = make_uint4(0, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 17; ++r) {
            const uint32_t *w = wrow + r * L.wp;
#ifdef JMME_ABL_NOLDS    // timing ablation only: no window reads
            const uint32_t w0 = r * 0x01010101u + tx, w1 = w0 ^ 1, w2 = w0 ^ 2, w3 = w0 ^ 3;
            (void)w;
#else
            const uint32_t w0 = w[0], w1 = w[4], w2 = w[8], w3 = w[12];
#endif
            if (r < 16) {   // row r of the MB against position y
              const uint4 c = cur4[r];
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
            if (r < 16) cprev = cur4[r];
            // bound the scheduler's look-ahead: a few rows of loads in flight,
            // not all 17 (which would pin ~140 VGPRs)
            if ((r & 1) == 1) __builtin_amdgcn_sched_barrier(0);
          }
          // pin the accumulators here: otherwise the SADs are sunk into the
          // (branchy) cost code and all 17 rows of loads stay live
#pragma unroll
          for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(a0[k]), "+v"(a1[k]));
        }
        const int ox = tx - R;
        const int candx = cqx + 4 * ox;     // candidate MV (qpel, relative to the block)
        auto eval_position = [&](const uint32_t (&acc)[16], int oyw) {
          const int oy = oyw - R;
          uint32_t ps[kNS];
          partition_sads(acc, ps);
          const int lring = max(abs(ox), abs(oy));
          const int sidx = spiral_index_bl(ox, oy);
          const int candy = cqy + 4 * oy;
          const bool is00 = (candx == 0) && (candy == 0);
          const uint32_t rank = ffs ? ((preseed && is00) ? 0u : (uint32_t)sidx + 1u) : (uint32_t)sidx;
          const MvCost mc = mv_cost<FFS>(candx, candy, cls_px, cls_py, cls_lam, p.max_mvd);
          SlotCtx c{mc.mvc, rank, lring, is00, mc.ok, chk00, cls_lam, preseed, rlim, L.slot, candx, candy, p.max_mvd};
          update_slots<KEY32, FFS, decltype(all_tag)::value>(ps, gmask, c, best64, best32);
        };
#ifdef JMME_ABL_NOCOST   // timing ablation only: keep the SADs live, skip the cost/minimum work
#pragma unroll
        for (int k = 0; k < 16; ++k) asm volatile("" :: "v"(a0[k]), "v"(a1[k]));
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

    // ---- workgroup reduction of this group's per-thread minima
#pragma unroll
    for (int s = 0; s < kNS; ++s) {
      if (!((gmask >> s) & 1)) continue;
      unsigned long long k;
      if (KEY32 && s >= kKey32First) {
        const uint32_t v = best32[s - kKey32First];
        k = (v == ~0u) ? ~0ull : ((((unsigned long long)(v >> 13)) << 32) | (v & 8191u));
      } else {
        k = best64[s];
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const unsigned lo = __shfl_xor((unsigned)k, off, 64);
        const unsigned hi = __shfl_xor((unsigned)(k >> 32), off, 64);
        const unsigned long long o = ((unsigned long long)hi << 32) | lo;
        k = o < k ? o : k;
      }
      if (lane == 0) L.red[wave * kNS + s] = k;
    }
    __syncthreads();
    if (tid < kNS && ((gmask >> tid) & 1)) {
      unsigned long long k = L.red[tid];
#pragma unroll
      for (int w = 1; w < kWaves; ++w) { const unsigned long long o = L.red[w * kNS + tid]; k = o < k ? o : k; }
      const int cx = cqx, cy = cqy;
      jmme_block_res res;
      res.reserved = 0;
      if (k == ~0ull) {
        // nothing eligible: JM leaves best_pos = 0 and returns the incoming min_mcost
        res.mv_x = (int16_t)cx; res.mv_y = (int16_t)cy; res.cost = JMME_DISTBLK_MAX;
      } else {
        const uint32_t rank = (uint32_t)(k & 0x7fffffffu);
        const int sidx = ffs ? (int)rank - 1 : (int)rank;
        int ox, oy;
        if (ffs && rank == 0) { ox = -(cx >> 2); oy = -(cy >> 2); }   // the pre-seeded (0,0)
        else spiral_offset(sidx, &ox, &oy);
        res.mv_x = (int16_t)(cx + 4 * ox);
        res.mv_y = (int16_t)(cy + 4 * oy);
        res.cost = (int64_t)(k >> 32);
      }
      p.out[(size_t)u * kNS + tid] = res;
    }
  }
}

// direct pass: one workgroup per unit (XCD-aware order)
template <bool KEY32, bool FFS>
__global__ __launch_bounds__(kWG, JMME_WAVES_PER_EU) void me_units_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int u = xcd_unit(blockIdx.x, gridDim.x);
  if (u >= p.n) return;
  unit_body<KEY32, FFS>(p, u, smem);
}

// deferred pass (64-bit keys): a small grid drains the device-side list of
// units whose 32-bit keys saturated; every workgroup exits when the list ends
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
  const int rawp = 4 * ((3 + 2 * R + 13 + 2) / 4 + 2);
  size_t off = (size_t)rows * wp * 4;
  off = (off + 15) & ~(size_t)15;
  off += (size_t)rows * rawp;
  off = (off + 15) & ~(size_t)15;
  off += 64 * 4 + kNS * 16 + 2 * kNS * 8 + kWaves * kNS * 8 + 16;
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
