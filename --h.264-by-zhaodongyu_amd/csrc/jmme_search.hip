// jmme_search.hip -- gfx950 kernels for JM 18.5 integer-pel full search (FS)
// and fast full search (FFS).
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
// Work decomposition:
//   * plan kernel (one wave per MB x ref unit): the unit's partitions are
//     grouped by identical search window AND predictor/lambda (FS: centre +
//     range + predictor; FFS: the MB's surface + predictor).  Each group is a
//     work Item; one SAD sweep serves every partition of the group.  Units
//     whose lambda could overflow the 32-bit key go to the 64-bit item list.
//   * item kernels (persistent, one 256-thread workgroup per CU slot, items
//     statically dealt in contiguous runs per XCD so neighbouring macroblocks'
//     overlapping windows hit the same L2): while item k is swept, item k+1's
//     reference window and current MB stream HBM -> LDS with
//     global_load_lds (no VGPRs held), so the sweep hides the fetch latency;
//   * window in LDS as "word[y][x] = pels x..x+3": every SAD row read is an
//     aligned ds_read_b32;
//   * the current MB lives in SGPRs (64 dwords, read once per item): every
//     v_sad uses it as its scalar operand, so the LDS only serves the window;
//   * a thread takes a vertical TRIPLE of search positions: the 18 reference
//     rows they need are read once and feed 3 x 16 4x4 SAD chains;
//   * key (fast path): 32 bits = cost << 11 | rank >> 2, built without a
//     shift per partition: a 4x4 chain starts from K(pos) = mvcost << 11 |
//     rank >> 2 and v_sad_hi_u8 adds SAD << 16 (= (32 * SAD) << 11), so the
//     chain ends on the 4x4 key; a larger partition's key is a + b - K (one
//     v_add3_u32); the 16x16 key, whose SAD may reach 65280, is a saturating
//     add.  One v_min_u32 per partition and position folds it.  The 2 dropped
//     rank bits are recovered exactly afterwards: the winner's rank lies in
//     [4c, 4c+4), and those <= 4 positions are re-evaluated per partition;
//   * JM's special (0,0) candidate (check_for_00's discount, FFS's pre-seed
//     with rank 0) is evaluated once per item after the sweep, not per position;
//   * key (exact fallback): 64 bits = cost << 32 | rank, for ranges > 44,
//     huge lambdas, FFS windows the GetMaxMVD gate cuts, and a 16x16 whose
//     every key saturated.
#include <hip/hip_runtime.h>
#include <type_traits>
#include "jmme.h"
#include "jmme_common.h"
#include "jmme_internal.h"
#include "jmme_subpel_dev.h"

namespace jmme {

namespace {

constexpr int kNS = JMME_NSLOT;
constexpr int kWaves = kWG / 64;
constexpr unsigned long long kAll = (1ull << kNS) - 1;
constexpr int kCostShift = 11;             // key32 = cost << 11 | rank >> 2
constexpr int kRankDrop = 2;
constexpr int kCand = 1 << kRankDrop;      // refine candidates per partition
constexpr int kPlanWaves = 16;             // plan kernel: units per workgroup
constexpr int kRed1 = (kNS + 3) / 4 * 2;      // reduce: registers after the permlane32 level (22)
constexpr int kRed2 = kRed1 / 2;              //         ... after the permlane16 level (11)

// v6 sweep (default): a fold reduce-scatters its keys across the wave at once
// into 11 registers (kRed2), so no wave keeps 41 per-lane minima through the
// sweep; the freed registers pay for 5 positions per task (13 task rows at
// R = 32, no redundant rows).
#ifndef JMME_SWEEP_P
#define JMME_SWEEP_P 5   // positions per sweep task (vertical run)
#endif
#ifndef JMME_WAVES_PER_EU
#define JMME_WAVES_PER_EU 4
#endif

// dwords per staged raw row: the words of a row read pels x0 .. x0+2R+15,
// fetched as aligned dwords from floor4(x0) (+1 dword for alignbyte's high half)
__host__ __device__ inline int raw_row_dwords(int R) { return (3 + 2 * R + 13 + 2) / 4 + 2; }
// the fetch also carries the item's current MB behind the window (LDS DMA only
// ever targets the raw area, never what the sweep reads)
constexpr int kRawExtra = 64;

struct Lds {
  int wp;                   // words per window row
  int wv;                   // this wave's index in the workgroup (uniform)
  uint32_t *words;          // current item's window, rows x wp
  uint32_t *raw;            // next item as fetched: window rows x nd dwords (dense),
                            // then its current MB (64 dwords)
  uint32_t *cur;            // 64 words: MB row r, column group c at [r*4+c] (static LDS)
  unsigned long long *red;  // kWaves x 41 reduction scratch
  uint4 *tx, *ty;           // per-item position tables (2R+1 each), see build_tabs
  uint32_t *spec;           // 16 4x4 SADs at the special (0,0) candidate, then its 41 keys
  uint32_t *ctr;            // the window centre's 41 keys, then its 16 4x4 SADs (exact elimination)
  uint32_t *tmax;           // per wave: 8 words, the centre's per-size key bounds (elimination test)
  unsigned long long *fb;   // exact 16x16 result of the saturation fallback
};

// words per window row in LDS: the 2R+13 words a row needs, rounded up to the
// expand's groups of 4 (it writes whole groups, 16-B aligned: one ds_write_b128);
// every launch up to R = 32 uses the R = 32 pitch, a compile-time constant of
// the sweep (its row offsets then fold into the ds_read2 offset fields).
// 84, not the 80 a row needs: the sweep's last wave-task (window column 64 at
// R = 32) has its 13 lanes 5 rows apart, and ds_read2_b32 banks are (a/4) mod 32
// -- with 80 they fell on 2 banks (up to 7-way conflicts), with 84 on 8 (at most
// 2-way): SQ_LDS_BANK_CONFLICT 9.0e6 -> 4.4e6 cycles per 1080p launch
// (profiles/round6/lds_pitch/)
#ifndef JMME_WP32
#define JMME_WP32 84
#endif
constexpr int kWP32 = JMME_WP32;
static_assert(kWP32 % 4 == 0 && kWP32 >= 80, "window pitch: whole 16-B groups of the 80 words a row needs at R = 32");
__host__ __device__ inline int words_pitch(int R) { return R <= 32 ? kWP32 : 4 * ((2 * R + 13 + 3) / 4); }
// 16-bit planes (SourceBitDepthLuma 9..14, KEY32 = false only): word[y][x] =
// samples x, x + 1 (a 4-sample chunk is words x and x + 2), 2R + 15 words a
// row, expanded in groups of 4 from the raw dwords of 2 samples each
__host__ __device__ inline int groups16(int R) { return (2 * R + 15 + 3) / 4; }
__host__ __device__ inline int words_pitch16(int R) { return R <= 32 ? kWP32 : 4 * groups16(R); }
__host__ __device__ inline int raw_row_dwords16(int R) { return 2 * groups16(R) + 2; }
constexpr int kRawExtra16 = 128;   // the current MB: 16 rows x 8 dwords

// one layout for the kernel (carve) and the host (items_lds_bytes)
struct LdsPlan { size_t words, raw, red, tx, ty, spec, ctr, tmax, fb, total; };
__host__ __device__ inline LdsPlan lds_plan(int R, bool hbd = false) {
  LdsPlan q;
  const int rows = 2 * R + 16, wp = hbd ? words_pitch16(R) : words_pitch(R), d = 2 * R + 1;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t at = off; off = (off + bytes + 15) & ~(size_t)15; return at; };
  q.words = take((size_t)rows * wp * 4);
  q.raw = take(hbd ? ((size_t)rows * raw_row_dwords16(R) + kRawExtra16) * 4
                   : ((size_t)rows * raw_row_dwords(R) + kRawExtra) * 4);
  q.red = take((size_t)kWaves * kNS * 8);
  q.tx = take((size_t)d * 16);
  q.ty = take((size_t)d * 16);
  q.spec = take((16 + kNS) * 4);
  q.ctr = take((kNS + 16) * 4);
  q.tmax = take(kWaves * 8 * 4);
  q.fb = take(2 * kWaves * 8);   // two halves: successive exact_slot calls alternate
  q.total = off;
  return q;
}

__device__ __forceinline__ Lds carve(unsigned char *smem, int R, bool hbd = false) {
  Lds L;
  const LdsPlan q = lds_plan(R, hbd);
  L.wp = hbd ? words_pitch16(R) : words_pitch(R);
  L.wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  L.words = reinterpret_cast<uint32_t *>(smem + q.words);
  L.raw = reinterpret_cast<uint32_t *>(smem + q.raw);
  L.red = reinterpret_cast<unsigned long long *>(smem + q.red);
  L.tx = reinterpret_cast<uint4 *>(smem + q.tx);
  L.ty = reinterpret_cast<uint4 *>(smem + q.ty);
  L.spec = reinterpret_cast<uint32_t *>(smem + q.spec);
  L.ctr = reinterpret_cast<uint32_t *>(smem + q.ctr);
  L.tmax = reinterpret_cast<uint32_t *>(smem + q.tmax);
  L.fb = reinterpret_cast<unsigned long long *>(smem + q.fb);
  return L;
}

// Diagnostic phase clocks (build with -DJMME_STAMPS; never in the shipped
// library): s_memtime at phase boundaries, summed per unit by lane 0.
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

// the thread index, rebuilt where it is used from the lane count (an opaque
// v_mbcnt pair the compiler can neither hoist nor merge) and the wave index,
// which is uniform and lives in an SGPR: nothing derived from threadIdx.x is
// hoisted out of the item loop and kept live -- spilled -- across the sweep
__device__ __forceinline__ int opaque_tid(const Lds &L) {
  unsigned t;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(t));
  return (int)(t + ((unsigned)L.wv << 6));
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// LDS reads of the sweep.  Plain loads: the compiler tracks them (an inline-asm
// load would let it copy the destination before the data lands).
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const uint32_t lds_u32;
__device__ __forceinline__ uint32_t lds_addr(const void *p) { return (uint32_t)(uintptr_t)p; }
__device__ __forceinline__ u32x2 ds_read2_0_4(uint32_t a) { const lds_u32 *q = (const lds_u32 *)(uintptr_t)a; return u32x2{q[0], q[4]}; }
__device__ __forceinline__ u32x2 ds_read2_8_12(uint32_t a) { const lds_u32 *q = (const lds_u32 *)(uintptr_t)a; return u32x2{q[8], q[12]}; }
__device__ __forceinline__ u32x4 ds_read_b128(uint32_t a) {
  return *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>((const lds_u32 *)(uintptr_t)a);
}

// slot request fields from the int4 image of jmme_block_req
__device__ __forceinline__ int rq_pred_x(int4 q) { return (int)(short)(q.x & 0xffff); }
__device__ __forceinline__ int rq_pred_y(int4 q) { return (int)(short)((unsigned)q.x >> 16); }
__device__ __forceinline__ int rq_cen_x(int4 q) { return (int)(short)(q.y & 0xffff); }
__device__ __forceinline__ int rq_cen_y(int4 q) { return (int)(short)((unsigned)q.y >> 16); }
__device__ __forceinline__ int rq_range(int4 q) { return (int)(short)(q.z & 0xffff); }
__device__ __forceinline__ int rq_flags(int4 q) { return (int)(short)((unsigned)q.z >> 16); }
__device__ __forceinline__ int rq_lambda(int4 q) { return q.w; }

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

// spiral_offset (jmme_common.h) without the ring loop: ring l = (isqrt(idx)+1)/2
__device__ __forceinline__ void spiral_offset_fast(int idx, int *ox, int *oy) {
  int q = (int)sqrtf((float)idx);
  q -= q * q > idx;
  q += (q + 1) * (q + 1) <= idx;
  const int l = (q + 1) >> 1;
  int r = idx - (2 * l - 1) * (2 * l - 1);
  if (idx <= 0) { *ox = 0; *oy = 0; return; }
  if (r < 2 * (2 * l - 1)) {
    *ox = r / 2 - l + 1;
    *oy = (r & 1) ? l : -l;
  } else {
    r -= 2 * (2 * l - 1);
    *oy = r / 2 - l;
    *ox = (r & 1) ? l : -l;
  }
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
  unsigned long long gmask;
  int rs;
};

// FFS eligibility of a position for the item's partitions: the GetMaxMVD gate
// (me_fullfast.c:663) and the partition's own range when it is below the
// surface's (me_fullfast.c:627) -- the pre-seeded (0,0) is always a candidate.
// Uniform over the item: partitions are grouped by their range too.
template <bool FFS>
__device__ __forceinline__ bool pos_eligible(const GroupCtx &g, bool gate_ok, int lring, bool is00) {
  if (!FFS) return true;
  return gate_ok && (lring <= g.rs || (g.preseed && is00));
}

template <bool KEY32, bool FFS, bool ALL, typename Best, bool HBD = false>
__device__ __forceinline__ void update_slots(const uint32_t (&ps)[kNS], const GroupCtx &g, const PosCtx &c,
                                             Best (&best)[kNS]) {
  if (KEY32 && HBD) {   // 16-bit samples: a partition SAD may pass 2^16, its key saturates (exact re-search)
    const uint32_t k32 = (c.mvc << kCostShift) | (c.rank >> kRankDrop);
    const uint32_t k32_0 = (c.mvc0 << kCostShift) | (c.rank >> kRankDrop);
#pragma unroll
    for (int s = 0; s < kNS; ++s) {
      if (!ALL && !((g.gmask >> s) & 1)) continue;
      const uint32_t k = ps[s] > 0xffffu ? ~0u : __builtin_elementwise_add_sat(ps[s] << (5 + kCostShift),
                                                                               s == 0 ? k32_0 : k32);
      const uint32_t kk = FFS ? (c.ok ? k : ~0u) : k;
      best[s] = min((uint32_t)best[s], kk);
    }
  } else if (KEY32) {
    const uint32_t k32 = (c.mvc << kCostShift) | (c.rank >> kRankDrop);
    const uint32_t k32_0 = (c.mvc0 << kCostShift) | (c.rank >> kRankDrop);
#pragma unroll
    for (int s = 0; s < kNS; ++s) {
      if (!ALL && !((g.gmask >> s) & 1)) continue;
      // cost<<11 | rank>>2  ==  (SAD << 16) + ((mvc << 11) | rank >> 2); the
      // 16x16 SAD may reach 65280, so its key saturates instead of wrapping
      const uint32_t k = s == 0 ? __builtin_elementwise_add_sat(ps[0] << (5 + kCostShift), k32_0)
                                : (ps[s] << (5 + kCostShift)) + k32;
      const uint32_t kk = FFS ? (c.ok ? k : ~0u) : k;
      best[s] = min((uint32_t)best[s], kk);
    }
  } else {
#pragma unroll
    for (int s = 0; s < kNS; ++s) {
      if (!ALL && !((g.gmask >> s) & 1)) continue;
      const uint32_t hi = (ps[s] << 5) + (s == 0 ? c.mvc0 : c.mvc);
      const unsigned long long k = ((unsigned long long)hi << 32) | c.rank;
      const unsigned long long kk = FFS ? (c.ok ? k : ~0ull) : k;
      best[s] = best[s] < kk ? best[s] : kk;
    }
  }
}

// exact SAD of partition s at window offset (oxw, oyw), for the refine pass
__device__ __forceinline__ uint32_t partition_sad_at(const Lds &L, const uint32_t *cur, int s, int oxw, int oyw) {
  const SlotGeom gm = slot_geom(s);
  uint32_t sad = 0;
  for (int r = 0; r < 4 * gm.h; ++r) {
    const int row = gm.by * 4 + r;
    const uint32_t *w = L.words + (oyw + row) * L.wp + oxw + gm.bx * 4;
    for (int c = 0; c < gm.w; ++c) sad = __builtin_amdgcn_sad_u8(w[4 * c], cur[row * 4 + gm.bx + c], sad);
  }
  return sad;
}

// One 4-pel row of a 4x4 block against the current MB: the window word at
// the block's column (w[0]; 16-bit planes: words x and x + 2 hold the 4
// samples) and the MB row (8-bit: one dword a block; 16-bit: two).
constexpr int cur_words(bool hbd) { return hbd ? 8 : 4; }   // L.cur dwords per MB row
template <bool HBD>
__device__ __forceinline__ uint32_t sad4(const uint32_t *w, const uint32_t *cur_row, int bx, uint32_t acc) {
  if constexpr (HBD)
    return __builtin_amdgcn_sad_u16(w[2], cur_row[2 * bx + 1], __builtin_amdgcn_sad_u16(w[0], cur_row[2 * bx], acc));
  return __builtin_amdgcn_sad_u8(w[0], cur_row[bx], acc);
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {   // full row / bank masks: every lane reads a valid source
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true);
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_min(uint32_t v) {
  // full row/bank masks and in-row patterns: every lane reads a valid source,
  // so the mov folds into v_min_u32_dpp (GCNDPPCombine)
  return min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true));
}

// ------------------------------------------------------------ plan kernel --
// One wave per unit: lane s holds slot s's request; groups found with
// readlane + ballot; items appended with one atomic per workgroup per list.
template <bool FFS>
__global__ __launch_bounds__(64 * kPlanWaves) void me_plan_kernel(KParams p) {
  __shared__ unsigned s_n[kPlanWaves], s_off[kPlanWaves];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int u = blockIdx.x * kPlanWaves + wave;
  // the next launch's counters (this launch's item kernel uses p.counts; stream
  // order puts the next launch after it)
  if (blockIdx.x == 0 && tid < kCountWords) p.counts_next[tid] = 0u;
  int ng = 0;
  bool slow = false;            // a lambda beyond the 32-bit keys: kItemSlow64 items
  unsigned long long my_gm = 0;
  int my_lead = 0;
  if (u < p.n) {
    const jmme_mb_req *rq = p.req + u;
    const unsigned long long mask = ufl64(rq->slot_mask) & kAll;
    const int4 me = lane < kNS ? reinterpret_cast<const int4 *>(&rq->blk[0])[lane] : make_int4(0, 0, 0, 0);
    const bool valid = lane < kNS && ((mask >> lane) & 1);
    slow = p.key32 && __builtin_amdgcn_ballot_w64(valid && (uint32_t)rq_lambda(me) > kMaxLambda32);
    unsigned long long rem = mask;
    while (rem) {
      const int lead = __builtin_ctzll(rem);
      const int ox = __builtin_amdgcn_readlane(me.x, lead);
      const int oy = __builtin_amdgcn_readlane(me.y, lead);
      const int oz = __builtin_amdgcn_readlane(me.z, lead);
      const int ow = __builtin_amdgcn_readlane(me.w, lead);
      // same predictor and lambda; FS also the same window (centre, range)
      // FFS: also the same own range (the eligibility test is then per item)
      const bool eq = valid && me.x == ox && me.w == ow && rq_range(me) == (int)(short)(oz & 0xffff) &&
                      (FFS || me.y == oy);
      const unsigned long long gm = __builtin_amdgcn_ballot_w64(eq) & rem;
      if (lane == ng) { my_gm = gm; my_lead = lead; }
      ++ng;
      rem &= ~gm;
    }
  }
  // list layout: a unit's first group is item u (raster order: neighbouring
  // macroblocks' windows overlap, and the item kernel deals contiguous runs to
  // an XCD); its further groups (1.5 % of the 1080p units) follow the n first
  // ones, one atomic per workgroup
  if (lane == 0) s_n[wave] = ng > 1 ? ng - 1 : 0;
  __syncthreads();
  if (tid == 0) {
    unsigned na = 0;
    for (int w = 0; w < kPlanWaves; ++w) {
      s_off[w] = na;
      na += s_n[w];
    }
    const unsigned ba = na ? atomicAdd(&p.counts[0], na) : 0u;
    for (int w = 0; w < kPlanWaves; ++w) s_off[w] += ba;
  }
  __syncthreads();
  if (u < p.n && ng == 0 && lane == 0) p.items[u].gmask = 0;   // nothing searched
  if (u < p.n && lane < ng) {
    const jmme_mb_req *rq = p.req + u;
    const int4 lq = reinterpret_cast<const int4 *>(&rq->blk[0])[my_lead];
    Item it;
    it.gmask = my_gm;
    it.rs = rq_range(lq);
    it.pad0 = 0;
    it.u = u;
    it.mb_x = rq->mb_x;
    it.mb_y = rq->mb_y;
    const int cqx = FFS ? rq->ffs_center_x : rq_cen_x(lq);
    const int cqy = FFS ? rq->ffs_center_y : rq_cen_y(lq);
    const int R = FFS ? rq->ffs_range : rq_range(lq);
    it.cqx = (int16_t)cqx;
    it.cqy = (int16_t)cqy;
    it.R = (int16_t)R;
    it.flags = (int16_t)(((!FFS && my_lead == 0 && (rq_flags(lq) & JMME_BLK_CHECK00)) ? kItemChk00 : 0) |
                         ((FFS && rq->ffs_pos00_valid) ? kItemPreseed : 0) | (slow ? kItemSlow64 : 0));
    it.px = (int16_t)rq_pred_x(lq);
    it.py = (int16_t)rq_pred_y(lq);
    it.lam = rq_lambda(lq);
    it.ref = rq->list * kMaxRefs + rq->ref_idx;
    it.pad = 0;
    // FFS: a partition's own range above the surface's would index past the
    // position tables and the staged window (device requests skip validate())
    const bool bad_range = R < 0 || R > p.lds_range || it.rs < 0 || it.rs > R;
    if (bad_range || ((cqx | cqy) & 3)) {
      // outside what this launch was sized for (or a sub-pel-grid centre):
      // refuse loudly instead of overrunning LDS; the host reports it
      atomicOr(&p.counts[2], bad_range ? 1u : 2u);
      it.gmask = 0;
    }
    p.items[lane == 0 ? (unsigned)u : (unsigned)p.n + s_off[wave] + lane - 1] = it;
  }
}

// ------------------------------------------------------------ item kernels --
struct Win { int R, x0, y0, wrows, wpr, xa, sh, nd; bool inner; };

template <bool HBD = false>
__device__ __forceinline__ Win win_of(const KParams &p, const Item &it) {
  Win w;
  w.R = it.R;
  w.x0 = it.mb_x + (it.cqx >> 2) - w.R;
  w.y0 = it.mb_y + (it.cqy >> 2) - w.R;
  w.wrows = 2 * w.R + 16;
  if (HBD) {   // two samples a dword: words 0 .. 2R+14, fetched from the even sample at or below x0
    w.wpr = 2 * w.R + 15;
    w.xa = w.x0 & ~1;
    w.sh = w.x0 - w.xa;                    // 0..1
    w.nd = raw_row_dwords16(w.R);
    w.inner = w.xa >= 0 && w.xa + 2 * w.nd <= p.width;
    return w;
  }
  w.wpr = 2 * w.R + 13;                    // words per window row
  w.xa = w.x0 & ~3;                        // dword-aligned start (floor)
  w.sh = w.x0 - w.xa;                      // 0..3
  w.nd = (w.sh + w.wpr + 2) / 4 + 2;       // dwords per row the words read (incl. alignbyte hi)
  w.inner = w.xa >= 0 && w.xa + 4 * w.nd <= p.width;
  return w;
}

// One LDS-DMA dword per lane: lane l's dword lands at LDS byte address
// lds + 4*l (lds wave-uniform, in M0).  Issued from inline asm on purpose:
// with the builtin (__builtin_amdgcn_global_load_lds) the compiler tracks the
// pending DMA and, for every LDS read that follows while it is in flight, waits
// with lgkmcnt(0) -- which undoes the sweep's one-row-ahead pipelining (each
// wait then covers the reads just issued for the next row).  Completion of these
// loads is awaited explicitly (s_waitcnt vmcnt(0) + barrier at the top of the
// next item) before anything reads the destination.
__device__ __forceinline__ void lds_dma_dword(const void *gptr, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(gptr), "s"(lds) : "memory", "m0");
}

// Issue the HBM -> LDS fetch of item `it` (window rows clamped into the
// picture, dword columns clamped into it -- UMVLine4X) and its current MB.  global_load_lds: per-lane global address, LDS destination
// contiguous per wave instruction; completion is awaited (vmcnt) only at the
// top of the next item.
template <bool HBD = false>
__device__ __forceinline__ void prefetch(const KParams &p, const Item &it, const Lds &L) {
  if (!it.gmask) return;
  const int tid = opaque_tid(L), lane = tid & 63, wave = ufl(tid >> 6);
  if constexpr (HBD) {   // 16-bit: pitch in samples, dword d of a row = samples xa + 2d, +1 (clamped dwords)
    const Win w = win_of<true>(p, it);
    const uint16_t *ref = reinterpret_cast<const uint16_t *>(p.refs[it.ref]);
    const int total = w.wrows * w.nd, w2 = p.width >> 1, xq = w.xa >> 1;
    if (w.nd > 64) {
      // rows wider than a wave instruction (R >= 55: nd = 2R + 18 rounded):
      // each row in 64-dword pieces, one wave instruction per piece
      for (int r = wave; r < w.wrows; r += kWaves) {
        const int gy = clampi(w.y0 + r, 0, p.height - 1);
        for (int c0 = 0; c0 < w.nd; c0 += 64) {
          const int d = c0 + lane;
          if (d < w.nd)
            lds_dma_dword(ref + 2 * clampi(xq + d, 0, w2 - 1) + (size_t)gy * p.pitch,
                          (uint32_t)ufl((int)lds_addr(L.raw + r * w.nd + c0)));
        }
      }
    } else {
      const int k = 64 / w.nd;   // >= 1 here
      const int dr = lane / w.nd, d = lane - dr * w.nd;
      const bool act = dr < k;
      const uint16_t *col = ref + 2 * clampi(xq + d, 0, w2 - 1);
      for (int r = wave * k; r < w.wrows; r += kWaves * k) {
        const int rr = r + dr;
        if (act && rr < w.wrows) {
          const int gy = clampi(w.y0 + rr, 0, p.height - 1);
          lds_dma_dword(col + (size_t)gy * p.pitch, (uint32_t)ufl((int)lds_addr(L.raw + r * w.nd)));
        }
      }
    }
    if (wave < 2) {   // the current MB: 16 rows x 8 dwords, rows 8 * wave ..
      const int r = 8 * wave + (lane >> 3), c = lane & 7;
      lds_dma_dword(reinterpret_cast<const uint16_t *>(p.cur) + (size_t)(it.mb_y + r) * p.pitch + it.mb_x + 2 * c,
                    (uint32_t)ufl((int)lds_addr(L.raw + total + 64 * wave)));
    }
    return;
  }
  const Win w = win_of(p, it);
  const uint8_t *ref = p.refs[it.ref];
  const int total = w.wrows * w.nd;
  const int w4 = p.width >> 2, xq = w.xa >> 2;
  // k = 64 / nd whole rows per wave instruction: lane l writes dword l of the
  // instruction's LDS span, i.e. dword l % nd of row l / nd (rows dense, nd
  // dwords each), so the per-lane column and row offset are fixed per item
  const int k = 64 / w.nd;
  const int dr = lane / w.nd, d = lane - dr * w.nd;
  const bool act = dr < k;
  const uint8_t *col = ref + 4 * clampi(xq + d, 0, w4 - 1);
  for (int r = wave * k; r < w.wrows; r += kWaves * k) {
    const int rr = r + dr;
    if (act && rr < w.wrows) {
      const int gy = clampi(w.y0 + rr, 0, p.height - 1);
      lds_dma_dword(col + (size_t)gy * p.pitch, (uint32_t)ufl((int)lds_addr(L.raw + r * w.nd)));
    }
  }
  // behind the window: the current MB (wave 0)
  if (wave == 0) {
    const int r = lane >> 2, c = lane & 3;
    lds_dma_dword(p.cur + (size_t)(it.mb_y + r) * p.pitch + it.mb_x + 4 * c, (uint32_t)ufl((int)lds_addr(L.raw + total)));
  }
}

// raw dwords -> words (word[y][x] = pels x..x+3 of the window)
// inner window, byte shift SH of its first pel inside the first fetched dword:
// words 4g..4g+3 of a row from its fetched dwords g..g+2 (rows r0, r0+rstep, ..;
// the next row's dwords are read before this row's words are written)
template <int SH>
__device__ __forceinline__ void expand_inner(const uint32_t *src, uint32_t *dst, int nd, int wp, int wrows, int r0,
                                             int rstep) {
  int r = r0;
  if (r >= wrows) return;
  uint32_t d0 = src[r * nd], d1 = src[r * nd + 1], d2 = src[r * nd + 2];
  for (;;) {
    const int rn = r + rstep;
    uint32_t e0 = 0, e1 = 0, e2 = 0;
    if (rn < wrows) { e0 = src[rn * nd]; e1 = src[rn * nd + 1]; e2 = src[rn * nd + 2]; }
    u32x4 v;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int b = k + SH;   // byte offset of word 4g+k from dword g (0..6), compile-time
      v[k] = b < 4 ? __builtin_amdgcn_alignbyte(d1, d0, b & 3) : __builtin_amdgcn_alignbyte(d2, d1, b & 3);
    }
    *reinterpret_cast<u32x4 *>(dst + r * wp) = v;   // ds_write_b128 (conflict-free: consecutive lanes, consecutive 16 B)
    if (rn >= wrows) break;
    r = rn; d0 = e0; d1 = e1; d2 = e2;
  }
}

// 16-bit: word x = samples x, x+1 of the window; the 4 words of group g come
// from raw dwords 2g .. 2g+2 (inner), or per sample through v_perm (edges)
__device__ __forceinline__ void expand16(const KParams &p, const Item &it, const Lds &L) {
  const int tid = opaque_tid(L);
  const Win w = win_of<true>(p, it);
  const uint32_t *tail = L.raw + w.wrows * w.nd;
  if (tid < 128) L.cur[tid] = tail[tid];
  const int ng = (w.wpr + 3) >> 2;
  const int rstep = kWG / ng;
  const int r0 = tid / ng, g = tid - r0 * ng;
  if (r0 >= rstep) return;
  uint32_t *dst = L.words + 4 * g;
  if (w.inner) {
    for (int r = r0; r < w.wrows; r += rstep) {
      const uint32_t *rw = L.raw + r * w.nd + 2 * g;
      const uint32_t d0 = rw[0], d1 = rw[1], d2 = rw[2];
      u32x4 v;
      if (w.sh == 0) {
        v[0] = d0; v[1] = __builtin_amdgcn_alignbyte(d1, d0, 2); v[2] = d1; v[3] = __builtin_amdgcn_alignbyte(d2, d1, 2);
      } else {
        v[0] = __builtin_amdgcn_alignbyte(d1, d0, 2); v[1] = d1; v[2] = __builtin_amdgcn_alignbyte(d2, d1, 2); v[3] = d2;
      }
      *reinterpret_cast<u32x4 *>(dst + r * L.wp) = v;
    }
  } else {
    // sample x of the window is picture column gx = clamp(x0 + x, 0, W-1) (UMVLine4X),
    // in fetched dword clamp(gx/2 - xa/2, 0, nd-1), half gx & 1
    const int xq = w.xa >> 1;
    int dq[4];
    uint32_t sel[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 4 * g + k;
      const int q0 = clampi((clampi(w.x0 + c, 0, p.width - 1) >> 1) - xq, 0, w.nd - 1);
      dq[k] = min(q0, w.nd - 2);
      uint32_t sl = 0;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int gx = clampi(w.x0 + c + b, 0, p.width - 1);
        const int q = clampi((gx >> 1) - xq, 0, w.nd - 1);
        const uint32_t byte0 = (uint32_t)(4 * (q - dq[k]) + 2 * (gx & 1));
        sl |= (byte0 | ((byte0 + 1) << 8)) << (16 * b);
      }
      sel[k] = sl;
    }
    for (int r = r0; r < w.wrows; r += rstep) {
      const uint32_t *rw = L.raw + r * w.nd;
      u32x4 v;
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_perm(rw[dq[k] + 1], rw[dq[k]], sel[k]);
      *reinterpret_cast<u32x4 *>(dst + r * L.wp) = v;
    }
  }
}

__device__ __forceinline__ void expand(const KParams &p, const Item &it, const Lds &L) {
  const int tid = opaque_tid(L);
  const Win w = win_of(p, it);
  const uint32_t *tail = L.raw + w.wrows * w.nd;
  if (tid < 64) L.cur[tid] = tail[tid];
  // a thread makes 4 consecutive words 4g..4g+3 of rows r0, r0+rstep, ...
  // (L.wp >= 4*ng: the words past wpr of the last group are scratch)
  const int ng = (w.wpr + 3) >> 2;          // word groups per row
  const int rstep = kWG / ng;               // rows per pass
  const int r0 = (int)(((unsigned)tid * ((65536u + (unsigned)ng - 1u) / (unsigned)ng)) >> 16);   // tid / ng (tid * ng < 2^16)
  const int g = tid - r0 * ng;
  if (r0 >= rstep) return;
  uint32_t *dst = L.words + 4 * g;
  if (w.inner) {
    const uint32_t *src = L.raw + g;
    switch (w.sh) {   // wave-uniform
      case 0: expand_inner<0>(src, dst, w.nd, L.wp, w.wrows, r0, rstep); break;
      case 1: expand_inner<1>(src, dst, w.nd, L.wp, w.wrows, r0, rstep); break;
      case 2: expand_inner<2>(src, dst, w.nd, L.wp, w.wrows, r0, rstep); break;
      default: expand_inner<3>(src, dst, w.nd, L.wp, w.wrows, r0, rstep); break;
    }
  } else {
    // window crosses (or lies beyond) the left/right picture edge: pel x of
    // the window is picture column gx = clamp(x, 0, W-1) (UMVLine4X); fetched
    // dword d holds picture dword clamp(xa/4 + d, 0, W/4-1), so gx sits in
    // dword clamp(gx/4 - xa/4, 0, nd-1), byte gx & 3.  The 4 pels of a word lie
    // in two neighbouring fetched dwords: one v_perm_b32 per word and row, with
    // the (dword, selector) pair fixed per column.
    const int xq = w.xa >> 2;
    int dq[4];
    uint32_t sel[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 4 * g + k;
      const int q0 = clampi((clampi(w.x0 + c, 0, p.width - 1) >> 2) - xq, 0, w.nd - 1);
      dq[k] = min(q0, w.nd - 2);
      uint32_t s = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int gx = clampi(w.x0 + c + b, 0, p.width - 1);
        const int q = clampi((gx >> 2) - xq, 0, w.nd - 1);
        s |= (uint32_t)(4 * (q - dq[k]) + (gx & 3)) << (8 * b);
      }
      sel[k] = s;
    }
    for (int r = r0; r < w.wrows; r += rstep) {
      const uint32_t *rw = L.raw + r * w.nd;
      u32x4 v;
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_perm(rw[dq[k] + 1], rw[dq[k]], sel[k]);
      *reinterpret_cast<u32x4 *>(dst + r * L.wp) = v;
    }
  }
}

// ------------------------------------------------------- v5 fast sweep --
// Is item `it` served by the v5 sweep?  32-bit keys, a sub-window of at least
// 3x3, and (FFS) no position of it cut by the GetMaxMVD gate (me_fullfast.c:663):
// the window's farthest vector from the predictor passes, so all do.
template <bool KEY32, bool FFS>
__device__ __forceinline__ bool item_fast(const KParams &p, const Item &it) {
  // the sweep's tasks are runs of JMME_SWEEP_P positions: at least that many rows
  if (!KEY32 || 2 * it.rs + 1 < JMME_SWEEP_P || it.rs < 1) return false;
  if (!FFS) return true;
  const int ex = max(abs(it.cqx - 4 * it.rs - it.px), abs(it.cqx + 4 * it.rs - it.px));
  const int ey = max(abs(it.cqy - 4 * it.rs - it.py), abs(it.cqy + 4 * it.rs - it.py));
  return max(ex, ey) < p.max_mvd - 1;
}

// Position tables of one item (LDS, built before its sweep).  For a window
// offset o in [-rs, rs] (entry o + rs):
//   tx[] = { lambda * mvbits(cqx + 4o - px) << 11, G', |o|, 2o }
//   ty[] = { lambda * mvbits(cqy + 4o - py) << 11, F', |o|, 2o }
// The spiral rank (spiral_index, jmme_common.h) splits by the side of the ring:
//   |oy| >  |ox| (top/bottom row of ring |oy|):   rank = F(oy) + 2 ox,
//       F(o) = 4a^2 - 2a - 1 + (o > 0), a = |o|
//   |oy| <= |ox| (left/right column of ring |ox|): rank = G(ox) + 2 oy,
//       G(o) = 4a^2 + 2a - 1 + (o > 0), G(0) = 0
// and F' = F + FFS, G' = G + FFS (FFS ranks are the spiral index + 1; rank 0
// is the pre-seeded (0,0), me_fullfast.c:650-657).
template <bool FFS>
__device__ __forceinline__ void build_tabs(const Item &it, const Lds &L) {
  const int tid = opaque_tid(L);
  const int rs = it.rs, D = 2 * rs + 1;
  for (int i = tid; i < 2 * D; i += kWG) {
    const bool y = i >= D;
    const int j = y ? i - D : i, o = j - rs, a = abs(o);
    const int cq = y ? it.cqy : it.cqx, pp = y ? it.py : it.px;
    const uint32_t m = ((uint32_t)it.lam * (uint32_t)mvbits(cq + 4 * o - pp)) << kCostShift;
    int f = y ? 4 * a * a - 2 * a - 1 + (o > 0) : (a == 0 ? 0 : 4 * a * a + 2 * a - 1 + (o > 0));
    f += FFS ? 1 : 0;
    (y ? L.ty : L.tx)[j] = make_uint4(m, (uint32_t)f, (uint32_t)a, (uint32_t)(2 * o));
  }
}

// The 41 partition keys of one position from its 16 4x4 keys (SAD << 16 + K
// each): a sum of two keys minus K is the key of the union (exact modulo 2^32
// because every true key is < 2^32 under kMaxLambda32); the 16x16 key
// saturates.  The sums are JM's (update_full_search_large_blocks,
// me_fullfast.c:196-260).
__device__ __forceinline__ uint32_t add3(uint32_t a, uint32_t b, uint32_t c) {
  // one v_add3_u32 (the compiler would split a + b - K into an add and a sub)
  uint32_t d;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

__device__ __forceinline__ void partition_keys(const uint32_t (&a)[16], uint32_t K, uint32_t (&ps)[kNS]) {
  const uint32_t nk = 0u - K;
#pragma unroll
  for (int k = 0; k < 16; ++k) ps[25 + k] = a[k];                                                    // 4x4
#pragma unroll
  for (int by = 0; by < 4; ++by)
#pragma unroll
    for (int h = 0; h < 2; ++h) ps[9 + by * 2 + h] = add3(a[by * 4 + 2 * h], a[by * 4 + 2 * h + 1], nk);      // 8x4
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int bx = 0; bx < 4; ++bx) ps[17 + v * 4 + bx] = add3(a[(2 * v) * 4 + bx], a[(2 * v + 1) * 4 + bx], nk);  // 4x8
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int h = 0; h < 2; ++h) ps[5 + v * 2 + h] = add3(ps[9 + (2 * v) * 2 + h], ps[9 + (2 * v + 1) * 2 + h], nk);  // 8x8
  ps[3] = add3(ps[5], ps[7], nk);
  ps[4] = add3(ps[6], ps[8], nk);   // 8x16
  ps[1] = add3(ps[5], ps[6], nk);
  ps[2] = add3(ps[7], ps[8], nk);   // 16x8
  ps[0] = __builtin_elementwise_add_sat(ps[1] + nk, ps[2]);   // 16x16: S_top << 16, + S_bot << 16 + K
}

// Exact elimination (fast path).  The keys of the window centre (offset (0,0)
// of the sweep: FS the search centre, FFS the surface centre -- an eligible
// candidate of every partition in the fast path) are real candidates' keys;
// the last wave writes them to L.ctr and they join the minima where the per-wave
// minima are combined.  A task of positions whose every partition key is
// provably >= the centre's holds no winner -- an equal key shares the centre's
// (cost, rank >> 2) group, whose ranks the refine re-evaluates exactly -- so its
// partition keys need not be formed: with e = (smallest 4x4 SAD) << 16 at a
// position, a partition of n 4x4 blocks has key >= K(pos) + n*e.  Each wave
// keeps, per size n in {1, 2, 4, 8, 16}, the largest centre key of that size
// plus n-1 (for a rounded-up division) in its 8-word L.tmax slot.
// On the bench clip 92 % of the 64-lane tasks skip the keys and minima.
template <bool FFS, bool HBD = false>
__device__ __forceinline__ void centre_bounds(const GroupCtx &g, const Lds &L, int lane, int wave) {
  const int b = lane & 15, i = lane >> 4;   // 4x4 block, row in it
  const int bx = b & 3, by = b >> 2;
  uint32_t sad = sad4<HBD>(&L.words[(g.R + 4 * by + i) * L.wp + g.R + 4 * bx], L.cur + (4 * by + i) * cur_words(HBD),
                           bx, 0u);
  sad += __shfl_xor(sad, 16, 64);
  sad += __shfl_xor(sad, 32, 64);           // every lane: the SAD of its block b
  // K at the centre: mvcost << 11 | rank >> 2, rank 0 (FFS 1: still 0 after >> 2)
  const uint32_t Kc = ((uint32_t)g.lam * (uint32_t)(mvbits(g.cqx - g.px) + mvbits(g.cqy - g.py))) << kCostShift;
  // every partition's SAD at lane b from its neighbours' (in VGPRs: as scalars the
  // sums spilled SGPRs, the MB holding 64 of them): lane b ^ 1 is the block to
  // the right / left (DPP quad_perm), b ^ 4 below / above, b ^ 2 two columns
  // over, b ^ 8 two rows over (ds_swizzle xor within 32 lanes)
  auto xs4 = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x101F); };   // lane ^ 4
  auto xs8 = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x201F); };   // lane ^ 8
  const uint32_t p2h = sad + dpp_mov<0xB1>(sad);   // 8x4 with block b
  const uint32_t p2v = sad + xs4(sad);        // 4x8
  const uint32_t p4 = p2h + xs4(p2h);         // 8x8
  const uint32_t p8h = p4 + dpp_mov<0x4E>(p4);     // 16x8
  const uint32_t p8v = p4 + xs8(p4);          // 8x16
  const uint32_t p16 = p8h + xs8(p8h);        // 16x16
  // the largest of each size over the row of 16 lanes (every lane of the row holds it)
  auto rmax = [&](uint32_t v) {
    v = max(v, dpp_mov<0xB1>(v));
    v = max(v, dpp_mov<0x4E>(v));
    v = max(v, dpp_mov<0x141>(v));
    return max(v, dpp_mov<0x140>(v));
  };
  // a key Kc + (SAD << 16), saturating (16-bit samples: a SAD may pass 2^16)
  auto key = [&](uint32_t m) { return m > 0xffffu ? ~0u : __builtin_elementwise_add_sat(Kc, m << 16); };
  const uint32_t m1 = rmax(sad), m2 = rmax(max(p2h, p2v)), m4 = rmax(p4), m8 = rmax(max(p8h, p8v));
  if (lane == 0) {   // per size n: the largest centre key plus n - 1 (a rounded-up division)
    uint32_t *t = L.tmax + wave * 8;
    t[0] = key(m1);
    t[1] = __builtin_elementwise_add_sat(key(m2), 1u);
    t[2] = __builtin_elementwise_add_sat(key(m4), 3u);
    t[3] = __builtin_elementwise_add_sat(key(m8), 7u);
    t[4] = __builtin_elementwise_add_sat(key(p16), 15u);
  }
  if (wave == kWaves - 1 && lane < 16) {   // the centre's keys for the combine (same form as the sweep's)
    L.ctr[25 + b] = key(sad);
    if (!(bx & 1)) L.ctr[9 + by * 2 + (bx >> 1)] = key(p2h);
    if (!(by & 1)) L.ctr[17 + (by >> 1) * 4 + bx] = key(p2v);
    if (!((bx | by) & 1)) L.ctr[5 + (by >> 1) * 2 + (bx >> 1)] = key(p4);
    if (bx == 0 && !(by & 1)) L.ctr[1 + (by >> 1)] = key(p8h);
    if (by == 0 && !(bx & 1)) L.ctr[3 + (bx >> 1)] = key(p8v);
    if (b == 0) L.ctr[0] = key(p16);
  }
}

// ---- v6 fold: keys reduce-scattered across the wave per fold --------------
// Four partitions m0..m3 (slots base .. base+3) per register: permlane32_swap
// pairs (m0, m1) and (m2, m3) (lanes 0-31 keep the first, 32-63 the second),
// permlane16_swap pairs again; row r of the result then holds the row-partial
// minimum of slot base + perm(r), perm = (0, 2, 1, 3).  The four DPP steps that
// finish a row run once per item (v6_write), not per fold.
__device__ __forceinline__ uint32_t v6_sr(uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3) {
  const auto s1 = __builtin_amdgcn_permlane32_swap(m0, m1, false, false);
  const auto s2 = __builtin_amdgcn_permlane32_swap(m2, m3, false, false);
  const uint32_t x = min((uint32_t)s1[0], (uint32_t)s1[1]), y = min((uint32_t)s2[0], (uint32_t)s2[1]);
  const auto s3 = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  return min((uint32_t)s3[0], (uint32_t)s3[1]);
}
// slot of register q's first partition: 4x4 (25-40), 4x8 (17-24), 8x4 (9-16),
// 8x8 (5-8), 16x8 / 8x16 (1-4), 16x16 (0, rows 1-3 padding)
__host__ __device__ constexpr int v6_base(int q) {
  return q < 4 ? 25 + 4 * q : q < 6 ? 17 + 4 * (q - 4) : q < 8 ? 9 + 4 * (q - 6) : q == 8 ? 5 : q == 9 ? 1 : 0;
}

// The fold of one task's P positions (their 16 4x4 keys each) into the 11
// reduce-scattered registers.  Phase A: the 4x4 slots straight from the keys.
// Phase B, position by position (a position's keys die with it): 8x4, 4x8,
// then 8x8 from the 8x4s, 16x8 / 8x16 from the 8x8s and the 16x16 -- the sums
// of partition_keys (update_full_search_large_blocks, me_fullfast.c:196-260).
// the key of the union of two partitions from theirs (each SAD << 16 + K):
// a + b - K, or for 16-bit samples (SAT) saturating -- a sum past 2^32 becomes
// ~0u, which the reduce sends to the exact re-search when it is the minimum
template <bool SAT>
__device__ __forceinline__ uint32_t ukey(uint32_t a, uint32_t b, uint32_t K) {
  if constexpr (SAT) return __builtin_elementwise_add_sat(a, b - K);
  return add3(a, b, 0u - K);
}

template <int P, bool SAT = false>
__device__ __forceinline__ void fold_v6(const uint32_t (&a)[P][16], const uint32_t (&K)[P], uint32_t (&b)[kRed2]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t m[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      m[i] = a[0][4 * q + i];
#pragma unroll
      for (int j = 1; j < P; ++j) m[i] = min(m[i], a[j][4 * q + i]);
    }
    b[q] = min(b[q], v6_sr(m[0], m[1], m[2], m[3]));
  }
  // 4x8: two registers of four partitions, straight from the 4x4 keys
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    uint32_t m[4];
#pragma unroll
    for (int bx = 0; bx < 4; ++bx) {
      m[bx] = ukey<SAT>(a[0][(2 * v) * 4 + bx], a[0][(2 * v + 1) * 4 + bx], K[0]);
#pragma unroll
      for (int j = 1; j < P; ++j) m[bx] = min(m[bx], ukey<SAT>(a[j][(2 * v) * 4 + bx], a[j][(2 * v + 1) * 4 + bx], K[j]));
    }
    b[4 + v] = min(b[4 + v], v6_sr(m[0], m[1], m[2], m[3]));
  }
  // 8x4 -> 8x8 -> 16x8 / 8x16 -> 16x16, position by position (its keys die with it)
  uint32_t e8[8], g4[4], t4[4], z;   // running minima over the positions
#pragma unroll
  for (int j = 0; j < P; ++j) {
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t nk = 0u - K[j];
    uint32_t e[8], g[4], t[4];
#pragma unroll
    for (int by = 0; by < 4; ++by)
#pragma unroll
      for (int h = 0; h < 2; ++h) e[by * 2 + h] = ukey<SAT>(a[j][by * 4 + 2 * h], a[j][by * 4 + 2 * h + 1], K[j]);   // 8x4
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int h = 0; h < 2; ++h) g[v * 2 + h] = ukey<SAT>(e[(2 * v) * 2 + h], e[(2 * v + 1) * 2 + h], K[j]);   // 8x8
    t[0] = ukey<SAT>(g[0], g[1], K[j]);   // 16x8 top
    t[1] = ukey<SAT>(g[2], g[3], K[j]);   // 16x8 bottom
    t[2] = ukey<SAT>(g[0], g[2], K[j]);   // 8x16 left
    t[3] = ukey<SAT>(g[1], g[3], K[j]);   // 8x16 right
    const uint32_t zz = __builtin_elementwise_add_sat(t[0] + nk, t[1]);   // 16x16 (saturating)
    if (j == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) e8[k] = e[k];
#pragma unroll
      for (int k = 0; k < 4; ++k) { g4[k] = g[k]; t4[k] = t[k]; }
      z = zz;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) e8[k] = min(e8[k], e[k]);
#pragma unroll
      for (int k = 0; k < 4; ++k) { g4[k] = min(g4[k], g[k]); t4[k] = min(t4[k], t[k]); }
      z = min(z, zz);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  b[6] = min(b[6], v6_sr(e8[0], e8[1], e8[2], e8[3]));
  b[7] = min(b[7], v6_sr(e8[4], e8[5], e8[6], e8[7]));
  b[8] = min(b[8], v6_sr(g4[0], g4[1], g4[2], g4[3]));
  b[9] = min(b[9], v6_sr(t4[0], t4[1], t4[2], t4[3]));
  b[10] = min(b[10], v6_sr(z, ~0u, ~0u, ~0u));
}

// The v5 sweep of the sub-window [-rs, rs]^2 (rs >= 1) of the staged window.
// A task is a vertical run of P positions (x, y..y+P-1); the 15+P window rows
// they need are read once; row r meets MB row r - j of position j.  The
// current MB comes from SGPRs (cs), so the only LDS traffic is the window.
// NB = kNS: per-lane minima of the 41 partition keys (v5); NB = kRed2: the
// v6 fold's reduce-scattered registers.  Returns whether any task folded.
// HBD: 16-bit samples (SourceBitDepthLuma <= 10): words x, x + 2 hold a block
// row's 4 samples, the MB rows come from LDS (128 dwords: no room in SGPRs), a
// block's SAD is accumulated plain and made a key (SAD << 16 + K) at the end,
// and partition keys saturate (fold_v6<P, true>).
// RS: the sub-window's range when known at compile time (32, the common +-32
// search: the task geometry folds to constants), else 0 (rs_in)
template <int WP, int P, int NB, bool HBD = false, int RS = 0>   // WP: words pitch when known at compile time (kWP32), else 0 (L.wp)
__device__ __forceinline__ bool sweep_v5(const Lds &L, const uint32_t (&cs)[64], int R, int rs_in,
                                         uint32_t (&best)[NB]) {
  bool folded = false;
  const int rs = RS ? RS : rs_in;
  const int tid = opaque_tid(L);
  const int D = 2 * rs + 1;
  const int DT = (D + P - 1) / P;        // tasks per column (the last one shifted up)
  const int ntask = D * DT;
  const int off = R - rs;
  const int qstep = kWG / D, rstep = kWG - qstep * D;
  // tid / D by a multiply: exact for tid * D < 2^16 (tid < 256, D <= 89)
  const unsigned dm = (65536u + (unsigned)D - 1u) / (unsigned)D;
  int tq = (int)(((unsigned)tid * dm) >> 16), tx = tid - tq * D;   // task column, task row
  // Windows of at least 64 columns: lane l takes column l of whole task rows
  // (a wave streams one row of tasks; task row = wave + 4k), so the 64 lanes
  // of an LDS read hit 64 consecutive words -- no bank conflicts.  Dealing
  // tasks in raster order instead wraps a wave across two task rows (P rows x
  // pitch apart), which put two lanes on one bank in most reads.  The columns
  // past 63 follow as extra tasks after the 64 * DT row tasks.
  const bool rows64 = D >= 64;
  const int nrow64 = 64 * DT;
  if (rows64) { tq = tid >> 6; tx = tid & 63; }
  const int wp = WP ? WP : L.wp;
  const uint32_t tb = lds_addr(L.tmax) + 32u * (uint32_t)ufl(tid >> 6);   // this wave's elimination bounds
  // The loop runs while the wave's first lane has a task (lane 0 holds the
  // wave's smallest t), so every lane stays active: the v6 fold's permlane swaps
  // read every lane.  A lane past the last task recomputes a valid position --
  // its row clamps to D - P below, its column stays inside the window -- which
  // cannot change a minimum.
  for (int t = tid; ufl(t) < ntask; t += kWG) {
    // a column past 63.  nrow64 is a multiple of 64, so the test is the same for
    // every lane of the wave: tested on the first lane it is a scalar branch, and
    // the division stays out of the row tasks (as a per-lane test the compiler
    // selected its result into every task: ~20 VALU a task)
    if (rows64 && ufl(t) >= nrow64) {
      const int e = t - nrow64;
      tq = e / (D - 64);
      tx = 64 + e - tq * (D - 64);
    }
    const int y0 = min(P * tq, D - P);
    uint32_t K[P];
    {
      const u32x4 cx = ds_read_b128(lds_addr(L.tx) + 16u * (uint32_t)tx);
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const u32x4 cy = ds_read_b128(lds_addr(L.ty) + 16u * (uint32_t)(y0 + j));
        const uint32_t rk = cy.z > cx.z ? cy.y + cx.w : cx.y + cy.w;
        K[j] = cx.x + cy.x + (rk >> kRankDrop);
      }
    }
    uint32_t a[P][16];
    // the row base with its sign bit provably clear: the compiler only folds DS
    // offsets onto a base known to be non-negative, and with the compile-time
    // pitch the row offsets then ride in the ds_read2 offset fields
    const uint32_t wbase = (lds_addr(L.words) + 4u * (uint32_t)((off + y0) * wp + off + tx)) & 0x7fffffffu;
    const lds_u32 *wrow = reinterpret_cast<const lds_u32 *>((uintptr_t)wbase);
    if constexpr (HBD) {
      const uint32_t cb = lds_addr(L.cur);
      uint32_t cm[16][8];   // MB rows as loaded (fully unrolled: P rows live at a time)
#pragma unroll
      for (int j = 0; j < P; ++j)
#pragma unroll
        for (int k = 0; k < 16; ++k) a[j][k] = 0u;
#pragma unroll
      for (int r = 0; r < 15 + P; ++r) {
        const lds_u32 *ad = wrow + r * wp;
        const u32x2 w0 = u32x2{ad[0], ad[2]}, w1 = u32x2{ad[4], ad[6]};
        const u32x2 w2 = u32x2{ad[8], ad[10]}, w3 = u32x2{ad[12], ad[14]};
        if (r < 16) {
          const u32x4 lo = ds_read_b128(cb + 32u * (uint32_t)r), hi = ds_read_b128(cb + 32u * (uint32_t)r + 16u);
          cm[r][0] = lo.x; cm[r][1] = lo.y; cm[r][2] = lo.z; cm[r][3] = lo.w;
          cm[r][4] = hi.x; cm[r][5] = hi.y; cm[r][6] = hi.z; cm[r][7] = hi.w;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < P; ++j) {
          const int mr = r - j;
          if (mr < 0 || mr > 15) continue;
          const int b = (mr >> 2) * 4;
          a[j][b + 0] = __builtin_amdgcn_sad_u16(w0.y, cm[mr][1], __builtin_amdgcn_sad_u16(w0.x, cm[mr][0], a[j][b + 0]));
          a[j][b + 1] = __builtin_amdgcn_sad_u16(w1.y, cm[mr][3], __builtin_amdgcn_sad_u16(w1.x, cm[mr][2], a[j][b + 1]));
          a[j][b + 2] = __builtin_amdgcn_sad_u16(w2.y, cm[mr][5], __builtin_amdgcn_sad_u16(w2.x, cm[mr][4], a[j][b + 2]));
          a[j][b + 3] = __builtin_amdgcn_sad_u16(w3.y, cm[mr][7], __builtin_amdgcn_sad_u16(w3.x, cm[mr][6], a[j][b + 3]));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // the 4x4 keys: exact for SAD < 2^14 (<= 10 bits) and lambda <= kMaxLambda32
#pragma unroll
      for (int j = 0; j < P; ++j)
#pragma unroll
        for (int k = 0; k < 16; ++k) a[j][k] = (a[j][k] << 16) + K[j];
    } else {
    u32x2 n01 = u32x2{wrow[0], wrow[4]}, n23 = u32x2{wrow[8], wrow[12]};
#pragma unroll
    for (int r = 0; r < 15 + P; ++r) {
      const u32x2 w01 = n01, w23 = n23;
      if (r < 14 + P) {
        const lds_u32 *ad = wrow + (r + 1) * wp;
        n01 = u32x2{ad[0], ad[4]};
        n23 = u32x2{ad[8], ad[12]};
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int mr = r - j;
        if (mr < 0 || mr > 15) continue;
        const int b = (mr >> 2) * 4;
        const bool first = (mr & 3) == 0;
        a[j][b + 0] = __builtin_amdgcn_sad_hi_u8(w01.x, cs[mr * 4 + 0], first ? K[j] : a[j][b + 0]);
        a[j][b + 1] = __builtin_amdgcn_sad_hi_u8(w01.y, cs[mr * 4 + 1], first ? K[j] : a[j][b + 1]);
        a[j][b + 2] = __builtin_amdgcn_sad_hi_u8(w23.x, cs[mr * 4 + 2], first ? K[j] : a[j][b + 2]);
        a[j][b + 3] = __builtin_amdgcn_sad_hi_u8(w23.y, cs[mr * 4 + 3], first ? K[j] : a[j][b + 3]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    }
    // exact elimination (centre_bounds): skip the keys and minima when no lane's
    // task can beat the centre in any partition
    bool fold = true;
    {
      uint32_t kmin = K[0], e = ~0u;
#pragma unroll
      for (int j = 1; j < P; ++j) kmin = min(kmin, K[j]);
#pragma unroll
      for (int j = 0; j < P; ++j) {
        uint32_t m = a[j][0];
#pragma unroll
        for (int k = 1; k < 16; ++k) m = min(m, a[j][k]);
        e = min(e, m - K[j]);
      }
      const u32x4 t = ds_read_b128(tb);
      const uint32_t t16 = reinterpret_cast<const lds_u32 *>((uintptr_t)tb)[4];
      uint32_t need = __builtin_elementwise_sub_sat(t.x, kmin);
      need = max(need, __builtin_elementwise_sub_sat(t.y, kmin) >> 1);
      need = max(need, __builtin_elementwise_sub_sat(t.z, kmin) >> 2);
      need = max(need, __builtin_elementwise_sub_sat(t.w, kmin) >> 3);
      need = max(need, __builtin_elementwise_sub_sat(t16, kmin) >> 4);
      fold = __builtin_amdgcn_ballot_w64(e < need) != 0;
    }
    if (fold) {
    folded = true;
    if constexpr (NB == kRed2) {
      fold_v6<P, HBD>(a, K, best);
    } else {
    // positions in pairs: both keys of a partition fold with one v_min3_u32
#pragma unroll
    for (int j = 0; j + 1 < P; j += 2) {
      uint32_t p0[kNS], p1[kNS];
      partition_keys(a[j], K[j], p0);
      partition_keys(a[j + 1], K[j + 1], p1);
#pragma unroll
      for (int s = 0; s < kNS; ++s) best[s] = min(best[s], min(p0[s], p1[s]));
    }
    if (P & 1) {
      uint32_t p0[kNS];
      partition_keys(a[P - 1], K[P - 1], p0);
#pragma unroll
      for (int s = 0; s < kNS; ++s) best[s] = min(best[s], p0[s]);
    }
    }
    }
    if (rows64) {
      tq += kWaves;
    } else {
      tx += rstep;
      tq += qstep;
      if (tx >= D) { tx -= D; ++tq; }
    }
  }
  return folded;
}

// v6: finish the 11 reduce-scattered registers (4 DPP steps per row) and store
// each row's slot to this wave's L.red row; a wave that never folded stores ~0
template <bool FOLDED>
__device__ __forceinline__ void v6_write(const Lds &L, const uint32_t (&b)[kRed2], int lane, int wave) {
  const int row = lane >> 4;
  const int pr = ((row & 1) << 1) | (row >> 1);
#pragma unroll
  for (int q = 0; q < kRed2; ++q) {
    uint32_t v = ~0u;
    if (FOLDED) {
      v = dpp_min<0xB1>(b[q]);   // quad_perm [1,0,3,2]
      v = dpp_min<0x4E>(v);      // quad_perm [2,3,0,1]
      v = dpp_min<0x141>(v);     // row_half_mirror
      v = dpp_min<0x140>(v);     // row_mirror
    }
    if ((lane & 15) == 0 && (q < kRed2 - 1 || row == 0)) L.red[wave * kNS + v6_base(q) + pr] = v;
  }
}

// JM's special (0,0) candidate, once per item instead of per position: FS
// check_for_00 (slot 0 at (0,0) costs mvcost - 16*lambda, me_fullsearch.c:61,
// 78-82) and the FFS pre-seed (every partition, rank 0, me_fullfast.c:650-657).
// Its keys are formed before the sweep (special_keys, last wave) and join the
// reduced minima where the reduce's per-wave minima are combined, so
// it adds no barrier; the sweep's own key for that position is never below it.
template <bool FFS>
__device__ __forceinline__ bool special_on(const GroupCtx &g) {
  const int ox = -(g.cqx >> 2), oy = -(g.cqy >> 2);   // the (0,0) vector as a window offset
  const bool inside = abs(ox) <= g.R && abs(oy) <= g.R;
  // FFS: JM pre-seeds with block_sad[pos_00], which setup_fast_full_search only
  // writes when (0,0) is in the window -- and with RDO off (the only case that
  // pre-seeds) it clips the centre so that (0,0) is (me_fullfast.c:319-324).
  // A caller-made window without (0,0) is outside JM's contract: no pre-seed.
  if (FFS) return g.preseed && inside && mv_cost<FFS>(0, 0, g.px, g.py, g.lam, g.max_mvd).ok;
  return g.chk00 && (g.gmask & 1) && inside;
}

// the special candidate's 32-bit key for slot s (~0u when it is not one)
template <bool FFS>
__device__ __forceinline__ uint32_t special_key(const GroupCtx &g, const Lds &L, int s) {
  if (!((g.gmask >> s) & 1) || !(FFS || s == 0)) return ~0u;
  const int ox = -(g.cqx >> 2), oy = -(g.cqy >> 2);
  const SlotGeom gm = slot_geom(s);
  uint32_t sad = 0;
  for (int j = 0; j < gm.h; ++j)
    for (int i = 0; i < gm.w; ++i) sad += L.spec[(gm.by + j) * 4 + gm.bx + i];
  const MvCost mc = mv_cost<FFS>(0, 0, g.px, g.py, g.lam, g.max_mvd);
  const uint32_t mvc = FFS ? mc.mvc : check00_adjust(mc.mvc, g.lam, true);
  const uint32_t rank = FFS ? 0u : (uint32_t)spiral_index_bl(ox, oy);
  const uint32_t cost = (sad << 5) + mvc;
  return cost < (1u << (32 - kCostShift)) ? (cost << kCostShift) | (rank >> kRankDrop) : ~0u;
}

// The last wave, before the sweep (the one the partial last round of sweep
// tasks leaves idle, so this work is off the critical path to the reduce's
// barrier): the special candidate's 16 4x4 SADs, then its key
// for every slot into L.spec[16 + s] (one wave: its LDS writes land before its
// own later reads, no barrier); read back after the reduce's barrier.
template <bool FFS, bool HBD = false>
__device__ __forceinline__ void special_keys(const GroupCtx &g, const Lds &L, int lane) {
  if (lane < 16) {
    const int ox = -(g.cqx >> 2), oy = -(g.cqy >> 2);
    const int bx = lane & 3, by = lane >> 2;
    const uint32_t *w = L.words + (oy + g.R + 4 * by) * L.wp + ox + g.R + 4 * bx;
    uint32_t sad = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) sad = sad4<HBD>(w + r * L.wp, L.cur + (4 * by + r) * cur_words(HBD), bx, sad);
    L.spec[lane] = sad;
  }
  if (lane < kNS) L.spec[16 + lane] = special_key<FFS>(g, L, lane);
}

// Exact search of one partition with 64-bit keys (cost << 32 | rank), every
// position of the window in the legacy per-position form.  Two users: a 16x16
// whose every 32-bit key saturated (only when lambda * mvbits > 8160 and its
// SADs are near 65280), and every partition of a unit whose lambda exceeds the
// 32-bit keys' range (kItemSlow64; no JM configuration comes near it).  The
// result is the min over this call's half of L.fb.  Successive calls of one
// item must pass alternating halves (a call counter, not the slot: the slots of
// a sparse group mask need not alternate), so one barrier per call suffices.
template <bool FFS, bool HBD = false>
__device__ __forceinline__ unsigned long long exact_slot(const GroupCtx &g, const Lds &L, int s, int half) {
  const int tid = opaque_tid(L), lane = tid & 63, wave = tid >> 6;
  const int R = g.R, D = 2 * R + 1;
  const SlotGeom gm = slot_geom(s);
  unsigned long long best = ~0ull;
  for (int i = tid; i < D * D; i += kWG) {
    const int oyw = i / D, oxw = i - oyw * D, ox = oxw - R, oy = oyw - R;
    const int candx = g.cqx + 4 * ox, candy = g.cqy + 4 * oy;
    const bool is00 = candx == 0 && candy == 0;
    const MvCost mc = mv_cost<FFS>(candx, candy, g.px, g.py, g.lam, g.max_mvd);
    if (!pos_eligible<FFS>(g, mc.ok, max(abs(ox), abs(oy)), is00)) continue;
    uint32_t sad = 0;
    for (int r = 0; r < 4 * gm.h; ++r)
      for (int c = 0; c < gm.w; ++c)
        sad = sad4<HBD>(&L.words[(oyw + 4 * gm.by + r) * L.wp + oxw + 4 * (gm.bx + c)],
                        L.cur + (4 * gm.by + r) * cur_words(HBD), gm.bx + c, sad);
    const int sidx = spiral_index_bl(ox, oy);
    const uint32_t rank = FFS ? ((g.preseed && is00) ? 0u : (uint32_t)sidx + 1u) : (uint32_t)sidx;
    const uint32_t mvc = (!FFS && g.chk00 && s == 0) ? check00_adjust(mc.mvc, g.lam, is00) : mc.mvc;
    const unsigned long long k = ((unsigned long long)((sad << 5) + mvc) << 32) | rank;
    best = k < best ? k : best;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned lo = __shfl_xor((unsigned)best, o, 64), hi = __shfl_xor((unsigned)(best >> 32), o, 64);
    const unsigned long long x = ((unsigned long long)hi << 32) | lo;
    best = x < best ? x : best;
  }
  unsigned long long *fb = L.fb + (half & 1) * kWaves;
  if (lane == 0) fb[wave] = best;
  __syncthreads();
  unsigned long long k = fb[0];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) k = fb[w] < k ? fb[w] : k;
  return k;
}

// one partition's result from its exact (cost, rank) -- JM leaves best_pos = 0
// and returns the incoming min_mcost when nothing was eligible
template <bool FFS>
__device__ __forceinline__ jmme_block_res block_result(const GroupCtx &g, bool found, uint32_t rank, uint32_t cost) {
  jmme_block_res res;
  res.reserved = 0;
  if (!found) {
    res.mv_x = (int16_t)g.cqx; res.mv_y = (int16_t)g.cqy; res.cost = JMME_DISTBLK_MAX;
    return res;
  }
  int ox, oy;
  if (FFS && rank == 0) { ox = -(g.cqx >> 2); oy = -(g.cqy >> 2); }   // the pre-seeded (0,0)
  else spiral_offset_fast(FFS ? (int)rank - 1 : (int)rank, &ox, &oy);
  res.mv_x = (int16_t)(g.cqx + 4 * ox);
  res.mv_y = (int16_t)(g.cqy + 4 * oy);
  res.cost = (int64_t)cost;
  return res;
}

// Refine + output for 32-bit keys, after the reduce's one barrier and without
// another: the winner of slot s has cost key >> 11 and a rank in [4c, 4c+4),
// c = key & 2047; those <= 4 candidates are re-evaluated exactly and the
// smallest matching rank wins.  Each lane owns (slot s, candidate j, part q of
// nq), at most two 4x4 blocks of one candidate, so every lane does <= 8 SADs:
//   wave 0: 4x4 slots (25-40), one block;    wave 1: 8x4 / 4x8 (9-24), two blocks;
//   wave 2: 8x8 (5-8) in 2 parts, 16x16 (0) in 8 parts;  wave 3: 16x8 / 8x16 (1-4) in 4 parts.
// The parts of a candidate are consecutive lanes (summed by DPP), its four
// candidates consecutive groups (the winner found by one ballot).  Every lane
// forms its slot's key from the per-wave minima itself, so nothing else needs
// the LDS combine.  skip0: slot 0 is served by the exact fallback instead.
template <bool FFS, bool HBD = false, int WP = 0>   // WP: words pitch when known at compile time (kWP32), else 0
__device__ __forceinline__ void refine_output32(const KParams &p, const GroupCtx &g, const Lds &L, bool spec,
                                                bool fast, unsigned long long skip, int u) {
  const int wp = WP ? WP : L.wp;
  const int tid = opaque_tid(L), lane = tid & 63, wave = ufl(tid >> 6);
  int s, j, q, nq;
  if (wave == 0) { s = 25 + (lane >> 2); j = lane & 3; q = 0; nq = 1; }
  else if (wave == 1) { s = 9 + (lane >> 2); j = lane & 3; q = 0; nq = 1; }
  else if (wave == 2) {
    if (lane < 32) { s = 5 + (lane >> 3); j = (lane >> 1) & 3; q = lane & 1; nq = 2; }
    else { s = 0; j = (lane >> 3) & 3; q = lane & 7; nq = 8; }
  } else { s = 1 + (lane >> 4); j = (lane >> 2) & 3; q = lane & 3; nq = 4; }
  const bool mine = ((g.gmask >> s) & 1) && !((skip >> s) & 1);
  uint32_t key = ~0u;
  if (mine) {
#pragma unroll
    for (int w = 0; w < kWaves; ++w) key = min(key, (uint32_t)L.red[w * kNS + s]);
    if (spec) key = min(key, L.spec[16 + s]);
    if (fast) key = min(key, L.ctr[s]);   // the centre (exact elimination)
  }
  // candidate j: its window offset, or none
  const int R = g.R, D = 2 * R + 1;
  const int rk = (int)(((key & ((1u << kCostShift) - 1)) << kRankDrop) + j);
  int ox = 0, oy = 0;
  bool exists = mine && key != ~0u;
  if (exists) {
    if (FFS && rk == 0) {            // the pre-seeded (0,0) vector
      ox = -(g.cqx >> 2); oy = -(g.cqy >> 2);
      exists = g.preseed && abs(ox) <= R && abs(oy) <= R;
    } else {
      const int sidx = FFS ? rk - 1 : rk;
      exists = sidx < D * D;
      if (exists) spiral_offset_fast(sidx, &ox, &oy);
    }
  }
  // this lane's blocks of the candidate: block q * per of the partition and,
  // when per = 2, the next one -- to its right, or below it for a 4x8 (w = 1);
  // partition widths are 1, 2, 4 blocks, so k / w is a shift by w >> 1
  uint32_t sad = 0;
  if (exists) {
    const SlotGeom gm = slot_geom(s);
    const int per = (gm.w * gm.h) / nq;   // 1 or 2, uniform per wave
    const int k0 = q * per;
    const int bx = gm.bx + (k0 & (gm.w - 1)), by = gm.by + (k0 >> (gm.w >> 1));
    const uint32_t *w = L.words + (oy + R + 4 * by) * wp + ox + R + 4 * bx;
    const uint32_t *c = L.cur + 4 * by * cur_words(HBD);
#pragma unroll
    for (int r = 0; r < 4; ++r) sad = sad4<HBD>(w + r * wp, c + r * cur_words(HBD), bx, sad);
    if (per == 2) {
      const bool vert = gm.w == 1;
      const uint32_t *w2 = vert ? w + 4 * wp : w + 4;
      const uint32_t *c2 = vert ? c + 4 * cur_words(HBD) : c;
      const int bx2 = vert ? bx : bx + 1;
#pragma unroll
      for (int r = 0; r < 4; ++r) sad = sad4<HBD>(w2 + r * wp, c2 + r * cur_words(HBD), bx2, sad);
    }
  }
  // sum the parts (groups of nq aligned lanes; every lane active here)
  {
    const uint32_t x1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)sad, 0xB1, 0xf, 0xf, true);    // lane ^ 1
    sad += nq >= 2 ? x1 : 0u;
    const uint32_t x2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)sad, 0x4E, 0xf, 0xf, true);    // lane ^ 2
    sad += nq >= 4 ? x2 : 0u;
    const uint32_t x4 = (uint32_t)__builtin_amdgcn_mov_dpp((int)sad, 0x141, 0xf, 0xf, true);   // the other quad of 8
    sad += nq >= 8 ? x4 : 0u;
  }
  // exact cost, rank and eligibility at the group leader
  bool m = false;
  if (exists && q == 0) {
    const int candx = g.cqx + 4 * ox, candy = g.cqy + 4 * oy;
    const bool is00 = (candx == 0) && (candy == 0);
    // the decoded position's rank is rk, except that under an FFS pre-seed the
    // (0,0) vector ranks 0 (me_fullfast.c:650-657) whatever its spiral index
    const bool rank_ok = !FFS || !(g.preseed && is00) || rk == 0;
    const MvCost mc = mv_cost<FFS>(candx, candy, g.px, g.py, g.lam, g.max_mvd);
    const bool ok = pos_eligible<FFS>(g, mc.ok, max(abs(ox), abs(oy)), is00);
    const uint32_t mv = (s == 0 && g.chk00) ? check00_adjust(mc.mvc, g.lam, is00) : mc.mvc;
    m = rank_ok && (sad << 5) + mv == (key >> kCostShift) && ok;
  }
  const unsigned long long M = __builtin_amdgcn_ballot_w64(m);
  // only leader lanes (q = 0) can match: bit jj * nq of M >> base is candidate jj
  // of this slot, the bits below j * nq its candidates before this one
  const int base = lane - q - j * nq;   // leader lane of (s, candidate 0)
  const unsigned long long grp = M >> base;
  const bool lower_hit = (grp & ((1ull << (j * nq)) - 1)) != 0;
  const bool any_hit = (grp & ((1ull << (kCand * nq)) - 1)) != 0;
  if (!mine || q != 0) return;
  jmme_block_res res;
  res.reserved = 0;
  if (m && !lower_hit) {
    res.mv_x = (int16_t)(g.cqx + 4 * ox);
    res.mv_y = (int16_t)(g.cqy + 4 * oy);
    res.cost = (int64_t)(key >> kCostShift);
  } else if (j == 0 && key == ~0u) {   // nothing eligible: JM leaves the centre and DISTBLK_MAX
    // DISTBLK_MAX built by the asm itself: a plain constant is hoisted out of
    // the item loop and spilled to scratch
    static_assert(JMME_DISTBLK_MAX == 0xfffffffe0ll, "DISTBLK_MAX halves below");
    uint32_t dlo, dhi;
    asm volatile("v_mov_b32 %0, 0xffffffe0" : "=v"(dlo));
    asm volatile("v_mov_b32 %0, 15" : "=v"(dhi));
    const int64_t dmax = (int64_t)(((uint64_t)dhi << 32) | dlo);
    res.mv_x = (int16_t)g.cqx; res.mv_y = (int16_t)g.cqy; res.cost = dmax;
  } else {
    if (j == 0 && !any_hit) atomicOr(&p.counts[2], 4u);   // cannot happen: refine lost the winner
    return;
  }
  p.out[(size_t)u * kNS + s] = res;
}

template <bool KEY32, bool FFS>
struct ItemStamps {
  unsigned long long wait = 0, expand = 0, sweep = 0, reduce = 0, refine = 0, out = 0;
};

// sweep + reduce + refine + output of one item whose window is in L.words
template <bool KEY32, bool FFS, bool HBD = false>
__device__ __forceinline__ void search_item(const KParams &p, const Item &it, const Lds &L, bool fast,
                                            const uint32_t (&cs)[64], unsigned *tick, unsigned *s_tick
#ifdef JMME_STAMPS
                                            , unsigned long long &t_last, ItemStamps<KEY32, FFS> &st
#endif
) {
  using Best = typename std::conditional<KEY32, uint32_t, unsigned long long>::type;
  int tid = opaque_tid(L);
  int lane = tid & 63;
  int wave = tid >> 6;
  const uint32_t *curw = L.cur;

  GroupCtx g;
  g.cqx = it.cqx;
  g.cqy = it.cqy;
  g.R = it.R;
  g.px = it.px;
  g.py = it.py;
  g.lam = it.lam;
  g.max_mvd = p.max_mvd;
  g.preseed = FFS && (it.flags & kItemPreseed);
  g.gmask = it.gmask;
  g.rs = it.rs;
  g.chk00 = !FFS && (it.flags & kItemChk00);
  const int R = g.R;
  const unsigned long long gmask = g.gmask;
  const int u = it.u;

  // per-thread running minima of the keys (v5 / generic sweep)
  Best best[kNS];
  auto init_best = [&]() {
#pragma unroll
    for (int s = 0; s < kNS; ++s) best[s] = (Best)~0ull;
  };
  // v6 fast sweep: the reduce-scattered minima
  uint32_t b11[kRed2];
  bool v6 = false, v6_folded = false;

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
      // the pair (yb, yb+1); D odd: the last pair is shifted up one row and
      // re-evaluates position D-2 (same key twice: harmless for a minimum)
      const int yb = D > 1 ? min(2 * ty, D - 2) : 0;
      uint32_t a0[16], a1[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) { a0[k] = 0; a1[k] = 0; }
      if constexpr (HBD) {
        // 16-bit samples: a 4x4 block row is words 4c and 4c+2 against the current
        // row's dwords 2c, 2c+1 (two v_sad_u16), the same one-row-ahead pipeline
        uint32_t zero;
        asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
        const uint32_t wrow = lds_addr(L.words) + 4u * (uint32_t)(yb * L.wp + tx);
        const uint32_t rowb = 4u * (uint32_t)L.wp;
        const uint32_t cb = lds_addr(curw) + zero;
        auto rd_row = [&](uint32_t a, uint32_t (&w)[8]) {
          const lds_u32 *q = (const lds_u32 *)(uintptr_t)a;
#pragma unroll
          for (int m = 0; m < 8; ++m) w[m] = q[2 * m];
        };
        auto rd_cur = [&](uint32_t a, uint32_t (&c)[8]) {
          const u32x4 lo = ds_read_b128(a), hi = ds_read_b128(a + 16u);
          c[0] = lo.x; c[1] = lo.y; c[2] = lo.z; c[3] = lo.w; c[4] = hi.x; c[5] = hi.y; c[6] = hi.z; c[7] = hi.w;
        };
        uint32_t nw[8], nc[8], cprev[8];
        rd_row(wrow, nw);
        rd_cur(cb, nc);
#pragma unroll
        for (int m = 0; m < 8; ++m) cprev[m] = 0;
#pragma unroll
        for (int r = 0; r < 17; ++r) {
          uint32_t w[8], c[8];
#pragma unroll
          for (int m = 0; m < 8; ++m) { w[m] = nw[m]; c[m] = nc[m]; }
          if (r < 16) {
            rd_row(wrow + (uint32_t)(r + 1) * rowb, nw);
            if (r < 15) rd_cur(cb + 32u * (uint32_t)(r + 1), nc);
          }
          __builtin_amdgcn_sched_barrier(0);
          if (r < 16) {   // row r of the MB against position y
            const int b = (r >> 2) * 4;
#pragma unroll
            for (int q = 0; q < 4; ++q)
              a0[b + q] = __builtin_amdgcn_sad_u16(w[2 * q + 1], c[2 * q + 1],
                                                   __builtin_amdgcn_sad_u16(w[2 * q], c[2 * q], a0[b + q]));
          }
          if (r > 0) {    // row r-1 of the MB against position y+1
            const int b = ((r - 1) >> 2) * 4;
#pragma unroll
            for (int q = 0; q < 4; ++q)
              a1[b + q] = __builtin_amdgcn_sad_u16(w[2 * q + 1], cprev[2 * q + 1],
                                                   __builtin_amdgcn_sad_u16(w[2 * q], cprev[2 * q], a1[b + q]));
          }
#pragma unroll
          for (int m = 0; m < 8; ++m) cprev[m] = c[m];
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(a0[k]), "+v"(a1[k]));
      } else {
        // opaque zero: keeps the broadcast reads of the current MB inside the
        // loop instead of letting LICM pin 64 VGPRs for them
        uint32_t zero;
        asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
        const uint32_t wrow = lds_addr(L.words) + 4u * (uint32_t)(yb * L.wp + tx);
        const uint32_t rowb = 4u * (uint32_t)L.wp;
        const uint32_t cb = lds_addr(curw) + zero;
        // software pipeline, one row ahead: row r+1's reference words and MB
        // row are requested before row r's v_sad_u8s, so each LDS round trip
        // hides behind a row of arithmetic (and the other waves of the SIMD)
        u32x2 n01, n23;
        u32x4 cn;
        n01 = ds_read2_0_4(wrow); n23 = ds_read2_8_12(wrow);
        cn = ds_read_b128(cb);
        u32x4 cprev = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int r = 0; r < 17; ++r) {
          const u32x2 w01 = n01, w23 = n23;
          const u32x4 c = cn;
          if (r < 16) {
            const uint32_t a = wrow + (uint32_t)(r + 1) * rowb;
            n01 = ds_read2_0_4(a); n23 = ds_read2_8_12(a);
            if (r < 15) cn = ds_read_b128(cb + 16u * (uint32_t)(r + 1));
          }
          __builtin_amdgcn_sched_barrier(0);
          if (r < 16) {   // row r of the MB against position y
            const int b = (r >> 2) * 4;
            a0[b + 0] = __builtin_amdgcn_sad_u8(w01.x, c.x, a0[b + 0]);
            a0[b + 1] = __builtin_amdgcn_sad_u8(w01.y, c.y, a0[b + 1]);
            a0[b + 2] = __builtin_amdgcn_sad_u8(w23.x, c.z, a0[b + 2]);
            a0[b + 3] = __builtin_amdgcn_sad_u8(w23.y, c.w, a0[b + 3]);
          }
          if (r > 0) {    // row r-1 of the MB against position y+1
            const int b = ((r - 1) >> 2) * 4;
            a1[b + 0] = __builtin_amdgcn_sad_u8(w01.x, cprev.x, a1[b + 0]);
            a1[b + 1] = __builtin_amdgcn_sad_u8(w01.y, cprev.y, a1[b + 1]);
            a1[b + 2] = __builtin_amdgcn_sad_u8(w23.x, cprev.z, a1[b + 2]);
            a1[b + 3] = __builtin_amdgcn_sad_u8(w23.y, cprev.w, a1[b + 3]);
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
      auto pos_ctx = [&](int oyw) {
        const int oy = oyw - R;
        PosCtx c;
        c.lring = max(abs(ox), abs(oy));
        const int sidx = spiral_index_bl(ox, oy);
        const int candy = g.cqy + 4 * oy;
        c.is00 = (candx == 0) && (candy == 0);
        c.rank = FFS ? ((g.preseed && c.is00) ? 0u : (uint32_t)sidx + 1u) : (uint32_t)sidx;
        const MvCost mc = mv_cost<FFS>(candx, candy, g.px, g.py, g.lam, g.max_mvd);
        c.mvc = mc.mvc;
        c.ok = pos_eligible<FFS>(g, mc.ok, c.lring, c.is00);
        c.mvc0 = g.chk00 ? check00_adjust(mc.mvc, g.lam, c.is00) : mc.mvc;
        return c;
      };
      auto eval_position = [&](const uint32_t (&acc)[16], int oyw) {
        uint32_t ps[kNS];
        partition_sads(acc, ps);
        update_slots<KEY32, FFS, decltype(all_tag)::value, Best, HBD>(ps, g, pos_ctx(oyw), best);
      };

      // range 0 (D == 1): one position -- the second is made a copy of it
      if (D == 1) {
#pragma unroll
        for (int k = 0; k < 16; ++k) a1[k] = a0[k];
      }
      // both positions unconditionally (one basic block): the two minima per
      // partition fold into one v_min3_u32
      eval_position(a0, yb);
      eval_position(a1, min(yb + 1, D - 1));
      tx += rstep;
      ty += qstep;
      if (tx >= D) { tx -= D; ++ty; }
    }
  };
  // every partition's minimum is tracked even when the group is a subset: the
  // slots outside gmask are simply never read back (one code path, no
  // per-partition masks in the loop)
  const bool spec = KEY32 && fast && special_on<FFS>(g);
  if (KEY32 && fast) {
    if (spec && wave == kWaves - 1) special_keys<FFS, HBD>(g, L, lane);   // the wave with the fewest sweep tasks; read back after the reduce's barrier
    if constexpr (KEY32) centre_bounds<FFS, HBD>(g, L, lane, ufl(wave));
    if constexpr (KEY32 && HBD) {   // 16-bit samples (<= 10 bits): 3 positions a task (the MB rows take VGPRs)
#pragma unroll
      for (int q = 0; q < kRed2; ++q) b11[q] = ~0u;
      v6 = true;
      v6_folded = L.wp == kWP32 ? sweep_v5<kWP32, 3, kRed2, true>(L, cs, R, g.rs, b11)
                                : sweep_v5<0, 3, kRed2, true>(L, cs, R, g.rs, b11);
    } else if constexpr (KEY32) {
#pragma unroll
      for (int q = 0; q < kRed2; ++q) b11[q] = ~0u;
      v6 = true;
      v6_folded = (L.wp == kWP32 && g.rs == 32) ? sweep_v5<kWP32, JMME_SWEEP_P, kRed2, false, 32>(L, cs, R, g.rs, b11)
                  : L.wp == kWP32                 ? sweep_v5<kWP32, JMME_SWEEP_P, kRed2>(L, cs, R, g.rs, b11)
                                                  : sweep_v5<0, JMME_SWEEP_P, kRed2>(L, cs, R, g.rs, b11);
    }
  } else {
    init_best();
    sweep(std::integral_constant<bool, true>{});
  }
  STAMP(st.sweep);

  // ---- workgroup reduction of this group's per-thread minima
  tid = opaque_tid(L);
  lane = tid & 63;
  wave = tid >> 6;
  // the workgroup's next ticket (see me_items_kernel): issued here, written to
  // LDS once the reduce and refine have hidden the atomic's round trip
  unsigned tk = 0;
  if (tick && tid == 0) tk = atomicAdd(tick, 1u);
  if (KEY32 && v6) {
    // (the fold's ballot makes v6_folded wave-uniform)
    if (__builtin_amdgcn_ballot_w64(v6_folded)) v6_write<true>(L, b11, lane, wave);
    else v6_write<false>(L, b11, lane, wave);
  } else if (KEY32) {
    // reduce-scatter through the wave: permlane32_swap pairs slots (lanes
    // 0-31 keep one, 32-63 the other), permlane16_swap pairs again (one slot
    // per row of 16), four DPP steps finish each row -- 11 registers carry
    // the 41 slots (padded to 44) instead of 41 full-wave reductions.
    uint32_t k1[kRed1];
#pragma unroll
    for (int m = 0; m < kRed1; ++m) {
      const uint32_t a = 2 * m < kNS ? (uint32_t)best[2 * m] : ~0u;
      const uint32_t b = 2 * m + 1 < kNS ? (uint32_t)best[2 * m + 1] : ~0u;
      const auto sw = __builtin_amdgcn_permlane32_swap(a, b, false, false);
      k1[m] = min((uint32_t)sw[0], (uint32_t)sw[1]);
    }
    const int row = lane >> 4;
#pragma unroll
    for (int q = 0; q < kRed2; ++q) {
      const auto sw = __builtin_amdgcn_permlane16_swap(k1[2 * q], k1[2 * q + 1], false, false);
      uint32_t v = min((uint32_t)sw[0], (uint32_t)sw[1]);
      v = dpp_min<0xB1>(v);    // quad_perm [1,0,3,2]
      v = dpp_min<0x4E>(v);    // quad_perm [2,3,0,1]
      v = dpp_min<0x141>(v);   // row_half_mirror
      v = dpp_min<0x140>(v);   // row_mirror: every lane of the row holds its minimum
      // row 0: slot 4q, row 1: 4q+2, row 2: 4q+1, row 3: 4q+3
      const int s = 4 * q + (((row & 1) << 1) | (row >> 1));
      if ((lane & 15) == 0 && s < kNS) L.red[wave * kNS + s] = v;
    }
  } else {
#pragma unroll
    for (int s = 0; s < kNS; ++s) {
      if (!((gmask >> s) & 1)) continue;
      unsigned long long k = best[s];
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const unsigned lo = __shfl_xor((unsigned)k, off, 64);
        const unsigned hi = __shfl_xor((unsigned)(k >> 32), off, 64);
        const unsigned long long o = ((unsigned long long)hi << 32) | lo;
        k = o < k ? o : k;
      }
      if (lane == 0) L.red[wave * kNS + s] = k;
    }
  }
  __syncthreads();
  if constexpr (KEY32) {
    // partitions whose every key saturated go to the exact 64-bit search: at
    // 8 bits only the 16x16 can (uniform: every thread forms slot 0's key); with
    // 16-bit samples any partition of 8x8 or more (each wave finds them itself:
    // lane s forms slot s's key)
    unsigned long long satm = 0;
    if constexpr (HBD) {
      bool m = false;
      if (lane < kNS && ((gmask >> lane) & 1)) {
        uint32_t k0 = ~0u;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) k0 = min(k0, (uint32_t)L.red[w * kNS + lane]);
        if (spec) k0 = min(k0, L.spec[16 + lane]);
        if (fast) k0 = min(k0, L.ctr[lane]);
        m = k0 == ~0u;
      }
      satm = __builtin_amdgcn_ballot_w64(m);
    } else if (gmask & 1) {
      uint32_t k0 = ~0u;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) k0 = min(k0, (uint32_t)L.red[w * kNS]);
      if (spec) k0 = min(k0, L.spec[16]);
      if (fast) k0 = min(k0, L.ctr[0]);
      satm = k0 == ~0u ? 1ull : 0ull;
    }
#ifdef JMME_DBG_CHECKS   // diagnostic: every wave computed the same saturated-slot mask
    {
      __shared__ unsigned long long s_dbg_satm[kWaves];
      if (lane == 0) s_dbg_satm[ufl(wave)] = satm;
      __syncthreads();
      for (int w = 0; w < kWaves; ++w)
        if (s_dbg_satm[w] != satm && lane == 0) atomicOr(&p.counts[2], 8u);
      __syncthreads();
    }
#endif
    STAMP(st.reduce);
    if (L.wp == kWP32) refine_output32<FFS, HBD, kWP32>(p, g, L, spec, fast, satm, u);
    else refine_output32<FFS, HBD, 0>(p, g, L, spec, fast, satm, u);
    if (tick && opaque_tid(L) == 0) *s_tick = tk;
    STAMP(st.refine);
    int call = 0;
    for (unsigned long long m = satm; m; m &= m - 1) {   // search those again with exact keys
      const int sl = __builtin_ctzll(m);
      const unsigned long long k = exact_slot<FFS, HBD>(g, L, sl, call++);
      if (opaque_tid(L) == 0)
        p.out[(size_t)u * kNS + sl] =
            block_result<FFS>(g, k != ~0ull, (uint32_t)(k & 0x7fffffffu), (uint32_t)(k >> 32));
    }
    STAMP(st.out);
    return;
  }
  if (tid < kNS) {
    unsigned long long k = L.red[tid];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) { const unsigned long long o = L.red[w * kNS + tid]; k = o < k ? o : k; }
    if (spec) k = min(k, (unsigned long long)L.spec[16 + tid]);
    L.red[tid] = k;   // wave 0's row now holds the group result
  }
  __syncthreads();
  STAMP(st.reduce);

  STAMP(st.refine);

  // ---- results of this group (64-bit keys: cost << 32 | rank)
  tid = opaque_tid(L);
  if (tick && tid == 0) *s_tick = tk;
  if (tid < kNS && ((gmask >> tid) & 1)) {
    const unsigned long long k = L.red[tid];
    p.out[(size_t)u * kNS + tid] =
        block_result<FFS>(g, k != ~0ull, (uint32_t)(k & 0x7fffffffu), (uint32_t)(k >> 32));
  }
  STAMP(st.out);
}

// A unit whose lambda exceeds the 32-bit keys' range (kItemSlow64): every
// partition of the item by the exact 64-bit search, one after the other.
template <bool FFS, bool HBD = false>
__device__ __forceinline__ void search_item_slow64(const KParams &p, const Item &it, const Lds &L) {
  GroupCtx g;
  g.cqx = it.cqx; g.cqy = it.cqy; g.R = it.R; g.px = it.px; g.py = it.py; g.lam = it.lam;
  g.max_mvd = p.max_mvd;
  g.preseed = FFS && (it.flags & kItemPreseed);
  g.gmask = it.gmask;
  g.rs = it.rs;
  g.chk00 = !FFS && (it.flags & kItemChk00);
  int call = 0;
  for (int s = 0; s < kNS; ++s) {
    if (!((g.gmask >> s) & 1)) continue;
    const unsigned long long k = exact_slot<FFS, HBD>(g, L, s, call++);
    if (opaque_tid(L) == 0)
      p.out[(size_t)it.u * kNS + s] =
          block_result<FFS>(g, k != ~0ull, (uint32_t)(k & 0x7fffffffu), (uint32_t)(k >> 32));
  }
}

// Wave-uniform loads through the scalar data cache (s_load): the constant
// address space tells the compiler the bytes do not change during the kernel.
// For data another launch (or the host) wrote before this one started.
typedef int v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const v4i const_v4i;
__device__ __forceinline__ v4i sload16(const void *p) { return *reinterpret_cast<const_v4i *>((uintptr_t)p); }

// item descriptors are wave-uniform: keep every field in SGPRs (the plan
// kernel wrote them in the previous launch)
__device__ __forceinline__ Item load_item(const Item *items, unsigned j) {
  Item it;
  v4i *dst = reinterpret_cast<v4i *>(&it);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(Item) / 16); ++k) dst[k] = sload16(reinterpret_cast<const v4i *>(items + j) + k);
  return it;
}

// Persistent item kernel.  The KEY32 instance drains the 32-bit list, the
// other the 64-bit list.  XCD x (= blockIdx % 8) serves every 8th chunk of
// p.chunk consecutive items -- one eighth of a macroblock row when that
// divides, the stripes rotating every p.rot rows, else 16 items (neighbouring
// macroblocks' windows overlap in its L2; with
// whole eighths of the list instead, the last eighth -- the bottom rows, whose
// padded, flat blocks defeat the elimination, and all further groups, which
// the bottom row holds -- made one XCD end 30 us after the others).  Inside
// its list the first two items of each workgroup
// are static (lb, lb + nbx); the rest are dealt by tickets,
// one atomic per item on the XCD's counter: the workgroups resident on one CU
// do not progress at the same rate (the oldest wave wins the SIMD's issue
// arbitration: on MI355X a CU's four workgroups finished equal static shares
// at 131, 171, 220 and 257 us), so a static deal leaves CUs with one or two
// workgroups for the last third of the launch.  A workgroup takes its ticket
// for the item after next while it serves an item, so the index is in LDS by
// the next item's first barrier.  Every ticket below the run's end is served by
// the workgroup that drew it: tickets are only drawn while a next item exists.
// LR: the launch's LDS range when fixed at compile time (32: every LDS offset
// and the window pitch are constants, no SGPRs hold them), else 0 (p.lds_range)
template <bool KEY32, bool FFS, bool HBD = false, int LR = 0>
__global__ __launch_bounds__(kWG, KEY32 ? JMME_WAVES_PER_EU : 2) void me_items_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ __attribute__((aligned(16))) uint32_t s_cur[HBD ? 128 : 64];
  __shared__ unsigned s_tick;
  const unsigned cnt = (unsigned)p.n + p.counts[0];   // first groups, then the further groups
  const Item *items = p.items;
  const int x = blockIdx.x & 7, lb = blockIdx.x >> 3, nbx = (gridDim.x - x + 7) >> 3;
  // XCD x's list: the chunks of p.chunk consecutive items c with c % 8 == x
  // (a chunk's macroblocks are neighbours: their windows overlap in the XCD's
  // L2); k-th item of the list = list index (k / ch * 8 + x) * ch + k % ch
  const unsigned ch = (unsigned)ufl(p.chunk), rot = (unsigned)ufl(p.rot);
  // the stripe XCD x serves in round r
  auto stripe = [&](unsigned r) { return rot ? ((unsigned)x + r / rot) & 7u : (unsigned)x; };
  const unsigned rounds = cnt / (8u * ch), rest = cnt - rounds * 8u * ch;
  const unsigned end = rounds * ch + (unsigned)min(max((int)rest - (int)stripe(rounds) * (int)ch, 0), (int)ch);
  auto item_at = [&](unsigned k) { const unsigned r = k / ch; return (r * 8u + stripe(r)) * ch + k % ch; };
  const unsigned j = (unsigned)lb;
  if (j >= end) return;
  unsigned jn = j + nbx;                                  // the second item (static)
  const unsigned dyn0 = 2u * (unsigned)nbx;               // ticket t serves item dyn0 + t
  unsigned *const tick = p.counts + 8 + x;

  Lds L = carve(smem, LR ? LR : p.lds_range, HBD);
  L.cur = s_cur;
  const unsigned long long dbg_slot =
      p.debug_words ? (1ull << __builtin_ctzll((ufl64(p.req[0].slot_mask) & kAll) | (1ull << 63))) : 0ull;
#ifdef JMME_STAMPS
  unsigned long long t_last = __builtin_amdgcn_s_memtime();
#endif

  Item it = load_item(items, item_at(j));
  prefetch<HBD>(p, it, L);
#ifdef JMME_STAMPS
  // per-workgroup record behind the per-unit ones: start / end (s_memrealtime,
  // 100 MHz), HW_ID, XCC_ID, items served
  const unsigned long long wg_t0 = __builtin_amdgcn_s_memrealtime();
  unsigned wg_items = 0;
#endif
  for (bool first = true;; first = false) {
#ifdef JMME_STAMPS
    ItemStamps<KEY32, FFS> st;
#endif
    // this item's fetch has landed (every wave waits for its own loads, the
    // barrier for everyone's); the previous item is completely done with LDS,
    // and the ticket it drew is visible
    // lgkmcnt(0) too: the ticket wave 0 stored to s_tick (and every other LDS
    // store of the previous item) must have landed before any wave passes the
    // barrier.  With vmcnt(0) alone here the compiler dropped the barrier's own
    // LDS wait, and waves on the other SIMDs now and then read the old ticket:
    // the workgroup's waves then served different items (wrong results for
    // whole refine waves, ~1 launch in 5 at 10 bits)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (!first) jn = dyn0 + (unsigned)ufl((int)s_tick);
#ifdef JMME_DBG_CHECKS   // diagnostic: every wave serves the same item and draws the same next one
    {
      __shared__ unsigned s_dbg_it[2 * kWaves];
      const int wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      if ((threadIdx.x & 63) == 0) { s_dbg_it[2 * wv] = (unsigned)it.u; s_dbg_it[2 * wv + 1] = jn; }
      __syncthreads();
      for (int w = 0; w < kWaves; ++w)
        if ((s_dbg_it[2 * w] != (unsigned)it.u || s_dbg_it[2 * w + 1] != jn) && (threadIdx.x & 63) == 0)
          atomicOr(&p.counts[2], 16u);
      __syncthreads();
    }
#endif
    const bool more = jn < end;
    Item nx;
    if (more) nx = load_item(items, item_at(jn));
    STAMP(st.wait);
    const bool fast = it.gmask && item_fast<KEY32, FFS>(p, it);
    if (it.gmask) {
      if constexpr (HBD) expand16(p, it, L);
      else expand(p, it, L);
    }
    if (fast) build_tabs<FFS>(it, L);
    __syncthreads();
    if (p.debug_words && it.u == 0 && (it.gmask & dbg_slot)) {
      const Win w = win_of<HBD>(p, it);
      for (int i = opaque_tid(L); i < w.wrows * w.wpr; i += kWG) {
        const int r = i / w.wpr;
        p.debug_words[i] = L.words[r * L.wp + i - r * w.wpr];
      }
    }
    STAMP(st.expand);
    // the raw buffer is free: start fetching the next item behind this sweep
    if (more) prefetch<HBD>(p, nx, L);
    bool ticketed = false;
    if (it.gmask) {
      // the current MB into SGPRs: every v_sad of the v5 sweep takes it as
      // its scalar operand
      uint32_t cs[64];
      if constexpr (!HBD) {
        // straight from the current picture (s_load_dwordx4 per MB row)
        const uint8_t *mb = p.cur + (size_t)it.mb_y * p.pitch + it.mb_x;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const v4i q = sload16(mb + (size_t)r * p.pitch);
          cs[4 * r + 0] = (uint32_t)q.x; cs[4 * r + 1] = (uint32_t)q.y;
          cs[4 * r + 2] = (uint32_t)q.z; cs[4 * r + 3] = (uint32_t)q.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 64; ++k) cs[k] = 0;   // (the v5 sweep's operand: 8-bit only)
      }
      if (KEY32 && (it.flags & kItemSlow64)) {
        search_item_slow64<FFS, HBD>(p, it, L);
      } else {
        ticketed = true;
#ifdef JMME_STAMPS
        search_item<KEY32, FFS, HBD>(p, it, L, fast, cs, more ? tick : nullptr, &s_tick, t_last, st);
#else
        search_item<KEY32, FFS, HBD>(p, it, L, fast, cs, more ? tick : nullptr, &s_tick);
#endif
      }
    }
    if (more && !ticketed && opaque_tid(L) == 0) s_tick = atomicAdd(tick, 1u);
#ifdef JMME_STAMPS
    if (p.stamps && threadIdx.x == 0) {
      unsigned long long *o = p.stamps + (size_t)it.u * 8;
      atomicAdd(o + 0, st.wait); atomicAdd(o + 1, st.expand); atomicAdd(o + 2, st.sweep);
      atomicAdd(o + 3, st.reduce); atomicAdd(o + 4, st.refine); atomicAdd(o + 5, st.out);
      atomicAdd(o + 6, (unsigned long long)__builtin_popcountll(it.gmask)); atomicAdd(o + 7, 1ull);
    }
    ++wg_items;
#endif
    if (!more) break;
    it = nx;
  }
#ifdef JMME_STAMPS
  if (p.stamps && threadIdx.x == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    unsigned long long *o = p.stamps + (size_t)p.n * 8 + (size_t)blockIdx.x * 4;
    o[0] = wg_t0; o[1] = __builtin_amdgcn_s_memrealtime(); o[2] = hw; o[3] = ((unsigned long long)xcc << 32) | wg_items;
  }
#endif
}

// ------------------------------------------------------- small batches --
// Latency form (the drop-in's speculative batches after a failed guess are one
// or two macroblocks; a launch + sync round trip costs ~10 us and a lightly
// loaded GPU runs at a low clock, so the critical path is what counts):
//   * search launch: one workgroup per (item, 16x16 tile of window
//     positions), one position per thread.  The tile's reference pels are
//     staged as aligned dwords (clamped into the picture as UMVLine4X does),
//     expanded to words (word[y][x] = pels x..x+3); per position only the 4x4
//     SADs the item's partitions use are formed.  Per served partition the
//     wave's minimum cost comes from 4 DPP steps + 4 readlanes, the smallest
//     rank among the lanes holding it from a ballot (and, on a tie, one more
//     such reduction); the 4 waves meet in LDS and the tile's exact key
//     cost << 32 | rank is stored (no atomics, no fences);
//   * finish launch: one thread per (item, partition) takes the minimum over
//     the item's tiles and writes the result (mapped host memory).
__host__ __device__ inline int small_rows() { return kSmallTile + 15; }
constexpr int kSmallWP = kSmallTile + 12;   // words per staged row
constexpr int kSmallRaw = 9;                // raw dwords per staged row (36 pels >= 3 + 28 + 3)

// wave minimum of a u32, the same in every lane (scalar)
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = dpp_min<0xB1>(v);    // quad_perm [1,0,3,2]
  v = dpp_min<0x4E>(v);    // quad_perm [2,3,0,1]
  v = dpp_min<0x141>(v);   // row_half_mirror
  v = dpp_min<0x140>(v);   // row_mirror: every lane of a row of 16 holds the row's minimum
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0), r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
  const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32), r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
  return min(min(r0, r1), min(r2, r3));
}

// High bit depth (SourceBitDepthLuma > 8: JM's imgpel holds up to 14 bits,
// JM/lencod/inc/defines.h:37): the planes are 16-bit and the staged words hold
// two pels, so a 4x4 row is two v_sad_u16 (|a.lo - b.lo| + |a.hi - b.hi|).
constexpr int kSmallWP16 = kSmallTile + 14;   // 2-pel words per staged row (c = tx + 4 bx + {0, 2})
constexpr int kSmallRaw16 = 16;               // raw dwords per staged row (32 pels >= 1 + 31)

template <bool FFS, bool HBD>
__global__ __launch_bounds__(kWG) void me_small_kernel(SmallParams p) {
  constexpr int kRows = kSmallTile + 15;
  constexpr int kWP = HBD ? kSmallWP16 : kSmallWP, kRaw = HBD ? kSmallRaw16 : kSmallRaw;
  __shared__ uint32_t s_w[kRows * kWP];
  __shared__ uint32_t s_raw[kRows * kRaw];
  __shared__ uint32_t s_cur[HBD ? 128 : 64];
  __shared__ uint32_t s_cost[kWaves][kNS], s_rank[kWaves][kNS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tpi = p.tiles * p.tiles;
  const int ii = blockIdx.x / tpi, t = blockIdx.x - ii * tpi;
  const SmallItem it = ii < p.n_inline ? p.inl[ii] : p.items[ii];
  const int R = it.R;
  const int ox0 = -R + kSmallTile * (t % p.tiles), oy0 = -R + kSmallTile * (t / p.tiles);
  unsigned long long *part = p.keys + ((size_t)ii * tpi + t) * kNS;
  // what the finish launch needs of the item, in device memory (it would
  // otherwise read the mapped host copy again)
  if (!p.host_finish && t == 0 && tid == 0) p.info[ii] = make_int4((int)(unsigned)it.gmask, (int)(unsigned)(it.gmask >> 32),
                                                 (int)(unsigned short)it.cqx | ((int)it.cqy << 16), it.u);
  if (ox0 > R || oy0 > R) {                              // a tile past this item's window
    if (tid < kNS && ((it.gmask >> tid) & 1)) part[tid] = ~0ull;
    return;
  }
  if constexpr (!HBD) {
    const int X0 = it.mb_x + (it.cqx >> 2) + ox0, Y0 = it.mb_y + (it.cqy >> 2) + oy0;
    const int xa = X0 & ~3, sh = X0 - xa;
    for (int i = tid; i < kRows * kSmallRaw; i += kWG) {
      const int r = i / kSmallRaw, k = i - r * kSmallRaw;
      const uint8_t *row = it.ref + (size_t)clampi(Y0 + r, 0, p.height - 1) * p.pitch;
      const int x = xa + 4 * k;
      uint32_t w;
      if (x >= 0 && x + 3 < p.width) {
        w = *reinterpret_cast<const uint32_t *>(row + x);
      } else {
        w = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) w |= (uint32_t)row[clampi(x + b, 0, p.width - 1)] << (8 * b);
      }
      s_raw[i] = w;
    }
    if (tid < 64)
      s_cur[tid] = *reinterpret_cast<const uint32_t *>(p.cur + (size_t)(it.mb_y + (tid >> 2)) * p.pitch + it.mb_x +
                                                       4 * (tid & 3));
    __syncthreads();
    for (int i = tid; i < kRows * kSmallWP; i += kWG) {
      const int r = i / kSmallWP, c = i - r * kSmallWP, q = (sh + c) >> 2;
      s_w[i] = __builtin_amdgcn_alignbyte(s_raw[r * kSmallRaw + q + 1], s_raw[r * kSmallRaw + q], (sh + c) & 3);
    }
    __syncthreads();
  } else {
    // pitch in pels; word c of a staged row = pels (X0 + c, X0 + c + 1)
    const int X0 = it.mb_x + (it.cqx >> 2) + ox0, Y0 = it.mb_y + (it.cqy >> 2) + oy0;
    const int xa = X0 & ~1, sh = X0 - xa;
    const uint16_t *ref16 = reinterpret_cast<const uint16_t *>(it.ref);
    const uint16_t *cur16 = reinterpret_cast<const uint16_t *>(p.cur);
    for (int i = tid; i < kRows * kSmallRaw16; i += kWG) {
      const int r = i / kSmallRaw16, k = i - r * kSmallRaw16;
      const uint16_t *row = ref16 + (size_t)clampi(Y0 + r, 0, p.height - 1) * p.pitch;
      const int x = xa + 2 * k;
      uint32_t w;
      if (x >= 0 && x + 1 < p.width)
        w = *reinterpret_cast<const uint32_t *>(row + x);
      else
        w = (uint32_t)row[clampi(x, 0, p.width - 1)] | ((uint32_t)row[clampi(x + 1, 0, p.width - 1)] << 16);
      s_raw[i] = w;
    }
    if (tid < 128)
      s_cur[tid] = *reinterpret_cast<const uint32_t *>(cur16 + (size_t)(it.mb_y + (tid >> 3)) * p.pitch + it.mb_x +
                                                       2 * (tid & 7));
    __syncthreads();
    for (int i = tid; i < kRows * kSmallWP16; i += kWG) {
      const int r = i / kSmallWP16, c = i - r * kSmallWP16, q = (sh + c) >> 1;
      const uint32_t lo = s_raw[r * kSmallRaw16 + q];
      s_w[i] = ((sh + c) & 1) ? __builtin_amdgcn_alignbyte(s_raw[r * kSmallRaw16 + q + 1], lo, 2) : lo;
    }
    __syncthreads();
  }
  const int tx = tid % kSmallTile, ty = tid / kSmallTile;
  const int ox = ox0 + tx, oy = oy0 + ty;
  uint32_t a[16];
#pragma unroll
  for (int b = 0; b < 16; ++b) {
    a[b] = 0;
    if ((it.bmask >> b) & 1) {
      const int by = b >> 2, bx = b & 3;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr (!HBD) {
          a[b] = __builtin_amdgcn_sad_u8(s_w[(ty + 4 * by + r) * kSmallWP + tx + 4 * bx], s_cur[(4 * by + r) * 4 + bx],
                                         a[b]);
        } else {
          const uint32_t *w = &s_w[(ty + 4 * by + r) * kSmallWP16 + tx + 4 * bx];
          a[b] = __builtin_amdgcn_sad_u16(w[0], s_cur[(4 * by + r) * 8 + 2 * bx], a[b]);
          a[b] = __builtin_amdgcn_sad_u16(w[2], s_cur[(4 * by + r) * 8 + 2 * bx + 1], a[b]);
        }
      }
    }
  }
  uint32_t ps[kNS];
  partition_sads(a, ps);
  GroupCtx g;
  g.R = R; g.cqx = it.cqx; g.cqy = it.cqy; g.px = it.px; g.py = it.py; g.lam = it.lam;
  g.max_mvd = p.max_mvd; g.preseed = FFS && (it.flags & kItemPreseed); g.gmask = it.gmask; g.rs = it.rs;
  g.chk00 = !FFS && (it.flags & kItemChk00);
  const int candx = it.cqx + 4 * ox, candy = it.cqy + 4 * oy;
  const bool is00 = candx == 0 && candy == 0;
  const MvCost mc = mv_cost<FFS>(candx, candy, it.px, it.py, it.lam, p.max_mvd);
  const bool ok = ox <= R && oy <= R && pos_eligible<FFS>(g, mc.ok, max(abs(ox), abs(oy)), is00);
  const int sidx = spiral_index_bl(ox, oy);
  const uint32_t rank = FFS ? ((g.preseed && is00) ? 0u : (uint32_t)sidx + 1u) : (uint32_t)sidx;
#pragma unroll
  for (int sl = 0; sl < kNS; ++sl) {
    if (!((it.gmask >> sl) & 1)) continue;
    const uint32_t mvc = (!FFS && g.chk00 && sl == 0) ? check00_adjust(mc.mvc, it.lam, is00) : mc.mvc;
    const uint32_t cost = ok ? (ps[sl] << 5) + mvc : ~0u;
    const uint32_t cmin = wave_min_u32(cost);
    const unsigned long long at = __builtin_amdgcn_ballot_w64(cost == cmin);
    uint32_t rmin = (uint32_t)__builtin_amdgcn_readlane((int)rank, __builtin_ctzll(at));
    if (at & (at - 1)) rmin = wave_min_u32(cost == cmin ? rank : ~0u);   // a tie: the first in spiral order
    if (lane == 0) { s_cost[wave][sl] = cmin; s_rank[wave][sl] = rmin; }
  }
  __syncthreads();
  if (tid < kNS && ((it.gmask >> tid) & 1)) {
    unsigned long long k = ~0ull;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const uint32_t c = s_cost[w][tid];
      const unsigned long long kw = c == ~0u ? ~0ull : (((unsigned long long)c << 32) | s_rank[w][tid]);
      k = kw < k ? kw : k;
    }
    part[tid] = k;
  }
}

// the results of a small batch: one thread per (item, partition), the minimum
// over the item's tiles (the kernel boundary orders it after the search launch)
template <bool FFS>
__global__ __launch_bounds__(kWG) void small_finish_kernel(SmallParams p) {
  const int i = blockIdx.x * kWG + threadIdx.x;
  if (i >= p.n_items * kNS) return;
  const int j = i / kNS, sl = i - j * kNS;
  const int4 q = p.info[j];
  const unsigned long long gmask = (unsigned)q.x | ((unsigned long long)(unsigned)q.y << 32);
  if (!((gmask >> sl) & 1)) return;
  const int tpi = p.tiles * p.tiles;
  const unsigned long long *part = p.keys + (size_t)j * tpi * kNS + sl;
  unsigned long long k = ~0ull;
  for (int t = 0; t < tpi; ++t) {
    const unsigned long long v = part[(size_t)t * kNS];
    k = v < k ? v : k;
  }
  GroupCtx g{};
  g.cqx = (int16_t)(q.z & 0xffff); g.cqy = (int16_t)((unsigned)q.z >> 16);
  p.out[(size_t)q.w * kNS + sl] = block_result<FFS>(g, k != ~0ull, (uint32_t)(k & 0xffffffffu), (uint32_t)(k >> 32));
}

// ------------------------------------------------------ chained searches --
// One workgroup per chain (jmme.h, jmme_search_mbs_chains).  Per step, thread 0
// derives the step's predictor and centre as JM would from the chain's
// neighbours (GetMotionVectorPredictorNormal, JM/lcommon/src/mv_prediction.c:
// 192-300; BlockMotionSearch, mv_search.c:930-956; CheckSearchRange :822-848;
// clip_mv_range, conformance.c:463-469), the window around it is staged in LDS
// (clamped as UMVLine4X does), every position's SAD over the partition is
// formed from the staged words, and the (cost, spiral rank) minimum wins, as
// in full_search_motion_estimation / fast_full_search_motion_estimation.  The
// step's answer, clipped as BlockMotionSearch clips it after the search
// (mv_search.c:983), is what the next steps read as that partition's vector.
constexpr int kChainWG = 1024, kChainWaves = kChainWG / 64;

// The staged window may carry a margin of kChainMargin pels on every side, so
// that a later step whose centre moved by up to that much searches the same
// staging.  Measured in the 1080p drop-in: a 12-pel margin left the chain
// kernel at 26.5 us (26.2 without) -- the larger first staging costs what the
// avoided restagings save -- so none.
constexpr int kChainMargin = 0;
__host__ __device__ inline int chain_wpr(int R) { return 2 * R + 13 + 2 * kChainMargin; }   // words per staged row
__host__ __device__ inline int chain_rows(int R) { return 2 * R + 16 + 2 * kChainMargin; }
__host__ __device__ inline int chain_raw(int R) { return (chain_wpr(R) + 9) / 4 + 1; }   // raw dwords per row
// 16-bit planes (SourceBitDepthLuma 9..14): words[x] = pels x, x+1, two more
// words a row (a 4-pel chunk is words x and x+2), two samples per raw dword
__host__ __device__ inline int chain_wpr16(int R) { return chain_wpr(R) + 2; }
__host__ __device__ inline int chain_raw16(int R) { return (chain_wpr16(R) + 5) / 2 + 1; }

__device__ __forceinline__ int imedian3(int a, int b, int c) {
  return a > b ? (b > c ? b : (a > c ? c : a)) : (a > c ? a : (b > c ? c : b));
}

#ifdef JMME_CHAIN_PROF
// diagnostic builds: block 0's phase times (100 MHz realtime; [30], [31] shader
// clocks at start / end), read with jmme_debug_chain_prof
__device__ unsigned long long g_chain_prof[32];
#define CPROF(i) do { if (blockIdx.x == 0 && tid == 0) g_chain_prof[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define CPROF(i) do { } while (0)
#endif

// a step's predictor, centre and ranges from its neighbours and the earlier
// steps' vectors (mv[j] for j < k): computed by every thread (uniform values,
// no barrier to hand them out)
struct ChainStepIn {
  int px, py, cx, cy, rmin, rmax;
};

__device__ __forceinline__ ChainStepIn chain_derive(const jmme_chain &c, const jmme_chain_step &st, const int (&mvx)[4],
                                                    const int (&mvy)[4], int max_mvd) {
  const SlotGeom sg = slot_geom(st.slot);
  const int bsx = 4 * sg.w, bsy = 4 * sg.h;
  // neighbours: (available, ref_idx, mv)
  int av[3], rf[3], mx[3], my[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const jmme_chain_nb nb = st.nb[j];
    av[j] = nb.src != JMME_NB_UNAVAILABLE;
    if (nb.src >= 0) {
      const int q = nb.src;   // < k <= 3
      rf[j] = c.ref_idx;
      mx[j] = q == 0 ? mvx[0] : q == 1 ? mvx[1] : mvx[2];
      my[j] = q == 0 ? mvy[0] : q == 1 ? mvy[1] : mvy[2];
    } else {
      rf[j] = nb.ref_idx; mx[j] = nb.mv_x; my[j] = nb.mv_y;
    }
  }
  const int r = c.ref_idx;
  const int rL = av[0] ? rf[0] : -1, rU = av[1] ? rf[1] : -1, rUR = av[2] ? rf[2] : -1;
  int type = 0;   // 0 median, 1 L, 2 U, 3 UR
  if (rL == r && rU != r && rUR != r) type = 1;
  else if (rL != r && rU == r && rUR != r) type = 2;
  else if (rL != r && rU != r && rUR == r) type = 3;
  if (bsx == 8 && bsy == 16) {
    if (sg.bx == 0) { if (rL == r) type = 1; }
    else { if (rUR == r) type = 3; }
  } else if (bsx == 16 && bsy == 8) {
    if (sg.by == 0) { if (rU == r) type = 2; }
    else { if (rL == r) type = 1; }
  }
  int px = 0, py = 0;
  if (type == 0) {
    if (!(av[1] || av[2])) {
      if (av[0]) { px = mx[0]; py = my[0]; }
    } else {
      px = imedian3(av[0] ? mx[0] : 0, av[1] ? mx[1] : 0, av[2] ? mx[2] : 0);
      py = imedian3(av[0] ? my[0] : 0, av[1] ? my[1] : 0, av[2] ? my[2] : 0);
    }
  } else {
    const int j = type - 1;
    if (av[j]) { px = mx[j]; py = my[j]; }
  }
  px = (int16_t)px; py = (int16_t)py;
  // BlockMotionSearch's centre: JM_INT_DIVIDE rounding, the (0,0)-inside clip
  // with CheckSearchRange when RDO is off, then the level's vector range
  int cx = (int16_t)(((px + 2) >> 2) * 4), cy = (int16_t)(((py + 2) >> 2) * 4);
  int mnx = st.sr_min_x, mxx = st.sr_max_x, mny = st.sr_min_y, mxy = st.sr_max_y;
  if (!c.rdopt) {
    const int ccx = cx, ccy = cy;
    cx = clampi(cx, mnx, mxx);
    cy = clampi(cy, mny, mxy);
    if (cx != ccx || cy != ccy) {
      const int md = max_mvd - 2;
      int left = cx + mnx, right = cx + mxx, top = cy + mny, down = cy + mxy;
      left = clampi(left, ccx - md, ccx + md);
      right = clampi(right, ccx - md, ccx + md);
      top = clampi(top, ccy - md, ccy + md);
      down = clampi(down, ccy - md, ccy + md);
      if (left < right && top < down) {
        cx = (int16_t)((left + right) >> 1);
        cy = (int16_t)((top + down) >> 1);
        mnx = left - cx; mxx = min(cx - left, right - cx);
        mny = top - cy; mxy = min(cy - top, down - cy);
      } else {
        cx = ccx; cy = ccy;
      }
    }
  }
  ChainStepIn o;
  o.px = px; o.py = py;
  o.cx = clampi(cx, c.mv_lim_x0, c.mv_lim_x1);
  o.cy = clampi(cy, c.mv_lim_y0, c.mv_lim_y1);
  o.rmin = min(mxx, mxy) >> 2;
  o.rmax = max(mxx, mxy) >> 2;
  return o;
}

// every position of the (2R+1)^2 window for a W x H (4x4 units) partition at
// (BX, BY): this thread's best (cost, rank).  Thread t owns window column
// t % D and every G-th row from t / D (G = 1024 / D row groups), so the column
// part of the vector cost is formed once; the spiral rank -- which only breaks
// ties -- is formed when a position ties the thread's best, and for the winner
// at the end.
template <bool FFS, int W, int H, bool HBD>
__device__ __forceinline__ void chain_sweep(const GroupCtx &g, const uint32_t *words, int wpr, const uint32_t *s_cur,
                                            int bx, int by, int tid, uint32_t &bc, uint32_t &br) {
  const int R = g.R, D = 2 * R + 1;
  const int G = kChainWG / D;                      // D <= 2 * kChainMaxR + 1 = 89 < 1024: G >= 11
  const int col = tid % D, grp = tid / D;
  if (grp >= G) return;
  const int ox = col - R, candx = g.cqx + 4 * ox, dx = candx - g.px;
  const uint32_t bits_x = (uint32_t)mvbits(dx);
  for (int iy = grp; iy < D; iy += G) {
    const int oy = iy - R, candy = g.cqy + 4 * oy, dy = candy - g.py;
    const bool is00 = candx == 0 && candy == 0;
    if (FFS) {
      const bool gate = max(abs(dx), abs(dy)) < g.max_mvd - 1;   // me_fullfast.c:663
      if (!pos_eligible<FFS>(g, gate, max(abs(ox), abs(oy)), is00)) continue;
    }
    uint32_t mvc = (uint32_t)g.lam * (bits_x + (uint32_t)mvbits(dy));
    if (g.chk00) mvc = check00_adjust(mvc, g.lam, is00);
    uint32_t sad = 0;
    const uint32_t *wb = words + (iy + 4 * by) * wpr + (col + 4 * bx);
#pragma unroll
    for (int r = 0; r < 4 * H; ++r)
#pragma unroll
      for (int wc = 0; wc < W; ++wc) {
        if constexpr (HBD) {   // a 4-pel chunk: words x and x+2 against two current dwords (v_sad_u16)
          const uint32_t *cr = s_cur + (4 * by + r) * 8 + 2 * (bx + wc);
          sad = __builtin_amdgcn_sad_u16(wb[r * wpr + 4 * wc], cr[0], sad);
          sad = __builtin_amdgcn_sad_u16(wb[r * wpr + 4 * wc + 2], cr[1], sad);
        } else {
          sad = __builtin_amdgcn_sad_u8(wb[r * wpr + 4 * wc], s_cur[(4 * by + r) * 4 + bx + wc], sad);
        }
      }
    const uint32_t cost = (sad << 5) + mvc;
    if (cost > bc) continue;
    const int sidx = spiral_index_bl(ox, oy);
    const uint32_t rank = FFS ? ((g.preseed && is00) ? 0u : (uint32_t)sidx + 1u) : (uint32_t)sidx;
    if (cost < bc || rank < br) { bc = cost; br = rank; }
  }
}

// SubPelME of a chain step (sub_pel_motion_estimation, me_fullsearch.c:186-289,
// the refinement BlockMotionSearch runs after IntPelME when DisableSubpelME is
// 0, mv_search.c:960-976).  Per phase (half-pel ring, quarter-pel ring) one
// thread forms one (candidate, 4x4 block) sum (jmme_subpel_dev.h job_sum: the
// metric's block sum at UMVLine4X-clamped sub-image coordinates) and adds it
// into the candidate's LDS slot; after the barrier every thread walks the
// candidates in JM's order with JM's comparisons and early-exit rule (dist),
// so the result is uniform with no broadcast.  No 8x8-transform SATD: the
// caller refuses JMME_SP_TEST8x8 for chains.
template <typename T>
__device__ __forceinline__ void chain_subpel_phase(const ChainParams &p, const T *sub, const T *org, int lg_nbx,
                                                   int lg_nb, int mx, int my, int p0, int p1, int sc, int metric,
                                                   int *sums, int tid) {
  const int ymax = p.height + 2 * spd::kPadY - 1 - 16 - spd::kPadY, xmax = p.width + 2 * spd::kPadX - 1 - 16 - spd::kPadX;
  if (tid < ((p1 - p0) << lg_nb)) {
    const int cnd = tid >> lg_nb, b = tid & ((1 << lg_nb) - 1), pos = p0 + cnd;
    const int bxo = (b & ((1 << lg_nbx) - 1)) * 4, byo = (b >> lg_nbx) * 4;
    const int s = spd::job_sum(sub, p.plane_stride, p.sub_pitch, org, p.pitch, ymax, xmax, metric, false,
                               mx + sc * spd::spiral_x(pos), my + sc * spd::spiral_y(pos), bxo, byo);
    atomicAdd(&sums[cnd], s);
  }
}

template <typename T>
__device__ __forceinline__ jmme_block_res chain_subpel(const ChainParams &p, const jmme_chain &c,
                                                       const jmme_subpel_req &sp, const SlotGeom &sg, int px, int py,
                                                       const jmme_block_res &r, int (*sums)[10], int tid) {
  const T *sub = reinterpret_cast<const T *>(p.subs[c.list * kMaxRefs + c.ref_idx]);
  const int pos_x = c.mb_x + 4 * sg.bx, pos_y = c.mb_y + 4 * sg.by;
  const int pxp = pos_x << 2, pyp = pos_y << 2;   // pos_x_padded (mv_search.c:685-686)
  const int lg_nbx = sg.w == 4 ? 2 : sg.w == 2 ? 1 : 0, lg_nb = lg_nbx + (sg.h == 4 ? 2 : sg.h == 2 ? 1 : 0);
  const T *org = reinterpret_cast<const T *>(p.cur) + (size_t)pos_y * p.pitch + pos_x;
  int mvx = r.mv_x, mvy = r.mv_y;
  int64_t min_mcost = sp.start_hp ? r.cost : spd::kDistMax;
  const bool chk0 = (sp.flags & JMME_SP_CHECK0) && c.ref_idx == 0 && sg.bt == 1 && mvx == 0 && mvy == 0;
  // half-pel ring (me_fullsearch.c:209-251)
  {
    const int p0 = sp.start_hp, p1 = !sp.start_hp ? max(1, (int)sp.search_pos2) : (int)sp.search_pos2;
    chain_subpel_phase(p, sub, org, lg_nbx, lg_nb, pxp + mvx, pyp + mvy, p0, p1, 2, sp.metric_h, sums[0], tid);
    __syncthreads();
    int best = 0;
    for (int pos = p0; pos < p1; ++pos) {
      const int cx = mvx + 2 * spd::spiral_x(pos), cy = mvy + 2 * spd::spiral_y(pos);
      int64_t mcost = spd::mv_cost(sp.lambda_h, cx, cy, px, py);
      if (mcost >= min_mcost) continue;
      mcost += spd::dist(sums[0][pos - p0], min_mcost - mcost);
      if (pos == 0 && chk0) mcost -= (int64_t)sp.lambda_h * 16;   // weighted_cost(lambda_factor, 16)
      if (mcost < min_mcost) { min_mcost = mcost; best = pos; }
    }
    if (best) { mvx += 2 * spd::spiral_x(best); mvy += 2 * spd::spiral_y(best); }
  }
  if (!sp.start_qp) min_mcost = spd::kDistMax;
  // quarter-pel ring (me_fullsearch.c:252-285)
  {
    const int p0 = sp.start_qp, p1 = sp.search_pos4;
    chain_subpel_phase(p, sub, org, lg_nbx, lg_nb, pxp + mvx, pyp + mvy, p0, p1, 1, sp.metric_q, sums[1], tid);
    __syncthreads();
    int best = 0;
    for (int pos = p0; pos < p1; ++pos) {
      const int cx = mvx + spd::spiral_x(pos), cy = mvy + spd::spiral_y(pos);
      int64_t mcost = spd::mv_cost(sp.lambda_q, cx, cy, px, py);
      if (mcost >= min_mcost) continue;
      mcost += spd::dist(sums[1][pos - p0], min_mcost - mcost);
      if (mcost < min_mcost) { min_mcost = mcost; best = pos; }
    }
    if (best) { mvx += spd::spiral_x(best); mvy += spd::spiral_y(best); }
  }
  jmme_block_res o;
  o.mv_x = (int16_t)mvx; o.mv_y = (int16_t)mvy; o.reserved = 0; o.cost = min_mcost;
  return o;
}

template <bool FFS, bool HBD>
__global__ __launch_bounds__(kChainWG) void chain_kernel(ChainParams p) {
  extern __shared__ uint32_t dyn[];
  __shared__ uint32_t s_cur[HBD ? 128 : 64];
  __shared__ uint32_t s_minc[2][kChainWaves], s_minr[2][kChainWaves];   // by step parity: one barrier per step
  __shared__ jmme_chain s_chain;                                         // out of the kernel arguments once
  __shared__ int s_sps[2][2][10];   // in-chain SubPelME: by step parity, per phase, per candidate
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#ifdef JMME_CHAIN_PROF
  if (blockIdx.x == 0 && tid == 0) g_chain_prof[30] = __builtin_amdgcn_s_memtime();
#endif
  CPROF(0);
  {
    // one parallel round of dword loads instead of a dependent scalar load per field
    constexpr int kWords = sizeof(jmme_chain) / 4;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(&p.chains[blockIdx.x]);
    uint32_t *dst = reinterpret_cast<uint32_t *>(&s_chain);
    if (tid >= 64 && tid < 64 + kWords) dst[tid - 64] = src[tid - 64];
  }
  __syncthreads();
  CPROF(1);
  const jmme_chain &c = s_chain;
  const int n_steps = c.n_steps;
  const uint8_t *ref = p.refs[c.list * kMaxRefs + c.ref_idx];
  if constexpr (HBD) {
    if (tid < 128)
      s_cur[tid] = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint16_t *>(p.cur) +
                                                       (size_t)(c.mb_y + (tid >> 3)) * p.pitch + c.mb_x + 2 * (tid & 7));
  } else if (tid < 64) {
    s_cur[tid] = *reinterpret_cast<const uint32_t *>(p.cur + (size_t)(c.mb_y + (tid >> 2)) * p.pitch + c.mb_x +
                                                     4 * (tid & 3));
  }
  // every thread holds the steps' vectors (as the next steps read them) and,
  // for thread 0's final write, their results
  int mvx[4] = {0, 0, 0, 0}, mvy[4] = {0, 0, 0, 0};
  jmme_chain_res res[4];
  bool alive = true;
  int st_x = 0, st_y = 0, st_w = 0, st_h = 0;   // the staged window in LDS (origin, words per row, rows)
#pragma unroll
  for (int k = 0; k < JMME_CHAIN_MAX_STEPS; ++k) {
    if (k >= n_steps) break;
    const jmme_chain_step &st = c.steps[k];
    const ChainStepIn in = chain_derive(c, st, mvx, mvy, p.max_mvd);
    const int cqx = FFS ? c.ffs_center_x : in.cx, cqy = FFS ? c.ffs_center_y : in.cy;
    const int R = FFS ? c.ffs_range : in.rmin, rs = FFS ? in.rmax : in.rmin;
    res[k].pred_x = (int16_t)in.px; res[k].pred_y = (int16_t)in.py;
    res[k].center_x = (int16_t)in.cx; res[k].center_y = (int16_t)in.cy;
    res[k].range_min = (int16_t)in.rmin; res[k].range_max = (int16_t)in.rmax;
    res[k].mv_x = res[k].mv_y = 0;
    CPROF(2 + 4 * k);
    // the window must fit the staged LDS and (FS) start on an integer vector
    alive = alive && R >= 0 && R <= p.max_r && rs >= 0 && !((cqx | cqy) & 3);
    if (!alive) {   // this step and the rest: no answer
      res[k].cost = -1;
      mvx[k] = cqx; mvy[k] = cqy;
      continue;
    }
    // stage the window of the whole macroblock: words[y][x] = pels x..x+3 of
    // window row y, clamped into the picture (UMVLine4X), with a margin; a step
    // whose window (origin: macroblock origin + centre - R) lies inside the
    // staged one searches it in place (FFS: one staging per chain)
    const int X0 = c.mb_x + (cqx >> 2) - R, Y0 = c.mb_y + (cqy >> 2) - R;
    if (!(X0 >= st_x && Y0 >= st_y && X0 + 2 * R + (HBD ? 15 : 13) <= st_x + st_w && Y0 + 2 * R + 16 <= st_y + st_h)) {
      st_x = X0 - kChainMargin; st_y = Y0 - kChainMargin; st_w = HBD ? chain_wpr16(R) : chain_wpr(R);
      st_h = chain_rows(R);
      if constexpr (HBD) {   // raw[r][q] = samples xa + 2q, +1 (clamped); words[x] = samples x, x + 1
        const int wpr = st_w, nraw = chain_raw16(R), rows = st_h;
        uint32_t *words = dyn, *raw = dyn + (size_t)rows * wpr;
        const int xa = st_x & ~1, sh = st_x - xa, Y0s = st_y;
        for (int i = tid; i < rows * nraw; i += kChainWG) {
          const int r = i / nraw, q = i - r * nraw;
          const uint16_t *row = reinterpret_cast<const uint16_t *>(ref) + (size_t)clampi(Y0s + r, 0, p.height - 1) * p.pitch;
          const int x = xa + 2 * q;
          raw[i] = (x >= 0 && x + 1 < p.width)
                       ? *reinterpret_cast<const uint32_t *>(row + x)
                       : (uint32_t)row[clampi(x, 0, p.width - 1)] | ((uint32_t)row[clampi(x + 1, 0, p.width - 1)] << 16);
        }
        __syncthreads();
        for (int i = tid; i < rows * wpr; i += kChainWG) {
          const int r = i / wpr, x = i - r * wpr, q = (sh + x) >> 1;
          words[i] = __builtin_amdgcn_alignbyte(raw[r * nraw + q + 1], raw[r * nraw + q], 2 * ((sh + x) & 1));
        }
        __syncthreads();
      } else {
      const int wpr = st_w, nraw = chain_raw(R), rows = st_h;
      uint32_t *words = dyn, *raw = dyn + (size_t)rows * wpr;
      const int xa = st_x & ~3, sh = st_x - xa, Y0s = st_y;
      for (int i = tid; i < rows * nraw; i += kChainWG) {
        const int r = i / nraw, q = i - r * nraw;
        const uint8_t *row = ref + (size_t)clampi(Y0s + r, 0, p.height - 1) * p.pitch;
        const int x = xa + 4 * q;
        uint32_t w;
        if (x >= 0 && x + 3 < p.width) {
          w = *reinterpret_cast<const uint32_t *>(row + x);
        } else {
          w = 0;
#pragma unroll
          for (int b = 0; b < 4; ++b) w |= (uint32_t)row[clampi(x + b, 0, p.width - 1)] << (8 * b);
        }
        raw[i] = w;
      }
      __syncthreads();
      for (int i = tid; i < rows * wpr; i += kChainWG) {
        const int r = i / wpr, x = i - r * wpr, q = (sh + x) >> 2;
        words[i] = __builtin_amdgcn_alignbyte(raw[r * nraw + q + 1], raw[r * nraw + q], (sh + x) & 3);
      }
      __syncthreads();
      }
    }
    const int wpr = st_w;
    const uint32_t *words = dyn + (size_t)(Y0 - st_y) * wpr + (X0 - st_x);   // this step's window in the staging
    CPROF(3 + 4 * k);
    GroupCtx g{};
    g.R = R; g.rs = rs; g.cqx = cqx; g.cqy = cqy; g.px = in.px; g.py = in.py; g.lam = c.lambda; g.max_mvd = p.max_mvd;
    g.preseed = FFS && c.ffs_pos00_valid;
    g.chk00 = !FFS && st.slot == 0 && (st.flags & JMME_CHAIN_CHECK00);
    const SlotGeom sg = slot_geom(st.slot);
    uint32_t bc = ~0u, br = ~0u;   // this thread's best (cost, rank)
    switch (sg.bt) {
      case 1: chain_sweep<FFS, 4, 4, HBD>(g, words, wpr, s_cur, sg.bx, sg.by, tid, bc, br); break;
      case 2: chain_sweep<FFS, 4, 2, HBD>(g, words, wpr, s_cur, sg.bx, sg.by, tid, bc, br); break;
      case 3: chain_sweep<FFS, 2, 4, HBD>(g, words, wpr, s_cur, sg.bx, sg.by, tid, bc, br); break;
      case 4: chain_sweep<FFS, 2, 2, HBD>(g, words, wpr, s_cur, sg.bx, sg.by, tid, bc, br); break;
      case 5: chain_sweep<FFS, 2, 1, HBD>(g, words, wpr, s_cur, sg.bx, sg.by, tid, bc, br); break;
      case 6: chain_sweep<FFS, 1, 2, HBD>(g, words, wpr, s_cur, sg.bx, sg.by, tid, bc, br); break;
      default: chain_sweep<FFS, 1, 1, HBD>(g, words, wpr, s_cur, sg.bx, sg.by, tid, bc, br); break;
    }
    // wave minimum of the cost (DPP), then the smallest rank among its holders;
    // after the one barrier every thread combines the 16 waves itself
    {
      const uint32_t cmin = wave_min_u32(bc);
      const uint32_t rmin = wave_min_u32(bc == cmin ? br : ~0u);
      if (lane == 0) { s_minc[k & 1][wave] = cmin; s_minr[k & 1][wave] = rmin; }
      // (this parity's sub-pel slots were last read in step k - 2, before step k - 1's barrier)
      if (p.subs && tid < 20) (&s_sps[k & 1][0][0])[tid] = 0;
    }
    __syncthreads();
    CPROF(4 + 4 * k);
    uint32_t bcost = s_minc[k & 1][0], brank = s_minr[k & 1][0];
#pragma unroll
    for (int w = 1; w < kChainWaves; ++w) {
      const uint32_t cw = s_minc[k & 1][w], rw = s_minr[k & 1][w];
      if (cw < bcost || (cw == bcost && rw < brank)) { bcost = cw; brank = rw; }
    }
    const jmme_block_res r = block_result<FFS>(g, brank != ~0u, brank, bcost);
    res[k].mv_x = r.mv_x; res[k].mv_y = r.mv_y; res[k].cost = r.cost;
    int fx = r.mv_x, fy = r.mv_y;
    if (p.subs) {   // SubPelME of the step's answer (mv_search.c:960-976)
      const jmme_block_res f = chain_subpel<std::conditional_t<HBD, uint16_t, uint8_t>>(
          p, c, p.sp[blockIdx.x], sg, in.px, in.py, r, s_sps[k & 1], tid);
      if (tid == 0) p.sp_res[(size_t)blockIdx.x * JMME_CHAIN_MAX_STEPS + k] = f;
      fx = f.mv_x; fy = f.mv_y;
    }
    // as BlockMotionSearch leaves it for the next partitions' predictors (mv_search.c:981)
    mvx[k] = clampi(fx, c.mv_lim_x0, c.mv_lim_x1);
    mvy[k] = clampi(fy, c.mv_lim_y0, c.mv_lim_y1);
    CPROF(5 + 4 * k);
  }
  if (tid == 0) {
    jmme_chain_res *out = p.res + (size_t)blockIdx.x * JMME_CHAIN_MAX_STEPS;
#pragma unroll
    for (int k = 0; k < JMME_CHAIN_MAX_STEPS; ++k)
      if (k < n_steps) out[k] = res[k];
    // the host polls this word instead of synchronising the stream: every
    // result of this chain (written by this thread) is visible before it
    if (p.done) {
      __threadfence_system();
      __hip_atomic_store(p.done + blockIdx.x, p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  CPROF(18);
#ifdef JMME_CHAIN_PROF
  if (blockIdx.x == 0 && tid == 0) g_chain_prof[31] = __builtin_amdgcn_s_memtime();
#endif
}


struct Occupancy {
  int cus = 0;
  int wg[8][JMME_MAX_RANGE + 1] = {};   // resident workgroups per CU, by kernel variant and lds range
};

template <typename K>
int resident_grid(Occupancy &o, int dev, int variant, K kernel, int lds_range, size_t lds) {
  if (!o.cus) {
    if (hipDeviceGetAttribute(&o.cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || o.cus <= 0)
      o.cus = 256;
  }
  int &nb = o.wg[variant][lds_range];
  if (!nb) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, kWG, lds) != hipSuccess || nb <= 0) nb = 1;
  }
  return nb * o.cus;
}

}  // namespace

size_t items_lds_bytes(int R, bool hbd) { return lds_plan(R, hbd).total; }

#ifdef JMME_CHAIN_PROF
}  // namespace jmme
extern "C" int jmme_debug_chain_prof(unsigned long long *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(jmme::g_chain_prof), sizeof jmme::g_chain_prof) == hipSuccess ? 0 : -1;
}
namespace jmme {
#endif


hipError_t launch_search(const KParams &p, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  // occupancy per device: the caller (jmme_capi) has made the context's device current
  constexpr int kMaxDev = 64;
  static thread_local Occupancy occ_tab[kMaxDev];
  int dev = 0;
  (void)hipGetDevice(&dev);
  Occupancy spare;
  Occupancy &occ = (dev >= 0 && dev < kMaxDev) ? occ_tab[dev] : spare;
  const size_t lds = items_lds_bytes(p.lds_range, p.hbd != 0);
  const bool ffs = p.mode == JMME_FAST_FULL_SEARCH;
  const int plan_grid = (p.n + kPlanWaves - 1) / kPlanWaves;
  if (ffs) hipLaunchKernelGGL(me_plan_kernel<true>, dim3(plan_grid), dim3(64 * kPlanWaves), 0, s, p);
  else hipLaunchKernelGGL(me_plan_kernel<false>, dim3(plan_grid), dim3(64 * kPlanWaves), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // the common +-32 launch: the instance with its LDS layout fixed at compile time
  auto k32 = p.lds_range == 32 ? (ffs ? me_items_kernel<true, true, false, 32> : me_items_kernel<true, false, false, 32>)
                               : (ffs ? me_items_kernel<true, true> : me_items_kernel<true, false>);
  auto k64 = ffs ? me_items_kernel<false, true> : me_items_kernel<false, false>;
  const int v = ffs ? 2 : 0;
  if (ev0) (void)hipEventRecord(ev0, s);
  if (p.hbd) {   // 16-bit planes: v_sad_u16; 32-bit keys up to 10 bits (p.key32), else 64-bit keys and the generic sweep
    auto k16 = p.key32 ? (ffs ? me_items_kernel<true, true, true> : me_items_kernel<true, false, true>)
                       : (ffs ? me_items_kernel<false, true, true> : me_items_kernel<false, false, true>);
    if (lds > 65536) {   // 16-bit staging above R = 36: raise the kernel's dynamic-LDS limit (once per instance and device)
      static thread_local bool raised[kMaxDev][4] = {};
      bool spare_flag = false;
      bool &done = (dev >= 0 && dev < kMaxDev) ? raised[dev][ffs + 2 * (p.key32 != 0)] : spare_flag;
      if (!done) {
        if ((e = hipFuncSetAttribute(reinterpret_cast<const void *>(k16), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds)) != hipSuccess)
          return e;
        done = true;
      }
    }
    hipLaunchKernelGGL(k16, dim3(resident_grid(occ, dev, (p.key32 ? 6 : 4) + v / 2, k16, p.lds_range, lds)), dim3(kWG),
                       lds, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ev1) (void)hipEventRecord(ev1, s);
  } else if (p.key32) {
    // (units whose lambda is beyond the 32-bit keys are served in this kernel
    // too, by the exact per-partition search: no second launch)
    hipLaunchKernelGGL(k32, dim3(resident_grid(occ, dev, v, k32, p.lds_range, lds)), dim3(kWG), lds, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ev1) (void)hipEventRecord(ev1, s);
  } else {
    hipLaunchKernelGGL(k64, dim3(resident_grid(occ, dev, v + 1, k64, p.lds_range, lds)), dim3(kWG), lds, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ev1) (void)hipEventRecord(ev1, s);
  }
  return hipGetLastError();
}

size_t chain_lds_bytes(int max_r, bool hbd) {
  return hbd ? (size_t)chain_rows(max_r) * (chain_wpr16(max_r) + chain_raw16(max_r)) * 4
             : (size_t)chain_rows(max_r) * (chain_wpr(max_r) + chain_raw(max_r)) * 4;
}

hipError_t launch_search_chains(const ChainParams &p, hipStream_t s) {
  if (p.n <= 0) return hipSuccess;
  const size_t lds = chain_lds_bytes(p.max_r, p.hbd);
  const bool ffs = p.mode == JMME_FAST_FULL_SEARCH;
  auto k = p.hbd ? (ffs ? chain_kernel<true, true> : chain_kernel<false, true>)
                 : (ffs ? chain_kernel<true, false> : chain_kernel<false, false>);
  if (lds > 65536) {   // 16-bit staging at R = 44: 65,728 B of the CU's 160 KiB (once per kernel, device and thread)
    constexpr int kMaxDev = 64;
    static thread_local bool raised[kMaxDev][2] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    bool spare_flag = false;
    bool &done = (dev >= 0 && dev < kMaxDev) ? raised[dev][ffs] : spare_flag;
    if (!done) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
      done = true;
    }
  }
  hipLaunchKernelGGL(k, dim3(p.n), dim3(kChainWG), lds, s, p);
  return hipGetLastError();
}

hipError_t launch_search_small(const SmallParams &p, hipStream_t s) {
  if (p.n_items <= 0) return hipSuccess;
  const dim3 grid((unsigned)(p.n_items * p.tiles * p.tiles)), g2((unsigned)((p.n_items * kNS + kWG - 1) / kWG));
  const bool ffs = p.mode == JMME_FAST_FULL_SEARCH;
  void (*search)(SmallParams) = p.hbd ? (ffs ? me_small_kernel<true, true> : me_small_kernel<false, true>)
                                      : (ffs ? me_small_kernel<true, false> : me_small_kernel<false, false>);
  void (*finish)(SmallParams) = ffs ? small_finish_kernel<true> : small_finish_kernel<false>;
  hipLaunchKernelGGL(search, grid, dim3(kWG), 0, s, p);
  if (!p.host_finish) hipLaunchKernelGGL(finish, g2, dim3(kWG), 0, s, p);
  return hipGetLastError();
}

}  // namespace jmme
