// jmme_fractal_pool.hip -- the thesis's full_search over a large domain pool
// (BASELINE configs[2]: "4x4 range blocks, full domain pool"), exact, with
// least-squares pruning.  ZL = /root/reference/2.论文程序/ZhangLing_Yu_
// version1/H264Fractal; full_search ZL/src/block_enc.c:1933-1977, compute_rms
// ZL/src/compute.c:6-189, QUAN_A ZL/inc/defines_enc.h:591-601.
//
// Why pruning is exact.  compute_rms evaluates, for the quantised scale
// α = a/100 and the block's quantised offset βq = QUAN_A(Σr/n) (the same for
// every candidate of a range block),
//     rms = Σ ((r − βq) − α (d − mean d))²                       (expanded form)
// so for every candidate, whatever α the quantiser picks,
//     rms ≥ LB = K − C²/D,   K = Σ(r − βq)²,  C = Σr·d − Σr·Σd/n,  D = Σd² − (Σd)²/n
// (the minimum of that parabola over real α; LB = K when D = 0).  In n·C and
// n·D only the integer sums Σrd, Σd, Σd² enter, so LB needs four v_dot4 and
// three float ops per (range, domain) pair instead of compute_rms's ~45 FP64
// operations and a division.  A candidate with LB > T + m, T = the exact rms
// of a candidate already evaluated, has rms > T (m = 1/64 covers the FP64
// rounding of the thesis's polynomial, < 1e-5 at 16x16), so it cannot be
// full_search's first strict minimum: only the rest ("survivors") are
// evaluated exactly (rms_of, bit-identical to the thesis) and folded into the
// lexicographic (rms, spiral rank) minimum.  The float test
//     fma(thr, D', −num'²) > 0 ⇒ prune,  num' = n·C/n (one fma), D' = n·D
// is made one-sided by shrinking thr = (K − T − m)/n by 2^-18 (≫ the ≤ 6
// float roundings of the test).
//
// Mapping (gfx950): one workgroup = 64 range blocks, one per lane, in all four
// waves; the waves split the rows of the wave's domain window.  The domain
// side of a pair is wave-uniform, so every domain quantity -- the four words of
// the block (the reference's words image), Σd and D (the per-size "pool
// image" pool_prep_kernel builds once per reference) -- arrives through scalar
// loads into SGPRs, and each pair is pure VALU: 4 v_dot4_u32_u8 (VGPR range
// word x SGPR domain word), cvt, fma, 2 mul, cmp.  Survivors branch to the
// exact FP64 path for their lane only.  The four waves' minima are merged in
// LDS.  Seeds (T before the first pair) come from the windowed kernel at a
// small radius, whose result is the exact minimum over a prefix of the same
// spiral.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "jmme.h"
#include "jmme_fractal_device.h"
#include "jmme_fractal_internal.h"

namespace jmme {

namespace {

constexpr int kPoolWG = 256;
constexpr int kPoolWaves = kPoolWG / 64;
constexpr int kChunk = 8;                    // domain positions per unrolled step
constexpr double kMargin = 1.0 / 64;         // ≫ the FP64 error of compute_rms's polynomial
constexpr float kShrink = 1.0f - 1.0f / 262144.0f;   // 1 - 2^-18

__device__ __forceinline__ int size_index(int bsx, int bsy) {
  switch ((bsx << 8) | bsy) {
    case (16 << 8) | 16: return 0;
    case (16 << 8) | 8: return 1;
    case (8 << 8) | 16: return 2;
    case (8 << 8) | 8: return 3;
    case (8 << 8) | 4: return 4;
    case (4 << 8) | 8: return 5;
    case (4 << 8) | 4: return 6;
    default: return -1;
  }
}

__global__ __launch_bounds__(kPoolWG) void pool_flags_kernel(const jmme_fractal_req *__restrict__ req, int n,
                                                             int *__restrict__ flags) {
  const int i = blockIdx.x * kPoolWG + threadIdx.x;
  if (i >= n) return;
  const int s = size_index(req[i].bsx, req[i].bsy);
  if (s >= 0) flags[s] = 1;          // benign race: every writer stores 1
}

// pool image of one block size: {Σd, n·Σd² − (Σd)²} per domain position, as
// floats (Σd exact; D rounded, 0 replaced by 1e-30 so that the pair test
// degenerates to "K − T − m > 0", the exact rule for a flat domain block)
template <int BSX, int BSY>
__global__ __launch_bounds__(kPoolWG) void pool_prep_kernel(const uint32_t *__restrict__ words, int wpitch, int W,
                                                            int H, const int *__restrict__ flags, int sidx,
                                                            float2 *__restrict__ pool) {
  if (!flags[sidx]) return;
  constexpr int NQ = BSX / 4, NO = BSX * BSY;
  const int x = blockIdx.x * kPoolWG + threadIdx.x, y = blockIdx.y;
  if (x > W - BSX || y > H - BSY) return;
  unsigned s1 = 0, s2 = 0;
#pragma unroll
  for (int r = 0; r < BSY; ++r)
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t d = words[(size_t)(y + r) * wpitch + x + 4 * q];
      s1 = __builtin_amdgcn_sad_u8(d, 0u, s1);
      s2 = __builtin_amdgcn_udot4(d, d, s2, false);
    }
  const unsigned det = NO * s2 - s1 * s1;      // < 2^32 for every thesis size, >= 0
  pool[(size_t)y * wpitch + x] = make_float2((float)s1, det ? (float)det : 1e-30f);
}

struct PoolBest { double rms; int rank, a; };

template <int BSX, int BSY, bool FULL>
__global__ __launch_bounds__(kPoolWG) void pool_search_kernel(
    const uint8_t *__restrict__ org, int pitch, const uint32_t *__restrict__ words, int wpitch,
    const float2 *__restrict__ pool, int W, int H, int R, const jmme_fractal_req *__restrict__ req, int n,
    const int *__restrict__ flags, int sidx, jmme_fractal_res *__restrict__ out,
    unsigned long long *__restrict__ stats) {
#pragma clang fp contract(off)
  constexpr int NQ = BSX / 4, ND = NQ * BSY, NO = BSX * BSY;
  __shared__ PoolBest s_best[kPoolWaves][64];
  if (!flags[sidx]) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = blockIdx.x * 64 + lane;
  const bool active = i < n && req[i].bsx == BSX && req[i].bsy == BSY;
  if (!__any(active)) return;                  // same answer in all four waves

  // ---- the lane's range block (search_one's prologue) ----
  int bx = 0, by = 0;
  uint32_t rw[ND];
  unsigned s1 = 0, s2 = 0;
  if (active) {
    bx = req[i].block_x;
    by = req[i].block_y;
  }
#pragma unroll
  for (int r = 0; r < BSY; ++r)
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t v = active ? *reinterpret_cast<const uint32_t *>(org + (size_t)(by + r) * pitch + bx + 4 * q) : 0u;
      rw[r * NQ + q] = v;
      s1 = __builtin_amdgcn_sad_u8(v, 0u, s1);
      s2 = __builtin_amdgcn_udot4(v, v, s2, false);
    }
  RangeStats rg;
  rg.rs1 = (double)s1;
  rg.rs2 = (double)s2;
  rg.beta = (double)quan_a((int)(rg.rs1 / NO));     // compute.c:161-164
  rg.bad_beta = rg.beta < -60 || rg.beta > 255;
  const double K = rg.rs2 - 2.0 * rg.beta * rg.rs1 + NO * rg.beta * rg.beta;   // Σ(r − βq)², exact integer
  const float nsr = -(float)s1 / NO;                                            // exact (power-of-two divisor)

  // ---- seed: the windowed search's exact minimum over a spiral prefix ----
  PoolBest best{2e30, 0x7fffffff, 0};
  if (active) {
    const jmme_fractal_res sd = out[i];
    best.rms = sd.rms;
    best.rank = spiral_rank(sd.x, sd.y);
    best.a = (int)lrint(sd.scale * 100);
  }
  auto threshold = [&](double T) -> float {
    if (!active) return INFINITY;                    // prunes every pair
    if (rg.bad_beta) return INFINITY;                // every candidate is 1e30: rank 0 (the seed) stands
    return (float)(((K - T) - kMargin) / NO) * kShrink;
  };
  float thr = threshold(best.rms);

  // ---- this wave's share of the domain window ----
  const int ilow = max(bx - R, 0), ihigh = min(bx + R, W - BSX);
  const int jlow = max(by - R, 0), jhigh = min(by + R, H - BSY);
  int xa, xb, ya, yb;
  if (FULL) {
    xa = 0; xb = W - BSX; ya = 0; yb = H - BSY;
  } else {
    int a0 = active ? ilow : 0x7fffffff, a1 = active ? ihigh : -1;
    int b0 = active ? jlow : 0x7fffffff, b1 = active ? jhigh : -1;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      a0 = min(a0, __shfl_xor(a0, off, 64));
      a1 = max(a1, __shfl_xor(a1, off, 64));
      b0 = min(b0, __shfl_xor(b0, off, 64));
      b1 = max(b1, __shfl_xor(b1, off, 64));
    }
    xa = __builtin_amdgcn_readfirstlane(a0);
    xb = __builtin_amdgcn_readfirstlane(a1);
    ya = __builtin_amdgcn_readfirstlane(b0);
    yb = __builtin_amdgcn_readfirstlane(b1);
  }
  const int rows = yb - ya + 1;
  const int y0 = ya + (int)((long long)rows * wave / kPoolWaves);
  const int y1 = ya + (int)((long long)rows * (wave + 1) / kPoolWaves);

  unsigned long long surv_count = 0;
  // one step over kChunk domain positions x0.. of row y; TAIL clamps the
  // positions past xb (loads stay inside the picture, the pairs are masked)
  auto step = [&](const uint32_t *wrow, const float2 *prow, int y, int x0, bool rowok, auto tail) {
    constexpr bool TAIL = decltype(tail)::value;
    unsigned srd[kChunk];
    float nm[kChunk], dt[kChunk];
    float emin = 1.0f;
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      const int x = TAIL ? min(x0 + k, xb) : x0 + k;
      unsigned acc = 0;
#pragma unroll
      for (int r = 0; r < BSY; ++r)
#pragma unroll
        for (int q = 0; q < NQ; ++q)
          acc = __builtin_amdgcn_udot4(rw[r * NQ + q], wrow[(size_t)r * wpitch + x + 4 * q], acc, false);
      srd[k] = acc;
      const float2 pd = prow[x];
      nm[k] = __builtin_fmaf(nsr, pd.x, (float)acc);     // (n·Σrd − Σr·Σd)/n, one rounding
      dt[k] = pd.y;
      // e <= 0  <=>  LB <= T + m (up to the shrink): the pair survives
      float e = __builtin_fmaf(thr, dt[k], -(nm[k] * nm[k]));
      if (!FULL) e = (x >= ilow && x <= ihigh) ? e : 1.0f;
      if (TAIL) e = (x0 + k <= xb) ? e : 1.0f;
      emin = fminf(emin, e);
    }
    bool any = !(emin > 0.0f);
    if (!FULL) any = any && rowok;
    if (!__any(any)) return;
    surv_count += __popcll(__ballot(any));
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      const int x = x0 + k;
      bool s = !(__builtin_fmaf(thr, dt[k], -(nm[k] * nm[k])) > 0.0f);   // thr may have tightened since
      if (!FULL) s = s && rowok && x >= ilow && x <= ihigh;
      if (TAIL) s = s && x <= xb;
      if (s) {
        unsigned ds1 = 0, ds2 = 0;
#pragma unroll
        for (int r = 0; r < BSY; ++r)
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const uint32_t d = wrow[(size_t)r * wpitch + x + 4 * q];
            ds1 = __builtin_amdgcn_sad_u8(d, 0u, ds1);
            ds2 = __builtin_amdgcn_udot4(d, d, ds2, false);
          }
        int a;
        const double rms = rms_of(ds1, ds2, srd[k], NO, rg, a);
        const int rank = spiral_rank(x - bx, y - by);
        if (rms < best.rms || (rms == best.rms && rank < best.rank)) {
          best.rms = rms;
          best.rank = rank;
          best.a = a;
          thr = threshold(rms);
        }
      }
    }
  };
  for (int y = y0; y < y1; ++y) {
    const uint32_t *wrow = words + (size_t)y * wpitch;
    const float2 *prow = pool + (size_t)y * wpitch;
    const bool rowok = FULL || (y >= jlow && y <= jhigh);
    int x0 = xa;
    for (; x0 + kChunk - 1 <= xb; x0 += kChunk) step(wrow, prow, y, x0, rowok, std::false_type{});
    if (x0 <= xb) step(wrow, prow, y, x0, rowok, std::true_type{});
  }

  // ---- merge the four waves' minima; lane 'lane' of wave 0 writes ----
  s_best[wave][lane] = best;
  if (lane == 0 && surv_count) atomicAdd(stats, surv_count);
  __syncthreads();
  if (wave == 0 && active) {
#pragma unroll
    for (int w = 1; w < kPoolWaves; ++w) {
      const PoolBest o = s_best[w][lane];
      if (o.rms < best.rms || (o.rms == best.rms && o.rank < best.rank)) best = o;
    }
    int xi, yj;
    spiral_xy(best.rank, xi, yj);
    jmme_fractal_res res;
    res.rms = best.rms;
    res.scale = (double)best.a / 100;
    res.offset = rg.beta;
    res.x = xi;
    res.y = yj;
    out[i] = res;
  }
}

// ---------------------------------------------------------------------------
// 4x4 full pool on the matrix cores.  For a 32 x 32 tile of (domain position,
// range block) pairs, Σrd is one v_mfma_f32_32x32x16_bf16: pels are integers
// 0..255, exact in bf16, their products exact in f32 and every partial sum of
// 16 of them (< 2^24) too, so D = Σrd exactly -- the same integer the VALU path
// forms with v_dot4.  Operands: A = 32 domain positions of one row (lane l:
// position x0 + (l & 31), pels of block rows 2h, 2h+1, h = l >> 5, from the
// "bf16 words" image: 4 bf16 per position), B = 32 range blocks (lane l: block
// l & 31, the same pel order -- A and B share the lane map, so the k order is
// irrelevant).  D: lane l holds column l & 31 (its range block) and rows
// (v&3) + 8(v>>2) + 4h (domain positions).  Epilogue per pair: one fma for
// num', one mul and one fma for the bound test, a min -- the domain's {Σd, n·D}
// come from the pool image through LDS.  A workgroup owns 128 range blocks
// (4 column groups, B fragments in VGPRs for the whole stream) and its four
// waves split the rows; survivors are evaluated exactly, one at a time, by the
// whole wave (uniform), and update the wave's LDS copy of the block's best.
typedef __bf16 mf_bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t mf_u32x4 __attribute__((ext_vector_type(4)));
typedef float mf_f32x16 __attribute__((ext_vector_type(16)));
typedef float mf_f32x2 __attribute__((ext_vector_type(2)));

constexpr int kMfCols = 4;
constexpr int kMfBlocks = 32 * kMfCols;

__device__ __forceinline__ uint32_t bf16_bits(uint32_t pel) { return __float_as_uint((float)pel) >> 16; }

// bw[y][x] = pels x..x+3 of row y as 4 bf16 (x <= W-4)
__global__ __launch_bounds__(kPoolWG) void bf16_words_kernel(const uint32_t *__restrict__ words, int wpitch, int W,
                                                             int H, const int *__restrict__ flags,
                                                             uint2 *__restrict__ bw) {
  if (!flags[6]) return;
  const int x = blockIdx.x * kPoolWG + threadIdx.x, y = blockIdx.y;
  if (x > W - 4 || y >= H) return;
  const uint32_t w = words[(size_t)y * wpitch + x];
  bw[(size_t)y * wpitch + x] = make_uint2(bf16_bits(w & 255) | bf16_bits((w >> 8) & 255) << 16,
                                          bf16_bits((w >> 16) & 255) | bf16_bits(w >> 24) << 16);
}

struct MfRange { double rs1, rs2, beta, K; int bx, by, bad, active; };

__global__ __launch_bounds__(kPoolWG, 4) void pool_mfma44_kernel(
    const uint8_t *__restrict__ org, int pitch, const uint32_t *__restrict__ words, const uint2 *__restrict__ bw,
    int wpitch, const float2 *__restrict__ pool, int W, int H, const jmme_fractal_req *__restrict__ req, int n,
    const int *__restrict__ flags, jmme_fractal_res *__restrict__ out, unsigned long long *__restrict__ stats) {
#pragma clang fp contract(off)
  constexpr int NO = 16;
  __shared__ MfRange s_rg[kMfBlocks];
  __shared__ PoolBest s_best[kPoolWaves][kMfBlocks];
  __shared__ float s_thr[kPoolWaves][kMfBlocks];
  __shared__ float4 s_dt[2][kPoolWaves][8];        // a tile's 32 1/sqrt(n·D), double-buffered
  if (!flags[6]) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hh = lane >> 5, col = lane & 31;
  const int base = blockIdx.x * kMfBlocks;

  // ---- range blocks: stats (one thread per block) and seeds ----
  bool mine = false;
  if (threadIdx.x < kMfBlocks) {
    const int i = base + threadIdx.x;
    MfRange rr{};
    rr.active = i < n && req[i].bsx == 4 && req[i].bsy == 4;
    mine = rr.active;
    if (rr.active) {
      rr.bx = req[i].block_x;
      rr.by = req[i].block_y;
      unsigned s1 = 0, s2 = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t v = *reinterpret_cast<const uint32_t *>(org + (size_t)(rr.by + r) * pitch + rr.bx);
        s1 = __builtin_amdgcn_sad_u8(v, 0u, s1);
        s2 = __builtin_amdgcn_udot4(v, v, s2, false);
      }
      rr.rs1 = (double)s1;
      rr.rs2 = (double)s2;
      rr.beta = (double)quan_a((int)(rr.rs1 / NO));
      rr.bad = rr.beta < -60 || rr.beta > 255;
      rr.K = rr.rs2 - 2.0 * rr.beta * rr.rs1 + NO * rr.beta * rr.beta;
    }
    s_rg[threadIdx.x] = rr;
  }
  if (!__syncthreads_or(mine)) return;
  auto threshold = [&](const MfRange &rr, double T) -> float {
    if (!rr.active || rr.bad) return INFINITY;
    return (float)(((rr.K - T) - kMargin) / NO) * kShrink;
  };
  for (int t = lane; t < kMfBlocks; t += 64) {
    const MfRange &rr = s_rg[t];
    PoolBest b{2e30, 0x7fffffff, 0};
    if (rr.active) {
      const jmme_fractal_res sd = out[base + t];
      b.rms = sd.rms;
      b.rank = spiral_rank(sd.x, sd.y);
      b.a = (int)lrint(sd.scale * 100);
    }
    s_best[wave][t] = b;
    s_thr[wave][t] = threshold(rr, b.rms);
  }
  __syncthreads();

  // the bound test compares |num'| / sqrt(n·D) with sqrt(thr): thr <= 0 prunes nothing (st = -1),
  // thr = inf prunes everything; the <= 1 ulp errors of sqrt and rsq and the product's rounding
  // (< 2^-21 together) are far inside the 2^-18 shrink.  A flat domain block has n·D = 1e-30 in the
  // pool image and num' = 0 exactly, so its ratio is 0: pruned iff thr > 0, the exact rule
  auto st_of = [](float t) { return t > 0.0f ? __builtin_sqrtf(t) : -1.0f; };
  // ---- B fragments (range blocks, centred) and per-lane constants, whole stream ----
  // r~ = r - Σr/16 is a multiple of 1/16 below 256: hi = its top 8 significant
  // bits (a bf16), lo = r~ - hi (exact in bf16 too), so two MFMAs give
  // num' = Σ d·r~ = Σrd - Σr·Σd/16 exactly: every product and partial sum is a
  // multiple of 1/16 below 2^20
  mf_bf16x8 Bh[kMfCols], Bl[kMfCols];
  float thr[kMfCols];
#pragma unroll
  for (int cb = 0; cb < kMfCols; ++cb) {
    const MfRange &rr = s_rg[cb * 32 + col];
    mf_u32x4 fh = {0u, 0u, 0u, 0u}, fl = fh;
    if (rr.active) {
      const float mean = (float)rr.rs1 / NO;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const uint32_t v = *reinterpret_cast<const uint32_t *>(org + (size_t)(rr.by + 2 * hh + r) * pitch + rr.bx);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float rt = (float)((v >> (8 * c)) & 255) - mean;
          const uint32_t hb = __float_as_uint(rt) >> 16;
          const uint32_t lb = __float_as_uint(rt - __uint_as_float(hb << 16)) >> 16;
          fh[2 * r + (c >> 1)] |= hb << (16 * (c & 1));
          fl[2 * r + (c >> 1)] |= lb << (16 * (c & 1));
        }
      }
    }
    Bh[cb] = __builtin_bit_cast(mf_bf16x8, fh);
    Bl[cb] = __builtin_bit_cast(mf_bf16x8, fl);
    thr[cb] = st_of(s_thr[wave][cb * 32 + col]);
  }

  const int xb = W - 4, yb = H - 4;
  const int rows = yb + 1;
  const int y0 = (int)((long long)rows * wave / kPoolWaves);
  const int y1 = (int)((long long)rows * (wave + 1) / kPoolWaves);
  unsigned long long surv_count = 0;
  auto dtl_of = [&](int b) { return reinterpret_cast<float *>(s_dt[b][wave]); };
  float *dtl = dtl_of(0);

  // exact evaluation of one survivor (wave-uniform arguments; ds1, ds2 are the
  // domain block's integer sums, taken from the A fragment -- no memory access
  // here, so the tile loop's vmcnt accounting stays exact)
  auto exact = [&](int t, int xs, int y, unsigned rd, unsigned ds1, unsigned ds2) {
    const MfRange &rr = s_rg[t];
    RangeStats rg;
    rg.rs1 = rr.rs1;
    rg.rs2 = rr.rs2;
    rg.beta = rr.beta;
    rg.bad_beta = rr.bad;
    int a;
    const double rms = rms_of(ds1, ds2, rd, NO, rg, a);
    const int rank = spiral_rank(xs - rr.bx, y - rr.by);
    const PoolBest b = s_best[wave][t];
    if (rms < b.rms || (rms == b.rms && rank < b.rank)) {
      if (lane == 0) {
        s_best[wave][t] = PoolBest{rms, rank, a};
        s_thr[wave][t] = threshold(rr, rms);
      }
    }
    __builtin_amdgcn_wave_barrier();
  };


  // tiles (y, x0) in row-major order; the next tile's global loads are issued
  // before the current tile's arithmetic, its {Σd, n·D} land in the other LDS
  // buffer at the end of the step
  const int ntx = xb / 32 + 1;                     // tiles per row
  const int ntiles = (y1 - y0) * ntx;
  struct TileIn { uint2 a0, a1; float2 pd; };
  // tile coordinates advance incrementally (no divisions in the loop)
  auto adv = [&](int &ty, int &tx) {
    tx += 32;
    if (tx > xb) {
      tx = 0;
      ++ty;
    }
  };
  auto load = [&](int ty, int tx, TileIn &in) {
    if (ty >= y1) return;
    const int xc = min(tx + col, xb);
    const uint2 *r0 = bw + (size_t)(ty + 2 * hh) * wpitch;
    in.a0 = r0[xc];
    in.a1 = r0[wpitch + xc];
    in.pd = pool[(size_t)ty * wpitch + xc];        // both lane halves (one address per column)
  };
  int buf = 0;
  // one tile: its {Σd, sqrt(n·D)} are in LDS buffer `buf`; at the end the next
  // tile's (already loaded) values go to the other buffer
  auto step = [&](int y, int x0, const TileIn &cur, const TileIn &nxt) {
    const mf_u32x4 af = {cur.a0.x, cur.a0.y, cur.a1.x, cur.a1.y};
    const mf_bf16x8 A = __builtin_bit_cast(mf_bf16x8, af);
    __builtin_amdgcn_wave_barrier();
    float dt[16];
#pragma unroll
    for (int g = 0; g < 4; ++g) {                             // positions 8g + 4h .. +3
      const float4 r = s_dt[buf][wave][2 * g + hh];
      dt[4 * g] = r.x; dt[4 * g + 1] = r.y; dt[4 * g + 2] = r.z; dt[4 * g + 3] = r.w;
    }
    const bool tail = x0 + 31 > xb;
    // q < st  <=>  |num'| / sqrt(n·D) < sqrt(thr): pruned; otherwise the pair survives
    // (st = sqrt(thr) per lane, dt = 1/sqrt(n·D) per position; the slow path recomputes q bit-identically)
    auto test = [&](const mf_f32x16 &D, float st, int v) {
      const float q = __builtin_fabsf(D[v] * dt[v]);
      return (tail && x0 + (v & 3) + 8 * (v >> 2) + 4 * hh > xb) ? false : !(q < st);
    };
    auto num_of = [&](int cb) {
      const mf_f32x16 Dh = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, Bh[cb], mf_f32x16{}, 0, 0, 0);
      return __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, Bl[cb], Dh, 0, 0, 0);
    };
    unsigned hit = 0;
    // does any pair of the column group survive?  Products two at a time (v_pk_mul_f32), their
    // magnitudes folded by v_max3_f32 with abs modifiers: 16 VALU per 16 pairs
    auto any_of = [&](const mf_f32x16 &D, int cb) {
      if (!tail) {                    // the same arithmetic without the column mask
        float qm = 0.0f;
#pragma unroll
        for (int v = 0; v < 16; v += 2) {
          const mf_f32x2 pr = mf_f32x2{D[v], D[v + 1]} * mf_f32x2{dt[v], dt[v + 1]};
          qm = fmaxf(fmaxf(qm, __builtin_fabsf(pr[0])), __builtin_fabsf(pr[1]));
        }
        return !(qm < thr[cb]);
      }
      bool any = false;
#pragma unroll
      for (int v = 0; v < 16; ++v) any |= test(D, thr[cb], v);
      return any;
    };
    // column groups in pairs: both hi MFMAs, then both lo MFMAs (each lo finds its hi
    // done), then the two epilogues -- two accumulators live, no MFMA waits on its own chain
#pragma unroll
    for (int cb = 0; cb < kMfCols; cb += 2) {
      mf_f32x16 D0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, Bh[cb], mf_f32x16{}, 0, 0, 0);
      mf_f32x16 D1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, Bh[cb + 1], mf_f32x16{}, 0, 0, 0);
      D0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, Bl[cb], D0, 0, 0, 0);
      D1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, Bl[cb + 1], D1, 0, 0, 0);
      if (__any(any_of(D0, cb))) hit |= 1u << cb;
      if (__any(any_of(D1, cb + 1))) hit |= 2u << cb;
    }
    if (hit) {                                           // rare: survivors, one at a time
      for (int cb = 0; cb < kMfCols; ++cb) {
        if (!((hit >> cb) & 1)) continue;
        const mf_f32x16 D = num_of(cb);
        for (int v = 0; v < 16; ++v) {
          unsigned long long m = __ballot(test(D, thr[cb], v));
          while (m) {
            const int ln = __ffsll((long long)m) - 1;
            m &= m - 1;
            ++surv_count;
            const int tb = cb * 32 + (ln & 31);
            const int xs = x0 + (v & 3) + 8 * (v >> 2) + 4 * (ln >> 5);
            const float num = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(D[v]), ln));
            const int pos = (v & 3) + 8 * (v >> 2) + 4 * (ln >> 5);   // lanes pos (rows 0-1), pos + 32 (rows 2-3)
            unsigned ds1 = 0, ds2 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
              for (int hl = 0; hl < 2; ++hl) {
                const unsigned w = (unsigned)__builtin_amdgcn_readlane((int)af[k], pos + 32 * hl);
                const unsigned p0 = (unsigned)__uint_as_float(w << 16), p1 = (unsigned)__uint_as_float(w & 0xffff0000u);
                ds1 += p0 + p1;
                ds2 += p0 * p0 + p1 * p1;
              }
            // Σrd = num' + Σr·Σd/16, an integer (both terms are multiples of 1/16, exact in double)
            const unsigned rd = (unsigned)((double)num + s_rg[tb].rs1 * (double)ds1 / NO);
            exact(tb, xs, y, rd, ds1, ds2);
          }
        }
        thr[cb] = st_of(s_thr[wave][cb * 32 + col]);
      }
    }
    buf ^= 1;
    dtl_of(buf)[col] = __builtin_amdgcn_rsqf(nxt.pd.y);  // both halves store the same value: no branch,
                                                         // so the waitcnt pass sees one straight path
  };
  // two register sets X, Y alternate (unrolled by two, so no register copies
  // wait on loads in flight): the tile after next loads while one computes
  TileIn X{make_uint2(0, 0), make_uint2(0, 0), make_float2(0.f, 1.f)}, Y = X;
  int cy = y0, cx = 0;                 // the tile being computed
  int ly = y0, lx = 0;                 // the next tile to load
  load(ly, lx, X);
  adv(ly, lx);
  load(ly, lx, Y);
  adv(ly, lx);
  dtl[col] = __builtin_amdgcn_rsqf(X.pd.y);
  int t = 0;
  for (; t + 1 < ntiles; t += 2) {       // both steps on every trip: exact vmcnt at the loop head
    step(cy, cx, X, Y);
    adv(cy, cx);
    load(ly, lx, X);
    adv(ly, lx);
    step(cy, cx, Y, X);
    adv(cy, cx);
    load(ly, lx, Y);
    adv(ly, lx);
  }
  if (t < ntiles) step(cy, cx, X, Y);

  if (lane == 0 && surv_count) atomicAdd(stats, surv_count);
  __syncthreads();
  if (threadIdx.x < kMfBlocks && s_rg[threadIdx.x].active) {
    const int t = threadIdx.x;
    PoolBest best = s_best[0][t];
#pragma unroll
    for (int w = 1; w < kPoolWaves; ++w) {
      const PoolBest o = s_best[w][t];
      if (o.rms < best.rms || (o.rms == best.rms && o.rank < best.rank)) best = o;
    }
    int xi, yj;
    spiral_xy(best.rank, xi, yj);
    jmme_fractal_res res;
    res.rms = best.rms;
    res.scale = (double)best.a / 100;
    res.offset = s_rg[t].beta;
    res.x = xi;
    res.y = yj;
    out[base + t] = res;
  }
}

template <int BSX, int BSY>
hipError_t launch_size(const FractalPoolParams &p, int sidx, hipStream_t s) {
  const int W = p.base.width, H = p.base.height;
  float2 *pool = reinterpret_cast<float2 *>(p.pool[sidx]);
  hipLaunchKernelGGL((pool_prep_kernel<BSX, BSY>), dim3((W - BSX + kPoolWG) / kPoolWG, H - BSY + 1), dim3(kPoolWG),
                     0, s, p.base.words, p.base.wpitch, W, H, p.flags, sidx, pool);
  const bool full = p.base.range >= std::max(W - BSX, H - BSY);
  const dim3 grid((p.base.n + 63) / 64);
  if (BSX == 4 && BSY == 4 && full && p.bw && p.use_mfma) {
    hipLaunchKernelGGL(bf16_words_kernel, dim3((W - 4 + kPoolWG) / kPoolWG, H), dim3(kPoolWG), 0, s, p.base.words,
                       p.base.wpitch, W, H, p.flags, reinterpret_cast<uint2 *>(p.bw));
    hipLaunchKernelGGL(pool_mfma44_kernel, dim3((p.base.n + kMfBlocks - 1) / kMfBlocks), dim3(kPoolWG), 0, s,
                       p.base.org, p.base.pitch, p.base.words, reinterpret_cast<const uint2 *>(p.bw), p.base.wpitch,
                       pool, W, H, p.base.req, p.base.n, p.flags, p.base.out, p.stats);
  } else if (full)
    hipLaunchKernelGGL((pool_search_kernel<BSX, BSY, true>), grid, dim3(kPoolWG), 0, s, p.base.org, p.base.pitch,
                       p.base.words, p.base.wpitch, pool, W, H, p.base.range, p.base.req, p.base.n, p.flags, sidx,
                       p.base.out, p.stats);
  else
    hipLaunchKernelGGL((pool_search_kernel<BSX, BSY, false>), grid, dim3(kPoolWG), 0, s, p.base.org, p.base.pitch,
                       p.base.words, p.base.wpitch, pool, W, H, p.base.range, p.base.req, p.base.n, p.flags, sidx,
                       p.base.out, p.stats);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_fractal_pool(const FractalPoolParams &p, hipStream_t s) {
  hipError_t e = hipMemsetAsync(p.flags, 0, 8 * sizeof(int), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(pool_flags_kernel, dim3((p.base.n + kPoolWG - 1) / kPoolWG), dim3(kPoolWG), 0, s, p.base.req,
                     p.base.n, p.flags);
  // seeds: the windowed kernel at a small radius writes each request's exact
  // minimum over the first (2*seed+1)^2 spiral ranks into out[]
  FractalParams seed = p.base;
  seed.range = std::min(p.base.range, p.seed_range);
  if ((e = launch_fractal_search(seed, s)) != hipSuccess) return e;
  if ((e = launch_size<16, 16>(p, 0, s)) != hipSuccess) return e;
  if ((e = launch_size<16, 8>(p, 1, s)) != hipSuccess) return e;
  if ((e = launch_size<8, 16>(p, 2, s)) != hipSuccess) return e;
  if ((e = launch_size<8, 8>(p, 3, s)) != hipSuccess) return e;
  if ((e = launch_size<8, 4>(p, 4, s)) != hipSuccess) return e;
  if ((e = launch_size<4, 8>(p, 5, s)) != hipSuccess) return e;
  return launch_size<4, 4>(p, 6, s);
}

}  // namespace jmme
