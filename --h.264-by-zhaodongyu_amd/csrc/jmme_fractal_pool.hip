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

template <int BSX, int BSY>
hipError_t launch_size(const FractalPoolParams &p, int sidx, hipStream_t s) {
  const int W = p.base.width, H = p.base.height;
  float2 *pool = reinterpret_cast<float2 *>(p.pool[sidx]);
  hipLaunchKernelGGL((pool_prep_kernel<BSX, BSY>), dim3((W - BSX + kPoolWG) / kPoolWG, H - BSY + 1), dim3(kPoolWG),
                     0, s, p.base.words, p.base.wpitch, W, H, p.flags, sidx, pool);
  const bool full = p.base.range >= std::max(W - BSX, H - BSY);
  const dim3 grid((p.base.n + 63) / 64);
  if (full)
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
