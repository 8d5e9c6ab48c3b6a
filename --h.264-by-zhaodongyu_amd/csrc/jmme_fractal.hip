// jmme_fractal.hip -- gfx950 kernels for the thesis codec's fractal
// domain-range block matching, ZL =
// /root/reference/2.论文程序/ZhangLing_Yu_version1/H264Fractal:
//
//   compute_domain_Sum / compute_range_Sum   ZL/src/compute.c:277-~1091   (box sums)
//   compute_rms + compute_rdSum + QUAN_A     ZL/src/compute.c:6-215,
//                                            ZL/inc/defines_enc.h:19-22, 591-601
//   full_search + bound_chk                  ZL/src/block_enc.c:1933-1977, 2894-2919
//
// Exactness.  Every sum the thesis keeps in doubles (Σd, Σd², Σr, Σr², Σrd,
// n·Σd² − (Σd)², n·Σrd − Σr·Σd) is an integer below 2^53, so it is formed in
// integer arithmetic here (v_sad_u8 / v_dot4_u32_u8) and converted: the same
// doubles.  The remaining FP64 steps -- α = num/det, (int)(α·100), a/100 and
// the rms polynomial -- are evaluated with the thesis's operand order and no
// FMA contraction (#pragma clang fp contract(off)), IEEE-rounded division
// included, so every candidate's rms is bit-identical to the thesis's.  The
// search returns the lexicographic minimum of (rms, spiral rank), which is
// what full_search's strict '<' walk over its spiral keeps.
//
// Mapping: one wave per range block (request); the (2R+1)^2 spiral ranks are
// dealt across its 64 lanes; domain rows are read as aligned dwords from a
// "words" image of the reference (word[y][x] = pels x..x+3, built once per
// reference) that stays cache-resident; the range block sits in LDS and is
// read by broadcast.
#include <hip/hip_runtime.h>
#include "jmme.h"
#include "jmme_fractal_internal.h"

namespace jmme {

namespace {

constexpr int kWG = 256;
constexpr int kWaves = kWG / 64;

// QUAN_A, ZL/inc/defines_enc.h:591-601
__device__ __forceinline__ int quan_a(int x) {
  int b = x % 10, c = x / 10;
  if (b > 2 && b < 8) b = 5;
  else if (b > 7) { b = 0; c += 1; }
  else b = 0;
  return c * 10 + b;
}

// thesis spiral (block_enc.c:1944-1973): rank 0 = (0,0); ring l starts at
// (-l,-l) and walks right, down, left, up over 8l steps
__device__ __forceinline__ void spiral_xy(int rank, int &i, int &j) {
  if (rank == 0) { i = 0; j = 0; return; }
  int q = (int)sqrtf((float)rank);
  q -= q * q > rank;
  q += (q + 1) * (q + 1) <= rank;
  const int l = (q + 1) >> 1;                 // (2l-1)^2 <= rank < (2l+1)^2
  const int k = rank - (2 * l - 1) * (2 * l - 1);
  if (k < 2 * l) { i = -l + k; j = -l; }
  else if (k < 4 * l) { i = l; j = -l + (k - 2 * l); }
  else if (k < 6 * l) { i = l - (k - 4 * l); j = l; }
  else { i = -l; j = l - (k - 6 * l); }
}

struct RangeStats { double rs1, rs2, beta; int bad_beta; };

// compute_rms (compute.c:152-188) from the integer sums of one candidate.
// Returns rms (1e30 if the quantised parameters are out of range) and the
// quantised alpha numerator a (alpha = a / 100).
__device__ __forceinline__ double rms_of(unsigned ds1u, unsigned ds2u, unsigned rdu, int no, const RangeStats &rg,
                                         int &a_out) {
#pragma clang fp contract(off)
  const double dsum1 = (double)ds1u, dsum2 = (double)ds2u, rdsum = (double)rdu;
  const double det = no * dsum2 - dsum1 * dsum1;
  const double alpha = det == 0.0 ? 0.0 : (no * rdsum - rg.rs1 * dsum1) / det;
  const int a = quan_a((int)(alpha * 100));
  a_out = a;
  const double al = (double)a / 100;
  if (al < -2.35 || al > 4.0 || rg.bad_beta) return 1e30;   // MIN/MAX_ALPHA, MIN/MAX_BETA
  const double be = rg.beta;
  const double t = be - al * dsum1 / no;
  return rg.rs2 + al * (al * dsum2 - 2.0 * rdsum + 2.0 * t * dsum1) + t * (t * no - 2.0 * rg.rs1);
}

// lexicographic (rms, rank) minimum across the wave; lane 0 ends with it
__device__ __forceinline__ void wave_min(double &rms, int &rank, int &a) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double o_rms = __shfl_xor(rms, off, 64);
    const int o_rank = __shfl_xor(rank, off, 64);
    const int o_a = __shfl_xor(a, off, 64);
    if (o_rms < rms || (o_rms == rms && o_rank < rank)) { rms = o_rms; rank = o_rank; a = o_a; }
  }
}

template <int BSX, int BSY>
__device__ __forceinline__ void search_one(const FractalParams &p, const jmme_fractal_req &rq, uint32_t *rng,
                                           int lane, jmme_fractal_res *out) {
  constexpr int NQ = BSX / 4;            // dwords per row
  constexpr int ND = NQ * BSY;           // dwords per block
  constexpr int NO = BSX * BSY;
  const int bx = rq.block_x, by = rq.block_y;
  // range block -> LDS (per wave), and its sums
  unsigned s1 = 0, s2 = 0;
  if (lane < ND) {
    const int r = lane / NQ, q = lane - r * NQ;
    const uint32_t v = *reinterpret_cast<const uint32_t *>(p.org + (size_t)(by + r) * p.pitch + bx + 4 * q);
    rng[lane] = v;
    s1 = __builtin_amdgcn_sad_u8(v, 0u, 0u);
    s2 = __builtin_amdgcn_udot4(v, v, 0u, false);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    s1 += __shfl_xor(s1, off, 64);
    s2 += __shfl_xor(s2, off, 64);
  }
  RangeStats rg;
  rg.rs1 = (double)s1;
  rg.rs2 = (double)s2;
  {
#pragma clang fp contract(off)
    rg.beta = (double)quan_a((int)(rg.rs1 / NO));    // beta = QUAN_A(rsum1 / no), compute.c:161-164
  }
  rg.bad_beta = rg.beta < -60 || rg.beta > 255;
  __builtin_amdgcn_wave_barrier();

  // bound_chk window (block_enc.c:2894-2919)
  const int R = p.range;
  const int ilow = max(bx - R, 0), ihigh = min(bx + R, p.width - BSX);
  const int jlow = max(by - R, 0), jhigh = min(by + R, p.height - BSY);
  const int ncand = (2 * R + 1) * (2 * R + 1);
  double best = 1e30 * 2;   // above any rms, so rank decides among equals
  int best_rank = 0x7fffffff, best_a = 0;
  for (int rank = lane; rank < ncand; rank += 64) {
    int i, j;
    spiral_xy(rank, i, j);
    const int m = bx + i, n = by + j;
    if (rank != 0 && !(m >= ilow && m <= ihigh && n >= jlow && n <= jhigh)) continue;
    unsigned ds1 = 0, ds2 = 0, rd = 0;
    const uint32_t *w = p.words + (size_t)n * p.wpitch + m;
#pragma unroll
    for (int r = 0; r < BSY; ++r)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const uint32_t d = w[(size_t)r * p.wpitch + 4 * q];
        ds1 = __builtin_amdgcn_sad_u8(d, 0u, ds1);
        ds2 = __builtin_amdgcn_udot4(d, d, ds2, false);
        rd = __builtin_amdgcn_udot4(rng[r * NQ + q], d, rd, false);
      }
    int a;
    const double rms = rms_of(ds1, ds2, rd, NO, rg, a);
    if (rms < best || (rms == best && rank < best_rank)) { best = rms; best_rank = rank; best_a = a; }
  }
  wave_min(best, best_rank, best_a);
  if (lane == 0) {
    int i, j;
    spiral_xy(best_rank, i, j);
    jmme_fractal_res res;
    res.rms = best;
    {
#pragma clang fp contract(off)
      res.scale = (double)best_a / 100;
    }
    res.offset = rg.beta;
    res.x = i;                  // (0,0) winner: the thesis leaves the caller's 0, 0
    res.y = j;
    *out = res;
  }
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(kWG) void fractal_search_kernel(FractalParams p) {
  __shared__ uint32_t s_rng[kWaves][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int t = blockIdx.x * kWaves + wave; t < p.n; t += gridDim.x * kWaves) {
    const jmme_fractal_req rq = p.req[t];
    uint32_t *rng = s_rng[wave];
    jmme_fractal_res *o = p.out + t;
    switch ((rq.bsx << 8) | rq.bsy) {
      case (16 << 8) | 16: search_one<16, 16>(p, rq, rng, lane, o); break;
      case (16 << 8) | 8: search_one<16, 8>(p, rq, rng, lane, o); break;
      case (8 << 8) | 16: search_one<8, 16>(p, rq, rng, lane, o); break;
      case (8 << 8) | 8: search_one<8, 8>(p, rq, rng, lane, o); break;
      case (8 << 8) | 4: search_one<8, 4>(p, rq, rng, lane, o); break;
      case (4 << 8) | 8: search_one<4, 8>(p, rq, rng, lane, o); break;
      case (4 << 8) | 4: search_one<4, 4>(p, rq, rng, lane, o); break;
      default: break;   // validated on the host
    }
  }
}

// word[y][x] = pels x..x+3 of the reference (x <= W-4), from two aligned dwords
__global__ __launch_bounds__(kWG) void words_kernel(const uint8_t *__restrict__ ref, int pitch, int W, int H,
                                                    uint32_t *__restrict__ words, int wpitch) {
  const int x = blockIdx.x * kWG + threadIdx.x, y = blockIdx.y;
  if (x > W - 4 || y >= H) return;
  const uint8_t *row = ref + (size_t)y * pitch;
  const int xa = x & ~3;
  const uint32_t lo = *reinterpret_cast<const uint32_t *>(row + xa);
  const uint32_t hi = (xa + 4 < pitch) ? *reinterpret_cast<const uint32_t *>(row + xa + 4) : 0u;
  words[(size_t)y * wpitch + x] = __builtin_amdgcn_alignbyte(hi, lo, x & 3);
}

// compute_domain_Sum for one block size: horizontal then vertical integer box
// sums, stored as doubles (exact)
__global__ __launch_bounds__(kWG) void box_hsum_kernel(const uint8_t *__restrict__ p, int pitch, int W, int H,
                                                       int bsx, uint32_t *__restrict__ hs, uint32_t *__restrict__ hs2) {
  const int x = blockIdx.x * kWG + threadIdx.x, y = blockIdx.y;
  const int w = W - bsx + 1;
  if (x >= w || y >= H) return;
  unsigned s = 0, s2 = 0;
  for (int c = 0; c < bsx; ++c) {
    const unsigned v = p[(size_t)y * pitch + x + c];
    s += v;
    s2 += v * v;
  }
  hs[(size_t)y * w + x] = s;
  hs2[(size_t)y * w + x] = s2;
}

__global__ __launch_bounds__(kWG) void box_vsum_kernel(const uint32_t *__restrict__ hs, const uint32_t *__restrict__ hs2,
                                                       int w, int H, int bsy, double *__restrict__ sum,
                                                       double *__restrict__ sum2) {
  const int x = blockIdx.x * kWG + threadIdx.x, y = blockIdx.y;
  if (x >= w || y > H - bsy) return;
  unsigned s = 0, s2 = 0;
  for (int r = 0; r < bsy; ++r) {
    s += hs[(size_t)(y + r) * w + x];
    s2 += hs2[(size_t)(y + r) * w + x];
  }
  sum[(size_t)y * w + x] = (double)s;
  sum2[(size_t)y * w + x] = (double)s2;
}

}  // namespace

hipError_t launch_fractal_words(const uint8_t *ref, int pitch, int W, int H, uint32_t *words, int wpitch,
                                hipStream_t s) {
  hipLaunchKernelGGL(words_kernel, dim3((W + kWG - 1) / kWG, H), dim3(kWG), 0, s, ref, pitch, W, H, words, wpitch);
  return hipGetLastError();
}

hipError_t launch_fractal_search(const FractalParams &p, hipStream_t s) {
  int grid = (p.n + kWaves - 1) / kWaves;
  if (grid > 65535) grid = 65535;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(fractal_search_kernel, dim3(grid), dim3(kWG), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_box_sums(const uint8_t *p, int pitch, int W, int H, int bsx, int bsy, uint32_t *hs, uint32_t *hs2,
                           double *sum, double *sum2, hipStream_t s) {
  const int w = W - bsx + 1;
  hipLaunchKernelGGL(box_hsum_kernel, dim3((w + kWG - 1) / kWG, H), dim3(kWG), 0, s, p, pitch, W, H, bsx, hs, hs2);
  hipLaunchKernelGGL(box_vsum_kernel, dim3((w + kWG - 1) / kWG, H - bsy + 1), dim3(kWG), 0, s, hs, hs2, w, H, bsy,
                     sum, sum2);
  return hipGetLastError();
}

}  // namespace jmme
