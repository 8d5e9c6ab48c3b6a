// jmme_fractal_device.h -- device helpers shared by the fractal kernels
// (jmme_fractal.hip: windowed search and quadtree; jmme_fractal_pool.hip:
// the pruned domain-pool search).  ZL = /root/reference/2.论文程序/
// ZhangLing_Yu_version1/H264Fractal.
#pragma once
#include <hip/hip_runtime.h>

namespace jmme {
namespace {

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

// inverse of spiral_xy: the rank of offset (i, j) in the thesis's walk
__device__ __forceinline__ int spiral_rank(int i, int j) {
  const int l = max(abs(i), abs(j));
  if (l == 0) return 0;
  int k;
  if (j == -l && i < l) k = i + l;                  // top edge, walking right
  else if (i == l && j < l) k = 3 * l + j;          // right edge, walking down
  else if (j == l && i > -l) k = 5 * l - i;         // bottom edge, walking left
  else k = 7 * l - j;                               // left edge, walking up
  return (2 * l - 1) * (2 * l - 1) + k;
}

}  // namespace
}  // namespace jmme
