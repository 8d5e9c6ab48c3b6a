/*
 * fractal_oracle.c -- TEST INFRASTRUCTURE: restatement of the thesis fractal
 * block matching; see fractal_oracle.h (parity unpinned, known-answer tested).
 * Written from the behaviour of ZL/src/compute.c and ZL/src/block_enc.c; no
 * thesis code is copied.  Floating-point expressions keep the thesis's
 * operand order (compiled without FP contraction: -ffp-contract=off).
 */
#include "fractal_oracle.h"

#define MIN_ALPHA (-2.35)   /* ZL/inc/defines_enc.h:19-22 */
#define MAX_ALPHA 4.0
#define MIN_BETA (-60)
#define MAX_BETA 255

/* QUAN_A, ZL/inc/defines_enc.h:591-601: units digit of (int)x -> 0 or 5,
 * 8 and 9 round up to the next ten, negative remainders -> 0 */
static int quan_a(int x)
{
  int b = x % 10, c = x / 10;
  if (b > 2 && b < 8) b = 5;
  else if (b > 7) { b = 0; c += 1; }
  else b = 0;
  return c * 10 + b;
}

void fro_box_sums(const uint8_t *p, int pitch, int W, int H, int bsx, int bsy, double *sum, double *sum2)
{
  const int w = W - bsx + 1, h = H - bsy + 1;
  int i, j, r, c;
  for (i = 0; i < h; i++)
    for (j = 0; j < w; j++) {
      double s = 0.0, s2 = 0.0;
      for (r = 0; r < bsy; r++)
        for (c = 0; c < bsx; c++) {
          const int v = p[(i + r) * pitch + j + c];
          s += v;
          s2 += v * v;
        }
      sum[i * w + j] = s;
      sum2[i * w + j] = s2;
    }
}

/* compute_rms, ZL/src/compute.c:6-189; the box sums are the same exact
 * integers the thesis reads from its sum_*_org / sum_*_ref_temp tables */
double fro_compute_rms(const uint8_t *org, const uint8_t *ref, int pitch, int bx, int by, int m, int n, int bsx,
                       int bsy, double *alpha, double *beta)
{
  double rms = 1e30, det, dsum1 = 0, dsum2 = 0, rsum1 = 0, rsum2 = 0, rdsum = 0;
  const int no = bsx * bsy;
  int a, i, j;
  for (i = 0; i < bsy; i++)
    for (j = 0; j < bsx; j++) {
      const int rv = org[(by + i) * pitch + bx + j], dv = ref[(n + i) * pitch + m + j];
      rsum1 += rv;
      rsum2 += rv * rv;
      dsum1 += dv;
      dsum2 += dv * dv;
      rdsum += rv * dv;       /* compute_rdSum, compute.c:192-215 */
    }
  det = no * dsum2 - dsum1 * dsum1;
  if (det == 0.0) *alpha = 0.0;
  else *alpha = (no * rdsum - rsum1 * dsum1) / det;
  a = (int)(*alpha * 100);
  *beta = rsum1 / no;
  a = quan_a(a);
  *beta = quan_a((int)*beta);
  *alpha = (double)a / 100;
  if (*alpha < MIN_ALPHA || *alpha > MAX_ALPHA) return rms;
  if (*beta < MIN_BETA || *beta > MAX_BETA) return rms;
  rms = rsum2 + (*alpha) * ((*alpha) * dsum2 - 2.0 * rdsum + 2.0 * ((*beta) - (*alpha) * dsum1 / no) * dsum1) +
        ((*beta) - (*alpha) * dsum1 / no) * (((*beta) - (*alpha) * dsum1 / no) * no - 2.0 * rsum1);
  return rms;
}

/* bound_chk, ZL/src/block_enc.c:2894-2919 */
static int bound_chk(int m, int n, int cx, int cy, int bsx, int bsy, int W, int H, int R)
{
  int ilow = cx - R, ihigh = cx + R, jlow = cy - R, jhigh = cy + R;
  if (ilow < 0) ilow = 0;
  if (ihigh > W - bsx) ihigh = W - bsx;
  if (jlow < 0) jlow = 0;
  if (jhigh > H - bsy) jhigh = H - bsy;
  return m <= ihigh && m >= ilow && n <= jhigh && n >= jlow;
}

/* full_search, ZL/src/block_enc.c:1933-1977 */
double fro_full_search(const uint8_t *org, const uint8_t *ref, int pitch, int W, int H, int R, int bx, int by,
                       int bsx, int bsy, int *out_x, int *out_y, double *scale, double *offset)
{
  double alpha, beta, rms, best;
  int l, k, i, j;
  best = fro_compute_rms(org, ref, pitch, bx, by, bx, by, bsx, bsy, &alpha, &beta);
  *scale = alpha;
  *offset = beta;
  *out_x = 0;
  *out_y = 0;
  for (l = 1; l <= R; l++) {
    i = j = -l;
    for (k = 0; k < 8 * l; k++) {
      const int m = bx + i, n = by + j;
      if (bound_chk(m, n, bx, by, bsx, bsy, W, H, R)) {
        rms = fro_compute_rms(org, ref, pitch, bx, by, m, n, bsx, bsy, &alpha, &beta);
        if (rms < best) {
          best = rms;
          *out_x = m - bx;
          *out_y = n - by;
          *scale = alpha;
          *offset = beta;
        }
      }
      if (k < 2 * l) i++;
      else if (k < 4 * l) j++;
      else if (k < 6 * l) i--;
      else j--;
    }
  }
  return best;
}

void fro_full_search_batch(const uint8_t *org, const uint8_t *ref, int pitch, int W, int H, int R, int n,
                           const int32_t *req, double *out, int32_t *xy)
{
  int t;
  for (t = 0; t < n; t++) {
    int x, y;
    double s, o;
    out[3 * t] = fro_full_search(org, ref, pitch, W, H, R, req[4 * t], req[4 * t + 1], req[4 * t + 2],
                                 req[4 * t + 3], &x, &y, &s, &o);
    out[3 * t + 1] = s;
    out[3 * t + 2] = o;
    xy[2 * t] = x;
    xy[2 * t + 1] = y;
  }
}
