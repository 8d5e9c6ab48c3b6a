/*
 * tq_oracle.c -- TEST INFRASTRUCTURE: plain-C restatement of JM 18.5's
 * block transforms, 4x4 quantisation and Hadamard SATD (SURVEY.md §8 rows
 * a12, a13).  The CHECKER for the HIP kernels of csrc/jmme_tq.hip; only
 * tests/ (and smoke/bench CPU legs) load it.  Pinned against the real JM
 * functions by tests/golden/tq_jm.npz (oracle/capture/jm_tq_harness.c).
 *
 * Blocks are passed as flat row-major arrays: b[r*N + c] is JM's
 * block[pos_y + r][pos_x + c].  Written from the behaviour of the JM sources
 * (JM = /root/reference/4.对比程序/jm18.5/JM); no JM code is copied.
 */
#include "tq_oracle.h"
#include <stdlib.h>

/* ---- 1-D butterflies --------------------------------------------------- */

/* H.264 forward core transform of 4 samples, lcommon/src/transform.c:32-44 */
static void fwd4(const int *x, int s, int *y, int t)
{
  const int a = x[0] + x[3 * s], b = x[s] + x[2 * s];
  const int c = x[s] - x[2 * s], d = x[0] - x[3 * s];
  y[0] = a + b;
  y[t] = 2 * d + c;
  y[2 * t] = a - b;
  y[3 * t] = d - 2 * c;
}

/* inverse core transform, transform.c:82-94 */
static void inv4(const int *x, int s, int *y, int t)
{
  const int e = x[0] + x[2 * s], f = x[0] - x[2 * s];
  const int g = (x[s] >> 1) - x[3 * s], h = x[s] + (x[3 * s] >> 1);
  y[0] = e + h;
  y[t] = f + g;
  y[2 * t] = f - g;
  y[3 * t] = e - h;
}

/* 4-point Hadamard as JM orders it, transform.c:133-145 */
static void had4(const int *x, int s, int *y, int t)
{
  const int a = x[0] + x[3 * s], b = x[s] + x[2 * s];
  const int c = x[s] - x[2 * s], d = x[0] - x[3 * s];
  y[0] = a + b;
  y[t] = d + c;
  y[2 * t] = a - b;
  y[3 * t] = d - c;
}

/* inverse 4-point Hadamard, transform.c:183-195 */
static void ihad4(const int *x, int s, int *y, int t)
{
  const int e = x[0] + x[2 * s], f = x[0] - x[2 * s];
  const int g = x[s] - x[3 * s], h = x[s] + x[3 * s];
  y[0] = e + h;
  y[t] = f + g;
  y[2 * t] = f - g;
  y[3 * t] = e - h;
}

/* 8-point forward (H.264 high-profile integer DCT), transform.c:365-402 */
static void fwd8(const int *x, int s, int *y, int t)
{
  const int s07 = x[0] + x[7 * s], s16 = x[s] + x[6 * s], s25 = x[2 * s] + x[5 * s], s34 = x[3 * s] + x[4 * s];
  const int d07 = x[0] - x[7 * s], d16 = x[s] - x[6 * s], d25 = x[2 * s] - x[5 * s], d34 = x[3 * s] - x[4 * s];
  const int e0 = s07 + s34, e1 = s16 + s25, e2 = s07 - s34, e3 = s16 - s25;
  const int o4 = d16 + d25 + ((d07 >> 1) + d07);
  const int o5 = d07 - d34 - ((d25 >> 1) + d25);
  const int o6 = d07 + d34 - ((d16 >> 1) + d16);
  const int o7 = d16 - d25 + ((d34 >> 1) + d34);
  y[0] = e0 + e1;
  y[t] = o4 + (o7 >> 2);
  y[2 * t] = e2 + (e3 >> 1);
  y[3 * t] = o5 + (o6 >> 2);
  y[4 * t] = e0 - e1;
  y[5 * t] = o6 - (o5 >> 2);
  y[6 * t] = (e2 >> 1) - e3;
  y[7 * t] = (o4 >> 2) - o7;
}

/* 8-point inverse, transform.c:474-506 */
static void inv8(const int *x, int s, int *y, int t)
{
  const int p0 = x[0], p1 = x[s], p2 = x[2 * s], p3 = x[3 * s];
  const int p4 = x[4 * s], p5 = x[5 * s], p6 = x[6 * s], p7 = x[7 * s];
  const int a0 = p0 + p4, a1 = p0 - p4, a2 = p6 - (p2 >> 1), a3 = p2 + (p6 >> 1);
  const int b0 = a0 + a3, b2 = a1 - a2, b4 = a1 + a2, b6 = a0 - a3;
  const int c0 = -p3 + p5 - p7 - (p7 >> 1);
  const int c1 = p1 + p7 - p3 - (p3 >> 1);
  const int c2 = -p1 + p7 + p5 + (p5 >> 1);
  const int c3 = p3 + p5 + p1 + (p1 >> 1);
  const int b1 = c0 + (c3 >> 2), b3 = c1 + (c2 >> 2), b5 = c2 - (c1 >> 2), b7 = c3 - (c0 >> 2);
  y[0] = b0 + b7;
  y[t] = b2 - b5;
  y[2 * t] = b4 + b3;
  y[3 * t] = b6 + b1;
  y[4 * t] = b6 - b1;
  y[5 * t] = b4 - b3;
  y[6 * t] = b2 + b5;
  y[7 * t] = b0 - b7;
}

typedef void (*line_fn)(const int *, int, int *, int);

/* separable 2-D transform: rows first into tmp, then columns (the order JM
 * uses -- it matters for the >> steps) */
static void sep2d(const int *in, int *out, int n, line_fn rows, line_fn cols)
{
  int tmp[64];
  int r, c;
  for (r = 0; r < n; r++) rows(in + r * n, 1, tmp + r * n, 1);
  for (c = 0; c < n; c++) cols(tmp + c, n, out + c, n);
}

void tqo_forward4x4(const int *in, int *out) { sep2d(in, out, 4, fwd4, fwd4); }   /* transform.c:20-68 */
void tqo_inverse4x4(const int *in, int *out) { sep2d(in, out, 4, inv4, inv4); }   /* transform.c:70-119 */
void tqo_forward8x8(const int *in, int *out) { sep2d(in, out, 8, fwd8, fwd8); }   /* transform.c:353-448 */
void tqo_inverse8x8(const int *in, int *out) { sep2d(in, out, 8, inv8, inv8); }   /* transform.c:450-528 */
void tqo_ihadamard4x4(const int *in, int *out) { sep2d(in, out, 4, ihad4, ihad4); } /* transform.c:171-218 */

/* hadamard4x4, transform.c:121-169: the vertical pass halves (>> 1) */
void tqo_hadamard4x4(const int *in, int *out)
{
  int tmp[16];
  int r, c;
  for (r = 0; r < 4; r++) had4(in + r * 4, 1, tmp + r * 4, 1);
  for (c = 0; c < 4; c++) {
    int y[4], k;
    had4(tmp + c, 4, y, 1);
    for (k = 0; k < 4; k++) out[k * 4 + c] = y[k] >> 1;
  }
}

/* hadamard4x2, transform.c:220-258: 2 rows x 4 columns (chroma DC, 4:2:2),
 * a 2-point butterfly down the columns, then the 4-point Hadamard per row */
void tqo_hadamard4x2(const int *in, int *out)
{
  int tmp[8], c;
  for (c = 0; c < 4; c++) {
    tmp[c] = in[c] + in[4 + c];
    tmp[4 + c] = in[c] - in[4 + c];
  }
  had4(tmp, 1, out, 1);
  had4(tmp + 4, 1, out + 4, 1);
}

/* ihadamard4x2, transform.c:260-300: output is 4 rows x 2 columns
 * (out[r*2 + i]), "coefficients (transposed)" */
void tqo_ihadamard4x2(const int *in, int *out)
{
  int tmp[8], c, i;
  for (c = 0; c < 4; c++) {
    tmp[c] = in[c] + in[4 + c];
    tmp[4 + c] = in[c] - in[4 + c];
  }
  for (i = 0; i < 2; i++) {
    int y[4], k;
    ihad4(tmp + 4 * i, 1, y, 1);
    for (k = 0; k < 4; k++) out[k * 2 + i] = y[k];
  }
}

/* hadamard2x2 / ihadamard2x2, transform.c:302-331 (the active versions):
 * in = {b00, b01, b10, b11} (JM reads block[0][0],[0][4],[4][0],[4][4]) */
void tqo_hadamard2x2(const int *in, int *out)
{
  const int p0 = in[0] + in[1], p1 = in[0] - in[1], p2 = in[2] + in[3], p3 = in[2] - in[3];
  out[0] = p0 + p2;
  out[1] = p1 + p3;
  out[2] = p0 - p2;
  out[3] = p1 - p3;
}
void tqo_ihadamard2x2(const int *in, int *out) { tqo_hadamard2x2(in, out); }

/* ---- SATD, lencod/src/me_distortion.c ----------------------------------- */

/* Every output of JM's HadamardSAD4x4 / 8x8 is a +-1 combination of the
 * inputs with a distinct sign pattern (a full Walsh-Hadamard transform), so
 * the sum of magnitudes does not depend on the output order JM uses. */
static int wht_abs_sum(const int *d, int n)
{
  int v[64], len, i, j, sum = 0;
  for (i = 0; i < n * n; i++) v[i] = d[i];
  for (i = 0; i < n; i++)                       /* rows */
    for (len = 1; len < n; len <<= 1)
      for (j = 0; j < n; j++)
        if (!(j & len)) {
          int a = v[i * n + j], b = v[i * n + j + len];
          v[i * n + j] = a + b;
          v[i * n + j + len] = a - b;
        }
  for (i = 0; i < n; i++)                       /* columns */
    for (len = 1; len < n; len <<= 1)
      for (j = 0; j < n; j++)
        if (!(j & len)) {
          int a = v[j * n + i], b = v[(j + len) * n + i];
          v[j * n + i] = a + b;
          v[(j + len) * n + i] = a - b;
        }
  for (i = 0; i < n * n; i++) sum += abs(v[i]);
  return sum;
}

/* HadamardSAD4x4, me_distortion.c:175-258 */
int tqo_hadamard_sad4x4(const int16_t *diff)
{
  int d[16], i;
  for (i = 0; i < 16; i++) d[i] = diff[i];
  return (wht_abs_sum(d, 4) + 1) >> 1;
}

/* HadamardSAD8x8, me_distortion.c:266-341 */
int tqo_hadamard_sad8x8(const int16_t *diff)
{
  int d[64], i;
  for (i = 0; i < 64; i++) d[i] = diff[i];
  return (wht_abs_sum(d, 8) + 2) >> 2;
}

/* ---- quantisation, lencod/src/quant4x4_normal.c:39-110 ------------------ */

int tqo_quant_4x4_normal(int *coef, const tqo_quant4x4_params *q, int32_t *levels, int32_t *runs,
                         int32_t *coeff_cost)
{
  const int q_bits = 15 + q->qp_per;           /* Q_BITS = 15, defines.h:311 */
  int k, run = 0, nz = 0, nout = 0;
  for (k = 0; k < 16; k++) {
    const int i = q->scan[k][0], j = q->scan[k][1];   /* (horizontal, vertical) */
    int *c = &coef[j * 4 + i];
    const int pq = j * 4 + i;
    if (*c == 0) { run++; continue; }
    {
      const int mag = abs(*c) * q->scale[pq];
      int level = (mag + q->offset[pq]) >> q_bits;
      if (level == 0) { *c = 0; run++; continue; }
      if (q->is_cavlc && level > 2063) level = 2063;   /* CAVLC_LEVEL_LIMIT, defines.h:99 */
      *coeff_cost += level > 1 ? 999999 : q->c_cost[run];   /* MAX_VALUE, defines.h:123 */
      if (*c < 0) level = -level;
      /* rshift_rnd_sf(x, 4) = (x + 8) >> 4, lcommon/inc/ifunctions.h:176 */
      *c = ((level * q->inv_scale[pq] << q->qp_per) + 8) >> 4;
      levels[nout] = level;
      runs[nout] = run;
      nout++;
      run = 0;
      nz = 1;
    }
  }
  levels[nout] = 0;   /* *ACL = 0 terminator */
  return nz;
}
