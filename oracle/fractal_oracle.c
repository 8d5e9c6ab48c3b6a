/*
 * fractal_oracle.c -- TEST INFRASTRUCTURE: restatement of the thesis fractal
 * block matching; see fractal_oracle.h (parity unpinned, known-answer tested).
 * Written from the behaviour of ZL/src/compute.c and ZL/src/block_enc.c; no
 * thesis code is copied.  Floating-point expressions keep the thesis's
 * operand order (compiled without FP contraction: -ffp-contract=off).
 */
#include "fractal_oracle.h"

#include <math.h>
#include <string.h>

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

/* ------------------------------------------------------------------ a17 --
 * encode_one_macroblock and the block encoders it calls, restated for
 * search_mode 0, num_regions 1 and the C view (currentVideo == 'C'), whose
 * every level runs full_search on its own reference and then on the H, M, N
 * views, keeping the first strict minimum (block_enc.c:563-700, 1131-1250,
 * 1396-1510, 1730-1845). */

typedef struct tree_ctx {
  const uint8_t *org;
  const uint8_t *const *refs;
  int n_refs, pitch, W, H, R;
  double tol_16, tol_8;
} tree_ctx;

/* full_search over every reference in view order; quirk4: encode_block_4
 * writes `trans->partition = trans->reference = 1` when the H view wins
 * (block_enc.c:1773), a partition that later views do not reset */
static double search_views(const tree_ctx *c, int bx, int by, int bsx, int bsy, fro_node *t, int quirk4)
{
  int k, x, y;
  double s, o, rl, rms;
  rms = fro_full_search(c->org, c->refs[0], c->pitch, c->W, c->H, c->R, bx, by, bsx, bsy, &x, &y, &s, &o);
  t->x = x;
  t->y = y;
  t->scale = s;
  t->offset = o;
  t->reference = 0;
  for (k = 1; k < c->n_refs; k++) {
    rl = fro_full_search(c->org, c->refs[k], c->pitch, c->W, c->H, c->R, bx, by, bsx, bsy, &x, &y, &s, &o);
    if (rl < rms) {
      rms = rl;
      t->x = x;
      t->y = y;
      t->scale = s;
      t->offset = o;
      t->reference = k;
      if (quirk4 && k == 1) t->partition = 1;
    }
  }
  t->rms = rms;
  return rms;
}

/* encode_block_rect, block_enc.c:1072-1336: half `half` of mode 1 (16x8 /
 * 8x4) or mode 2 (8x16 / 4x8) at depth 1 or 2; matched when rms is not above
 * tol_8^2 * no (no = the block's pel count, the global compute_rms sets) */
static int encode_rect(const tree_ctx *c, int bx, int by, int half, fro_node *t, int mode, int depth)
{
  int bsx, bsy;
  if (mode == 1) {
    bsx = 16 / depth;
    bsy = 8 / depth;
    by += bsy * half;
  } else {
    bsx = 8 / depth;
    bsy = 16 / depth;
    bx += bsx * half;
  }
  return !(search_views(c, bx, by, bsx, bsy, t, 0) > c->tol_8 * c->tol_8 * (bsx * bsy));
}

/* encode_block_4, block_enc.c:1676-1932 */
static void encode_b4(const tree_ctx *c, int bx, int by, fro_node *t)
{
  t->x = t->y = 0;
  search_views(c, bx, by, 4, 4, t, 1);
}

/* encode_block_8, block_enc.c:1337-1675: 8x8; if unmatched (rms >
 * tol_8^2 * 64) the 8x4 pair, then the 4x8 pair (a pair stops at its first
 * unmatched half), else four 4x4 */
static void encode_b8(const tree_ctx *c, int bx, int by, fro_node *t, fro_node *next)
{
  int mode, i, j, ok;
  t->partition = 0;
  t->reference = 0;
  t->x = 0;
  t->y = 0;
  if (search_views(c, bx, by, 8, 8, t, 0) > c->tol_8 * c->tol_8 * 64) {
    for (mode = 1; mode < 3; mode++) {
      ok = 0;
      t->partition = mode;
      for (i = 0; i < 2; i++) {
        next[i].x = 0;
        next[i].y = 0;
        if (!encode_rect(c, bx, by, i, &next[i], mode, 2)) break;
        ok++;
      }
      if (ok == 2) break;
    }
    if (mode == 3) {
      t->partition = 3;
      for (i = 0; i < 2; i++)
        for (j = 0; j < 2; j++) encode_b4(c, bx + j * 4, by + i * 4, &next[i * 2 + j]);
    }
  }
}

/* the 16x16 gate's chun: squared correlation of the range block with the
 * co-located block of the own reference, summed column by column
 * (block_enc.c:760-796) */
static double mb_chun(const tree_ctx *c, int bx, int by)
{
  double R[256], D[256], sumR = 0, sumD = 0, r, d, sR = 0, sD = 0, mr = 0;
  int i, j, ii = 0;
  for (j = bx; j < bx + 16; j++)
    for (i = by; i < by + 16; i++) {
      R[ii] = c->org[i * c->pitch + j];
      D[ii] = c->refs[0][i * c->pitch + j];
      sumR += R[ii];
      sumD += D[ii];
      ii++;
    }
  r = sumR / 256;
  d = sumD / 256;
  for (ii = 0; ii < 256; ii++) {
    sR += (R[ii] - r) * (R[ii] - r);
    sD += (D[ii] - d) * (D[ii] - d);
  }
  for (ii = 0; ii < 256; ii++) mr += ((R[ii] - r) / (sqrt(sR))) * ((D[ii] - d) / (sqrt(sD)));
  return mr * mr;
}

/* encode_one_macroblock, block_enc.c:508-1050 (region 0 branch, k == 0).
 * Split when 0.9 <= chun <= 1 and rms > tol_16^2 * 256.  Its 16x8 / 8x16
 * loop (block_enc.c:798-855) never leaves early (a matched pair does not set
 * mode = 4), so the 8x8 split always follows and overwrites the pair's
 * next[0..1] and stored vectors: the pair searches are dead stores and are
 * not restated. */
void fro_encode_mbs(const uint8_t *org, const uint8_t *const *refs, int n_refs, int pitch, int W, int H, int R,
                    double tol_16, double tol_8, fro_mb *out)
{
  tree_ctx c;
  int mbs_x = W / 16, n_mb = mbs_x * (H / 16), mb, i, j;
  c.org = org;
  c.refs = refs;
  c.n_refs = n_refs;
  c.pitch = pitch;
  c.W = W;
  c.H = H;
  c.R = R;
  c.tol_16 = tol_16;
  c.tol_8 = tol_8;
  for (mb = 0; mb < n_mb; mb++) {
    fro_mb *m = &out[mb];
    const int bx = (mb % mbs_x) * 16, by = (mb / mbs_x) * 16;
    double rms;
    memset(m, 0, sizeof(*m));
    rms = search_views(&c, bx, by, 16, 16, &m->mb, 0);
    m->chun = mb_chun(&c, bx, by);
    if (m->chun <= 1 && m->chun >= 0.9 && rms > tol_16 * tol_16 * 256) {
      m->mb.partition = 3;
      for (i = 0; i < 2; i++)
        for (j = 0; j < 2; j++) encode_b8(&c, bx + j * 8, by + i * 8, &m->b8[i * 2 + j], m->sub[i * 2 + j]);
    }
  }
}

/* ---- decoder: block_dec.c -------------------------------------------------
 * Leaf kinds and the view each one reads, per component and reference index
 * (num_regions == 1 branches):
 *   16x16  decode_one_macroblock  :126-209  reference 0..3 -> that view
 *   8x8    decode_block_8         :861-904  reference 0 -> 0, anything else -> 1
 *   8x4    decode_block_rect      :558-628  0, 1, 2 -> same; anything else -> 3
 *   4x8    decode_block_rect      :637-701  0, 1, 2 -> same; anything else -> 3
 *   4x4    decode_block_4         :1078-1146 0, 1, 2 -> same, else 3; for V
 *          the second test repeats `reference==0` (:1135), so 1 -> 3
 * The box sum is always taken from the same view as the pixels for these
 * kinds (the mismatched 16x8 U branch, :437-440, belongs to the 16x8 / 8x16
 * macroblock partitions the encoder never leaves behind). */
enum { FRO_L16, FRO_L8, FRO_L84, FRO_L48, FRO_L4 };

static int fro_leaf_view(int kind, int component, int ref) {
  switch (kind) {
    case FRO_L16: return (ref >= 0 && ref <= 3) ? ref : -1;
    case FRO_L8: return ref == 0 ? 0 : 1;
    case FRO_L84:
    case FRO_L48: return (ref == 0 || ref == 1 || ref == 2) ? ref : 3;
    default:
      if (component == 3) return ref == 0 ? 0 : ref == 2 ? 2 : 3;
      return (ref == 0 || ref == 1 || ref == 2) ? ref : 3;
  }
}

/* one leaf: block_dec.c:212-227 (16x16), :712-727 (rect), :912-928 (8x8),
 * :1150-1163 (4x4) -- avg = sum / (double)(bsx*bsy) with the box sum of the
 * domain block (compute_domain_Sum's exact integer as a double) */
static int fro_decode_leaf(const fro_node *t, int kind, int bx, int by, int bsx, int bsy,
                           const uint8_t *const *views, int n_views, int pitch, int W, int H, int component,
                           uint8_t *rec) {
  const int v = fro_leaf_view(kind, component, t->reference);
  if (v < 0 || v >= n_views) return -1;
  const int dx = bx + t->x, dy = by + t->y;
  if (dx < 0 || dy < 0 || dx + bsx > W || dy + bsy > H) return -1;
  const uint8_t *ref = views[v];
  long sum = 0;
  for (int j = 0; j < bsy; ++j)
    for (int i = 0; i < bsx; ++i) sum += ref[(size_t)(dy + j) * pitch + dx + i];
  const double scale = t->scale, offset = t->offset;
  const double average_domain = (double)sum / (double)(bsx * bsy);
  for (int j = 0; j < bsy; ++j)
    for (int i = 0; i < bsx; ++i) {
      const double a = 0.5 + scale * ref[(size_t)(dy + j) * pitch + dx + i] + offset - scale * average_domain;
      rec[(size_t)(by + j) * pitch + bx + i] = (unsigned char)(a < 0.0 ? 0 : (a > 255.0 ? 255 : a));   /* bound() */
    }
  return 0;
}

int fro_decode_mbs(const fro_mb *mbs, const uint8_t *const *views, int n_views, int pitch, int W, int H,
                   int component, uint8_t *rec) {
  const int mbs_x = W / 16, n_mb = mbs_x * (H / 16);
  for (int m = 0; m < n_mb; ++m) {
    const fro_mb *t = &mbs[m];
    const int bx = (m % mbs_x) * 16, by = (m / mbs_x) * 16;
    if (t->mb.partition == 0) {                                 /* :34 16x16 */
      if (fro_decode_leaf(&t->mb, FRO_L16, bx, by, 16, 16, views, n_views, pitch, W, H, component, rec)) return -1;
      continue;
    }
    for (int q = 0; q < 4; ++q) {                               /* :238-245 four 8x8 */
      const int x8 = bx + (q & 1) * 8, y8 = by + (q >> 1) * 8;
      const fro_node *b = &t->b8[q];
      int e = 0;
      if (b->partition == 0)                                    /* decode_block_8 :771 */
        e = fro_decode_leaf(b, FRO_L8, x8, y8, 8, 8, views, n_views, pitch, W, H, component, rec);
      else if (b->partition == 1)                               /* :932-937 rect pair, depth 2 */
        for (int h = 0; h < 2 && !e; ++h)
          e = fro_decode_leaf(&t->sub[q][h], FRO_L84, x8, y8 + 4 * h, 8, 4, views, n_views, pitch, W, H,
                              component, rec);
      else if (b->partition == 2)
        for (int h = 0; h < 2 && !e; ++h)
          e = fro_decode_leaf(&t->sub[q][h], FRO_L48, x8 + 4 * h, y8, 4, 8, views, n_views, pitch, W, H,
                              component, rec);
      else                                                      /* :940-945 four 4x4 */
        for (int c = 0; c < 4 && !e; ++c)
          e = fro_decode_leaf(&t->sub[q][c], FRO_L4, x8 + (c & 1) * 4, y8 + (c >> 1) * 4, 4, 4, views, n_views,
                              pitch, W, H, component, rec);
      if (e) return -1;
    }
  }
  return 0;
}
