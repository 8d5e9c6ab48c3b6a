/*
 * subpel_oracle.c -- TEST INFRASTRUCTURE (the checker, never the product).
 * Plain-C restatement of JM 18.5's quarter-pel interpolation and sub-pel
 * motion refinement; see subpel_oracle.h.  JM = /root/reference/4.对比程序/jm18.5/JM.
 */
#include <stdlib.h>
#include <string.h>
#include "subpel_oracle.h"

#define DISTBLK_MAX (((int64_t)0x7fffffff) << 5)   /* JM/lencod/inc/defines.h:135 */

/* p_Vid->max_imgpel_value = (1 << bitdepth_luma) - 1 (image.c init_img); 255 unless set */
static int g_max_pel = 255;
void spo_set_bitdepth(int bits) { g_max_pel = (1 << bits) - 1; }
static inline int clip255(int v) { return v < 0 ? 0 : (v > g_max_pel ? g_max_pel : v); }   /* iClip1(max_imgpel_value) */
static inline int rnd_sf(int x, int a) { return (x + (1 << (a - 1))) >> a; }    /* rshift_rnd_sf, ifunctions.h */
static inline int imin_(int a, int b) { return a < b ? a : b; }
static inline int imax_(int a, int b) { return a > b ? a : b; }
static inline int iabs_(int a) { return a < 0 ? -a : a; }

/* ---------------------------------------------------------------------------
 * getSubImagesLuma (img_luma.c:611-680).  All arrays here are indexed in
 * padded coordinates: row r = j + PAD_Y in [0, ph), column c = i + PAD_X in
 * [0, pw).  Each helper follows the JM function named in its comment,
 * including its first/last row and column special cases. */
#define SP(p, r, c) (p)[(size_t)(r) * pw + (c)]

/* getSubImageInteger (img_luma.c:40-86): copy + edge replication */
static void sub_integer(const uint16_t *src, int W, int H, uint16_t *dst, int pw, int ph)
{
  for (int r = 0; r < ph; r++) {
    int j = imin_(imax_(r - SPO_PAD_Y, 0), H - 1);
    for (int c = 0; c < pw; c++) {
      int i = imin_(imax_(c - SPO_PAD_X, 0), W - 1);
      SP(dst, r, c) = src[(size_t)j * W + i];
    }
  }
}

/* getHorSubImageSixTap (img_luma.c:151-241): taps clamped to the padded row;
 * also fills the unrounded int image (p_Vid->imgY_sub_tmp) */
static void hor_six_tap(const uint16_t *s, uint16_t *dst, int *tmp, int pw, int ph)
{
  for (int r = 0; r < ph; r++)
    for (int c = 0; c < pw; c++) {
      int a = SP(s, r, c), d = SP(s, r, imin_(c + 1, pw - 1));
      int b = SP(s, r, imax_(c - 1, 0)), e = SP(s, r, imin_(c + 2, pw - 1));
      int cc = SP(s, r, imax_(c - 2, 0)), f = SP(s, r, imin_(c + 3, pw - 1));
      int is = 20 * (a + d) - 5 * (b + e) + (cc + f);     /* ONE_FOURTH_TAP[0], img_luma.h:21 */
      SP(tmp, r, c) = is;
      SP(dst, r, c) = (uint16_t)clip255(rnd_sf(is, 5));
    }
}

/* getVerSubImageSixTap (img_luma.c:256-335) and getVerSubImageSixTapTmp
 * (:350-431, over the int image, rounding by 10): rows clamped to [0, ph-1] */
static void ver_six_tap(const uint16_t *s, const int *si, uint16_t *dst, int pw, int ph)
{
  for (int r = 0; r < ph; r++) {
    int ra = r, rd = imin_(r + 1, ph - 1), rb = imax_(r - 1, 0), re = imin_(r + 2, ph - 1);
    int rc = imax_(r - 2, 0), rf = imin_(r + 3, ph - 1);
    for (int c = 0; c < pw; c++) {
      if (si) {
        int is = 20 * (SP(si, ra, c) + SP(si, rd, c)) - 5 * (SP(si, rb, c) + SP(si, re, c)) +
                 (SP(si, rc, c) + SP(si, rf, c));
        SP(dst, r, c) = (uint16_t)clip255(rnd_sf(is, 10));
      } else {
        int is = 20 * (SP(s, ra, c) + SP(s, rd, c)) - 5 * (SP(s, rb, c) + SP(s, re, c)) +
                 (SP(s, rc, c) + SP(s, rf, c));
        SP(dst, r, c) = (uint16_t)clip255(rnd_sf(is, 5));
      }
    }
  }
}

/* getSubImageBiLinear (img_luma.c:448-466): same position */
static void bilin(uint16_t *dst, const uint16_t *a, const uint16_t *b, int pw, int ph)
{
  for (size_t k = 0; k < (size_t)pw * ph; k++) dst[k] = (uint16_t)rnd_sf(a[k] + b[k], 1);
}

/* getHorSubImageBiLinear (img_luma.c:484-505): R one column right, last column clamped */
static void bilin_h(uint16_t *dst, const uint16_t *l, const uint16_t *rr, int pw, int ph)
{
  for (int r = 0; r < ph; r++)
    for (int c = 0; c < pw; c++)
      SP(dst, r, c) = (uint16_t)rnd_sf(SP(l, r, c) + SP(rr, r, imin_(c + 1, pw - 1)), 1);
}

/* getVerSubImageBiLinear (img_luma.c:523-552): B one row down, last row clamped */
static void bilin_v(uint16_t *dst, const uint16_t *t, const uint16_t *b, int pw, int ph)
{
  for (int r = 0; r < ph; r++)
    for (int c = 0; c < pw; c++)
      SP(dst, r, c) = (uint16_t)rnd_sf(SP(t, r, c) + SP(b, imin_(r + 1, ph - 1), c), 1);
}

/* getDiagSubImageBiLinear (img_luma.c:570-600): T one row down, B one column right */
static void bilin_d(uint16_t *dst, const uint16_t *t, const uint16_t *b, int pw, int ph)
{
  for (int r = 0; r < ph; r++)
    for (int c = 0; c < pw; c++)
      SP(dst, r, c) = (uint16_t)rnd_sf(SP(t, imin_(r + 1, ph - 1), c) + SP(b, r, imin_(c + 1, pw - 1)), 1);
}

void spo_sub_images(const uint16_t *src, int W, int H, uint16_t *out)
{
  int pw = W + 2 * SPO_PAD_X, ph = H + 2 * SPO_PAD_Y;
  size_t n = (size_t)pw * ph;
  uint16_t *S[4][4];
  int *tmp = (int *)malloc(n * sizeof(int));
  for (int dy = 0; dy < 4; dy++)
    for (int dx = 0; dx < 4; dx++) S[dy][dx] = out + (size_t)(dy * 4 + dx) * n;
  /* the call order of getSubImagesLuma, img_luma.c:621-679 */
  sub_integer(src, W, H, S[0][0], pw, ph);
  hor_six_tap(S[0][0], S[0][2], tmp, pw, ph);
  ver_six_tap(S[0][0], NULL, S[2][0], pw, ph);
  ver_six_tap(NULL, tmp, S[2][2], pw, ph);
  bilin(S[0][1], S[0][0], S[0][2], pw, ph);
  bilin(S[1][0], S[0][0], S[2][0], pw, ph);
  bilin(S[1][1], S[0][2], S[2][0], pw, ph);
  bilin(S[1][2], S[0][2], S[2][2], pw, ph);
  bilin(S[2][1], S[2][0], S[2][2], pw, ph);
  bilin_h(S[0][3], S[0][2], S[0][0], pw, ph);
  bilin_h(S[1][3], S[0][2], S[2][0], pw, ph);
  bilin_h(S[2][3], S[2][2], S[2][0], pw, ph);
  bilin_v(S[3][0], S[2][0], S[0][0], pw, ph);
  bilin_v(S[3][1], S[2][0], S[0][2], pw, ph);
  bilin_v(S[3][2], S[2][2], S[0][2], pw, ph);
  bilin_d(S[3][3], S[0][2], S[2][0], pw, ph);
  free(tmp);
}
#undef SP

/* ---------------------------------------------------------------------------
 * Distortion of one candidate, restating computeSAD / computeSSE / computeSATD
 * with their early exits (they return the threshold, dist_scale_f =
 * min_mcost, mv_search.h:19-20). */
typedef struct view {
  const uint16_t *cur, *sub;
  int W, H, pw, ph;
} view;

/* UMVLine4X (JM/lencod/inc/refbuf.h:22-26): origin clamp, then the row runs on */
static inline const uint16_t *umv_line(const view *v, int y, int x)
{
  int size_y_pad = v->H + 2 * SPO_PAD_Y - 1 - 16 - SPO_PAD_Y;   /* mbuffer.c:550 */
  int size_x_pad = v->W + 2 * SPO_PAD_X - 1 - 16 - SPO_PAD_X;   /* mbuffer.c:549 */
  int yy = imin_(imax_(y >> 2, -SPO_PAD_Y), size_y_pad);
  int xx = imin_(imax_(x >> 2, -SPO_PAD_X), size_x_pad);
  const uint16_t *plane = v->sub + (size_t)((y & 3) * 4 + (x & 3)) * v->pw * v->ph;
  return plane + (size_t)(yy + SPO_PAD_Y) * v->pw + (xx + SPO_PAD_X);
}

static int had4(const int16_t *d);   /* HadamardSAD4x4 */
static int had8(const int16_t *d);   /* HadamardSAD8x8 */

/* cand = absolute (padded) qpel position, as pad_MVs makes it (mv_search.h:66-72) */
static int64_t distortion(const view *v, const spo_req *r, int metric, int64_t min_mcost, int cx, int cy)
{
  int imin_cost = (int)(min_mcost >> 5);    /* dist_down */
  int mcost = 0;
  const uint16_t *org = v->cur;             /* orig block: cur[(pos_y+y)*W + pos_x+x] */
  if (metric == 0 || metric == 1) {
    /* computeSAD me_distortion.c:349-426 / computeSSE :1189-1240 */
    const uint16_t *ref = umv_line(v, cy, cx);
    for (int y = 0; y < r->bsy; y++) {
      for (int x = 0; x < r->bsx; x++) {
        int d = org[(size_t)(r->pos_y + y) * v->W + r->pos_x + x] - ref[(size_t)y * v->pw + x];
        mcost += metric == 0 ? iabs_(d) : d * d;
      }
      if (mcost > imin_cost) return min_mcost;
    }
    return (int64_t)mcost << 5;
  }
  /* computeSATD me_distortion.c:745-825 */
  int bs = r->test8x8 ? 8 : 4;
  int16_t diff[64];
  for (int by = 0; by < r->bsy; by += bs)
    for (int bx = 0; bx < r->bsx; bx += bs) {
      const uint16_t *ref = umv_line(v, cy + (by << 2), cx + (bx << 2));
      for (int y = 0; y < bs; y++)
        for (int x = 0; x < bs; x++)
          diff[y * bs + x] = (int16_t)(org[(size_t)(r->pos_y + by + y) * v->W + r->pos_x + bx + x] -
                                       ref[(size_t)y * v->pw + x]);
      mcost += bs == 4 ? had4(diff) : had8(diff);
      if (mcost > imin_cost) return min_mcost;
    }
  return (int64_t)mcost << 5;
}

/* mvbits closed form (mv_search.c:366-374) and mv_cost (mv_search.h:100-104) */
static inline int64_t mvbits(int v)
{
  unsigned a = (unsigned)iabs_(v);
  int lg = -1;
  while (a) { lg++; a >>= 1; }
  return (int64_t)(2 * lg + 3);
}
static inline int64_t mv_cost(int lambda, int cx, int cy, int px, int py)
{
  return (int64_t)lambda * (mvbits(cx - px) + mvbits(cy - py));
}

/* spiral_search / spiral_hpel_search (mv_search.c:406-442): first 9 entries
 * are (0,0),(0,-1),(0,1),(-1,-1),(1,-1),(-1,0),(1,0),(-1,1),(1,1) */
static const int SPIRAL9[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {1, 1}};

int64_t spo_sub_pel_me(const uint16_t *cur, const uint16_t *sub, int W, int H, const spo_req *r, int16_t *out_mv)
{
  view v = {cur, sub, W, H, W + 2 * SPO_PAD_X, H + 2 * SPO_PAD_Y};
  int mvx = r->mv_x, mvy = r->mv_y;
  int64_t min_mcost = r->min_mcost;
  int px = r->pred_x, py = r->pred_y;
  int pos_xp = r->pos_x << 2, pos_yp = r->pos_y << 2;     /* pos_x_padded, mv_search.c:685-686 */
  /* me_fullsearch.c:205 */
  int check_position0 = (!r->rdopt && r->slice_type != 1 && r->ref == 0 && r->blocktype == 1 && mvx == 0 && mvy == 0);
  int max_pos2 = !r->start_hp ? imax_(1, r->search_pos2) : r->search_pos2;   /* :209 */
  int best_pos, pos;
  int lambda = r->lambda_h;
  /* half-pel, :221-250; spiral_hpel_search = spiral_search * 2 */
  for (best_pos = 0, pos = r->start_hp; pos < max_pos2; pos++) {
    int cx = mvx + 2 * SPIRAL9[pos][0], cy = mvy + 2 * SPIRAL9[pos][1];
    int64_t mcost = mv_cost(lambda, cx, cy, px, py);
    if (mcost >= min_mcost) continue;
    mcost += distortion(&v, r, r->metric_h, min_mcost - mcost, cx + pos_xp, cy + pos_yp);
    if (pos == 0 && check_position0) mcost -= (int64_t)lambda * 16;   /* weighted_cost(lambda,16) */
    if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
  }
  if (best_pos) { mvx += 2 * SPIRAL9[best_pos][0]; mvy += 2 * SPIRAL9[best_pos][1]; }
  if (!r->start_qp) min_mcost = DISTBLK_MAX;                          /* :252-253 */
  lambda = r->lambda_q;
  /* quarter-pel, :263-282 */
  for (best_pos = 0, pos = r->start_qp; pos < r->search_pos4; pos++) {
    int cx = mvx + SPIRAL9[pos][0], cy = mvy + SPIRAL9[pos][1];
    int64_t mcost = mv_cost(lambda, cx, cy, px, py);
    if (mcost >= min_mcost) continue;
    mcost += distortion(&v, r, r->metric_q, min_mcost - mcost, cx + pos_xp, cy + pos_yp);
    if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
  }
  if (best_pos) { mvx += SPIRAL9[best_pos][0]; mvy += SPIRAL9[best_pos][1]; }
  out_mv[0] = (int16_t)mvx;
  out_mv[1] = (int16_t)mvy;
  return min_mcost;
}

/* me_epzs.h:23-42 */
static const int NEXT_START[25] = {0, 8, 5, 6, 7, 8, 0, 5, 8, 8, 5, 5, 0, 6, 5, 6, 6, 6, 0, 7, 7, 8, 7, 7, 0};
static const int NEXT_END[25] = {0, 10, 7, 8, 9, 10, 0, 6, 10, 9, 7, 6, 0, 7, 7, 8, 8, 7, 0, 8, 9, 9, 9, 8, 0};
static const int SP_PT[10][2] = {{0, 0}, {-1, 0}, {0, 1}, {1, 0}, {0, -1}, {-1, 1}, {1, 1}, {1, -1}, {-1, -1}, {-1, 1}};

int64_t spo_epzs_sub_pel_me(const uint16_t *cur, const uint16_t *sub, int W, int H, const spo_req *r,
                            int16_t *out_mv)
{
  view v = {cur, sub, W, H, W + 2 * SPO_PAD_X, H + 2 * SPO_PAD_Y};
  int mvx = r->mv_x, mvy = r->mv_y;
  int64_t min_mcost = r->min_mcost, second_mcost = DISTBLK_MAX, mcost;
  int best_pos = 0, second_pos = 0, pos;
  /* me_epzs_sub.c:43 */
  int max_pos2 = (!r->start_hp || !r->start_qp) ? imax_(1, r->search_pos2) : r->search_pos2;
  int pxp = r->pos_x << 2, pyp = r->pos_y << 2;
  int padx = mvx + pxp, pady = mvy + pyp;                  /* padded_mv */
  int ppx = r->pred_x + pxp, ppy = r->pred_y + pyp;        /* pred_mv (padded) */
  int start_pos = 5, end_pos = max_pos2;
  int lambda = r->lambda_h;
  int64_t sub_threshold = r->subthres + (int64_t)lambda * 2;   /* :56-57 */

  /* half-pel, :66-88 */
  for (best_pos = 0, pos = r->start_hp; pos < imin_(5, max_pos2); ++pos) {
    int cx = padx + 2 * SP_PT[pos][0], cy = pady + 2 * SP_PT[pos][1];
    mcost = mv_cost(lambda, cx, cy, ppx, ppy);
    if (mcost < second_mcost) {
      mcost += distortion(&v, r, r->metric_h, second_mcost - mcost, cx, cy);
      if (mcost < min_mcost) {
        second_mcost = min_mcost; second_pos = best_pos; min_mcost = mcost; best_pos = pos;
      } else if (mcost < second_mcost) {
        second_mcost = mcost; second_pos = pos;
      }
    }
  }
  /* :90-93 */
  if (best_pos == 0 && r->pred_x == mvx && r->pred_y == mvy && min_mcost < sub_threshold) {
    out_mv[0] = (int16_t)mvx; out_mv[1] = (int16_t)mvy;
    return min_mcost;
  }
  /* :96-121 */
  if (r->search_pos2 >= 9) {
    if (best_pos != 0 || (iabs_(r->pred_x - mvx) + iabs_(r->pred_y - mvy))) {
      start_pos = NEXT_START[best_pos * 5 + second_pos];
      end_pos = NEXT_END[best_pos * 5 + second_pos];
      for (pos = start_pos; pos < end_pos; ++pos) {
        int cx = padx + 2 * SP_PT[pos][0], cy = pady + 2 * SP_PT[pos][1];
        mcost = mv_cost(lambda, cx, cy, ppx, ppy);
        if (mcost < min_mcost) {
          mcost += distortion(&v, r, r->metric_h, min_mcost - mcost, cx, cy);
          if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
        }
      }
    }
  }
  /* :123-127 */
  if (best_pos) {
    mvx += 2 * SP_PT[best_pos][0]; mvy += 2 * SP_PT[best_pos][1];
    padx = mvx + pxp; pady = mvy + pyp;
  }
  /* quarter-pel, :135-172 */
  end_pos = (min_mcost < sub_threshold) ? 1 : 5;
  second_mcost = DISTBLK_MAX;
  if (!r->start_qp) { best_pos = -1; min_mcost = DISTBLK_MAX; } else best_pos = 0;
  lambda = r->lambda_q;
  for (pos = r->start_qp; pos < end_pos; ++pos) {
    int cx = padx + SP_PT[pos][0], cy = pady + SP_PT[pos][1];
    mcost = mv_cost(lambda, cx, cy, ppx, ppy);
    if (mcost < second_mcost) {
      mcost += distortion(&v, r, r->metric_q, second_mcost - mcost, cx, cy);
      if (mcost < min_mcost) {
        second_mcost = min_mcost; second_pos = best_pos; min_mcost = mcost; best_pos = pos;
      } else if (mcost < second_mcost) {
        second_mcost = mcost; second_pos = pos;
      }
    }
  }
  /* :175-204 */
  if (min_mcost > sub_threshold) {
    if (best_pos != 0 || (iabs_(r->pred_x - mvx) + iabs_(r->pred_y - mvy))) {
      /* With start_qp == 0 the first improvement moves best_pos = -1 into
       * second_pos, and JM then reads next_start_pos[best][-1]: for best >= 1
       * that is row-major [best-1][4]; for best == 0 it is the word before
       * each table, which in the JM build (gcc, me_epzs_sub.o .rodata: both
       * tables 32-byte aligned after zero padding) reads 0 -> an empty loop. */
      int k = best_pos * 5 + second_pos;
      start_pos = k >= 0 ? NEXT_START[k] : 0;
      end_pos = k >= 0 ? NEXT_END[k] : 0;
      for (pos = start_pos; pos < end_pos; ++pos) {
        int cx = padx + SP_PT[pos][0], cy = pady + SP_PT[pos][1];
        mcost = mv_cost(lambda, cx, cy, ppx, ppy);
        if (mcost < min_mcost) {
          mcost += distortion(&v, r, r->metric_q, min_mcost - mcost, cx, cy);
          if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
        }
      }
    }
  }
  if (best_pos > 0) { mvx += SP_PT[best_pos][0]; mvy += SP_PT[best_pos][1]; }
  out_mv[0] = (int16_t)mvx;
  out_mv[1] = (int16_t)mvy;
  return min_mcost;
}

void spo_sub_pel_batch(const uint16_t *cur, const uint16_t *sub, int W, int H, const spo_req *r, int n,
                       int epzs, int16_t *out_mv, int64_t *out_cost)
{
  for (int k = 0; k < n; k++)
    out_cost[k] = epzs ? spo_epzs_sub_pel_me(cur, sub, W, H, &r[k], out_mv + 2 * k)
                       : spo_sub_pel_me(cur, sub, W, H, &r[k], out_mv + 2 * k);
}

/* HadamardSAD4x4, me_distortion.c:175-258 (JM's butterfly order) */
static int had4(const int16_t *diff)
{
  int m[16], d[16], satd = 0;
  m[0] = diff[0] + diff[12]; m[1] = diff[1] + diff[13]; m[2] = diff[2] + diff[14]; m[3] = diff[3] + diff[15];
  m[4] = diff[4] + diff[8]; m[5] = diff[5] + diff[9]; m[6] = diff[6] + diff[10]; m[7] = diff[7] + diff[11];
  m[8] = diff[4] - diff[8]; m[9] = diff[5] - diff[9]; m[10] = diff[6] - diff[10]; m[11] = diff[7] - diff[11];
  m[12] = diff[0] - diff[12]; m[13] = diff[1] - diff[13]; m[14] = diff[2] - diff[14]; m[15] = diff[3] - diff[15];
  d[0] = m[0] + m[4]; d[1] = m[1] + m[5]; d[2] = m[2] + m[6]; d[3] = m[3] + m[7];
  d[4] = m[8] + m[12]; d[5] = m[9] + m[13]; d[6] = m[10] + m[14]; d[7] = m[11] + m[15];
  d[8] = m[0] - m[4]; d[9] = m[1] - m[5]; d[10] = m[2] - m[6]; d[11] = m[3] - m[7];
  d[12] = m[12] - m[8]; d[13] = m[13] - m[9]; d[14] = m[14] - m[10]; d[15] = m[15] - m[11];
  m[0] = d[0] + d[3]; m[1] = d[1] + d[2]; m[2] = d[1] - d[2]; m[3] = d[0] - d[3];
  m[4] = d[4] + d[7]; m[5] = d[5] + d[6]; m[6] = d[5] - d[6]; m[7] = d[4] - d[7];
  m[8] = d[8] + d[11]; m[9] = d[9] + d[10]; m[10] = d[9] - d[10]; m[11] = d[8] - d[11];
  m[12] = d[12] + d[15]; m[13] = d[13] + d[14]; m[14] = d[13] - d[14]; m[15] = d[12] - d[15];
  d[0] = m[0] + m[1]; d[1] = m[0] - m[1]; d[2] = m[2] + m[3]; d[3] = m[3] - m[2];
  d[4] = m[4] + m[5]; d[5] = m[4] - m[5]; d[6] = m[6] + m[7]; d[7] = m[7] - m[6];
  d[8] = m[8] + m[9]; d[9] = m[8] - m[9]; d[10] = m[10] + m[11]; d[11] = m[11] - m[10];
  d[12] = m[12] + m[13]; d[13] = m[12] - m[13]; d[14] = m[14] + m[15]; d[15] = m[15] - m[14];
  for (int k = 0; k < 16; ++k) satd += iabs_(d[k]);
  return (satd + 1) >> 1;
}

/* HadamardSAD8x8, me_distortion.c:266-341: rows then columns, 3 butterfly
 * stages each; (sum + 2) >> 2 */
static int had8(const int16_t *diff)
{
  int m1[8][8], m2[8][8], m3[8][8], sad = 0;
  for (int j = 0; j < 8; j++) {
    const int16_t *d = diff + 8 * j;
    m2[j][0] = d[0] + d[4]; m2[j][1] = d[1] + d[5]; m2[j][2] = d[2] + d[6]; m2[j][3] = d[3] + d[7];
    m2[j][4] = d[0] - d[4]; m2[j][5] = d[1] - d[5]; m2[j][6] = d[2] - d[6]; m2[j][7] = d[3] - d[7];
    m1[j][0] = m2[j][0] + m2[j][2]; m1[j][1] = m2[j][1] + m2[j][3];
    m1[j][2] = m2[j][0] - m2[j][2]; m1[j][3] = m2[j][1] - m2[j][3];
    m1[j][4] = m2[j][4] + m2[j][6]; m1[j][5] = m2[j][5] + m2[j][7];
    m1[j][6] = m2[j][4] - m2[j][6]; m1[j][7] = m2[j][5] - m2[j][7];
    m2[j][0] = m1[j][0] + m1[j][1]; m2[j][1] = m1[j][0] - m1[j][1];
    m2[j][2] = m1[j][2] + m1[j][3]; m2[j][3] = m1[j][2] - m1[j][3];
    m2[j][4] = m1[j][4] + m1[j][5]; m2[j][5] = m1[j][4] - m1[j][5];
    m2[j][6] = m1[j][6] + m1[j][7]; m2[j][7] = m1[j][6] - m1[j][7];
  }
  for (int i = 0; i < 8; i++) {
    m3[0][i] = m2[0][i] + m2[4][i]; m3[1][i] = m2[1][i] + m2[5][i];
    m3[2][i] = m2[2][i] + m2[6][i]; m3[3][i] = m2[3][i] + m2[7][i];
    m3[4][i] = m2[0][i] - m2[4][i]; m3[5][i] = m2[1][i] - m2[5][i];
    m3[6][i] = m2[2][i] - m2[6][i]; m3[7][i] = m2[3][i] - m2[7][i];
    m1[0][i] = m3[0][i] + m3[2][i]; m1[1][i] = m3[1][i] + m3[3][i];
    m1[2][i] = m3[0][i] - m3[2][i]; m1[3][i] = m3[1][i] - m3[3][i];
    m1[4][i] = m3[4][i] + m3[6][i]; m1[5][i] = m3[5][i] + m3[7][i];
    m1[6][i] = m3[4][i] - m3[6][i]; m1[7][i] = m3[5][i] - m3[7][i];
    m2[0][i] = m1[0][i] + m1[1][i]; m2[1][i] = m1[0][i] - m1[1][i];
    m2[2][i] = m1[2][i] + m1[3][i]; m2[3][i] = m1[2][i] - m1[3][i];
    m2[4][i] = m1[4][i] + m1[5][i]; m2[5][i] = m1[4][i] - m1[5][i];
    m2[6][i] = m1[6][i] + m1[7][i]; m2[7][i] = m1[6][i] - m1[7][i];
  }
  for (int j = 0; j < 8; j++)
    for (int i = 0; i < 8; i++) sad += iabs_(m2[j][i]);
  return (sad + 2) >> 2;
}
