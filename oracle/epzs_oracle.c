/*
 * epzs_oracle.c -- TEST INFRASTRUCTURE: restatement of JM 18.5's EPZS
 * integer-pel search; see epzs_oracle.h.  Written from the behaviour of
 * JM/lencod/src/me_epzs.c; no JM code is copied.  Only tests/ and the bench
 * CPU legs load this library.
 */
#include "epzs_oracle.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define DMAX (((int64_t)0x7fffffff) << 5)   /* DISTBLK_MAX, JM/lencod/inc/defines.h:135 */

/* refinement patterns (me_epzs_common.c:46-80 data, 176-230 wiring):
 * (dx, dy, start_nmbr, next_points) in qpel */
typedef struct pat {
  int n;
  short pt[12][4];
  int stop, next_last, next;
} pat;

enum { P_SDIAMOND, P_SQUARE, P_EDIAMOND, P_LDIAMOND, P_SBDIAMOND, P_PMVFAST };

static const pat PATS[6] = {
  {4, {{0, 4, 3, 3}, {4, 0, 0, 3}, {0, -4, 1, 3}, {-4, 0, 2, 3}}, 1, 1, P_SDIAMOND},
  {8, {{0, 4, 7, 3}, {4, 4, 7, 5}, {4, 0, 1, 3}, {4, -4, 1, 5}, {0, -4, 3, 3}, {-4, -4, 3, 5}, {-4, 0, 5, 3},
       {-4, 4, 5, 5}}, 1, 1, P_SQUARE},
  {12, {{-4, 4, 10, 5}, {0, 8, 10, 8}, {0, 4, 10, 7}, {4, 4, 1, 5}, {8, 0, 1, 8}, {4, 0, 1, 7}, {4, -4, 4, 5},
        {0, -8, 4, 8}, {0, -4, 4, 7}, {-4, -4, 7, 5}, {-8, 0, 7, 8}, {-4, 0, 7, 7}}, 1, 1, P_EDIAMOND},
  {8, {{0, 8, 6, 5}, {4, 4, 0, 3}, {8, 0, 0, 5}, {4, -4, 2, 3}, {0, -8, 2, 5}, {-4, -4, 4, 3}, {-8, 0, 4, 5},
       {-4, 4, 6, 3}}, 1, 1, P_LDIAMOND},
  {12, {{0, 8, 6, 12}, {4, 4, 0, 12}, {8, 0, 0, 12}, {4, -4, 2, 12}, {0, -8, 2, 12}, {-4, -4, 4, 12},
        {-8, 0, 4, 12}, {-4, 4, 6, 12}, {0, 2, 6, 12}, {2, 0, 0, 12}, {0, -2, 2, 12}, {-2, 0, 4, 12}}, 0, 1,
   P_SDIAMOND},
  {8, {{0, 8, 6, 5}, {4, 4, 0, 3}, {8, 0, 0, 5}, {4, -4, 2, 3}, {0, -8, 2, 5}, {-4, -4, 4, 3}, {-8, 0, 4, 5},
       {-4, 4, 6, 3}}, 0, 1, P_SDIAMOND},
};

/* EPZSPattern / EPZSDualRefinement -> pattern (me_epzs_common.c:530-565) */
static int primary_pattern(int v)
{
  switch (v) {
    case 5: return P_PMVFAST;
    case 4: return P_SBDIAMOND;
    case 3: return P_LDIAMOND;
    case 2: return P_EDIAMOND;
    case 1: return P_SQUARE;
    default: return P_SDIAMOND;
  }
}

static int dual_pattern(int v)
{
  switch (v) {
    case 6: return P_PMVFAST;
    case 5: return P_SBDIAMOND;
    case 4: return P_LDIAMOND;
    case 3: return P_EDIAMOND;
    case 2: return P_SQUARE;
    default: return P_SDIAMOND;
  }
}

static int mvbits(int v)   /* JM/lencod/src/mv_search.c:366-374 */
{
  unsigned a = (unsigned)(v < 0 ? -v : v), w = 2u * a + 1u;
  int b = 0;
  while (w >> (b + 1)) b++;
  return 2 * b + 1;
}

typedef struct ctx {
  const eo_req *q;
  const eo_pel *cur, *ref;
  int pitch, W, H;
  /* EPZSMap restated as the set of visited integer offsets from the centre */
  int side_x, side_y;
  unsigned char *map;
} ctx;

static int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* mv_cost + computeSAD<<5 for an integer qpel vector (UMVLine4X clamps each
 * sample into the picture) */
static int64_t cost_of(const ctx *c, int mx, int my)
{
  const eo_req *q = c->q;
  int64_t mvc = (int64_t)q->lambda * (mvbits(mx - q->pred_x) + mvbits(my - q->pred_y));
  int x, y, sad = 0;
  const int ox = q->pos_x + (mx >> 2), oy = q->pos_y + (my >> 2);
  for (y = 0; y < q->bsy; y++) {
    const eo_pel *rrow = c->ref + (size_t)clampi(oy + y, 0, c->H - 1) * c->pitch;
    const eo_pel *crow = c->cur + (size_t)(q->pos_y + y) * c->pitch + q->pos_x;
    for (x = 0; x < q->bsx; x++) {
      int d = crow[x] - rrow[clampi(ox + x, 0, c->W - 1)];
      sad += d < 0 ? -d : d;
    }
  }
  return mvc + ((int64_t)sad << 5);
}

static int in_range(const ctx *c, int mx, int my)
{
  int dx = mx - c->q->center_x, dy = my - c->q->center_y;
  return (dx < 0 ? -dx : dx) <= c->q->max_x && (dy < 0 ? -dy : dy) <= c->q->max_y;
}

/* test-and-set of the map cell of an in-range integer vector */
static int visit(ctx *c, int mx, int my)
{
  int cx = (mx - c->q->center_x + c->q->max_x) >> 2, cy = (my - c->q->center_y + c->q->max_y) >> 2;
  unsigned char *m = &c->map[cy * c->side_x + cx];
  if (*m) return 0;
  *m = 1;
  return 1;
}

static int16_t int_mv(int16_t v) { return (int16_t)(v & 0xFFFC); }   /* set_integer_mv, me_epzs.c:39-43 */

/* ---- validity intervals (the drop-in's speculative searches) -------------
 * Every comparison the search makes with the stop criterion S or the prevSad
 * value P is monotone in that value, so it reads "x >= t" for a threshold t
 * formed from the other operands.  ge() returns the outcome and narrows [lo, hi]
 * to the values that give the same outcome; the search's result is then the
 * same for every (S, P) inside the two intervals. */
typedef struct iv {
  int64_t lo, hi;
} iv;
static int ge(int64_t x, int64_t t, iv *v)
{
  if (x >= t) {
    if (t > v->lo) v->lo = t;
    return 1;
  }
  if (t - 1 < v->hi) v->hi = t - 1;
  return 0;
}
static int64_t fdiv(int64_t a, int64_t b) { return a / b - ((a % b) != 0 && a < 0); }   /* floor, b > 0 */
static int64_t cdiv(int64_t a, int64_t b) { return -fdiv(-a, b); }
/* P <= S with both inputs: pinned on the guessed P so each interval stands alone */
static int le2(int64_t p, int64_t s, iv *pv, iv *sv)
{
  if (p <= s) {
    if (p < pv->hi) pv->hi = p;
    if (p > sv->lo) sv->lo = p;
    return 1;
  }
  if (p > pv->lo) pv->lo = p;
  if (p - 1 < sv->hi) sv->hi = p - 1;
  return 0;
}
/* whether a JMME_EPZS_PRED_* entry joins the list for centre cost g and stop S
 * (me_epzs_common.c:1550 temporal, me_epzs.c:184-199 window, :205 block type) */
static int cond_ok(int c, int64_t g, int64_t S, iv *sv)
{
  switch (c) {
    case 1: return !ge(S, g, sv);                    /* g > S */
    case 2: return !ge(S, fdiv(g - 1, 2) + 1, sv);   /* g > 2 S */
    case 3: return !ge(S, fdiv(g - 1, 3) + 1, sv);   /* g > 3 S */
    default: return 1;
  }
}

void eo_epzs_ex(const eo_req *q, const int16_t *preds, const uint8_t *cond, const int16_t *stale, const eo_pel *cur,
                const eo_pel *ref, int pitch, int W, int H, eo_res *out, eo_bounds *bnd, int16_t *vis, int max_vis)
{
  ctx c;
  const int frame = q->flags & 1, pslice = (q->flags >> 1) & 1, bt = q->blocktype, refi = q->ref_idx;
  const int64_t lambda_dist = (int64_t)q->lambda * (q->variant ? 3 : 2);
  const int mv_range = q->variant ? 12 : 10;
  int64_t stop = q->medthres + lambda_dist, prev = q->prev_sad, min;
  int tmpx = q->center_x, tmpy = q->center_y, i, written = 0;
  iv sv = {INT64_MIN, INT64_MAX}, pv = {INT64_MIN, INT64_MAX};
  memset(out, 0, sizeof(*out));
  c.q = q;
  c.cur = cur;
  c.ref = ref;
  c.pitch = pitch;
  c.W = W;
  c.H = H;
  c.side_x = (2 * q->max_x >> 2) + 1;
  c.side_y = (2 * q->max_y >> 2) + 1;
  c.map = calloc((size_t)c.side_x * c.side_y, 1);
  for (i = 0; i < q->n_stale; i++) {       /* cells left holding this BlkCount */
    int dx = stale[2 * i], dy = stale[2 * i + 1];
    if ((dx & 3) == 0 && (dy & 3) == 0 && in_range(&c, q->center_x + dx, q->center_y + dy))
      visit(&c, q->center_x + dx, q->center_y + dy);
  }
  visit(&c, q->center_x, q->center_y);
  min = cost_of(&c, q->center_x, q->center_y);

  if (refi > 0 && frame && !ge(prev, stop < min ? stop : min, &pv)) {   /* prev < min(stop, min) */
    out->path = 1;
    goto done_noupdate;
  }
  if (min > stop) {
    int64_t second = DMAX;
    int check_median = 0, tmp2x = 0, tmp2y = 0, P, ok[4] = {1, 1, 1, 1};
    const int64_t gen_min = min;
    stop = q->stop_crit;
    if (ge(stop, 2 * min + 2, &sv)) {      /* min < (stop >> 1) */
      out->path = 2;
      goto done_noupdate;
    }
    if (cond)   /* the conditional parts of the list, generated with min_mcost = the centre's cost */
      for (i = 0; i < q->n_pred; i++)
        if (cond[i] && ok[cond[i]] == 1) ok[cond[i]] = 2 + cond_ok(cond[i], gen_min, stop, &sv);
    for (i = 0; i < q->n_pred; i++) {
      const int mx = int_mv(preds[2 * i]), my = int_mv(preds[2 * i + 1]);
      if (cond && cond[i] && ok[cond[i]] != 3) continue;   /* not in JM's list */
      if (in_range(&c, mx, my) && visit(&c, mx, my)) {
        const int64_t mc = cost_of(&c, mx, my);
        if (mc < min) {
          tmp2x = tmpx;
          tmp2y = tmpy;
          tmpx = mx;
          tmpy = my;
          second = min;
          min = mc;
          check_median = 1;
        } else if (mc < second) {
          tmp2x = mx;
          tmp2y = my;
          second = mc;
          check_median = 1;
        }
      }
      if (q->variant && ge(stop, cdiv(4 * min + 4, 3), &sv)) {     /* min < (3 stop) >> 2, me_epzs.c:583-596 */
        out->path = 3;
        goto done_mv_noupdate;
      }
    }
    if (!ge(stop, min, &sv)) {             /* min > stop */
      int cenx, ceny, point = 0, pstop = 0, next_last = 0, total, dir = 0;
      P = primary_pattern(q->pattern);
      if (q->pattern != 0) {
        if (ge(stop, min - ((3 * q->medthres) >> 1) + 1, &sv)) {   /* min < stop + 3 medthres / 2 */
          const int dx = abs(tmpx - q->center_x), dy = abs(tmpy - q->center_y);
          P = ((tmpx == 0 && tmpy == 0) || (dx < mv_range && dy < mv_range)) ? P_SDIAMOND : P_SQUARE;
        } else if (q->variant || bt > 4 || (refi > 0 && bt != 1)) {
          P = P_SQUARE;
        }
      }
      cenx = tmpx;
      ceny = tmpy;
      for (;;) {
        total = PATS[P].n;
        do {
          int left = total;
          do {
            const int mx = cenx + PATS[P].pt[point][0], my = ceny + PATS[P].pt[point][1];
            if (in_range(&c, mx, my) && visit(&c, mx, my)) {
              const int64_t mc = cost_of(&c, mx, my);
              if (mc < min) {
                tmpx = mx;
                tmpy = my;
                min = mc;
                dir = point;
              }
            }
            if (++point >= PATS[P].n) point -= PATS[P].n;
          } while (--left > 0);
          if (next_last || (tmpx == cenx && tmpy == ceny)) {
            pstop = PATS[P].stop;
            P = PATS[P].next;
            total = PATS[P].n;
            next_last = PATS[P].next_last;
            dir = 0;
            point = 0;
          } else {
            total = PATS[P].pt[dir][3];
            point = PATS[P].pt[dir][2];
            cenx = tmpx;
            ceny = tmpy;
          }
        } while (pstop != 1);

        /* 4 prev < min || (3 prev < min && prev <= stop) */
        if (refi > 0 && frame &&
            (!ge(prev, fdiv(min - 1, 4) + 1, &pv) || (!ge(prev, fdiv(min - 1, 3) + 1, &pv) && le2(prev, stop, &pv, &sv)))) {
          out->path = 4;
          goto done_mv_noupdate;
        }
        if (!(check_median && (pslice || (!q->variant && bt < 5)) && !ge(stop, min, &sv) && q->dual > 0)) break;
        point = 0;
        pstop = 0;
        dir = 0;
        next_last = 0;
        if ((tmpx == 0 && tmpy == 0) || (tmpx == q->center_x && tmpy == q->center_y)) {
          const int dx = abs(tmpx - q->center_x), dy = abs(tmpy - q->center_y);
          P = (dx < mv_range && dy < mv_range) ? P_SDIAMOND : P_SQUARE;
        } else {
          P = dual_pattern(q->dual);
        }
        cenx = tmp2x;
        ceny = tmp2y;
        check_median = 0;
      }
    }
  }
  out->path = out->path ? out->path : 5;
  if (refi == 0 || ge(prev, min + 1, &pv)) {   /* prev > min */
    prev = min;
    written = 1;
  }
done_mv_noupdate:
  out->mv_x = (int16_t)tmpx;
  out->mv_y = (int16_t)tmpy;
  goto finish;
done_noupdate:
  out->mv_x = q->center_x;
  out->mv_y = q->center_y;
finish:
  out->cost = min;
  out->prev_sad = prev;
  if (bnd) {
    bnd->stop_lo = sv.lo;
    bnd->stop_hi = sv.hi;
    bnd->prev_lo = pv.lo;
    bnd->prev_hi = pv.hi;
    bnd->prev_written = written;
    bnd->n_visited = 0;
    for (i = 0; i < c.side_x * c.side_y; i++)   /* every stamped cell, (dx, dy) qpel from the centre, in cell order */
      if (c.map[i]) {
        if (vis && bnd->n_visited < max_vis) {
          vis[2 * bnd->n_visited] = (int16_t)(4 * (i % c.side_x) - q->max_x);
          vis[2 * bnd->n_visited + 1] = (int16_t)(4 * (i / c.side_x) - q->max_y);
        }
        bnd->n_visited++;
      }
  }
  free(c.map);
}

void eo_epzs(const eo_req *q, const int16_t *preds, const int16_t *stale, const eo_pel *cur, const eo_pel *ref,
             int pitch, int W, int H, eo_res *out)
{
  eo_epzs_ex(q, preds, NULL, stale, cur, ref, pitch, W, H, out, NULL, NULL, 0);
}

void eo_epzs_batch(const eo_req *q, int n, const int16_t *preds, const int16_t *stale, const eo_pel *cur,
                   const eo_pel *const *refs, int pitch, int W, int H, eo_res *out)
{
  int i;
  for (i = 0; i < n; i++)
    eo_epzs(&q[i], preds + 2 * (size_t)q[i].pred_off, stale + 2 * (size_t)q[i].stale_off, cur, refs[q[i].plane],
            pitch, W, H, &out[i]);
}


/* ===========================================================================
 * EPZSSubPelGrid = 1: EPZS_integer_motion_estimation (variant 2) and
 * EPZS_integer_subMB_motion_estimation (variant 3), JM/lencod/src/
 * me_epzs_int.c:41-380 / 431-782.  Same skeleton as the integer-grid
 * functions above, with: the centre and the predictors kept at quarter-pel
 * precision (no set_integer_mv), the EPZSMap indexed per quarter-pel
 * position, computePredFPel = computeSAD on the quarter-pel sub-images
 * (UMVLine4X), and the control-flow differences marked inline.
 * subs: the reference's 16 sub-images, plane dy*4+dx, (H+40) x (W+64) 8-bit,
 * padded row 0 = picture row -20 (getSubImagesLuma layout). */
typedef struct gctx {
  const eo_req *q;
  const eo_pel *cur, *subs;
  int pitch, W, H, sp, sh;   /* cur pitch; sub-image pitch / rows */
  int side_x;
  unsigned char *map;
} gctx;

/* mv_cost + computeSAD<<5 at quarter-pel vector (mx, my) (me_distortion.c:349-426) */
static int64_t gcost_of(const gctx *c, int mx, int my)
{
  const eo_req *q = c->q;
  int64_t mvc = (int64_t)q->lambda * (mvbits(mx - q->pred_x) + mvbits(my - q->pred_y));
  const int cx = mx + (q->pos_x << 2), cy = my + (q->pos_y << 2);   /* pad_MVs */
  /* UMVLine4X (refbuf.h:22-26): size_y_pad = H+3, size_x_pad = W+15 (mbuffer.c:549-550) */
  const int yy = clampi(cy >> 2, -20, c->H + 3), xx = clampi(cx >> 2, -32, c->W + 15);
  const eo_pel *plane = c->subs + (size_t)((cy & 3) * 4 + (cx & 3)) * c->sp * c->sh;
  int x, y, sad = 0;
  for (y = 0; y < q->bsy; y++) {
    const eo_pel *rrow = plane + (size_t)(yy + 20 + y) * c->sp + (xx + 32);
    const eo_pel *crow = c->cur + (size_t)(q->pos_y + y) * c->pitch + q->pos_x;
    for (x = 0; x < q->bsx; x++) {
      int d = crow[x] - rrow[x];
      sad += d < 0 ? -d : d;
    }
  }
  return mvc + ((int64_t)sad << 5);
}

static int gin_range(const gctx *c, int mx, int my)
{
  int dx = mx - c->q->center_x, dy = my - c->q->center_y;
  return (dx < 0 ? -dx : dx) <= c->q->max_x && (dy < 0 ? -dy : dy) <= c->q->max_y;
}

/* EPZSMap[max_y - mv.y + my][max_x - mv.x + mx] (me_epzs_int.c:214-219): one cell per qpel position */
static int gvisit(gctx *c, int mx, int my)
{
  unsigned char *m = &c->map[(my - c->q->center_y + c->q->max_y) * c->side_x + (mx - c->q->center_x + c->q->max_x)];
  if (*m) return 0;
  *m = 1;
  return 1;
}

void eo_epzs_grid_ex(const eo_req *q, const int16_t *preds, const uint8_t *cond, const int16_t *stale,
                     const eo_pel *cur, int pitch, const eo_pel *subs, int W, int H, eo_res *out, eo_bounds *bnd,
                     int16_t *vis, int max_vis)
{
  gctx c;
  const int frame = q->flags & 1, pslice = (q->flags >> 1) & 1, bt = q->blocktype, refi = q->ref_idx;
  const int sub = q->variant == 3;
  const int64_t lambda_dist = (int64_t)q->lambda * (sub ? 3 : 2);
  const int mv_range = sub ? 12 : 10;
  int64_t stop = q->medthres + lambda_dist, prev = q->prev_sad, min;
  int tmpx = q->center_x, tmpy = q->center_y, i, written = 0;
  iv sv = {INT64_MIN, INT64_MAX}, pv = {INT64_MIN, INT64_MAX};
  memset(out, 0, sizeof(*out));
  c.q = q;
  c.cur = cur;
  c.subs = subs;
  c.pitch = pitch;
  c.W = W;
  c.H = H;
  c.sp = W + 64;
  c.sh = H + 40;
  c.side_x = 2 * q->max_x + 1;
  c.map = calloc((size_t)c.side_x * (2 * q->max_y + 1), 1);
  for (i = 0; i < q->n_stale; i++) {       /* cells left holding this BlkCount */
    int dx = stale[2 * i], dy = stale[2 * i + 1];
    if (gin_range(&c, q->center_x + dx, q->center_y + dy)) gvisit(&c, q->center_x + dx, q->center_y + dy);
  }
  gvisit(&c, q->center_x, q->center_y);
  min = gcost_of(&c, q->center_x, q->center_y);

  /* :67-80 / :496-507: the ref > 0 early exit also fires when prevSad * 8 (6 for subMB) < min */
  if (refi > 0 && frame &&
      (!ge(prev, stop < min ? stop : min, &pv) || !ge(prev, fdiv(min - 1, sub ? 6 : 8) + 1, &pv))) {
    out->path = 1;
    goto done_noupdate;
  }
  if (min > stop) {
    int64_t second = DMAX;
    int check_median = 0, tmp2x = 0, tmp2y = 0, P, ok[4] = {1, 1, 1, 1};
    const int64_t gen_min = min;
    stop = q->stop_crit;
    if (ge(stop, 2 * min + 2, &sv)) {      /* min < (stop >> 1): :112-124 (variant 2 updates prevSad) / :525-536 */
      out->path = 2;
      if (!sub && (refi == 0 || ge(prev, min + 1, &pv))) {
        prev = min;
        written = 1;
      }
      goto done_noupdate;
    }
    if (cond)   /* the conditional parts of the list, generated with min_mcost = the centre's cost */
      for (i = 0; i < q->n_pred; i++)
        if (cond[i] && ok[cond[i]] == 1) ok[cond[i]] = 2 + cond_ok(cond[i], gen_min, stop, &sv);
    for (i = 0; i < q->n_pred; i++) {
      const int mx = preds[2 * i], my = preds[2 * i + 1];   /* no set_integer_mv */
      if (cond && cond[i] && ok[cond[i]] != 3) continue;   /* not in JM's list */
      if (gin_range(&c, mx, my) && gvisit(&c, mx, my)) {
        int64_t mc = (int64_t)q->lambda * (mvbits(mx - q->pred_x) + mvbits(my - q->pred_y));
        if (mc < second) {   /* :224-226: the SAD of a candidate whose mv cost reaches second is skipped */
          mc = gcost_of(&c, mx, my);
          if (mc < min) {
            tmp2x = tmpx;
            tmp2y = tmpy;
            tmpx = mx;
            tmpy = my;
            second = min;
            min = mc;
            check_median = 1;
          } else if (mc < second) {
            tmp2x = mx;
            tmp2y = my;
            second = mc;
            check_median = 1;
          }
        }
      }
      if (sub) {
        if (refi > 0 && frame && !ge(prev, fdiv(min - 1, 3) + 1, &pv)) {   /* prev * 3 < min, :590-600 */
          out->path = 6;
          goto done_noupdate;
        }
        if (ge(stop, cdiv(4 * min + 4, 3), &sv)) {                          /* min < (3 stop) >> 2, :604-615 */
          out->path = 3;
          goto done_mv_noupdate;
        }
      }
    }
    if (!sub && refi > 0 && frame && !ge(prev, fdiv(min - 1, 3) + 1, &pv)) {   /* prev * 3 < min, :249-265 */
      out->path = 7;
      goto done_mv_noupdate;
    }
    if (!ge(stop, min, &sv)) {             /* min > stop */
      int cenx, ceny, point = 0, pstop = 0, next_last = 0, total, dir = 0;
      P = primary_pattern(q->pattern);
      if (q->pattern != 0) {
        if (ge(stop, min - ((3 * q->medthres) >> 1) + 1, &sv)) {   /* min < stop + 3 medthres / 2 */
          const int dx = abs(tmpx - q->center_x), dy = abs(tmpy - q->center_y);
          P = ((sub && bt == 7) || (tmpx == 0 && tmpy == 0) || (dx < mv_range && dy < mv_range)) ? P_SDIAMOND
                                                                                                  : P_SQUARE;
        } else if (sub || (refi > 0 && bt != 1)) {   /* variant 2 drops the bt > 4 test (:282) */
          P = P_SQUARE;
        }
      }
      cenx = tmpx;
      ceny = tmpy;
      for (;;) {
        total = PATS[P].n;
        do {
          int left = total;
          do {
            const int mx = cenx + PATS[P].pt[point][0], my = ceny + PATS[P].pt[point][1];
            if (gin_range(&c, mx, my) && gvisit(&c, mx, my)) {
              int64_t mc = (int64_t)q->lambda * (mvbits(mx - q->pred_x) + mvbits(my - q->pred_y));
              if (mc < min) {
                mc = gcost_of(&c, mx, my);
                if (mc < min) {
                  tmpx = mx;
                  tmpy = my;
                  min = mc;
                  dir = point;
                }
              }
            }
            if (++point >= PATS[P].n) point -= PATS[P].n;
          } while (--left > 0);
          if (next_last || (tmpx == cenx && tmpy == ceny)) {
            pstop = PATS[P].stop;
            P = PATS[P].next;
            total = PATS[P].n;
            next_last = PATS[P].next_last;
            dir = 0;
            point = 0;
          } else {
            total = PATS[P].pt[dir][3];
            point = PATS[P].pt[dir][2];
            cenx = tmpx;
            ceny = tmpy;
          }
        } while (pstop != 1);

        /* 4 prev < min || (3 prev < min && prev <= stop) */
        if (refi > 0 && frame &&
            (!ge(prev, fdiv(min - 1, 4) + 1, &pv) || (!ge(prev, fdiv(min - 1, 3) + 1, &pv) && le2(prev, stop, &pv, &sv)))) {
          out->path = 4;
          goto done_mv_noupdate;
        }
        /* second-best refinement, :337-340 / :298-301: min < 2 prev; min > (3 stop) >> 1 */
        if (!(check_median && (!sub || bt != 7) && (refi == 0 || ge(prev, cdiv(min + 1, 2), &pv)) && (!sub || pslice) &&
              !ge(stop, fdiv(2 * min - 1, 3) + 1, &sv) && q->dual > 0))
          break;
        point = 0;
        pstop = 0;
        dir = 0;
        next_last = 0;
        if ((tmpx == 0 && tmpy == 0) || (tmpx == q->center_x && tmpy == q->center_y)) {
          const int dx = abs(tmpx - q->center_x), dy = abs(tmpy - q->center_y);
          P = ((sub && bt == 7) || (dx < mv_range && dy < mv_range)) ? P_SDIAMOND : P_SQUARE;
        } else {
          P = dual_pattern(q->dual);
        }
        cenx = tmp2x;
        ceny = tmp2y;
        check_median = 0;
      }
    }
  }
  out->path = out->path ? out->path : 5;
  if (refi == 0 || ge(prev, min + 1, &pv)) {   /* prev > min */
    prev = min;
    written = 1;
  }
done_mv_noupdate:
  out->mv_x = (int16_t)tmpx;
  out->mv_y = (int16_t)tmpy;
  goto finish;
done_noupdate:
  out->mv_x = q->center_x;
  out->mv_y = q->center_y;
finish:
  out->cost = min;
  out->prev_sad = prev;
  if (bnd) {
    const int side_y = 2 * q->max_y + 1;
    bnd->stop_lo = sv.lo;
    bnd->stop_hi = sv.hi;
    bnd->prev_lo = pv.lo;
    bnd->prev_hi = pv.hi;
    bnd->prev_written = written;
    bnd->n_visited = 0;
    for (i = 0; i < c.side_x * side_y; i++)     /* every stamped cell, (dx, dy) qpel from the centre, in cell order */
      if (c.map[i]) {
        if (vis && bnd->n_visited < max_vis) {
          vis[2 * bnd->n_visited] = (int16_t)(i % c.side_x - q->max_x);
          vis[2 * bnd->n_visited + 1] = (int16_t)(i / c.side_x - q->max_y);
        }
        bnd->n_visited++;
      }
  }
  free(c.map);
}

void eo_epzs_grid(const eo_req *q, const int16_t *preds, const int16_t *stale, const eo_pel *cur, int pitch,
                  const eo_pel *subs, int W, int H, eo_res *out)
{
  eo_epzs_grid_ex(q, preds, NULL, stale, cur, pitch, subs, W, H, out, NULL, NULL, 0);
}

void eo_epzs_grid_batch(const eo_req *q, int n, const int16_t *preds, const int16_t *stale, const eo_pel *cur,
                        int pitch, const eo_pel *const *subs, int W, int H, eo_res *out)
{
  int i;
  for (i = 0; i < n; i++)
    eo_epzs_grid(&q[i], preds + 2 * (size_t)q[i].pred_off, stale + 2 * (size_t)q[i].stale_off, cur, pitch,
                 subs[q[i].plane], W, H, &out[i]);
}

void eo_epzs_ex_batch(const eo_req *q, int n, const int16_t *preds, const uint8_t *cond, const int16_t *stale,
                      const eo_pel *cur, const eo_pel *const *refs, int pitch, int W, int H, eo_res *out,
                      eo_bounds *bnd, int16_t *vis, int max_vis)
{
  int i;
  for (i = 0; i < n; i++)
    eo_epzs_ex(&q[i], preds + 2 * (size_t)q[i].pred_off, cond ? cond + q[i].pred_off : NULL,
               stale + 2 * (size_t)q[i].stale_off, cur, refs[q[i].plane], pitch, W, H, &out[i], &bnd[i],
               vis ? vis + 2 * (size_t)max_vis * i : NULL, max_vis);
}

void eo_epzs_grid_ex_batch(const eo_req *q, int n, const int16_t *preds, const uint8_t *cond, const int16_t *stale,
                           const eo_pel *cur, int pitch, const eo_pel *const *subs, int W, int H, eo_res *out,
                           eo_bounds *bnd, int16_t *vis, int max_vis)
{
  int i;
  for (i = 0; i < n; i++)
    eo_epzs_grid_ex(&q[i], preds + 2 * (size_t)q[i].pred_off, cond ? cond + q[i].pred_off : NULL,
                    stale + 2 * (size_t)q[i].stale_off, cur, pitch, subs[q[i].plane], W, H, &out[i], &bnd[i],
                    vis ? vis + 2 * (size_t)max_vis * i : NULL, max_vis);
}
