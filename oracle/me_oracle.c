/*
 * me_oracle.c -- TEST INFRASTRUCTURE: CPU restatement of JM 18.5 integer-pel
 * ME (full search + fast full search).  See me_oracle.h for the contract.
 * Written from the behaviour of the JM sources; no JM code is copied.
 * (JM = /root/reference/4.对比程序/jm18.5/JM)
 */
#include "me_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline int iabs_(int v) { return v < 0 ? -v : v; }

/* spiral order, JM lencod/src/mv_search.c:406-442:
 *   index 0 = (0,0); ring l = 1..R: for i=-l+1..l-1 push (i,-l),(i,+l);
 *   then for i=-l..l push (-l,i),(+l,i). */
int ora_spiral(int search_range, int16_t *out_xy)
{
  int k = 1, l, i;
  out_xy[0] = 0; out_xy[1] = 0;
  for (l = 1; l <= search_range; l++) {
    for (i = -l + 1; i < l; i++) {
      out_xy[2 * k] = (int16_t)i; out_xy[2 * k + 1] = (int16_t)-l; k++;
      out_xy[2 * k] = (int16_t)i; out_xy[2 * k + 1] = (int16_t)l;  k++;
    }
    for (i = -l; i <= l; i++) {
      out_xy[2 * k] = (int16_t)-l; out_xy[2 * k + 1] = (int16_t)i; k++;
      out_xy[2 * k] = (int16_t)l;  out_xy[2 * k + 1] = (int16_t)i; k++;
    }
  }
  return k;
}

/* JM lencod/src/mv_search.c:321-327 (sizes) and :366-374 (fill). */
int ora_mvbits_table(int search_range, int32_t *out, int out_len)
{
  int number_of_subpel_positions = 4 * (2 * search_range + 3);
  int max_mv_bits = 3 + 2 * (int)ceil(log(number_of_subpel_positions + 1) / log(2) + 1e-10);
  int max_mvd = (1 << (max_mv_bits >> 1)) - 1;
  int bits, i;
  if (out_len < 2 * max_mvd + 1) return -1;
  memset(out, 0, sizeof(int32_t) * (size_t)(2 * max_mvd + 1));
  out[max_mvd] = 1;
  for (bits = 3; bits <= max_mv_bits; bits += 2) {
    int i_max = 1 << (bits >> 1);
    int i_min = i_max >> 1;
    for (i = i_min; i < i_max; i++) {
      out[max_mvd + i] = bits;
      out[max_mvd - i] = bits;
    }
  }
  return max_mvd;
}

/* closed form of the table above: bits(0)=1, bits(+-v)=2*floor(log2 v)+3 */
static inline int64_t mvbits(int v)
{
  unsigned a = (unsigned)iabs_(v);
  int lg = -1;
  while (a) { lg++; a >>= 1; }
  return (int64_t)(2 * lg + 3);
}

/* mv_cost, JM lencod/inc/mv_search.h:100-104 (JCOST_CALC_SCALEUP = 1) */
static inline int64_t mv_cost(int lambda, int cx, int cy, int px, int py)
{
  return (int64_t)lambda * (mvbits(cx - px) + mvbits(cy - py));
}

/* pixel of the padded reference at integer (y,x): UMVLine4X origin clamp
 * (refbuf.h:22-26) over an edge-replicated pad (img_luma.c:40-86) is the
 * per-pixel clamp into the picture for blocks up to 16 wide. */
static inline int refpel(const uint16_t *ref, int W, int H, int y, int x)
{
  return ref[(size_t)clampi(y, 0, H - 1) * W + clampi(x, 0, W - 1)];
}

int64_t ora_full_search(const uint16_t *cur, const uint16_t *ref, int W, int H,
                        int pos_x, int pos_y, int bsx, int bsy,
                        int pred_x, int pred_y, int center_x, int center_y,
                        int search_range, int lambda, int check_for_00,
                        int64_t min_mcost_in, int16_t *out_mv)
{
  int R = search_range;
  int max_pos = (2 * R + 1) * (2 * R + 1);
  int16_t *sp;
  int pos, best_pos = 0;
  int64_t min_mcost = min_mcost_in;
  /* absolute (padded) qpel positions, me_fullsearch.c:62-65 */
  int pad_x = pos_x << 2, pad_y = pos_y << 2;
  int cx0 = pad_x + center_x, cy0 = pad_y + center_y;
  int px = pad_x + pred_x, py = pad_y + pred_y;

  if ((center_x & 3) || (center_y & 3)) return -1; /* sub-pel grid centre: not in this restatement */
  sp = (int16_t *)malloc(sizeof(int16_t) * 2 * (size_t)max_pos);
  ora_spiral(R, sp);

  for (pos = 0; pos < max_pos; pos++) {
    int cand_x = cx0 + (sp[2 * pos] << 2);
    int cand_y = cy0 + (sp[2 * pos + 1] << 2);
    int64_t mcost = mv_cost(lambda, cand_x, cand_y, px, py);
    if (check_for_00 && cand_x == pad_x && cand_y == pad_y) {
      int64_t tmp = (int64_t)lambda * 16;      /* weighted_cost(lambda,16), ifunctions.h:224 */
      mcost = mcost > tmp ? mcost - tmp : 0;
    }
    if (mcost >= min_mcost) continue;
    {
      /* computeSAD, me_distortion.c:349-426: row-wise early exit against
       * dist_down(min_mcost - mcost); on exit the threshold is returned. */
      int64_t thr = min_mcost - mcost;
      int imin_cost = (int)(thr >> 5);
      int sad = 0, y, x, early = 0;
      int ox = cand_x >> 2, oy = cand_y >> 2;
      for (y = 0; y < bsy && !early; y++) {
        const uint16_t *src = cur + (size_t)(pos_y + y) * W + pos_x;
        for (x = 0; x < bsx; x++) sad += iabs_((int)src[x] - refpel(ref, W, H, oy + y, ox + x));
        if (sad > imin_cost) early = 1;
      }
      mcost += early ? thr : ((int64_t)sad << 5);
    }
    if (mcost < min_mcost) { best_pos = pos; min_mcost = mcost; }
  }
  out_mv[0] = (int16_t)(center_x + (best_pos ? (sp[2 * best_pos] << 2) : 0));
  out_mv[1] = (int16_t)(center_y + (best_pos ? (sp[2 * best_pos + 1] << 2) : 0));
  free(sp);
  return min_mcost;
}

void ora_ffs_surface(const uint16_t *cur, const uint16_t *ref, int W, int H,
                     int mb_x, int mb_y, int center_x, int center_y,
                     int surf_range, uint32_t *out)
{
  int R = surf_range, P = (2 * R + 1) * (2 * R + 1), pos;
  int16_t *sp = (int16_t *)malloc(sizeof(int16_t) * 2 * (size_t)P);
  ora_spiral(R, sp);
  for (pos = 0; pos < P; pos++) {
    /* cand = search_center_padded + spiral (me_fullfast.c:329,493) */
    int ox = mb_x + (center_x >> 2) + sp[2 * pos];
    int oy = mb_y + (center_y >> 2) + sp[2 * pos + 1];
    int b;
    for (b = 0; b < 16; b++) {
      int bx = (b & 3) * 4, by = (b >> 2) * 4, y, x;
      uint32_t s = 0;
      for (y = 0; y < 4; y++)
        for (x = 0; x < 4; x++)
          s += (uint32_t)iabs_(refpel(ref, W, H, oy + by + y, ox + bx + x) -
                               (int)cur[(size_t)(mb_y + by + y) * W + mb_x + bx + x]);
      out[(size_t)b * P + pos] = s;
    }
  }
  free(sp);
}

void ora_ffs_aggregate(const uint32_t *t7, int P, uint32_t *all)
{
  /* all[bt][blk][pos]; blocktype 7 = 4x4, 6 = 4x8, 5 = 8x4, 4 = 8x8,
   * 3 = 8x16, 2 = 16x8, 1 = 16x16 (macroblock.h:58 block_size). */
#define A(bt, blk) (all + ((size_t)(bt) * 16 + (blk)) * (size_t)P)
  int i, pos;
  memset(all, 0, sizeof(uint32_t) * 8 * 16 * (size_t)P);
  memcpy(A(7, 0), t7, sizeof(uint32_t) * 16 * (size_t)P);
  for (i = 0; i < 16; i++) {
    int bx = i & 3, by = i >> 2;
    if (!(by & 1)) for (pos = 0; pos < P; pos++) A(6, i)[pos] = A(7, i)[pos] + A(7, i + 4)[pos];
    if (!(bx & 1)) for (pos = 0; pos < P; pos++) A(5, i)[pos] = A(7, i)[pos] + A(7, i + 1)[pos];
  }
  for (i = 0; i < 16; i++) {
    int bx = i & 3, by = i >> 2;
    if (!(bx & 1) && !(by & 1)) for (pos = 0; pos < P; pos++) A(4, i)[pos] = A(6, i)[pos] + A(6, i + 1)[pos];
  }
  for (i = 0; i <= 2; i += 2) for (pos = 0; pos < P; pos++) A(3, i)[pos] = A(4, i)[pos] + A(4, i + 8)[pos];
  for (i = 0; i <= 8; i += 8) for (pos = 0; pos < P; pos++) A(2, i)[pos] = A(4, i)[pos] + A(4, i + 2)[pos];
  for (pos = 0; pos < P; pos++) A(1, 0)[pos] = A(3, 0)[pos] + A(3, 2)[pos];
#undef A
}

int64_t ora_ffs_block(const uint32_t *all, int surf_range,
                      int blocktype, int block_x, int block_y,
                      int center_x, int center_y, int pred_x, int pred_y,
                      int block_range, int lambda, int max_mvd, int rdopt,
                      int pos00, int64_t min_mcost_in, int16_t *out_mv)
{
  int Ps = (2 * surf_range + 1) * (2 * surf_range + 1);
  int max_pos = (2 * block_range + 1) * (2 * block_range + 1);
  const uint32_t *bsad = all + ((size_t)blocktype * 16 + (size_t)((block_y << 2) + block_x)) * (size_t)Ps;
  int16_t *sp = (int16_t *)malloc(sizeof(int16_t) * 2 * (size_t)(max_pos > Ps ? max_pos : Ps));
  int64_t min_mcost = min_mcost_in;
  int best_pos = 0, pos;
  int gate = max_mvd - 1;  /* me_fullfast.c:637 */
  ora_spiral(block_range > surf_range ? block_range : surf_range, sp);

  /* (0,0) pre-seed, me_fullfast.c:650-657 */
  if (!rdopt && (iabs_(pred_x) > iabs_(pred_y) ? iabs_(pred_x) : iabs_(pred_y)) < gate) {
    min_mcost = ((int64_t)bsad[pos00] << 5) + mv_cost(lambda, 0, 0, pred_x, pred_y);
    best_pos = pos00;
  }
  for (pos = 0; pos < max_pos; pos++) {
    int64_t mcost = (int64_t)bsad[pos] << 5;
    int cx = center_x + (sp[2 * pos] << 2), cy = center_y + (sp[2 * pos + 1] << 2);
    int dmax = iabs_(cx - pred_x) > iabs_(cy - pred_y) ? iabs_(cx - pred_x) : iabs_(cy - pred_y);
    if (mcost < min_mcost && dmax < gate) {
      mcost += mv_cost(lambda, cx, cy, pred_x, pred_y);
      if (mcost < min_mcost) { min_mcost = mcost; best_pos = pos; }
    }
  }
  out_mv[0] = (int16_t)(center_x + (sp[2 * best_pos] << 2));
  out_mv[1] = (int16_t)(center_y + (sp[2 * best_pos + 1] << 2));
  free(sp);
  return min_mcost;
}

void ora_full_search_batch(const uint16_t *cur, const uint16_t *ref, int W, int H,
                           int nreq, const int32_t *req, int16_t *out_mv, int64_t *out_cost)
{
  int i;
  for (i = 0; i < nreq; i++) {
    const int32_t *r = req + (size_t)i * ORA_REQ_FIELDS;
    out_cost[i] = ora_full_search(cur, ref, W, H, r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7],
                                  r[8], r[9], r[10], ORA_DISTBLK_MAX, out_mv + 2 * (size_t)i);
  }
}

void ora_ffs_batch(const uint16_t *cur, const uint16_t *ref, int W, int H,
                   int surf_range, int max_mvd, int rdopt,
                   int nmb, const int32_t *mbs, int nblk, const int32_t *blk,
                   int16_t *out_mv, int64_t *out_cost)
{
  int P = (2 * surf_range + 1) * (2 * surf_range + 1);
  uint32_t *t7 = (uint32_t *)malloc(sizeof(uint32_t) * 16 * (size_t)P);
  uint32_t *all = (uint32_t *)malloc(sizeof(uint32_t) * 8 * 16 * (size_t)P);
  int m, b = 0;
  for (m = 0; m < nmb; m++) {
    const int32_t *mb = mbs + 4 * (size_t)m;
    ora_ffs_surface(cur, ref, W, H, mb[0], mb[1], mb[2], mb[3], surf_range, t7);
    ora_ffs_aggregate(t7, P, all);
    for (; b < nblk && blk[9 * (size_t)b] == m; b++) {
      const int32_t *q = blk + 9 * (size_t)b;
      out_cost[b] = ora_ffs_block(all, surf_range, q[1], q[2], q[3], mb[2], mb[3], q[4], q[5],
                                  q[6], q[7], max_mvd, rdopt, q[8], ORA_DISTBLK_MAX,
                                  out_mv + 2 * (size_t)b);
    }
  }
  free(t7);
  free(all);
}
