/*
 * jm_me_capture.c -- TEST INFRASTRUCTURE (oracle side), never shipped.
 *
 * Link-time interposer for an UNMODIFIED JM 18.5 lencod build
 * (`-Wl,--wrap=full_search_motion_estimation -Wl,--wrap=fast_full_search_motion_estimation`).
 * It logs, for every integer-pel search JM performs, the exact inputs the
 * search sees and the (mv, cost) JM returns, plus the luma planes it reads.
 * The log is the golden-vector source for tests/golden/ (see
 * tests/golden/make_golden.py).  Nothing here changes JM's behaviour: each
 * wrapper calls the real function and only records.
 *
 * Reference interfaces observed (JM = /root/reference/4.对比程序/jm18.5/JM):
 *   IntPelME signature            JM/lencod/inc/global.h:459
 *   full_search_motion_estimation JM/lencod/src/me_fullsearch.c:39-103
 *   fast_full_search_motion_est.  JM/lencod/src/me_fullfast.c:618-689
 *   call site (min_mcost=DISTBLK_MAX) JM/lencod/src/mv_search.c:878,960
 *   MEBlock fields                JM/lencod/inc/global.h:254-314
 *
 * Output: binary file named by env JMME_CAPTURE (no-op when unset).
 *   plane record : u32 'PLN0', i32 frame_no, i32 kind(0=cur,1=ref), i32 list,
 *                  i32 ref, i32 W, i32 H, then W*H u16 samples (row major)
 *   search record: u32 'SRC0', struct cap_search (packed, little endian)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#include "global.h"
#include "mbuffer.h"
#include "me_fullfast.h"

extern distblk __real_full_search_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int);
extern distblk __real_fast_full_search_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int);

#pragma pack(push, 1)
struct cap_search {
  int32_t mode;          /* -1 = FS, 0 = FFS */
  int32_t frame_no;
  int32_t mb_addr;
  int16_t pix_x, pix_y;  /* MB origin (luma pels) */
  int16_t blocktype, block_x, block_y; /* block_x/y in 4x4 units inside MB */
  int16_t pos_x, pos_y;  /* block origin (luma pels) */
  int16_t bsx, bsy;
  int16_t list, ref;
  int16_t pred_x, pred_y;     /* MV predictor, qpel */
  int16_t center_x, center_y; /* mv_block->mv[list] on entry, qpel */
  int32_t sr_min_x, sr_max_x, sr_min_y, sr_max_y; /* mv_block->searchRange, qpel */
  int32_t lambda;
  int32_t rdopt;
  int32_t slice_type;
  int64_t min_mcost_in;
  /* FFS-only state (after setup) */
  int16_t ffs_center_x, ffs_center_y; /* search_center[list][ref], qpel, unpadded */
  int32_t ffs_max_range;              /* max_search_range[list][ref], integer pels */
  int32_t ffs_pos00;
  int32_t max_mvd;
  int32_t img_w, img_h;
  /* outputs */
  int16_t out_mv_x, out_mv_y;
  int64_t out_cost;
};
#pragma pack(pop)

static FILE *g_fp = NULL;
static int g_init = 0;
static int g_last_cur_frame = -1000000;
static int g_ref_seen[2][64];
static int g_ref_seen_frame = -1000000;

static FILE *cap_file(void)
{
  if (!g_init) {
    const char *p = getenv("JMME_CAPTURE");
    g_init = 1;
    if (p && *p) {
      g_fp = fopen(p, "wb");
      if (!g_fp) { fprintf(stderr, "jm_me_capture: cannot open %s\n", p); exit(2); }
    }
  }
  return g_fp;
}

static void dump_plane(FILE *fp, int frame_no, int kind, int list, int ref, imgpel **rows, int w, int h)
{
  uint32_t tag = 0x304E4C50u; /* 'PLN0' */
  int32_t hdr[6] = { frame_no, kind, list, ref, w, h };
  int y;
  fwrite(&tag, 4, 1, fp);
  fwrite(hdr, 4, 6, fp);
  for (y = 0; y < h; y++) {
    /* imgpel is uint16 (IMGTYPE 1, JM/lencod/inc/defines.h:37) */
    fwrite(rows[y], sizeof(imgpel), (size_t)w, fp);
  }
}

static void record(int mode, Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                   distblk min_mcost, int lambda_factor, const MotionVector *center_in,
                   distblk out_cost)
{
  FILE *fp = cap_file();
  VideoParameters *p_Vid = currMB->p_Vid;
  InputParameters *p_Inp = currMB->p_Inp;
  Slice *currSlice = currMB->p_Slice;
  int list = mv_block->list;
  int ref = mv_block->ref_idx;
  StorablePicture *ref_pic = currSlice->listX[list + currMB->list_offset][ref];
  struct cap_search r;
  uint32_t tag = 0x30435253u; /* 'SRC0' */

  if (!fp) return;

  if (p_Vid->frame_no != g_last_cur_frame) {
    g_last_cur_frame = p_Vid->frame_no;
    dump_plane(fp, p_Vid->frame_no, 0, 0, 0, p_Vid->pCurImg, p_Vid->width, p_Vid->height);
  }
  if (p_Vid->frame_no != g_ref_seen_frame) {
    g_ref_seen_frame = p_Vid->frame_no;
    memset(g_ref_seen, 0, sizeof(g_ref_seen));
  }
  if (list < 2 && ref < 64 && !g_ref_seen[list][ref]) {
    g_ref_seen[list][ref] = 1;
    dump_plane(fp, p_Vid->frame_no, 1, list, ref, ref_pic->imgY, ref_pic->size_x, ref_pic->size_y);
  }

  memset(&r, 0, sizeof(r));
  r.mode = mode;
  r.frame_no = p_Vid->frame_no;
  r.mb_addr = currMB->mbAddrX;
  r.pix_x = currMB->pix_x;
  r.pix_y = currMB->opix_y;
  r.blocktype = mv_block->blocktype;
  r.block_x = mv_block->block_x;
  r.block_y = mv_block->block_y;
  r.pos_x = mv_block->pos_x;
  r.pos_y = mv_block->pos_y;
  r.bsx = mv_block->blocksize_x;
  r.bsy = mv_block->blocksize_y;
  r.list = (int16_t)list;
  r.ref = (int16_t)ref;
  r.pred_x = pred_mv->mv_x;
  r.pred_y = pred_mv->mv_y;
  r.center_x = center_in->mv_x;
  r.center_y = center_in->mv_y;
  r.sr_min_x = mv_block->searchRange.min_x;
  r.sr_max_x = mv_block->searchRange.max_x;
  r.sr_min_y = mv_block->searchRange.min_y;
  r.sr_max_y = mv_block->searchRange.max_y;
  r.lambda = lambda_factor;
  r.rdopt = p_Inp->rdopt;
  r.slice_type = currSlice->slice_type;
  r.min_mcost_in = (int64_t)min_mcost;
  if (mode == 0 && p_Vid->p_ffast_me) {
    r.ffs_center_x = p_Vid->p_ffast_me->search_center[list][ref].mv_x;
    r.ffs_center_y = p_Vid->p_ffast_me->search_center[list][ref].mv_y;
    r.ffs_max_range = p_Vid->p_ffast_me->max_search_range[list][ref];
    r.ffs_pos00 = p_Vid->p_ffast_me->pos_00[list][ref];
  }
  r.max_mvd = p_Vid->max_mvd;
  r.img_w = p_Vid->width;
  r.img_h = p_Vid->height;
  r.out_mv_x = mv_block->mv[list].mv_x;
  r.out_mv_y = mv_block->mv[list].mv_y;
  r.out_cost = (int64_t)out_cost;
  fwrite(&tag, 4, 1, fp);
  fwrite(&r, sizeof(r), 1, fp);
}

distblk __wrap_full_search_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                             distblk min_mcost, int lambda_factor)
{
  MotionVector center_in = mv_block->mv[(short)mv_block->list];
  distblk c = __real_full_search_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
  record(-1, currMB, pred_mv, mv_block, min_mcost, lambda_factor, &center_in, c);
  return c;
}

distblk __wrap_fast_full_search_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                                  distblk min_mcost, int lambda_factor)
{
  MotionVector center_in = mv_block->mv[(short)mv_block->list];
  distblk c = __real_fast_full_search_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
  record(0, currMB, pred_mv, mv_block, min_mcost, lambda_factor, &center_in, c);
  return c;
}
