/*
 * jm_subpel_capture.c -- TEST INFRASTRUCTURE (oracle side), never shipped.
 *
 * Link-time interposer for an UNMODIFIED JM 18.5 lencod build that records the
 * sub-pel half of JM's motion search:
 *
 *   -Wl,--wrap=sub_pel_motion_estimation       JM/lencod/src/me_fullsearch.c:186-289
 *   -Wl,--wrap=EPZS_sub_pel_motion_estimation  JM/lencod/src/me_epzs_sub.c:30-222
 *   -Wl,--wrap=getSubImagesLuma                JM/lencod/src/img_luma.c:611-680
 *
 * Every wrapper calls the real function and only records: the exact inputs the
 * refinement sees (mv_block->mv in, the predictor, min_mcost, the three lambda
 * factors, the metric JM bound to computePredHPel / computePredQPel, test8x8,
 * the start_me_refinement_hp/qp switches) and JM's (mv, cost) result, plus the
 * luma planes it reads.  getSubImagesLuma dumps the 16 padded quarter-pel
 * sub-images it built (the first JMME_CAPTURE_SUBIMG calls; default 0), with
 * the integer picture they were built from.
 *
 * Call sites: SubPelME from BlockMotionSearch, JM/lencod/src/mv_search.c:966-976
 * (SubPelME bound in init_ME_engine :139-175 / EPZS_setup_engine
 * me_epzs_common.c:155-160); getSubImagesLuma from UnifiedOneForthPix,
 * JM/lencod/src/image.c:2148-2164.
 *
 * Output: binary file named by env JMME_CAPTURE (no-op when unset).
 *   plane record  : u32 'PLN0', i32 frame_no, i32 kind (0 cur, 1 ref, 2 interpolation
 *                   source), i32 list, i32 ref, i32 W, i32 H, W*H u16 samples
 *   sub-image rec : u32 'SUB0', i32 seq, i32 W, i32 H, then 16 planes [dy*4+dx] of
 *                   (H+2*IMG_PAD_SIZE_Y) x (W+2*IMG_PAD_SIZE_X) u16 samples
 *   search record : u32 'SPL0', struct cap_subpel (packed, little endian)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#include "global.h"
#include "mbuffer.h"
#include "me_distortion.h"
#include "me_epzs.h"

extern distblk __real_sub_pel_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int *);
extern distblk __real_EPZS_sub_pel_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int *);
extern void __real_getSubImagesLuma(VideoParameters *, StorablePicture *);

#pragma pack(push, 1)
struct cap_subpel {
  int32_t kind;              /* 0 sub_pel_motion_estimation, 1 EPZS_sub_pel_motion_estimation */
  int32_t frame_no;
  int32_t mb_addr;
  int16_t pix_x, pix_y;
  int16_t blocktype, block_x, block_y;
  int16_t pos_x, pos_y, bsx, bsy;
  int16_t list, ref;
  int16_t pred_x, pred_y;    /* MV predictor, qpel */
  int16_t mv_in_x, mv_in_y;  /* mv_block->mv[list] on entry (integer-pel result), qpel */
  int64_t min_mcost_in;
  int32_t lambda_f, lambda_h, lambda_q;
  int32_t rdopt, slice_type;
  int32_t start_hp, start_qp;
  int32_t metric_h, metric_q; /* 0 SAD, 1 SSE, 2 SATD, -1 other (weighted / otf) */
  int32_t test8x8;
  int32_t search_pos2, search_pos4;
  int32_t chroma_me;
  int64_t subthres;          /* EPZS: p_EPZS->subthres[blocktype] */
  int32_t img_w, img_h;
  int16_t out_mv_x, out_mv_y;
  int64_t out_cost;
};
#pragma pack(pop)

static FILE *g_fp = NULL;
static int g_init = 0;
static int g_subimg_left = 0;
static int g_subimg_seq = 0;
static int g_last_cur_frame = -1000000;
static int g_ref_seen[2][64];
static int g_ref_seen_frame = -1000000;

static FILE *cap_file(void)
{
  if (!g_init) {
    const char *p = getenv("JMME_CAPTURE");
    const char *s = getenv("JMME_CAPTURE_SUBIMG");
    g_init = 1;
    g_subimg_left = s ? atoi(s) : 0;
    if (p && *p) {
      g_fp = fopen(p, "wb");
      if (!g_fp) { fprintf(stderr, "jm_subpel_capture: cannot open %s\n", p); exit(2); }
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
  for (y = 0; y < h; y++)
    fwrite(rows[y], sizeof(imgpel), (size_t)w, fp);
}

static int metric_of(distblk (*f)(StorablePicture *, MEBlock *, distblk, MotionVector *))
{
  if (f == computeSAD) return 0;
  if (f == computeSSE) return 1;
  if (f == computeSATD) return 2;
  return -1;
}

static void record(int kind, Macroblock *currMB, MotionVector *pred, MEBlock *mv_block, distblk min_mcost,
                   int *lambda, MotionVector mv_in, distblk out_cost)
{
  FILE *fp = cap_file();
  VideoParameters *p_Vid = currMB->p_Vid;
  InputParameters *p_Inp = currMB->p_Inp;
  Slice *currSlice = currMB->p_Slice;
  int list = mv_block->list;
  int ref = mv_block->ref_idx;
  StorablePicture *ref_pic = currSlice->listX[list + currMB->list_offset][ref];
  struct cap_subpel r;
  uint32_t tag = 0x304C5053u; /* 'SPL0' */

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
  r.kind = kind;
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
  r.pred_x = pred->mv_x;
  r.pred_y = pred->mv_y;
  r.mv_in_x = mv_in.mv_x;
  r.mv_in_y = mv_in.mv_y;
  r.min_mcost_in = (int64_t)min_mcost;
  r.lambda_f = lambda[F_PEL];
  r.lambda_h = lambda[H_PEL];
  r.lambda_q = lambda[Q_PEL];
  r.rdopt = p_Inp->rdopt;
  r.slice_type = currSlice->slice_type;
  r.start_hp = p_Vid->start_me_refinement_hp;
  r.start_qp = p_Vid->start_me_refinement_qp;
  r.metric_h = metric_of(mv_block->computePredHPel);
  r.metric_q = metric_of(mv_block->computePredQPel);
  r.test8x8 = mv_block->test8x8;
  r.search_pos2 = mv_block->search_pos2;
  r.search_pos4 = mv_block->search_pos4;
  r.chroma_me = mv_block->ChromaMEEnable;
  if (kind == 1 && currSlice->p_EPZS)
    r.subthres = (int64_t)currSlice->p_EPZS->subthres[mv_block->blocktype];
  r.img_w = p_Vid->width;
  r.img_h = p_Vid->height;
  r.out_mv_x = mv_block->mv[list].mv_x;
  r.out_mv_y = mv_block->mv[list].mv_y;
  r.out_cost = (int64_t)out_cost;
  fwrite(&tag, 4, 1, fp);
  fwrite(&r, sizeof(r), 1, fp);
}

distblk __wrap_sub_pel_motion_estimation(Macroblock *currMB, MotionVector *pred, MEBlock *mv_block,
                                         distblk min_mcost, int *lambda)
{
  MotionVector mv_in = mv_block->mv[(short)mv_block->list];
  distblk c = __real_sub_pel_motion_estimation(currMB, pred, mv_block, min_mcost, lambda);
  record(0, currMB, pred, mv_block, min_mcost, lambda, mv_in, c);
  return c;
}

distblk __wrap_EPZS_sub_pel_motion_estimation(Macroblock *currMB, MotionVector *pred, MEBlock *mv_block,
                                              distblk min_mcost, int *lambda)
{
  MotionVector mv_in = mv_block->mv[(short)mv_block->list];
  distblk c = __real_EPZS_sub_pel_motion_estimation(currMB, pred, mv_block, min_mcost, lambda);
  record(1, currMB, pred, mv_block, min_mcost, lambda, mv_in, c);
  return c;
}

void __wrap_getSubImagesLuma(VideoParameters *p_Vid, StorablePicture *s)
{
  FILE *fp = cap_file();
  __real_getSubImagesLuma(p_Vid, s);
  if (fp && g_subimg_left > 0 && s->p_curr_img == s->imgY) {
    uint32_t tag = 0x30425553u; /* 'SUB0' */
    int32_t hdr[3] = { g_subimg_seq, s->size_x, s->size_y };
    int dy, dx, y;
    int pw = s->size_x + 2 * IMG_PAD_SIZE_X, ph = s->size_y + 2 * IMG_PAD_SIZE_Y;
    g_subimg_left--;
    dump_plane(fp, g_subimg_seq, 2, 0, 0, s->imgY, s->size_x, s->size_y);
    fwrite(&tag, 4, 1, fp);
    fwrite(hdr, 4, 3, fp);
    for (dy = 0; dy < 4; dy++)
      for (dx = 0; dx < 4; dx++)
        for (y = -IMG_PAD_SIZE_Y; y < ph - IMG_PAD_SIZE_Y; y++)
          fwrite(&s->p_curr_img_sub[dy][dx][y][-IMG_PAD_SIZE_X], sizeof(imgpel), (size_t)pw, fp);
    g_subimg_seq++;
  }
}
