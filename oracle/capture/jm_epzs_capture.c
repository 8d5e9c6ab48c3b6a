/*
 * jm_epzs_capture.c -- TEST INFRASTRUCTURE (oracle side), never shipped.
 *
 * Link-time interposer for an UNMODIFIED JM 18.5 lencod build that records
 * every EPZS integer-pel search:
 *   EPZS_motion_estimation        JM/lencod/src/me_epzs.c:54-407
 *   EPZS_subMB_motion_estimation  JM/lencod/src/me_epzs.c:417-780
 *   EPZS_integer_motion_estimation / EPZS_integer_subMB_motion_estimation
 *                                 JM/lencod/src/me_epzs_int.c:41-380 / 431-782
 *                                 (EPZSSubPelGrid = 1: variants 2 / 3)
 * together with the host-side state each search reads -- the predictor list
 * JM generated for it (EPZS_spatial_predictors / _spatial_memory_ /
 * _temporal_ / EPZSWindowPredictors / EPZSBlockTypePredictors(MB),
 * me_epzs_common.c:1224-1764), its stop criterion
 * (EPZSDetermineStopCriterion :1764), the prevSad slot, and the cells of the
 * never-cleared EPZSMap that already hold this search's BlkCount (uint16
 * wrap-around, me_epzs.c:92-94) -- plus the search's (mv, cost).  Each
 * wrapper calls the real function; nothing in JM's behaviour changes.
 *
 * Output (env JMME_CAPTURE): plane records as in jm_me_capture.c, then per
 * search u32 'EPZ0', struct cap_epzs, n_pred x (i16 x, i16 y) predictors,
 * n_stale x (i16 dx, i16 dy) pre-marked map offsets (qpel, from the centre).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#include "global.h"
#include "mbuffer.h"
#include "me_epzs.h"
#include "me_epzs_common.h"

extern distblk __real_EPZS_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int);
extern distblk __real_EPZS_subMB_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int);
extern distblk __real_EPZS_integer_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int);
extern distblk __real_EPZS_integer_subMB_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int);
extern distblk __real_EPZSDetermineStopCriterion(EPZSParameters *, distblk *, MEBlock *, distblk);
extern short __real_EPZS_spatial_predictors(EPZSParameters *, MEBlock *, int, int, short, struct pic_motion_params **);
extern void __real_EPZS_spatial_memory_predictors(EPZSParameters *, MEBlock *, int, int *, int);
extern void __real_EPZS_temporal_predictors(Macroblock *, StorablePicture *, EPZSParameters *, MEBlock *, int *,
                                            distblk, distblk);
extern void __real_EPZSWindowPredictors(MotionVector *, EPZSStructure *, int *, EPZSStructure *);
extern void __real_EPZSBlockTypePredictorsMB(Slice *, MEBlock *, SPoint *, int *);
extern void __real_EPZSBlockTypePredictors(Slice *, MEBlock *, SPoint *, int *);

#define MAX_STALE 256

#pragma pack(push, 1)
struct cap_epzs {
  int32_t variant;       /* 0 EPZS_motion_estimation, 1 EPZS_subMB_motion_estimation,
                            2 EPZS_integer_motion_estimation, 3 EPZS_integer_subMB_motion_estimation */
  int32_t frame_no;
  int32_t mb_addr;
  int16_t mb_x, mb_y;    /* currMB->mb_x / mb_y (MB units) */
  int16_t blocktype, block_x, block_y;
  int16_t pos_x, pos_y;  /* block origin, luma pels */
  int16_t bsx, bsy;
  int16_t list, ref, list_offset;
  int16_t pred_x, pred_y;     /* qpel */
  int16_t center_x, center_y; /* mv_block->mv[list] on entry, qpel */
  int32_t sr_min_x, sr_max_x, sr_min_y, sr_max_y;
  int32_t lambda;
  int32_t slice_type, structure;
  int32_t epzs_pattern, epzs_dual;
  int32_t blk_count;          /* the BlkCount this search marks with */
  int64_t prev_sad_in;
  int64_t medthres;           /* p_EPZS->medthres[blocktype] */
  int64_t stop_crit;          /* EPZSDetermineStopCriterion's value, -1 if not called */
  int32_t n_pred;             /* predictor count, -1 if none were generated */
  int32_t n_stale;
  int32_t stale_overflow;
  int32_t img_w, img_h;
  int64_t min_mcost_in;
  int16_t out_mv_x, out_mv_y;
  int64_t out_cost;
  int64_t prev_sad_out;
};
#pragma pack(pop)

static FILE *g_fp = NULL;
static int g_init = 0;
static int g_last_cur_frame = -1000000;
static int g_ref_seen[2][64];
static int g_ref_seen_frame = -1000000;

static int64_t g_stop = -1;
static int g_npred = -1;

static FILE *cap_file(void)
{
  if (!g_init) {
    const char *p = getenv("JMME_CAPTURE");
    g_init = 1;
    if (p && *p) {
      g_fp = fopen(p, "wb");
      if (!g_fp) { fprintf(stderr, "jm_epzs_capture: cannot open %s\n", p); exit(2); }
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
  for (y = 0; y < h; y++) fwrite(rows[y], sizeof(imgpel), (size_t)w, fp);
}

static int map_side(Macroblock *currMB)
{
  InputParameters *p_Inp = currMB->p_Inp;
  VideoParameters *p_Vid = currMB->p_Vid;
  int sr = p_Inp->search_range[p_Vid->view_id];
  if (p_Inp->BiPredMotionEstimation && p_Inp->BiPredMESearchRange[p_Vid->view_id] > sr)
    sr = p_Inp->BiPredMESearchRange[p_Vid->view_id];
  return (2 * sr + 1) << 2;       /* me_epzs_common.c:428-431 */
}

static distblk call_real(int variant, Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block, distblk min_mcost,
                         int lambda_factor)
{
  switch (variant) {
    case 0: return __real_EPZS_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
    case 1: return __real_EPZS_subMB_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
    case 2: return __real_EPZS_integer_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
    default: return __real_EPZS_integer_subMB_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
  }
}

static distblk run(int variant, Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block, distblk min_mcost,
                   int lambda_factor)
{
  FILE *fp = cap_file();
  Slice *currSlice = currMB->p_Slice;
  VideoParameters *p_Vid = currMB->p_Vid;
  InputParameters *p_Inp = currMB->p_Inp;
  EPZSParameters *p_EPZS = currSlice->p_EPZS;
  int list = mv_block->list;
  int cur_list = list + currMB->list_offset;
  int ref = mv_block->ref_idx;
  int bt = mv_block->blocktype;
  distblk *prevSad = &p_EPZS->distortion[cur_list][bt - 1][mv_block->pos_x2];
  MotionVector center_in = mv_block->mv[list];
  struct cap_epzs r;
  int16_t stale[MAX_STALE][2];
  uint16 next = (uint16)(p_EPZS->BlkCount + 1);
  distblk c;
  int i, j, side;

  if (!fp) return call_real(variant, currMB, pred_mv, mv_block, min_mcost, lambda_factor);
  if (next == 0) next = 1;
  memset(&r, 0, sizeof(r));
  /* cells already equal to the BlkCount this search will use (left by the
     search 65535 calls earlier): JM treats them as visited */
  side = map_side(currMB);
  for (i = 0; i < side; i++)
    for (j = 0; j < side; j++)
      if (p_EPZS->EPZSMap[i][j] == next) {
        int dy = i - mv_block->searchRange.max_y, dx = j - mv_block->searchRange.max_x;
        if (dy < -mv_block->searchRange.max_y || dy > mv_block->searchRange.max_y ||
            dx < -mv_block->searchRange.max_x || dx > mv_block->searchRange.max_x)
          continue;
        if (r.n_stale < MAX_STALE) {
          stale[r.n_stale][0] = (int16_t)dx;
          stale[r.n_stale][1] = (int16_t)dy;
          r.n_stale++;
        } else {
          r.stale_overflow = 1;
        }
      }
  r.prev_sad_in = (int64_t)*prevSad;
  g_stop = -1;
  g_npred = -1;
  c = call_real(variant, currMB, pred_mv, mv_block, min_mcost, lambda_factor);

  if (p_Vid->frame_no != g_last_cur_frame) {
    g_last_cur_frame = p_Vid->frame_no;
    dump_plane(fp, p_Vid->frame_no, 0, 0, 0, p_Vid->pCurImg, p_Vid->width, p_Vid->height);
  }
  if (p_Vid->frame_no != g_ref_seen_frame) {
    g_ref_seen_frame = p_Vid->frame_no;
    memset(g_ref_seen, 0, sizeof(g_ref_seen));
  }
  if (list < 2 && ref < 64 && !g_ref_seen[list][ref]) {
    StorablePicture *ref_pic = currSlice->listX[cur_list][ref];
    g_ref_seen[list][ref] = 1;
    dump_plane(fp, p_Vid->frame_no, 1, list, ref, ref_pic->imgY, ref_pic->size_x, ref_pic->size_y);
  }

  r.variant = variant;
  r.frame_no = p_Vid->frame_no;
  r.mb_addr = currMB->mbAddrX;
  r.mb_x = (int16_t)currMB->mb_x;
  r.mb_y = (int16_t)currMB->mb_y;
  r.blocktype = (int16_t)bt;
  r.block_x = mv_block->block_x;
  r.block_y = mv_block->block_y;
  r.pos_x = mv_block->pos_x;
  r.pos_y = mv_block->pos_y;
  r.bsx = mv_block->blocksize_x;
  r.bsy = mv_block->blocksize_y;
  r.list = (int16_t)list;
  r.ref = (int16_t)ref;
  r.list_offset = (int16_t)currMB->list_offset;
  r.pred_x = pred_mv->mv_x;
  r.pred_y = pred_mv->mv_y;
  r.center_x = center_in.mv_x;
  r.center_y = center_in.mv_y;
  r.sr_min_x = mv_block->searchRange.min_x;
  r.sr_max_x = mv_block->searchRange.max_x;
  r.sr_min_y = mv_block->searchRange.min_y;
  r.sr_max_y = mv_block->searchRange.max_y;
  r.lambda = lambda_factor;
  r.slice_type = currSlice->slice_type;
  r.structure = currSlice->structure;
  r.epzs_pattern = p_Inp->EPZSPattern;
  r.epzs_dual = p_Inp->EPZSDual;
  r.blk_count = p_EPZS->BlkCount;
  r.medthres = (int64_t)p_EPZS->medthres[bt];
  r.stop_crit = g_stop;
  r.n_pred = g_npred;
  r.img_w = p_Vid->width;
  r.img_h = p_Vid->height;
  r.min_mcost_in = (int64_t)min_mcost;
  r.out_mv_x = mv_block->mv[list].mv_x;
  r.out_mv_y = mv_block->mv[list].mv_y;
  r.out_cost = (int64_t)c;
  r.prev_sad_out = (int64_t)*prevSad;
  {
    uint32_t tag = 0x305A5045u; /* 'EPZ0' */
    fwrite(&tag, 4, 1, fp);
    fwrite(&r, sizeof(r), 1, fp);
    for (i = 0; i < r.n_pred; i++) {
      int16_t xy[2] = { p_EPZS->predictor->point[i].motion.mv_x, p_EPZS->predictor->point[i].motion.mv_y };
      fwrite(xy, 2, 2, fp);
    }
    fwrite(stale, 4, (size_t)r.n_stale, fp);
  }
  return c;
}

distblk __wrap_EPZS_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                      distblk min_mcost, int lambda_factor)
{
  return run(0, currMB, pred_mv, mv_block, min_mcost, lambda_factor);
}

distblk __wrap_EPZS_subMB_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                            distblk min_mcost, int lambda_factor)
{
  return run(1, currMB, pred_mv, mv_block, min_mcost, lambda_factor);
}

distblk __wrap_EPZS_integer_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                              distblk min_mcost, int lambda_factor)
{
  return run(2, currMB, pred_mv, mv_block, min_mcost, lambda_factor);
}

distblk __wrap_EPZS_integer_subMB_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                                    distblk min_mcost, int lambda_factor)
{
  return run(3, currMB, pred_mv, mv_block, min_mcost, lambda_factor);
}

distblk __wrap_EPZSDetermineStopCriterion(EPZSParameters *p_EPZS, distblk *prevSad, MEBlock *mv_block,
                                          distblk lambda_dist)
{
  distblk s = __real_EPZSDetermineStopCriterion(p_EPZS, prevSad, mv_block, lambda_dist);
  g_stop = (int64_t)s;
  return s;
}

short __wrap_EPZS_spatial_predictors(EPZSParameters *p_EPZS, MEBlock *mv_block, int list, int list_offset,
                                     short ref, struct pic_motion_params **mv_info)
{
  short v = __real_EPZS_spatial_predictors(p_EPZS, mv_block, list, list_offset, ref, mv_info);
  g_npred = 5;            /* the caller's prednum starts at 5 (me_epzs.c:137) */
  return v;
}

void __wrap_EPZS_spatial_memory_predictors(EPZSParameters *p_EPZS, MEBlock *mv_block, int list, int *prednum,
                                           int img_width)
{
  __real_EPZS_spatial_memory_predictors(p_EPZS, mv_block, list, prednum, img_width);
  g_npred = *prednum;
}

void __wrap_EPZS_temporal_predictors(Macroblock *currMB, StorablePicture *ref_picture, EPZSParameters *p_EPZS,
                                     MEBlock *mv_block, int *prednum, distblk stopCriterion, distblk min_mcost)
{
  __real_EPZS_temporal_predictors(currMB, ref_picture, p_EPZS, mv_block, prednum, stopCriterion, min_mcost);
  g_npred = *prednum;
}

void __wrap_EPZSWindowPredictors(MotionVector *mv, EPZSStructure *predictor, int *prednum, EPZSStructure *windowPred)
{
  __real_EPZSWindowPredictors(mv, predictor, prednum, windowPred);
  g_npred = *prednum;
}

void __wrap_EPZSBlockTypePredictorsMB(Slice *currSlice, MEBlock *mv_block, SPoint *point, int *prednum)
{
  __real_EPZSBlockTypePredictorsMB(currSlice, mv_block, point, prednum);
  g_npred = *prednum;
}

void __wrap_EPZSBlockTypePredictors(Slice *currSlice, MEBlock *mv_block, SPoint *point, int *prednum)
{
  __real_EPZSBlockTypePredictors(currSlice, mv_block, point, prednum);
  g_npred = *prednum;
}
