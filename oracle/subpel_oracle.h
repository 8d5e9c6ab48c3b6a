/*
 * subpel_oracle.h -- TEST INFRASTRUCTURE: plain-C restatement of JM 18.5's
 * quarter-pel reference interpolation and sub-pel motion refinement
 * (SURVEY.md §8(f) rank 1).  The checker for csrc/jmme_subpel.hip; never
 * linked into libjmme.  Pinned against the real JM functions through
 * oracle/capture/jm_subpel_capture.c -> tests/golden/subpel_*.npz.
 *
 * JM = /root/reference/4.对比程序/jm18.5/JM.
 */
#ifndef SUBPEL_ORACLE_H
#define SUBPEL_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPO_PAD_Y 20   /* IMG_PAD_SIZE_Y, JM/lencod/inc/defines.h */
#define SPO_PAD_X 32   /* IMG_PAD_SIZE_X */

/* getSubImagesLuma (JM/lencod/src/img_luma.c:611-680, OnTheFlyFractMCP 0):
 * src = W x H luma (row stride W, 8-bit content in uint16), out = 16 planes
 * [dy*4+dx] of (H+2*SPO_PAD_Y) x (W+2*SPO_PAD_X) uint16, row (j+SPO_PAD_Y),
 * column (i+SPO_PAD_X) holding JM's p_curr_img_sub[dy][dx][j][i]. */
void spo_sub_images(const uint16_t *src, int W, int H, uint16_t *out);

/* The interpolation's clip bound, JM's max_imgpel_value = (1 << bits) - 1
 * (SourceBitDepthLuma); 8 unless set.  Process-wide. */
void spo_set_bitdepth(int bits);

/* One sub-pel refinement with JM's inputs.  sub = spo_sub_images() output of
 * the reference; cur = W x H current picture.  Metrics: 0 SAD (computeSAD,
 * me_distortion.c:349-426), 1 SSE (computeSSE :1189-1240), 2 SATD
 * (computeSATD :745-825, 4x4 or, with test8x8, 8x8 Hadamard). */
typedef struct spo_req {
  int pos_x, pos_y, bsx, bsy, blocktype, ref;
  int pred_x, pred_y;            /* qpel */
  int mv_x, mv_y;                /* mv_block->mv[list] on entry, qpel */
  int64_t min_mcost;
  int lambda_h, lambda_q;
  int rdopt, slice_type;         /* slice_type: JM's P_SLICE = 0, B_SLICE = 1 */
  int start_hp, start_qp;
  int metric_h, metric_q;
  int test8x8;
  int search_pos2, search_pos4;
  int64_t subthres;              /* EPZS only: p_EPZS->subthres[blocktype] */
} spo_req;

/* sub_pel_motion_estimation, JM/lencod/src/me_fullsearch.c:186-289.
 * Returns min_mcost; out_mv[0..1] = mv_block->mv[list] on return. */
int64_t spo_sub_pel_me(const uint16_t *cur, const uint16_t *sub, int W, int H, const spo_req *r, int16_t *out_mv);

/* EPZS_sub_pel_motion_estimation, JM/lencod/src/me_epzs_sub.c:30-222. */
int64_t spo_epzs_sub_pel_me(const uint16_t *cur, const uint16_t *sub, int W, int H, const spo_req *r,
                            int16_t *out_mv);

/* Batch helpers for the Python tests: rows of spo_req, one reference. */
void spo_sub_pel_batch(const uint16_t *cur, const uint16_t *sub, int W, int H, const spo_req *r, int n,
                       int epzs, int16_t *out_mv, int64_t *out_cost);

#ifdef __cplusplus
}
#endif
#endif
