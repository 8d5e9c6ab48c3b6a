/*
 * epzs_oracle.h -- TEST INFRASTRUCTURE: plain-C restatement of JM 18.5's EPZS
 * integer-pel search, the checker for
 * csrc/jmme_epzs.hip.  JM = /root/reference/4.对比程序/jm18.5/JM:
 *   EPZS_motion_estimation        JM/lencod/src/me_epzs.c:54-407   (variant 0)
 *   EPZS_subMB_motion_estimation  JM/lencod/src/me_epzs.c:417-780  (variant 1)
 *   search patterns               JM/lencod/src/me_epzs_common.c:46-80, 176-230, 530-565
 *   computeSAD / UMVLine4X        JM/lencod/src/me_distortion.c:349-426, inc/refbuf.h:22-26
 *   mv_cost, weighted_cost        JM/lencod/inc/mv_search.h:87-112
 * The predictor list, the stop criterion and the prevSad slot are the state
 * JM builds on the host before the candidate search (me_epzs_common.c), and
 * are inputs here, as are the EPZSMap cells that already hold the search's
 * BlkCount (the uint16 map is never cleared; me_epzs.c:92-94).
 * Pinned against JM itself: tests/golden/epzs_*.npz hold every EPZS call of
 * real lencod runs (oracle/capture/jm_epzs_capture.c).
 *
 * Request / result layouts equal jmme_epzs_req / jmme_epzs_res (include/jmme.h).
 */
#ifndef EPZS_ORACLE_H
#define EPZS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Sample type of the planes: 8-bit, or JM's 16-bit imgpel for SourceBitDepthLuma
 * 9..14 (build/libepzs_oracle16.so is this file compiled with -DEO_PEL16). */
#ifdef EO_PEL16
typedef uint16_t eo_pel;
#else
typedef uint8_t eo_pel;
#endif

typedef struct eo_req {
  int16_t pos_x, pos_y, bsx, bsy;
  int16_t blocktype, ref_idx;
  int16_t pred_x, pred_y, center_x, center_y;
  int16_t max_x, max_y;
  int32_t lambda;
  uint8_t variant, flags, pattern, dual;
  int32_t n_pred, pred_off;
  int32_t n_stale, stale_off;
  int32_t plane;
  int32_t pad;
  int64_t prev_sad, medthres, stop_crit;
} eo_req;                       /* 80 bytes */

typedef struct eo_res {
  int16_t mv_x, mv_y;
  int32_t path;
  int64_t cost, prev_sad;
} eo_res;                       /* 24 bytes */

/* one search; cur / ref 8-bit W x H planes with `pitch`; preds / stale are
 * (x, y) int16 pairs (stale: qpel offsets from the centre) */
void eo_epzs(const eo_req *q, const int16_t *preds, const int16_t *stale, const eo_pel *cur, const eo_pel *ref,
             int pitch, int W, int H, eo_res *out);

/* batch: request i searches ref plane refs[q.plane] */
void eo_epzs_batch(const eo_req *q, int n, const int16_t *preds, const int16_t *stale, const eo_pel *cur,
                   const eo_pel *const *refs, int pitch, int W, int H, eo_res *out);

/* EPZSSubPelGrid = 1 (variants 2 EPZS_integer_motion_estimation, 3
 * EPZS_integer_subMB_motion_estimation, JM/lencod/src/me_epzs_int.c:41-782):
 * subs = the reference's 16 padded sub-images (plane dy*4+dx, (H+40) x (W+64)
 * 8-bit, getSubImagesLuma layout, subpel_oracle.h).  Extra paths: 6 = the
 * subMB predictor-loop prevSad exit (mv untouched), 7 = the post-predictor
 * prevSad exit of variant 2 (mv = best). */
void eo_epzs_grid(const eo_req *q, const int16_t *preds, const int16_t *stale, const eo_pel *cur, int pitch,
                  const eo_pel *subs, int W, int H, eo_res *out);
void eo_epzs_grid_batch(const eo_req *q, int n, const int16_t *preds, const int16_t *stale, const eo_pel *cur,
                        int pitch, const eo_pel *const *subs, int W, int H, eo_res *out);

/* Speculative searches (the drop-in's EPZS batches): with the predictor
 * conditions of jmme_epzs_search_ex (cond[i] = JMME_EPZS_PRED_*, NULL: all
 * unconditional; the list JM searches is the entries whose condition holds for
 * the centre's cost) and the validity intervals of the result: the same result
 * (mv, cost, visited cells, p_motion) for every stop criterion in
 * [stop_lo, stop_hi] and prevSad in [prev_lo, prev_hi] (each comparison with
 * either value is monotone in it; P <= S, which holds both, is pinned on the
 * given P).  prev_written: JM stores *prevSad = cost at this return (else it
 * leaves *prevSad alone).  n_visited and vis (may be NULL; up to max_vis pairs):
 * the EPZSMap cells the search stamped, (dx, dy) qpel from the centre, in cell
 * (row-major) order.  Layout = jmme_epzs_bounds. */
typedef struct eo_bounds {
  int64_t stop_lo, stop_hi, prev_lo, prev_hi;
  int32_t prev_written, n_visited;
} eo_bounds;                    /* 40 bytes */

void eo_epzs_ex(const eo_req *q, const int16_t *preds, const uint8_t *cond, const int16_t *stale, const eo_pel *cur,
                const eo_pel *ref, int pitch, int W, int H, eo_res *out, eo_bounds *bnd, int16_t *vis, int max_vis);
void eo_epzs_grid_ex(const eo_req *q, const int16_t *preds, const uint8_t *cond, const int16_t *stale,
                     const eo_pel *cur, int pitch, const eo_pel *subs, int W, int H, eo_res *out, eo_bounds *bnd,
                     int16_t *vis, int max_vis);
/* batches: cond (may be NULL) parallel to preds, indexed by pred_off like them; vis: max_vis pairs per request */
void eo_epzs_ex_batch(const eo_req *q, int n, const int16_t *preds, const uint8_t *cond, const int16_t *stale,
                      const eo_pel *cur, const eo_pel *const *refs, int pitch, int W, int H, eo_res *out,
                      eo_bounds *bnd, int16_t *vis, int max_vis);
void eo_epzs_grid_ex_batch(const eo_req *q, int n, const int16_t *preds, const uint8_t *cond, const int16_t *stale,
                           const eo_pel *cur, int pitch, const eo_pel *const *subs, int W, int H, eo_res *out,
                           eo_bounds *bnd, int16_t *vis, int max_vis);

#ifdef __cplusplus
}
#endif
#endif
