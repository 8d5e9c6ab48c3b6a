/*
 * me_oracle.h -- TEST INFRASTRUCTURE: plain-C restatement of the JM 18.5
 * integer-pel motion-estimation path.  This is the CHECKER for the HIP
 * product path; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  It is never linked into libjmme.
 *
 * Parity of this restatement is pinned against golden vectors captured from
 * the real JM 18.5 lencod (oracle/_ref/lencod_capture, see
 * tests/golden/make_golden.py) -- tests/test_oracle_golden.py.
 *
 * Every function cites the JM file:line it restates
 * (JM = /root/reference/4.对比程序/jm18.5/JM).
 */
#ifndef ME_ORACLE_H
#define ME_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* JM lencod/inc/defines.h:135  DISTBLK_MAX = (int64)INT_MAX << LAMBDA_ACCURACY_BITS */
#define ORA_DISTBLK_MAX (((int64_t)0x7fffffff) << 5)

/* spiral_qpel_search[] of JM lencod/src/mv_search.c:406-442, in INTEGER pels
 * (qpel table = this << 2).  out must hold (2R+1)^2 pairs (x,y). */
int ora_spiral(int search_range, int16_t *out_xy);

/* mvbits[] of JM lencod/src/mv_search.c:342-374 built by JM's own loop.
 * Fills out[0 .. 2*max_mvd] with out[max_mvd + v] = mvbits[v]; returns max_mvd. */
int ora_mvbits_table(int search_range, int32_t *out, int out_len);

/* Full search, restating full_search_motion_estimation
 * (JM lencod/src/me_fullsearch.c:39-103) with computeSAD
 * (JM lencod/src/me_distortion.c:349-426, incl. the row early exit) and
 * UMVLine4X (JM lencod/inc/refbuf.h:22-26).
 * cur/ref: W x H uint16 luma planes (row stride W).
 * pos_x,pos_y: block origin (pels); bsx,bsy: block size;
 * pred, center: qpel MVs (relative to the block) as JM passes them;
 * search_range: integer pels (imin(max_x,max_y)>>2, me_fullsearch.c:49);
 * check_for_00: (blocktype==1 && !rdopt && !B && ref==0), me_fullsearch.c:61.
 * min_mcost_in: what BlockMotionSearch passes (DISTBLK_MAX, mv_search.c:878).
 * Returns min_mcost (int64); writes best mv (qpel) to out_mv[0..1].
 * Returns -1 for unsupported input (sub-pel centre). */
int64_t ora_full_search(const uint16_t *cur, const uint16_t *ref, int W, int H,
                        int pos_x, int pos_y, int bsx, int bsy,
                        int pred_x, int pred_y, int center_x, int center_y,
                        int search_range, int lambda, int check_for_00,
                        int64_t min_mcost_in, int16_t *out_mv);

/* FFS SAD surface, restating setup_fast_full_search's SAD loop
 * (JM lencod/src/me_fullfast.c:492-556): 16 4x4 SADs of the 16x16 MB at
 * every spiral position around the (unpadded, already clipped) search centre.
 * out: [16][ (2R+1)^2 ] uint32, block index = (by<<2)+bx. */
void ora_ffs_surface(const uint16_t *cur, const uint16_t *ref, int W, int H,
                     int mb_x, int mb_y, int center_x, int center_y,
                     int surf_range, uint32_t *out);

/* update_full_search_large_blocks (JM lencod/src/me_fullfast.c:196-260):
 * in: t7[16][P]; out: all[8][16][P] (blocktypes 1..7, JM block indexing). */
void ora_ffs_aggregate(const uint32_t *t7, int P, uint32_t *all);

/* fast_full_search_motion_estimation (JM lencod/src/me_fullfast.c:618-689)
 * for one block, given the MB's surface `all` from ora_ffs_aggregate.
 * block_range: imax(max_x,max_y)>>2 (me_fullfast.c:627).
 * max_mvd: p_Vid->max_mvd.  rdopt: p_Inp->rdopt.  pos00: p_ffast_me->pos_00.
 * Returns min_mcost; writes mv (qpel). */
int64_t ora_ffs_block(const uint32_t *all, int surf_range,
                      int blocktype, int block_x, int block_y,
                      int center_x, int center_y, int pred_x, int pred_y,
                      int block_range, int lambda, int max_mvd, int rdopt,
                      int pos00, int64_t min_mcost_in, int16_t *out_mv);

/* Batch helper for the CPU baseline / large tests: nreq full searches.
 * req: nreq x ORA_REQ_FIELDS int32 in the order of ora_full_search's args
 *   [pos_x,pos_y,bsx,bsy,pred_x,pred_y,center_x,center_y,search_range,lambda,check_for_00]
 * Single-threaded (JM is). */
#define ORA_REQ_FIELDS 11
void ora_full_search_batch(const uint16_t *cur, const uint16_t *ref, int W, int H,
                           int nreq, const int32_t *req, int16_t *out_mv, int64_t *out_cost);

/* Per-MB FFS for a batch of MBs (setup + all listed blocks), single-threaded.
 * mbs: nmb x 4 int32 [mb_x, mb_y, center_x, center_y] (centre qpel, unpadded)
 * blk: nblk x 9 int32 [mb_index, blocktype, block_x, block_y, pred_x, pred_y,
 *                       block_range, lambda, pos00]
 */
void ora_ffs_batch(const uint16_t *cur, const uint16_t *ref, int W, int H,
                   int surf_range, int max_mvd, int rdopt,
                   int nmb, const int32_t *mbs, int nblk, const int32_t *blk,
                   int16_t *out_mv, int64_t *out_cost);

#ifdef __cplusplus
}
#endif
#endif
