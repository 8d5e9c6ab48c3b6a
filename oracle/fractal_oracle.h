/*
 * fractal_oracle.h -- TEST INFRASTRUCTURE: plain-C restatement of the thesis
 * codec's fractal domain-range block matching:
 *   compute_domain_Sum / compute_range_Sum   ZL/src/compute.c:277-~1091
 *   compute_rms, compute_rdSum, QUAN_A       ZL/src/compute.c:6-215,
 *                                            ZL/inc/defines_enc.h:19-22,591-601
 *   full_search, bound_chk                   ZL/src/block_enc.c:1933-1977, 2894-2919
 *   encode_one_macroblock quadtree gating    ZL/src/block_enc.c:508-1050 (row a17),
 *     encode_block_rect / _8 / _4            ZL/src/block_enc.c:1072-1932
 * (ZL = /root/reference/2.论文程序/ZhangLing_Yu_version1/H264Fractal).
 *
 * PARITY UNPINNED: the thesis sources need a windows.h stand-in to compile,
 * which makes them unbuildable here under this project's rules, and the
 * reference ships no reproducible fixture for this path (ZLD/trans_show_*.txt
 * lack their input).  This restatement is therefore checked by known-answer
 * tests (planted affine maps) and is the checker for csrc/jmme_fractal.hip.
 *
 * Planes are 8-bit, row-major with a pitch.  Only tests/, smoke() and the
 * bench CPU legs may load this library.
 */
#ifndef FRACTAL_ORACLE_H
#define FRACTAL_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* compute_domain_Sum: sum and sum of squares of every bsx x bsy box, at every
 * position (i, j), i < H-bsy+1, j < W-bsx+1 (out row stride W-bsx+1). */
void fro_box_sums(const uint8_t *plane, int pitch, int W, int H, int bsx, int bsy, double *sum, double *sum2);

/* compute_rms for range block (bx, by) against domain block (m, n), both
 * bsx x bsy.  Writes alpha (scale) and beta (offset); returns rms (1e30 when
 * the quantised parameters fall outside [MIN_ALPHA, MAX_ALPHA] x
 * [MIN_BETA, MAX_BETA]). */
double fro_compute_rms(const uint8_t *org, const uint8_t *ref, int pitch, int bx, int by, int m, int n, int bsx,
                       int bsy, double *alpha, double *beta);

/* full_search: (0,0) first, then rings l = 1..R in the thesis spiral, domain
 * blocks restricted by bound_chk to the picture W x H; strict '<'.  out_x/out_y
 * stay 0 when (0,0) wins (the caller initialises the TRANS_NODE). */
double fro_full_search(const uint8_t *org, const uint8_t *ref, int pitch, int W, int H, int R, int bx, int by,
                       int bsx, int bsy, int *out_x, int *out_y, double *scale, double *offset);

/* batch form: req int32 [n][4] = (bx, by, bsx, bsy); out double [n][3] =
 * (rms, scale, offset), xy int32 [n][2] */
void fro_full_search_batch(const uint8_t *org, const uint8_t *ref, int pitch, int W, int H, int R, int n,
                           const int32_t *req, double *out, int32_t *xy);

/* One TRANS_NODE of the fractal tree (ZL/inc/defines_enc.h TRANS_NODE fields
 * x, y, scale, offset, reference, partition) plus the rms its search returned.
 * Same layout as jmme_fractal_node in include/jmme.h. */
typedef struct fro_node {
  double rms, scale, offset;
  int32_t x, y, reference, partition;
} fro_node;                                  /* 40 bytes */

/* one macroblock's tree: mb = trans[0][CurMb]; b8[q] = its next[q] (when
 * mb.partition == 3); sub[q][c] = b8[q].next[c] (2 rect halves for partition
 * 1/2, 4 4x4 blocks for partition 3); unused nodes are zero.  chun is the
 * squared correlation the 16x16 gate reads.  Same layout as jmme_fractal_mb. */
typedef struct fro_mb {
  fro_node mb, b8[4], sub[4][4];
  double chun;
} fro_mb;                                    /* 848 bytes */

/* encode_one_macroblock for every 16x16 macroblock of a W x H plane (raster
 * order, W and H multiples of 16), search_mode 0 (full search), one region
 * (num_regions == 1), the C view with n_refs reference planes searched in
 * order (refs[0] = its own reference frame, then the H, M, N views:
 * block_enc.c:563-700), tolerances tol_16 / tol_8 as in the config file. */
void fro_encode_mbs(const uint8_t *org, const uint8_t *const *refs, int n_refs, int pitch, int W, int H, int R,
                    double tol_16, double tol_8, fro_mb *out);

/* decode_one_macroblock / decode_block_rect / decode_block_8 / decode_block_4
 * (ZL/src/block_dec.c:20-1160), num_regions == 1, for every macroblock of a
 * W x H plane of component `component` (1 = Y, 2 = U, 3 = V), from the trees
 * fro_encode_mbs produces (16x16 leaves, 8x8 leaves, 8x4 / 4x8 pairs, 4x4).
 * views[k] is the plane the decoder reads for reference k (the thesis's
 * imgY_ref, _h, _m, _n, or the chroma equivalents).  Each leaf pixel is
 *   (unsigned char) bound(0.5 + scale*d + offset - scale*avg),
 * avg = (box sum of the domain block) / n.  Returns 0, or -1 when a leaf maps
 * to a view index >= n_views (the per-level view quirks can map reference 1
 * to view 3) or its domain block leaves the plane; rec is W x H, pitch bytes
 * per row. */
int fro_decode_mbs(const fro_mb *mbs, const uint8_t *const *views, int n_views, int pitch, int W, int H,
                   int component, uint8_t *rec);

#ifdef __cplusplus
}
#endif
#endif
