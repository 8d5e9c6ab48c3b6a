/*
 * tq_oracle.h -- TEST INFRASTRUCTURE: plain-C restatement of JM 18.5's
 * integer transforms (lcommon/src/transform.c), 4x4 quantisation
 * (lencod/src/quant4x4_normal.c) and Hadamard SATD (lencod/src/
 * me_distortion.c).  The checker for csrc/jmme_tq.hip; never linked into
 * libjmme.  Pinned against the real JM functions: tests/golden/tq_jm.npz.
 *
 * Blocks are flat row-major int arrays: b[r*N + c] == JM block[pos_y+r][pos_x+c].
 */
#ifndef TQ_ORACLE_H
#define TQ_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

void tqo_forward4x4(const int *in, int *out);     /* transform.c:20-68 */
void tqo_inverse4x4(const int *in, int *out);     /* transform.c:70-119 */
void tqo_hadamard4x4(const int *in, int *out);    /* transform.c:121-169 */
void tqo_ihadamard4x4(const int *in, int *out);   /* transform.c:171-218 */
void tqo_hadamard4x2(const int *in, int *out);    /* transform.c:220-258, 2x4 in, 2x4 out */
void tqo_ihadamard4x2(const int *in, int *out);   /* transform.c:260-300, 2x4 in, 4x2 out */
void tqo_hadamard2x2(const int *in, int *out);    /* transform.c:302-315 */
void tqo_ihadamard2x2(const int *in, int *out);   /* transform.c:317-331 */
void tqo_forward8x8(const int *in, int *out);     /* transform.c:353-448 */
void tqo_inverse8x8(const int *in, int *out);     /* transform.c:450-528 */

int tqo_hadamard_sad4x4(const int16_t *diff);     /* me_distortion.c:175-258 */
int tqo_hadamard_sad8x8(const int16_t *diff);     /* me_distortion.c:266-341 */

/* quant_4x4_normal's inputs for one block (quant4x4_normal.c:39-110):
 * scale/offset/inv_scale = q_params_4x4[j][i].{ScaleComp,OffsetComp,
 * InvScaleComp} at [j*4+i]; scan = pos_scan (horizontal, vertical);
 * c_cost = COEFF_COST4x4[disthres] (block.c:72). */
typedef struct tqo_quant4x4_params {
  int32_t scale[16], offset[16], inv_scale[16];
  int32_t qp_per;          /* p_Quant->qp_per_matrix[qp] */
  int32_t is_cavlc;
  uint8_t scan[16][2];
  uint8_t c_cost[16];
} tqo_quant4x4_params;

/* in place: coef = the dequantised block; levels[0..16] = ACLevel (0-terminated),
 * runs = ACRun; *coeff_cost accumulates; returns nonzero */
int tqo_quant_4x4_normal(int *coef, const tqo_quant4x4_params *q, int32_t *levels, int32_t *runs,
                         int32_t *coeff_cost);

#ifdef __cplusplus
}
#endif
#endif
