/*
 * jm_f3_gpu.c -- SURVEY §8(f)3 in the drop-in (JMME_F3=1; off by default):
 * mode decision's inter residual coding served from the GPU.
 *
 * JM codes the residual of every inter mode it evaluates one 4x4 block at a time
 * through currMB->residual_transform_quant_luma_4x4 (JM/lencod/src/block.c:660-724,
 * called from macroblock.c:874 / 975 for each 4x4 of an 8x8 prediction):
 * check_zero, forward4x4, the quantiser, and -- when a level survives --
 * inverse4x4 and sample_reconstruct into the encoded picture.  For an inter block
 * the inputs are the residual mb_ores (original - motion-compensated prediction)
 * and the prediction mb_pred, both set for the whole macroblock before its first
 * 4x4 is coded, so the first call of a macroblock sends all 16 blocks to
 * jmme_residual4x4 (one launch) and the calls that follow are answered from it.
 *
 * A call is served only when its inputs equal those the GPU computed with --
 * the 4x4 residual and prediction, and the quantiser's parameter set (scale,
 * offset and inverse scale of q_params_4x4[pl][0][qp], qp_per, CAVLC, scan,
 * COEFF_COST4x4[disthres]) -- and only for the plain form of the function with
 * quant_4x4_normal (no adaptive-rounding quantiser, no trellis, frame
 * macroblocks, 4:2:0 luma): everything else, and every intra call (whose
 * prediction is the reconstruction of the block before it), runs JM's own code
 * and is counted.  The served call leaves JM's state exactly as JM's own would:
 * cofAC levels / runs, *coeff_cost, subblock_x / y, tblk16x16, mb_rres and the
 * encoded picture.
 *
 * JM's two scan tables and the coefficient cost table are restated from
 * block.c:72-76 and 169-183 (static there).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "global.h"
#include "mbuffer.h"
#include "block.h"
#include "quant4x4.h"
#include "jmme.h"

extern jmme_ctx *jm_gpu_me_engine(VideoParameters *p_Vid, InputParameters *p_Inp);

static const byte kCoeffCost4x4[2][16] = {{3, 2, 2, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
                                         {9, 9, 9, 9, 9, 9, 9, 9, 9, 9, 9, 9, 9, 9, 9, 9}};
static const byte kSnglScan[16][2] = {{0, 0}, {1, 0}, {0, 1}, {0, 2}, {1, 1}, {2, 0}, {3, 0}, {2, 1},
                                      {1, 2}, {0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 2}, {2, 3}, {3, 3}};

static int g_on = -1;
static long long g_calls, g_served, g_batches, g_refused_form, g_refused_intra, g_refused_inputs;
static jmme_quant4x4_params g_par;                  /* the parameter set of the current batch */
static jmme_resid4x4_req g_req[16];                 /* the batch: the macroblock's 16 blocks, raster order */
static jmme_resid4x4_res g_res[16];
static int g_valid = 0;

int jm_f3_gpu_on(void)
{
  if (g_on < 0) {
    const char *e = getenv("JMME_F3");
    g_on = e && e[0] == '1';
  }
  return g_on;
}

/* the quantiser parameter set JM's call would use (block.c:679-692) */
static void f3_params(Macroblock *m, ColorPlane pl, jmme_quant4x4_params *q)
{
  Slice *s = m->p_Slice;
  VideoParameters *v = m->p_Vid;
  QuantParameters *pq = v->p_Quant;
  const int qp = m->qp_scaled[pl];
  LevelQuantParams **lq = pq->q_params_4x4[pl][0][qp];
  int i, j;
  memset(q, 0, sizeof *q);
  for (j = 0; j < 4; j++)
    for (i = 0; i < 4; i++) {
      q->scale[4 * j + i] = lq[j][i].ScaleComp;
      q->offset[4 * j + i] = lq[j][i].OffsetComp;
      q->inv_scale[4 * j + i] = lq[j][i].InvScaleComp;
    }
  q->qp_per = pq->qp_per_matrix[qp];
  q->is_cavlc = s->symbol_mode == CAVLC;
  memcpy(q->scan, kSnglScan, sizeof q->scan);
  memcpy(q->c_cost, kCoeffCost4x4[s->disthres], 16);
}

static void f3_block(Macroblock *m, ColorPlane pl, int bx, int by, jmme_resid4x4_req *r)
{
  Slice *s = m->p_Slice;
  int **ores = s->mb_ores[pl];
  imgpel **pred = s->mb_pred[pl];
  int i, j;
  for (j = 0; j < 4; j++)
    for (i = 0; i < 4; i++) {
      r->ores[4 * j + i] = ores[by + j][bx + i];
      r->pred[4 * j + i] = pred[by + j][bx + i];
    }
  r->param = 0;
  r->max_pel = m->p_Vid->max_imgpel_value;
}

int jm_f3_gpu_rq4(Macroblock *m, ColorPlane pl, int block_x, int block_y, int *coeff_cost, int intra)
{
  Slice *s = m->p_Slice;
  VideoParameters *v = m->p_Vid;
  jmme_quant4x4_params par;
  jmme_resid4x4_req want;
  const jmme_resid4x4_res *o;
  int k, i, j;
  ++g_calls;
  if (intra) {
    ++g_refused_intra;
    return residual_transform_quant_luma_4x4(m, pl, block_x, block_y, coeff_cost, intra);
  }
  if (pl != PLANE_Y || s->quant_4x4 != quant_4x4_normal || m->is_field_mode || v->yuv_format == YUV444 ||
      (block_x & 3) || (block_y & 3) || block_x > 12 || block_y > 12) {
    ++g_refused_form;
    return residual_transform_quant_luma_4x4(m, pl, block_x, block_y, coeff_cost, intra);
  }
  k = (block_y >> 2) * 4 + (block_x >> 2);
  f3_params(m, pl, &par);
  f3_block(m, pl, block_x, block_y, &want);
  if (!g_valid || memcmp(&par, &g_par, sizeof par) || memcmp(&want, &g_req[k], sizeof want)) {
    /* a new batch: every 4x4 of the macroblock with the inputs JM holds now */
    int b;
    jmme_ctx *ctx = jm_gpu_me_engine(v, m->p_Inp);
    g_par = par;
    for (b = 0; b < 16; b++) f3_block(m, pl, (b & 3) * 4, (b >> 2) * 4, &g_req[b]);
    if (jmme_residual4x4(ctx, &g_par, 1, g_req, g_res, 16)) {
      char buf[600];
      snprintf(buf, sizeof buf, "jm_f3_gpu: jmme_residual4x4: %s", jmme_last_error());
      error(buf, 500);
    }
    g_valid = 1;
    ++g_batches;
    if (memcmp(&want, &g_req[k], sizeof want)) {   /* (cannot differ: read back to back) */
      ++g_refused_inputs;
      g_valid = 0;
      return residual_transform_quant_luma_4x4(m, pl, block_x, block_y, coeff_cost, intra);
    }
  }
  o = &g_res[k];
  ++g_served;
  {
    const int pos_x = block_x >> 2, pos_y = block_y >> 2;
    const int b8 = 2 * (pos_y >> 1) + (pos_x >> 1) + (pl << 2), b4 = 2 * (pos_y & 1) + (pos_x & 1);
    imgpel **img = v->enc_picture->p_curr_img;
    int *acl = s->cofAC[b8][b4][0], *acr = s->cofAC[b8][b4][1];
    if (o->zero) {   /* check_zero found no coefficient (block.c:717-721) */
      acl[0] = 0;
    } else {
      int n;
      m->subblock_x = ((b8 & 1) == 0) ? (((b4 & 1) == 0) ? 0 : 4) : (((b4 & 1) == 0) ? 8 : 12);
      m->subblock_y = (b8 < 2) ? ((b4 < 2) ? 0 : 4) : ((b4 < 2) ? 8 : 12);
      for (j = 0; j < 4; j++)
        for (i = 0; i < 4; i++) s->tblk16x16[block_y + j][block_x + i] = o->coef[4 * j + i];
      for (n = 0; o->levels[n]; n++) {
        acl[n] = o->levels[n];
        acr[n] = o->runs[n];
      }
      acl[n] = 0;
      *coeff_cost += o->cost;
      if (o->nonzero)
        for (j = 0; j < 4; j++)
          for (i = 0; i < 4; i++) s->mb_rres[pl][block_y + j][block_x + i] = o->rres[4 * j + i];
    }
    for (j = 0; j < 4; j++)
      for (i = 0; i < 4; i++) img[m->pix_y + block_y + j][m->pix_x + block_x + i] = o->recon[4 * j + i];
    return o->nonzero;
  }
}

static void report(void) __attribute__((destructor));
static void report(void)
{
  if (g_on != 1) return;
  fprintf(stderr, "jm_f3_gpu: %lld 4x4 residual calls: %lld served from %lld GPU batches; on JM's code: %lld intra, "
          "%lld other forms, %lld input mismatches\n", g_calls, g_served, g_batches, g_refused_intra, g_refused_form,
          g_refused_inputs);
}
