/*
 * jm_noop_me.c -- measurement only, never a product: JM 18.5 lencod with its
 * integer-pel search replaced by a search that costs nothing (it returns at
 * once, keeping the centre).  JM's "Total ME time" (report.c:803) of this
 * binary is the part of the ME time that is JM's own loop around IntPelME
 * (mv_search.c BlockMotionSearch: neighbours, predictors, get_original_block,
 * set_me_parameters, mode-decision bookkeeping), which no search engine can
 * remove.  The bitstream is NOT the stock encoder's.
 */
#include "global.h"

distblk __wrap_full_search_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                             distblk min_mcost, int lambda_factor)
{
  (void)currMB; (void)pred_mv; (void)mv_block; (void)lambda_factor;
  return min_mcost;
}

distblk __wrap_fast_full_search_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                                  distblk min_mcost, int lambda_factor)
{
  (void)currMB; (void)pred_mv; (void)mv_block; (void)lambda_factor;
  return min_mcost;
}

/* sub_pel_motion_estimation (me_fullsearch.c:186-289): no refinement either,
 * so the sub-pel-on rows have a floor too (the vector stays the integer one) */
distblk __wrap_sub_pel_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                         distblk min_mcost, int *lambda_factor)
{
  (void)currMB; (void)pred_mv; (void)mv_block; (void)lambda_factor;
  return min_mcost;
}

/* the fast-full-search surface JM would build on the CPU: not built */
void __wrap_setup_fast_full_search(Macroblock *currMB, MEBlock *mv_block, int list)
{
  (void)currMB; (void)mv_block; (void)list;
}
