/*
 * jmme.h -- C ABI of the MI355X-native (gfx950) JM 18.5 integer-pel motion
 * estimation engine (libjmme.so).  Plain C types only; no HIP/torch types.
 *
 * What it replaces in JM 18.5 lencod (JM = /root/reference/4.对比程序/jm18.5/JM):
 *
 *   jmme_full_search_block()      <- currMB->IntPelME = full_search_motion_estimation
 *                                    signature JM/lencod/inc/global.h:459,
 *                                    body JM/lencod/src/me_fullsearch.c:39-103,
 *                                    assigned JM/lencod/src/mv_search.c:139-175
 *   jmme_fast_full_search_block() <- currMB->IntPelME = fast_full_search_motion_estimation
 *                                    (global.h:459, JM/lencod/src/me_fullfast.c:618-689) with
 *                                    currMB->p_SetupFastFullPelSearch = setup_fast_full_search
 *                                    (global.h:469, me_fullfast.c:269-608)
 *   jmme_search_mbs()             <- the same two searches batched per macroblock x
 *                                    reference: one unit = the 41 partitions
 *                                    PartitionMotionSearch / SubPartitionMotionSearch
 *                                    issue for one MB (mv_search.c:1564,1686)
 *   jmme_upload_cur/_ref()        <- the frame buffers JM's searches read:
 *                                    p_Vid->pCurImg (image.c:2868, get_mem2Dpel layout,
 *                                    JM/lcommon/src/memalloc.c:864) and the reference
 *                                    StorablePicture::imgY (get_mem2Dpel_pad,
 *                                    memalloc.c:881; filled at store_picture_in_dpb,
 *                                    mbuffer.c:2116-2122)
 *   jmme_config_parse()           <- Configure()/ParseContent for the ME keys of
 *                                    encoder.cfg (JM/lencod/src/configfile.c:314,
 *                                    Map[] JM/lencod/inc/configfile.h:32-615)
 *
 * Error behaviour: every call returns a status (0 = OK, <0 = error) and
 * jmme_last_error() describes the last failure of the calling thread.  The
 * JM-signature wrappers mirror JM's error(): they print and exit(500) on
 * failure, because JM has no error return on that path.
 *
 * Numerics: bit-exact with JM 18.5 (JCOST_CALC_SCALEUP=1, imgpel=uint16,
 * distblk=int64).  8-bit content only in this version (BitDepthLuma 8):
 * uploads with a sample > 255 are rejected.
 */
#ifndef JMME_H
#define JMME_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef uint16_t jmme_imgpel;   /* JM imgpel, IMGTYPE 1 (JM/lcommon/inc/typedefs.h:35) */
typedef int64_t  jmme_distblk;  /* JM distblk (typedefs.h:37) */

#define JMME_DISTBLK_MAX (((int64_t)0x7fffffff) << 5)  /* JM/lencod/inc/defines.h:135 */
#define JMME_NSLOT 41           /* partitions per macroblock (7 block types) */
#define JMME_MAX_RANGE 64       /* largest integer-pel search range supported */

typedef struct jmme_mv { int16_t mv_x, mv_y; } jmme_mv;  /* JM MotionVector, quarter-pel */

/* SearchMode values, JM/lcommon/inc/types.h:126-133 */
enum { JMME_FULL_SEARCH = -1, JMME_FAST_FULL_SEARCH = 0, JMME_UM_HEX = 1,
       JMME_UM_HEX_SIMPLE = 2, JMME_EPZS = 3 };

/* The motion-estimation subset of JM's InputParameters, with encoder.cfg key
 * names (JM/lencod/inc/configfile.h line of each Map entry in brackets). */
typedef struct jmme_config {
  int SourceWidth;            /* [76]  */
  int SourceHeight;           /* [77]  */
  int SearchMode;             /* [407] -1 FS, 0 FFS, 1 UMHEX, 2 sUMHEX, 3 EPZS */
  int SearchRange;            /* [62]  integer pels */
  int NumberReferenceFrames;  /* [63]  */
  int DisableSubpelME;        /* [61]  */
  int RDOptimization;         /* [153] rdopt */
  int MEDistortionFPel;       /* [278] 0 SAD, 1 SSE, 2 SATD */
  int MDDistortion;           /* [281] */
  int EPZSSubPelGrid;         /* [435] */
  int RestrictSearchRange;    /* [401] full_search */
  int UseMVLimits;            /* [403] */
  int SetMVXLimit;            /* [404] */
  int SetMVYLimit;            /* [405] */
  int ChromaMEEnable;         /* [275] must be 0 in this version */
  int SourceBitDepthLuma;     /* [332] must be 8 in this version */
} jmme_config;

/* ---- configuration ------------------------------------------------------ */
/* JM defaults (InitParams, JM/lcommon/src/config_common.c:297, for these keys). */
int jmme_config_default(jmme_config *cfg);
/* Parse a JM encoder.cfg (may be NULL) then `-p Key=Value` overrides
 * (argv holds "Key=Value" strings), as lencod -d file -p k=v does.
 * Unknown keys are ignored (JM warns); malformed values fail. */
int jmme_config_parse(jmme_config *cfg, const char *cfg_path, int argc, const char *const *argv);
/* p_Vid->max_mvd for this config (JM/lencod/src/mv_search.c:321-328). */
int jmme_max_mvd(const jmme_config *cfg);

/* ---- context ------------------------------------------------------------ */
typedef struct jmme_ctx jmme_ctx;
/* device < 0: current HIP device.  Returns NULL on error. */
jmme_ctx *jmme_create(const jmme_config *cfg, int device);
void jmme_destroy(jmme_ctx *ctx);
const char *jmme_last_error(void);
const char *jmme_version(void);

/* ---- frame buffers (JM get_mem2Dpel / get_mem2Dpel_pad layout) ----------
 * rows[y] points at sample (0, y) of the UNPADDED picture; rows are equally
 * spaced (one allocation), so a single strided copy moves the plane.
 * The reference must be the reconstructed picture JM stores in the DPB. */
int jmme_upload_cur(jmme_ctx *ctx, const jmme_imgpel *const *rows, int width, int height);
int jmme_upload_ref(jmme_ctx *ctx, int list, int ref_idx,
                    const jmme_imgpel *const *rows, int width, int height);

/* ---- batched search: one unit = one macroblock x one reference ----------
 * Slot order of the 41 partitions (jmme_slot()):
 *   0 16x16 | 1-2 16x8 | 3-4 8x16 | 5-8 8x8 | 9-16 8x4 | 17-24 4x8 | 25-40 4x4
 * Per-slot inputs are exactly what JM hands the IntPelME call for that
 * partition (BlockMotionSearch, mv_search.c:916-960). */
typedef struct jmme_block_req {
  int16_t pred_x, pred_y;     /* MV predictor (qpel)                           */
  int16_t center_x, center_y; /* FS: search centre mv_block->mv[list] (qpel)   */
  int16_t search_range;       /* FS: imin(max_x,max_y)>>2; FFS: imax(...)>>2    */
  int16_t flags;              /* JMME_BLK_* */
  int32_t lambda;             /* lambda_factor[F_PEL] */
} jmme_block_req;             /* 16 bytes */

#define JMME_BLK_CHECK00 1    /* FS: (0,0) bonus, me_fullsearch.c:61,78-82 */

typedef struct jmme_mb_req {
  int16_t mb_x, mb_y;         /* macroblock origin (luma pels)                 */
  int16_t list, ref_idx;      /* which uploaded reference                      */
  uint64_t slot_mask;         /* bit s set = slot s is searched                */
  int16_t ffs_center_x;       /* FFS: search_center[list][ref] (qpel)          */
  int16_t ffs_center_y;
  int16_t ffs_range;          /* FFS: max_search_range[list][ref] (pels)       */
  int16_t ffs_pos00_valid;    /* FFS: !rdopt pre-seed of (0,0) enabled          */
  int16_t reserved[4];        /* zero; keeps blk[] 16-byte aligned              */
  jmme_block_req blk[JMME_NSLOT];
} jmme_mb_req;                /* 32 + 41*16 = 688 bytes */

typedef struct jmme_block_res {
  int16_t mv_x, mv_y;         /* best mv (qpel), mv_block->mv[list] on return  */
  int32_t reserved;
  int64_t cost;               /* min_mcost JM returns (distblk)                 */
} jmme_block_res;             /* 16 bytes */

/* slot of (blocktype 1..7, block_x, block_y in 4x4 units), -1 if invalid */
int jmme_slot(int blocktype, int block_x, int block_y);

/* mode = JMME_FULL_SEARCH or JMME_FAST_FULL_SEARCH.  Host arrays, synchronous.
 * out has n * JMME_NSLOT entries (unsearched slots are left untouched). */
int jmme_search_mbs(jmme_ctx *ctx, int mode, const jmme_mb_req *req, int n, jmme_block_res *out);
/* ---- Chained partition searches (the drop-in's guesses inside one macroblock)
 * JM searches a macroblock's partitions one at a time, and a partition's MV
 * predictor (GetMotionVectorPredictorNormal, JM/lcommon/src/mv_prediction.c:192)
 * reads the vectors its neighbours inside the macroblock were just given
 * (set_me_parameters after each search, mv_search.c:1614,1705-1720).  A chain
 * is such a run of partitions -- the rest of a 16x8 / 8x16 pair, or one
 * sub-mode of one 8x8 quadrant -- whose neighbours are either fixed (decided
 * before the chain starts: neighbouring macroblocks, earlier quadrants) or an
 * earlier step of the same chain.  The GPU derives each step's predictor and
 * centre exactly as BlockMotionSearch does (mv_search.c:896-956) from those
 * neighbours and the previous steps' results, and searches it.  Single
 * reference, integer-pel only (the neighbours' vectors are integer results);
 * the caller uses a result only when JM's real call carries the same inputs. */
#define JMME_CHAIN_MAX_STEPS 4
#define JMME_NB_UNAVAILABLE (-1)
#define JMME_NB_FIXED (-2)
#define JMME_CHAIN_CHECK00 1   /* jmme_chain_step.flags: check_for_00 (a 16x16 step, FS, me_fullsearch.c:61) */

typedef struct jmme_chain_nb {
  int16_t src;                 /* JMME_NB_UNAVAILABLE, JMME_NB_FIXED, or k >= 0: step k's result */
  int16_t ref_idx;             /* JMME_NB_FIXED: mv_info[y][x].ref_idx[list] */
  int16_t mv_x, mv_y;          /* JMME_NB_FIXED: mv_info[y][x].mv[list] (qpel) */
} jmme_chain_nb;               /* 8 bytes */

typedef struct jmme_chain_step {
  int16_t slot;                /* partition (jmme_slot) */
  int16_t flags;               /* JMME_CHAIN_CHECK00 */
  jmme_chain_nb nb[3];         /* get_neighbors' block[0] (left), [1] (up), [2] (up-right, else up-left) */
  int16_t sr_min_x, sr_max_x;  /* mv_block->searchRange after get_search_range (qpel) */
  int16_t sr_min_y, sr_max_y;
} jmme_chain_step;             /* 36 bytes */

typedef struct jmme_chain {
  int16_t mb_x, mb_y;          /* macroblock origin (luma pels) */
  int16_t list, ref_idx;       /* the uploaded reference; also the in-chain neighbours' ref_idx */
  int16_t n_steps;             /* 1..JMME_CHAIN_MAX_STEPS */
  int16_t rdopt;               /* p_Inp->rdopt (the centre clip of mv_search.c:939-955 runs when 0) */
  int16_t ffs_center_x, ffs_center_y, ffs_range, ffs_pos00_valid;   /* FFS: the macroblock's surface */
  int16_t mv_lim_x0, mv_lim_x1;   /* p_Vid->MaxHmvR[4], [5] (clip_mv_range, Q_PEL) */
  int16_t mv_lim_y0, mv_lim_y1;   /* p_Vid->MaxVmvR[4], [5] */
  int32_t lambda;              /* lambda_factor[F_PEL] */
  jmme_chain_step steps[JMME_CHAIN_MAX_STEPS];
} jmme_chain;                  /* 32 + 4 * 36 = 176 bytes */

typedef struct jmme_chain_res {
  int16_t pred_x, pred_y;      /* the step's derived predictor (qpel) */
  int16_t center_x, center_y;  /* FS: mv_block->mv[list] on entry to IntPelME */
  int16_t range_min, range_max;   /* min / max(searchRange.max_x, .max_y) >> 2 after CheckSearchRange */
  int16_t mv_x, mv_y;          /* the search's answer (before JM's clip_mv_range) */
  int64_t cost;
} jmme_chain_res;              /* 24 bytes */

/* jmme_search_mbs plus chains, one launch round trip: res[i * JMME_CHAIN_MAX_STEPS + k] is step k of chain i. */
int jmme_search_mbs_chains(jmme_ctx *ctx, int mode, const jmme_mb_req *req, int n, jmme_block_res *out,
                           const jmme_chain *chains, int n_chains, jmme_chain_res *res);

/* jmme_search_mbs serves a batch of at most 32 units whose work items (partition
 * groups sharing a window and predictor) fit in at most `max_workgroups` workgroups of 16x16
 * window positions by a single low-latency launch (no device copies, results
 * written to mapped host memory) -- the speculative batches of the JM drop-in
 * are mostly one or two macroblocks.  Default 4096; 0 sends everything down the
 * throughput path.  Results are identical either way. */
int jmme_set_small_batch_limit(jmme_ctx *ctx, int max_workgroups);
/* Pay the one-time start-up costs (HIP loads a module's kernels at their first
 * launch; occupancy queries are cached on first use) with a search on a dummy
 * plane, so that the first real search is not charged for them.  Optional. */
int jmme_prepare(jmme_ctx *ctx);
/* Size the synchronous batch path's device and pinned host buffers for batches
 * of up to `max_units` units now (they otherwise grow on demand, each growth a
 * device allocation inside some search call) -- and, unless the configuration
 * has DisableSubpelME, jmme_subpel_refine's for batches of max_units *
 * JMME_NSLOT refinements.  Optional. */
int jmme_reserve(jmme_ctx *ctx, int max_units);

/* Device-resident variant for pipelines and the benchmark: d_req/d_out are
 * device pointers, planes are those already uploaded; enqueued on `stream`
 * (a hipStream_t, NULL = default stream); no host synchronisation. */
int jmme_search_mbs_async(jmme_ctx *ctx, int mode, const jmme_mb_req *d_req, int n,
                          jmme_block_res *d_out, void *stream);

/* Device-plane variant: d_cur/d_ref are 8-bit planes (pitch bytes per row)
 * already in device memory (e.g. from torch), for multi-frame pipelines.
 * Both base pointers and the pitch must be multiples of 4 bytes. */
int jmme_search_mbs_planes_async(jmme_ctx *ctx, int mode,
                                 const uint8_t *d_cur, const uint8_t *d_ref, int pitch,
                                 int width, int height,
                                 const jmme_mb_req *d_req, int n, jmme_block_res *d_out,
                                 void *stream);

/* Status of the last search launch of ctx (synchronises `stream`).  The device
 * request paths above are not validated on the host; the plan kernel refuses
 * requests that would overrun the launch (range above SearchRange, an FFS block
 * range above its surface's, a sub-pel centre) and this returns -1 for them,
 * with jmme_last_error() naming the cause. */
int jmme_search_status(jmme_ctx *ctx, void *stream);

/* ---- JM IntPelME-signature drop-ins (one partition per call) ------------
 * Same inputs/outputs as full_search_motion_estimation / the FFS pair, in C
 * types: mv_inout is mv_block->mv[list] (centre in, best out). */
jmme_distblk jmme_full_search_block(jmme_ctx *ctx, int list, int ref_idx,
                                    int pos_x, int pos_y, int blocktype,
                                    const jmme_mv *pred_mv, jmme_mv *mv_inout,
                                    jmme_distblk min_mcost, int lambda_factor,
                                    int search_range, int check_for_00);

/* fast_full_search_motion_estimation (me_fullfast.c:618-689) with the state
 * setup_fast_full_search leaves in p_Vid->p_ffast_me (me_fullfast.c:269-608):
 * search_center = p_ffast_me->search_center[list][ref] (qpel, integer grid),
 * surface_range = the SAD surface's range (p_ffast_me->max_search_range),
 * block_range   = imax(searchRange.max_x, max_y) >> 2 for this partition,
 * rdopt         = p_Inp->rdopt (0: the (0,0) vector is pre-seeded, :650-657).
 * mv_out = mv_block->mv[list]; returns the minimum motion cost. */
jmme_distblk jmme_fast_full_search_block(jmme_ctx *ctx, int list, int ref_idx,
                                         int pos_x, int pos_y, int blocktype,
                                         const jmme_mv *pred_mv, const jmme_mv *search_center,
                                         int surface_range, int block_range, int rdopt,
                                         jmme_mv *mv_out, jmme_distblk min_mcost, int lambda_factor);

/* ---- Block transforms, 4x4 quantisation, Hadamard SATD (batched) ---------
 * SURVEY.md §8 rows a12/a13.  n independent blocks, each a flat row-major
 * array (b[r*N + c] == JM's block[pos_y + r][pos_x + c]), back to back.
 * *_async take device pointers and run on the caller's HIP stream; the plain
 * forms take host arrays and synchronise.  All bit-exact with JM 18.5. */
typedef enum jmme_transform_op {
  JMME_TF_FORWARD4x4 = 0,   /* forward4x4,   JM/lcommon/src/transform.c:20-68   (16 -> 16) */
  JMME_TF_INVERSE4x4,       /* inverse4x4,   transform.c:70-119                  (16 -> 16) */
  JMME_TF_HADAMARD4x4,      /* hadamard4x4,  transform.c:121-169 (luma DC)       (16 -> 16) */
  JMME_TF_IHADAMARD4x4,     /* ihadamard4x4, transform.c:171-218                 (16 -> 16) */
  JMME_TF_HADAMARD4x2,      /* hadamard4x2,  transform.c:220-258 (2x4 chroma DC) ( 8 ->  8) */
  JMME_TF_IHADAMARD4x2,     /* ihadamard4x2, transform.c:260-300 (2x4 -> 4x2)    ( 8 ->  8) */
  JMME_TF_HADAMARD2x2,      /* hadamard2x2,  transform.c:302-315 ({b00,b04,b40,b44}) (4 -> 4) */
  JMME_TF_IHADAMARD2x2,     /* ihadamard2x2, transform.c:317-331                 ( 4 ->  4) */
  JMME_TF_FORWARD8x8,       /* forward8x8,   transform.c:353-448                 (64 -> 64) */
  JMME_TF_INVERSE8x8        /* inverse8x8,   transform.c:450-528                 (64 -> 64) */
} jmme_transform_op;

int jmme_transform(jmme_ctx *ctx, int op, const int32_t *in, int32_t *out, int n);
int jmme_transform_async(jmme_ctx *ctx, int op, const int32_t *d_in, int32_t *d_out, int n, void *stream);

/* HadamardSAD4x4 / HadamardSAD8x8 (JM/lencod/src/me_distortion.c:175-341) of
 * n residual blocks (int16, 16 or 64 per block) -> int32 per block, unscaled
 * (distortion4x4SATD, me_distortion.c:70-74, is this << 5). size = 4 or 8. */
int jmme_satd(jmme_ctx *ctx, int size, const int16_t *diff, int32_t *out, int n);
int jmme_satd_async(jmme_ctx *ctx, int size, const int16_t *d_diff, int32_t *d_out, int n, void *stream);

/* quant_4x4_normal (JM/lencod/src/quant4x4_normal.c:39-110) inputs for one
 * parameter set: scale/offset/inv_scale = q_params_4x4[j][i].{ScaleComp,
 * OffsetComp,InvScaleComp} at [j*4+i] (quant_params.h:17-21), qp_per =
 * p_Quant->qp_per_matrix[qp], is_cavlc = (symbol_mode == CAVLC), scan =
 * pos_scan as (horizontal, vertical), c_cost = COEFF_COST4x4[disthres]. */
typedef struct jmme_quant4x4_params {
  int32_t scale[16], offset[16], inv_scale[16];
  int32_t qp_per;
  int32_t is_cavlc;
  uint8_t scan[16][2];
  uint8_t c_cost[16];
} jmme_quant4x4_params;   /* 248 bytes */

/* Per block b (param set params[param_idx[b]], or params[0] if param_idx is
 * NULL): coef[b][16] in = tblock, out = the dequantised block JM leaves in
 * tblock; levels[b][17] = ACLevel (0-terminated), runs[b][16] = ACRun;
 * coeff_cost[b] in/out (JM's *coeff_cost += ...); nonzero[b] = return value. */
int jmme_quant4x4(jmme_ctx *ctx, const jmme_quant4x4_params *params, int n_params, const int32_t *param_idx,
                  int32_t *coef, int32_t *levels, int32_t *runs, int32_t *coeff_cost, int32_t *nonzero, int n);
int jmme_quant4x4_async(jmme_ctx *ctx, const jmme_quant4x4_params *d_params, const int32_t *d_param_idx,
                        int32_t *d_coef, int32_t *d_levels, int32_t *d_runs, int32_t *d_coeff_cost,
                        int32_t *d_nonzero, int n, void *stream);

/* residual_transform_quant_luma_4x4 (JM/lencod/src/block.c:660-724) of inter
 * blocks -- the mode-decision call SURVEY.md §8(f)3 names: check_zero,
 * forward4x4, quant_4x4_normal, then inverse4x4 + sample_reconstruct
 * (lcommon/src/blk_prediction.c:48-62) when a level survives, else the
 * prediction.  Per block: ores = mb_ores[block_y + r][block_x + c] (original -
 * prediction), pred = mb_pred[...], param = index of its jmme_quant4x4_params
 * (q_params_4x4[pl][0][qp], qp_per, CAVLC, scan, COEFF_COST4x4[disthres]),
 * max_pel = max_imgpel_value.  Results: what JM leaves -- zero (check_zero
 * found no coefficient: JM sets ACLevel[0] = 0 and copies the prediction),
 * nonzero (the return value), cost (added to *coeff_cost), levels / runs
 * (cofAC[b8][b4][0/1], levels 0-terminated), coef (tblk16x16 after the
 * quantiser: the dequantised block; not touched when zero), rres (mb_rres,
 * only when nonzero), recon (enc_picture rows). */
typedef struct jmme_resid4x4_req {
  int32_t ores[16];
  jmme_imgpel pred[16];
  int32_t param;
  int32_t max_pel;
} jmme_resid4x4_req;   /* 104 bytes */

typedef struct jmme_resid4x4_res {
  int32_t coef[16];
  int32_t rres[16];
  int32_t levels[17];
  int32_t runs[16];
  int32_t cost, nonzero, zero;
  jmme_imgpel recon[16];
} jmme_resid4x4_res;   /* 304 bytes */

int jmme_residual4x4(jmme_ctx *ctx, const jmme_quant4x4_params *params, int n_params,
                     const jmme_resid4x4_req *req, jmme_resid4x4_res *res, int n);

/* ---- EPZS integer-pel search --------------------------
 * EPZS_motion_estimation (variant 0) and EPZS_subMB_motion_estimation
 * (variant 1), JM/lencod/src/me_epzs.c:54-407 / 417-780 (EPZSSubPelGrid = 0),
 * and on the quarter-pel grid EPZS_integer_motion_estimation (variant 2) and
 * EPZS_integer_subMB_motion_estimation (variant 3), me_epzs_int.c:41-782
 * (EPZSSubPelGrid = 1 in the context's config; candidates costed on the
 * sub-images of jmme_interpolate_ref, built automatically): median check and
 * its early exits, the predictor list (deduplicated through the EPZSMap), the
 * refinement pattern walk (EPZSPattern 0-5; the half-pel SBP diamond 4 only
 * on the quarter-pel grid) and the dual refinement around the second best
 * (EPZSDualRefinement 0-6, 5 only on the quarter-pel grid).
 * What JM builds on the host before the candidate search is input: the
 * predictor list (EPZS_spatial / _spatial_memory / _temporal /
 * EPZSWindowPredictors / EPZSBlockTypePredictors(MB), me_epzs_common.c), the
 * stop criterion (EPZSDetermineStopCriterion :1764), the prevSad slot
 * (p_EPZS->distortion[list][blocktype-1][pos_x2]) and the EPZSMap cells that
 * already hold the search's BlkCount (the uint16 map is never cleared).
 * The result is JM's (mv, cost) and the prevSad value JM leaves. */
typedef struct jmme_epzs_req {
  int16_t pos_x, pos_y;        /* block origin, luma pels */
  int16_t bsx, bsy;            /* 16 / 8 / 4 */
  int16_t blocktype, ref_idx;  /* 1..7; reference index (the ref > 0 thresholds) */
  int16_t pred_x, pred_y;      /* MV predictor, qpel */
  int16_t center_x, center_y;  /* mv_block->mv[list] on entry, qpel (a multiple of 4 for variants 0/1) */
  int16_t max_x, max_y;        /* mv_block->searchRange.max_x / max_y, qpel */
  int32_t lambda;              /* lambda_factor[F_PEL] */
  uint8_t variant;             /* 0 EPZS_motion_estimation, 1 EPZS_subMB_motion_estimation,
                                  2 / 3 their EPZSSubPelGrid forms (me_epzs_int.c) */
  uint8_t flags;               /* JMME_EPZS_FRAME | JMME_EPZS_PSLICE */
  uint8_t pattern, dual;       /* EPZSPattern, EPZSDualRefinement */
  int32_t n_pred, pred_off;    /* predictor list: (x, y) qpel pairs at preds[pred_off ..] */
  int32_t n_stale, stale_off;  /* pre-marked EPZSMap cells: (dx, dy) qpel from the centre */
  int32_t ref_slot;            /* list * 32 + ref_idx of jmme_upload_ref */
  int32_t reserved;
  int64_t prev_sad;            /* *prevSad on entry */
  int64_t medthres;            /* p_EPZS->medthres[blocktype] */
  int64_t stop_crit;           /* EPZSDetermineStopCriterion's value (read only when JM calls it) */
} jmme_epzs_req;               /* 80 bytes */

#define JMME_EPZS_FRAME 1      /* currSlice->structure == FRAME */
#define JMME_EPZS_PSLICE 2     /* currSlice->slice_type == P_SLICE */

typedef struct jmme_epzs_res {
  int16_t mv_x, mv_y;          /* mv_block->mv[list] on return, qpel */
  int32_t path;                /* 1..7: which return of the JM function was taken (-1: refused) */
  int64_t cost;                /* return value (min_mcost) */
  int64_t prev_sad;            /* *prevSad on return */
  int16_t motion_x, motion_y;  /* JM's tmp at return: what EPZSSpatialMem stores to p_motion */
  int32_t n_visited;           /* EPZSMap cells the search stamped (jmme_epzs_search_ex) */
} jmme_epzs_res;               /* 32 bytes */

/* Predictor conditions (jmme_epzs_search_ex's pred_cond, one per predictor):
 * JM generates part of the list only when the centre's cost min_mcost passes a
 * bound on the stop criterion (me_epzs.c:170-212, me_epzs_int.c:163-212):
 * temporal neighbours (min_mcost > stop, EPZS_temporal_predictors), window
 * predictors (> 3 stop), block-type predictors for ref > 0 (> 2 stop).  The
 * caller generates the whole list with JM's own routines; the search keeps the
 * entries whose condition holds for the centre cost it computes. */
#define JMME_EPZS_PRED_ALWAYS   0
#define JMME_EPZS_PRED_GT_STOP  1
#define JMME_EPZS_PRED_GT_2STOP 2
#define JMME_EPZS_PRED_GT_3STOP 3

/* against the uploaded current frame and reference slots; host arrays */
int jmme_epzs_search(jmme_ctx *ctx, const jmme_epzs_req *req, int n, const int16_t *preds, int n_preds,
                     const int16_t *stale, int n_stale, jmme_epzs_res *out);
/* device arrays on `stream` (requests validated by the caller) */
int jmme_epzs_search_async(jmme_ctx *ctx, const jmme_epzs_req *d_req, int n, const int16_t *d_preds,
                           const int16_t *d_stale, jmme_epzs_res *d_out, void *stream);
/* The drop-in's form (integration/jm_gpu_me.c wraps JM's four EPZS functions
 * with it, one call per search): as jmme_epzs_search, plus pred_cond (may be
 * NULL) and, when visited is not NULL, the EPZSMap cells each search stamped
 * -- (dx, dy) qpel from its centre, max_visited pairs per request at
 * visited[2 * max_visited * i] -- so the caller can keep JM's map.  Fails when a
 * search stamps more than max_visited cells.  Host arrays; no device copies (the
 * kernel reads and writes mapped host memory), one launch and one sync. */
int jmme_epzs_search_ex(jmme_ctx *ctx, const jmme_epzs_req *req, int n, const int16_t *preds,
                        const uint8_t *pred_cond, int n_preds, const int16_t *stale, int n_stale,
                        jmme_epzs_res *out, int16_t *visited, int max_visited);

/* ---- Speculative EPZS batches (the drop-in's throughput form) -------------
 * A search reads the stop criterion (EPZSDetermineStopCriterion,
 * me_epzs_common.c:1764) and *prevSad only through comparisons, each monotone
 * in that value (JM/lencod/src/me_epzs.c:54-407, me_epzs_int.c:41-782), so a
 * search run with guessed values returns the intervals within which its whole
 * execution -- (mv, cost, the cells it stamps, p_motion, whether it writes
 * *prevSad) -- is unchanged.  The drop-in serves a cached answer to JM's call
 * when the call's other inputs equal the guessed ones and its real stop
 * criterion and prevSad lie inside. */
typedef struct jmme_epzs_bounds {
  int64_t stop_lo, stop_hi;    /* the result holds for every stop criterion in [stop_lo, stop_hi] */
  int64_t prev_lo, prev_hi;    /* ... and every *prevSad on entry in [prev_lo, prev_hi] */
  int32_t prev_written;        /* 1: the search stores *prevSad = cost; 0: it leaves *prevSad alone */
  int32_t n_visited;           /* = jmme_epzs_res.n_visited */
} jmme_epzs_bounds;            /* 40 bytes */

/* ---- Quarter-pel reference planes and sub-pel refinement -----------------
 * SURVEY.md §8(f) rank 1.
 *
 * Sub-images: getSubImagesLuma (JM/lencod/src/img_luma.c:611-680,
 * OnTheFlyFractMCP = 0) -- the 16 quarter-pel sub-images of a reference,
 * sub[dy][dx], built with JM's six-tap / bilinear filters over the
 * edge-replicated picture, padded by IMG_PAD_SIZE_Y = 20 rows and
 * IMG_PAD_SIZE_X = 32 columns (JM/lencod/inc/defines.h) exactly as
 * get_mem4Dpel_pad lays them out (memalloc.c:881-904).  Built on the device
 * for each uploaded reference slot when first needed (jmme_upload_ref marks a
 * slot's sub-images stale).  A context with SourceBitDepthLuma 9..14 keeps
 * 16-bit sub-images, the six-tap results clipped to (1 << bits) - 1
 * (max_imgpel_value), and refines on them; the SSE metric is refused above 11
 * bits, where JM's int sum (computeSSE, me_distortion.c:1197) can wrap. */
#define JMME_SUBPEL_PAD_Y 20
#define JMME_SUBPEL_PAD_X 32

/* (re)build the sub-images of an uploaded reference slot on `stream` */
int jmme_interpolate_ref(jmme_ctx *ctx, int list, int ref_idx, void *stream);
/* getSubImagesLuma drop-in: copy them out in JM's layout.  sub[dy][dx][j][i]
 * for j in [-20, H+20), i in [-32, W+32) (JM's s->imgY_sub after
 * UnifiedOneForthPix, image.c:2148-2164); row pointers as get_mem4Dpel_pad
 * makes them (sub[dy][dx][j] points at column 0 of padded row j). */
int jmme_get_sub_images(jmme_ctx *ctx, int list, int ref_idx, jmme_imgpel ****sub);
/* device form over caller planes (8-bit only): d_src = 8-bit W x H plane (src_pitch bytes
 * a row); d_dst = 16 planes, plane k = dy*4+dx at d_dst + k*plane_stride,
 * (H+40) rows of dst_pitch >= W+64 bytes, padded row 0 = picture row -20 */
int jmme_sub_images_async(jmme_ctx *ctx, const uint8_t *d_src, int src_pitch, int width, int height,
                          uint8_t *d_dst, int dst_pitch, size_t plane_stride, void *stream);

/* One sub-pel refinement: what BlockMotionSearch (mv_search.c:966-976) hands
 * currMB->SubPelME for one partition.
 *   variant 0: sub_pel_motion_estimation       (JM/lencod/src/me_fullsearch.c:186-289;
 *              SearchMode FS / FFS, and EPZS with EPZSSubPelME 0)
 *   variant 1: EPZS_sub_pel_motion_estimation  (JM/lencod/src/me_epzs_sub.c:30-222;
 *              EPZS with EPZSSubPelME 1)
 * Metrics (MEDistortionHPel / QPel): 0 SAD (computeSAD), 1 SSE (computeSSE),
 * 2 SATD (computeSATD: 4x4 Hadamard, or 8x8 when test8x8 is set), evaluated on
 * the sub-images with UMVLine4X clamping (refbuf.h:22-26). */
typedef struct jmme_subpel_req {
  int16_t pos_x, pos_y;       /* block origin (luma pels) */
  int16_t blocktype;          /* 1..7 (0: skip this entry, its output is left untouched) */
  int16_t ref_slot;           /* list * 32 + ref_idx of jmme_upload_ref */
  int16_t pred_x, pred_y;     /* MV predictor (qpel) */
  int16_t mv_x, mv_y;         /* mv_block->mv[list] on entry: the integer-pel result (qpel) */
  int32_t lambda_h, lambda_q; /* lambda_factor[H_PEL], lambda_factor[Q_PEL] */
  int64_t min_mcost;          /* what SubPelME receives (DISTBLK_MAX when start_hp == 0) */
  int64_t subthres;           /* variant 1: p_EPZS->subthres[blocktype] (me_epzs_common.c:448-466) */
  uint8_t variant;
  uint8_t flags;              /* JMME_SP_* */
  uint8_t metric_h, metric_q; /* 0 SAD, 1 SSE, 2 SATD */
  uint8_t start_hp, start_qp; /* p_Vid->start_me_refinement_hp / _qp (mv_search.c:445-446) */
  uint8_t search_pos2, search_pos4;   /* mv_block->search_pos2 / 4 (JM: 9, mv_search.c:720-721) */
} jmme_subpel_req;            /* 48 bytes */

#define JMME_SP_TEST8x8 1     /* mv_block->test8x8 (mv_search.c:1630,1770) */
#define JMME_SP_CHECK0  2     /* variant 0: !rdopt && slice_type != B_SLICE (check_position0's slice terms,
                                 me_fullsearch.c:205; ref 0, blocktype 1 and mv (0,0) are read from the request) */

/* host arrays, synchronous; out[i] = (mv, cost) SubPelME returns */
int jmme_subpel_refine(jmme_ctx *ctx, const jmme_subpel_req *req, int n, jmme_block_res *out);

/* jmme_search_mbs_chains with sub_pel_motion_estimation inside the chains (FS /
 * FFS with DisableSubpelME = 0: a partition's neighbours then hold refined
 * vectors).  sp[i] is chain i's SubPelME template -- lambda_h / lambda_q,
 * metric_h / metric_q, start_hp / start_qp, search_pos2 / 4 and flags
 * (JMME_SP_CHECK0; JMME_SP_TEST8x8 is refused) as JM hands them; variant must
 * be 0; its block, ref_slot, pred, mv, min_mcost and subthres are ignored:
 * step k refines its own integer answer under its derived predictor with
 * min_mcost = start_hp ? its cost : DISTBLK_MAX (mv_search.c:960-976), and
 * the refined vector, clipped as mv_search.c:981 clips it, is what the later
 * steps read as that partition's vector.  sp_res[i * JMME_CHAIN_MAX_STEPS + k]
 * = the (mv, cost) SubPelME returns; res[] as jmme_search_mbs_chains (the
 * integer answers).  sp == NULL: jmme_search_mbs_chains. */
int jmme_search_mbs_chains_sp(jmme_ctx *ctx, int mode, const jmme_mb_req *req, int n, jmme_block_res *out,
                              const jmme_chain *chains, int n_chains, const jmme_subpel_req *sp,
                              jmme_chain_res *res, jmme_block_res *sp_res);

/* EPZS speculative batch with its chained sub-pel refinements (jmme_epzs_bounds above). */
/* One launch over n searches, as jmme_epzs_search_ex (host arrays, one sync),
 * plus bounds[i] and, when sp_req is not NULL, one sub-pel refinement per search
 * chained on the device: sp_req[i] (blocktype 0: none; its mv and min_mcost are
 * ignored) refines search i's result -- mv = its mv, min_mcost = start_hp ? its
 * cost : DISTBLK_MAX, as BlockMotionSearch hands SubPelME (mv_search.c:960-976)
 * -- into sp_out[i].  A search that stamps more than max_visited cells is not
 * an error here: only max_visited pairs are written and n_visited tells. */
int jmme_epzs_speculate(jmme_ctx *ctx, const jmme_epzs_req *req, int n, const int16_t *preds,
                        const uint8_t *pred_cond, int n_preds, const int16_t *stale, int n_stale,
                        jmme_epzs_res *out, jmme_epzs_bounds *bounds, int16_t *visited, int max_visited,
                        const jmme_subpel_req *sp_req, jmme_block_res *sp_out);
/* device arrays on `stream`.  d_int (may be NULL): integer-pel results aligned
 * with the requests (e.g. the jmme_search_mbs_async output with requests in
 * unit x slot order); when given, entry i takes mv = d_int[i].mv and
 * min_mcost = start_hp ? d_int[i].cost : DISTBLK_MAX instead of the request's,
 * as BlockMotionSearch does (mv_search.c:960-976).  The requests must have
 * been validated (jmme_subpel_validate) and their sub-images built. */
int jmme_subpel_refine_async(jmme_ctx *ctx, const jmme_subpel_req *d_req, int n, const jmme_block_res *d_int,
                             jmme_block_res *d_out, void *stream);
/* host-side check of requests against the context (0 = OK) */
int jmme_subpel_validate(jmme_ctx *ctx, const jmme_subpel_req *req, int n);

/* ---- Fractal domain-range block matching (thesis codec) -------------------
 * SURVEY.md §8 rows a14-a16; ZL = /root/reference/2.论文程序/ZhangLing_Yu_
 * version1/H264Fractal.  full_search (ZL/src/block_enc.c:1933-1977) with
 * compute_rms / compute_rdSum / QUAN_A (ZL/src/compute.c:6-215,
 * ZL/inc/defines_enc.h:591-601) and bound_chk (block_enc.c:2894-2919), one
 * request per range block.  Planes are 8-bit (the thesis's byte**), rows
 * `pitch` bytes apart (pitch % 4 == 0, W and H the picture size bound_chk
 * uses, i.e. the component's own size).  Block sizes: 16x16, 16x8, 8x16,
 * 8x8, 8x4, 4x8, 4x4 with the range block aligned to its size.
 * rms/scale/offset are bit-identical doubles to the thesis's. */
typedef struct jmme_fractal_req {
  int16_t block_x, block_y;   /* range block origin (pels), multiple of bsx / bsy */
  int16_t bsx, bsy;
} jmme_fractal_req;           /* 8 bytes */

typedef struct jmme_fractal_res {
  double rms;                 /* full_search's return value (1e30: nothing in range) */
  double scale, offset;       /* TRANS_NODE scale (alpha), offset (beta) */
  int32_t x, y;               /* TRANS_NODE x, y: domain - range offset (0,0 when (0,0) wins) */
} jmme_fractal_res;           /* 32 bytes */

int jmme_fractal_search(jmme_ctx *ctx, const uint8_t *org, const uint8_t *ref, int pitch, int width, int height,
                        int search_range, const jmme_fractal_req *req, int n, jmme_fractal_res *out);
/* device-pointer form: d_words is the reference's words image built by
 * jmme_fractal_words_async (one per reference frame, width*height uint32). */
int jmme_fractal_words_async(jmme_ctx *ctx, const uint8_t *d_ref, int pitch, int width, int height,
                             uint32_t *d_words, void *stream);
int jmme_fractal_search_async(jmme_ctx *ctx, const uint8_t *d_org, int pitch, const uint32_t *d_words, int width,
                              int height, int search_range, const jmme_fractal_req *d_req, int n,
                              jmme_fractal_res *d_out, void *stream);

/* Large radii (search_range >= the pool radius, default 80; the BASELINE
 * "full domain pool" is search_range >= max(width, height)) run the pruned
 * pool search: every candidate whose least-squares bound
 *   K - C^2/D  (K = sum (r - offset)^2, C = sum r*d - sum r * sum d / n,
 *               D = sum d^2 - (sum d)^2 / n)
 * already exceeds an exactly evaluated rms is skipped, the rest are evaluated
 * exactly -- same results as the windowed kernel, bit for bit.  A radius
 * above max(width, height) is the same search as max(width, height).
 * set_pool_min_range chooses the switch-over radius (0: always pool, a huge
 * value: never); pool_survivors returns (and clears) the number of exactly
 * evaluated candidates since the last call (synchronises the device). */
int jmme_fractal_set_pool_min_range(jmme_ctx *ctx, int min_range);
int jmme_fractal_pool_survivors(jmme_ctx *ctx, unsigned long long *survivors);
/* 4x4 blocks over the full pool run the bound test on the matrix cores
 * (exact bf16 products, f32 sums of 16); on = 0 selects the VALU kernel
 * (for comparison; same results). */
int jmme_fractal_set_pool_mfma(jmme_ctx *ctx, int on);

/* compute_domain_Sum / compute_range_Sum (ZL/src/compute.c:277-~1091) for one
 * block size: sum and sum of squares of every bsx x bsy box of the plane,
 * (height-bsy+1) x (width-bsx+1) doubles each (exact integers). */
int jmme_fractal_box_sums(jmme_ctx *ctx, const uint8_t *plane, int pitch, int width, int height, int bsx, int bsy,
                          double *sum, double *sum2);

/* ---- Fractal macroblock encoder: the quadtree gate ------
 * encode_one_macroblock (ZL/src/block_enc.c:508-1050) with encode_block_rect
 * / _8 / _4 (block_enc.c:1072-1932) for every 16x16 macroblock of a plane, in
 * the configuration the thesis encodes its centre view with: search_mode 0
 * (full_search), one region (num_regions 1), currentVideo 'C'.  Each tree
 * level searches reference view 0 (the view's own reference frame) and then
 * views 1..n_refs-1 (the thesis's H, M, N) and keeps the first strict minimum;
 * `reference` is that view's index.
 *   16x16 splits when 0.9 <= chun <= 1 and rms > tol_16^2 * 256, chun being
 *   the squared correlation of the range block with the co-located block of
 *   view 0; then every 8x8 is searched (the thesis's 16x8 / 8x16 attempt at
 *   this level never ends the mode loop, block_enc.c:798-855, so it is
 *   overwritten and not run);
 *   8x8 with rms > tol_8^2 * 64 tries the 8x4 pair (partition 1), then the
 *   4x8 pair (partition 2), a pair matching when neither half has rms >
 *   tol_8^2 * 32; otherwise four 4x4 (partition 3);
 *   a 4x4 node gets partition 1 when view 1 beat view 0 (block_enc.c:1773).
 * Output nodes are bit-identical to the thesis's TRANS_NODE values (x, y,
 * scale, offset, reference, partition) plus the rms the node's search
 * returned; nodes the tree does not reach are zero (a fresh tree). */
#define JMME_FRACTAL_MAX_VIEWS 4

typedef struct jmme_fractal_node {
  double rms, scale, offset;
  int32_t x, y;
  int32_t reference;          /* winning view, 0 .. n_refs-1 */
  int32_t partition;          /* 0 leaf; 1 16x8/8x4 pair; 2 8x16/4x8 pair; 3 quadrants */
} jmme_fractal_node;          /* 40 bytes */

typedef struct jmme_fractal_mb {
  jmme_fractal_node mb;       /* trans[0][CurMb] */
  jmme_fractal_node b8[4];    /* its next[0..3] (raster order) when mb.partition == 3 */
  jmme_fractal_node sub[4][4];/* b8[q].next[0..1] (pairs) or [0..3] (4x4, raster) */
  double chun;                /* the 16x16 gate's squared correlation (NaN for a flat block) */
} jmme_fractal_mb;            /* 848 bytes */

/* host planes: org and refs[0..n_refs-1], all width x height with rows pitch
 * bytes apart; width, height multiples of 16; out[(width/16)*(height/16)]
 * in raster macroblock order */
int jmme_fractal_encode_mbs(jmme_ctx *ctx, const uint8_t *org, const uint8_t *const *refs, int n_refs, int pitch,
                            int width, int height, int search_range, double tol_16, double tol_8,
                            jmme_fractal_mb *out);
/* device form: d_ref0 = view 0's plane (the gate's co-located block),
 * d_words[k] = view k's words image (jmme_fractal_words_async); all work is
 * queued on `stream` with no host synchronisation (the tree levels size
 * themselves on the device) */
int jmme_fractal_encode_mbs_async(jmme_ctx *ctx, const uint8_t *d_org, const uint8_t *d_ref0, int pitch,
                                  const uint32_t *const *d_words, int n_refs, int width, int height,
                                  int search_range, double tol_16, double tol_8, jmme_fractal_mb *d_out,
                                  void *stream);
/* the same for the macroblock rows [mb_row0, mb_row1) of the plane only (an
 * MB-row band of a multi-GPU split): the searches still see the
 * whole picture (bound_chk's frame limits, domain blocks outside the band), so
 * the band's trees are identical to those rows of the whole-plane encode;
 * d_out[(width/16)*(mb_row1-mb_row0)], raster order from row mb_row0 */
int jmme_fractal_encode_mb_rows_async(jmme_ctx *ctx, const uint8_t *d_org, const uint8_t *d_ref0, int pitch,
                                      const uint32_t *const *d_words, int n_refs, int width, int height,
                                      int mb_row0, int mb_row1, int search_range, double tol_16, double tol_8,
                                      jmme_fractal_mb *d_out, void *stream);

/* ---- Fractal decoder (reconstruction of a P plane from its trees) -------
 * decode_one_macroblock, decode_block_rect, decode_block_8, decode_block_4
 * (ZL/src/block_dec.c:20-1160), num_regions == 1, for every macroblock of a
 * width x height plane (multiples of 16) of component 1 (Y), 2 (U) or 3 (V),
 * from the jmme_fractal_mb trees jmme_fractal_encode_mbs produces.  views[k]
 * is the plane the thesis's decoder reads for reference k (imgY_ref, _h, _m,
 * _n or the chroma equivalents).  Each leaf pel is
 *   (unsigned char) bound(0.5 + scale*d + offset - scale*avg),
 * avg = (box sum of the leaf's domain block) / n, with the thesis's per-level
 * view choice (8x8 leaves: reference 0 -> view 0, else view 1; V 4x4 leaves:
 * reference 1 -> view 3).  Fails (sync form) when a leaf
 * maps to a view >= n_views or its domain block leaves the plane; the async
 * form sets *d_status |= 1 instead (d_status may be NULL) and writes 0 there. */
int jmme_fractal_decode_mbs(jmme_ctx *ctx, const jmme_fractal_mb *mbs, const uint8_t *const *views, int n_views,
                            int pitch, int width, int height, int component, uint8_t *rec);
int jmme_fractal_decode_mbs_async(jmme_ctx *ctx, const jmme_fractal_mb *d_mbs, const uint8_t *const *d_views,
                                  int n_views, int pitch, int width, int height, int component, uint8_t *d_rec,
                                  int *d_status, void *stream);

/* ---- timing of the last jmme_search_mbs* launch (HIP events on its stream) */
float jmme_last_kernel_ms(jmme_ctx *ctx);

/* ---- exposed for host-side tests (no GPU needed) ------------------------ */
int jmme_spiral_index(int ox, int oy);                /* position in spiral_search order */
void jmme_spiral_offset(int index, int *ox, int *oy); /* inverse */
int jmme_mvbits(int v);                                /* mvbits[v], mv_search.c:366-374 */

/* Test hook (GPU): run one unit and copy out the first reference window it
 * staged in LDS, (2R+16) rows x (2R+13) words, word[y][x] = pels x..x+3
 * of the clamped reference; R = the context's SearchRange. */
int jmme_debug_window(jmme_ctx *ctx, int mode, const jmme_mb_req *req, uint32_t *out, int max_words);

/* Diagnostic builds only (-DJMME_STAMPS): per-unit phase clock sums of the
 * last launch, 8 x uint64 per unit; returns units copied or -1. */
int jmme_debug_stamps(jmme_ctx *ctx, uint64_t *out, int max_units);

#ifdef __cplusplus
}
#endif
#endif /* JMME_H */
