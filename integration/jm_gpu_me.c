/*
 * jm_gpu_me.c -- the JM side of the drop-in, built into a
 * JM 18.5 lencod whose integer-pel motion search runs on the MI355X through
 * libjmme (include/jmme.h).  JM's sources are not modified: this file is linked
 * with JM's own objects (compiled from /root/reference by oracle/Makefile) and
 * the GNU ld `--wrap` of three symbols, so the encoder's own call sites reach
 * the GPU:
 *
 *   full_search_motion_estimation       JM/lencod/src/me_fullsearch.c:39-103
 *       currMB->IntPelME for SearchMode = -1 (assigned mv_search.c:161,
 *       called mv_search.c:960; signature JM/lencod/inc/global.h:459)
 *   fast_full_search_motion_estimation  JM/lencod/src/me_fullfast.c:618-689
 *       currMB->IntPelME for SearchMode = 0 (mv_search.c:168)
 *   setup_fast_full_search              JM/lencod/src/me_fullfast.c:269-608
 *       p_Vid->p_SetupFastFullPelSearch (global.h:469, mv_search.c:172): here it
 *       only derives the search centre (me_fullfast.c:312-327) -- the SAD
 *       surface JM would build on the CPU is the GPU's job
 *   sub_pel_motion_estimation           JM/lencod/src/me_fullsearch.c:186-289
 *       currMB->SubPelME for FS / FFS (called mv_search.c:966-976): half- and
 *       quarter-pel refinement on the GPU's quarter-pel planes
 *
 * Frame buffers: p_Vid->pCurImg (image.c:2868) and the reference pictures'
 * imgY (StorablePicture, mbuffer.c:2116-2122) are uploaded once per coded
 * picture (jmme_upload_cur / jmme_upload_ref).  Errors follow JM's error()
 * convention (message, exit code 500).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <x86intrin.h>

#include "global.h"
#include "mbuffer.h"
#include "me_distortion.h"
#include "me_epzs_common.h"
#include "me_fullfast.h"
#include "mv_search.h"
#include "jmme.h"

extern distblk __real_sub_pel_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int *);
extern distblk __real_full_search_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int);
extern distblk __real_fast_full_search_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int);
extern void __real_setup_fast_full_search(Macroblock *, MEBlock *, int);
extern void __real_init_motion_search_module(VideoParameters *, InputParameters *);

extern void get_neighbors(Macroblock *currMB, PixelPos *block, int mb_x, int mb_y, int blockshape_x);

static jmme_ctx *g_me = NULL;
static int g_bits = 8;  /* SourceBitDepthLuma */
static long long g_calls = 0, g_cpu_calls = 0;
static FILE *g_trace = NULL, *g_trace_miss = NULL;   /* JMME_TRACE / JMME_TRACE_MISS */

/* What the uploaded planes and every cached answer belong to.  frame_no alone
 * does not identify a coded picture: MVC view 1 shares view 0's frame_no with
 * another pCurImg, and RDPictureDecision codes one frame again (rd_pass 1, 2)
 * with other reference lists or weights.  So the current plane is keyed on
 * (frame_no, pCurImg, view_id, structure, rd_pass) and each (list, ref) slot on
 * the StorablePicture* bound to it (currSlice->listX[list + list_offset][ref]).
 * Any change bumps a generation; the caches of a slot are valid only for the
 * generation its picture was uploaded in. */
typedef struct pic_key {
  int frame_no, view_id, structure, rd_pass;
  imgpel **cur;
} pic_key;
static pic_key g_pic = {-1000000, -1, -1, -1, NULL};
static StorablePicture *g_ref_pic[2][32];  /* picture uploaded into each slot (NULL: none) */
static unsigned g_slot_gen[2][32];         /* generation of that upload */
static unsigned g_gen = 0;

static void fail_jm(const char *what)
{
  char buf[600];
  snprintf(buf, sizeof buf, "jm_gpu_me: %s: %s", what, jmme_last_error());
  error(buf, 500);
}

/* the encoder's ME configuration, from JM's own parsed parameters
 * (JM/lencod/inc/configfile.h Map[] entries named in include/jmme.h) */
static void init_once(VideoParameters *p_Vid, InputParameters *p_Inp)
{
  jmme_config c;
  if (g_me) return;
  jmme_config_default(&c);
  /* the adapter numbers macroblocks of a frame picture; field pictures and MBAFF
   * pairs (other plane heights, list_offset 2..5) are not handled */
  if (p_Inp->PicInterlace || p_Inp->MbInterlace)
    error("jm_gpu_me: PicInterlace / MbInterlace are not supported by the GPU drop-in", 500);
  c.SourceWidth = p_Vid->width;
  c.SourceHeight = p_Vid->height;
  c.SearchMode = p_Inp->SearchMode[0];
  /* MVC: each view has its own SearchRange (configfile.h:62,539); the context
   * must admit the larger one */
  c.SearchRange = p_Inp->num_of_views > 1 ? imax(p_Inp->search_range[0], p_Inp->search_range[1])
                                           : p_Inp->search_range[0];
  c.NumberReferenceFrames = p_Inp->num_ref_frames;
  c.DisableSubpelME = p_Inp->DisableSubpelME[0];
  c.RDOptimization = p_Inp->rdopt;
  /* only SAD integer-pel searches reach the GPU (fs_on_cpu / ffs_on_cpu send
   * SSE, SATD and weighted ones to JM's own code), so the context is a SAD one */
  c.MEDistortionFPel = 0;
  c.MDDistortion = p_Inp->ModeDecisionMetric;
  c.EPZSSubPelGrid = p_Inp->EPZSSubPelGrid;
  c.RestrictSearchRange = p_Inp->full_search;
  c.UseMVLimits = p_Inp->UseMVLimits;
  c.SetMVXLimit = p_Inp->SetMVXLimit;
  c.SetMVYLimit = p_Inp->SetMVYLimit;
  c.ChromaMEEnable = p_Inp->ChromaMEEnable;
  /* the luma depth of JM's imgpel planes (init_img, lencod.c:1115): above 8 the
   * context keeps 16-bit planes and searches with v_sad_u16 */
  c.SourceBitDepthLuma = p_Vid->bitdepth_luma > 0 ? p_Vid->bitdepth_luma : p_Inp->source.bit_depth[0];
  g_bits = c.SourceBitDepthLuma;
  g_me = jmme_create(&c, -1);
  if (!g_me) fail_jm("jmme_create");
}

/* the encoder's GPU engine (created on first use): jm_f3_gpu.c's residual coding shares it */
jmme_ctx *jm_gpu_me_engine(VideoParameters *p_Vid, InputParameters *p_Inp)
{
  init_once(p_Vid, p_Inp);
  return g_me;
}

/* init_motion_search_module (mv_search.c:315, called once from init_encoder,
 * lencod.c:606) builds JM's ME tables; the GPU engine is created there too, and
 * its one-time start-up (code-object loading, first-launch setup) is paid
 * before any frame is timed, like JM's own table setup */
static void prefault_tables(VideoParameters *p_Vid, InputParameters *p_Inp);
static void reserve_batches(void);
static void calibrate_clock(void);

void __wrap_init_motion_search_module(VideoParameters *p_Vid, InputParameters *p_Inp)
{
  __real_init_motion_search_module(p_Vid, p_Inp);
  calibrate_clock();   /* (before any picture is timed) */
  if (p_Inp->SearchMode[0] == FULL_SEARCH || p_Inp->SearchMode[0] == FAST_FULL_SEARCH || p_Inp->SearchMode[0] == EPZS) {
    init_once(p_Vid, p_Inp);
    if (jmme_prepare(g_me)) fail_jm("jmme_prepare");
    reserve_batches();
  }
  if (p_Inp->SearchMode[0] == FULL_SEARCH || p_Inp->SearchMode[0] == FAST_FULL_SEARCH) prefault_tables(p_Vid, p_Inp);
}

/* planes of the picture being coded and of the reference (list, ref) */
static double g_t_planes = 0, g_t_plane_max = 0;   /* in jmme_upload_cur / _ref (reported when tracing) */
static long long g_n_uploads = 0;
static double now_us(void);
static void ensure_planes(Macroblock *currMB, int list, int ref)
{
  VideoParameters *p_Vid = currMB->p_Vid;
  Slice *currSlice = currMB->p_Slice;
  StorablePicture *pic;
  pic_key k;
  init_once(p_Vid, currMB->p_Inp);
  k.frame_no = p_Vid->frame_no;
  k.view_id = p_Vid->view_id;
  k.structure = p_Vid->structure;
  k.rd_pass = p_Vid->rd_pass;
  k.cur = p_Vid->pCurImg;
  if (k.frame_no != g_pic.frame_no || k.view_id != g_pic.view_id || k.structure != g_pic.structure ||
      k.rd_pass != g_pic.rd_pass || k.cur != g_pic.cur) {   /* another coded picture: every slot is stale */
    g_pic = k;
    memset(g_ref_pic, 0, sizeof g_ref_pic);
    double t0 = now_us();
    ++g_gen;
    if (jmme_upload_cur(g_me, (const jmme_imgpel *const *)p_Vid->pCurImg, p_Vid->width, p_Vid->height))
      fail_jm("jmme_upload_cur");
    t0 = now_us() - t0;
    g_t_planes += t0;
    g_t_plane_max = t0 > g_t_plane_max ? t0 : g_t_plane_max;
    ++g_n_uploads;
  }
  if (list < 0 || list > 1 || ref < 0 || ref >= 32) error("jm_gpu_me: reference index out of range", 500);
  pic = currSlice->listX[list + currMB->list_offset][ref];
  if (g_ref_pic[list][ref] != pic) {           /* first use, or the slot now names another picture */
    double t0 = now_us();
    if (jmme_upload_ref(g_me, list, ref, (const jmme_imgpel *const *)pic->imgY, pic->size_x, pic->size_y))
      fail_jm("jmme_upload_ref");
    g_ref_pic[list][ref] = pic;
    g_slot_gen[list][ref] = ++g_gen;
    t0 = now_us() - t0;
    g_t_planes += t0;
    g_t_plane_max = t0 > g_t_plane_max ? t0 : g_t_plane_max;
    ++g_n_uploads;
  }
}

/* JM's integer-pel metric for this block is not the plain SAD the GPU computes:
 * SSE / SATD (MEDistortionFPel 1/2, lencod.c:782-796), the weighted variants
 * (mv_search.c:741-755) or the on-the-fly ones (mv_search.c:456-473).  Full
 * search calls mv_block->computePredFPel, so that pointer decides. */
static int fs_on_cpu(const MEBlock *mv_block)
{
  return mv_block->computePredFPel != computeSAD || mv_block->ChromaMEEnable;
}

/* setup_fast_full_search builds its surface with its own rule
 * (me_fullfast.c:274,294-295): squared differences for MEDistortionFPel 1 and
 * weighted samples when weighted prediction and UseWeightedReferenceME are on */
static int ffs_on_cpu(Macroblock *currMB, const MEBlock *mv_block)
{
  VideoParameters *p_Vid = currMB->p_Vid;
  InputParameters *p_Inp = currMB->p_Inp;
  Slice *currSlice = currMB->p_Slice;
  int apply_weights = ((p_Vid->active_pps->weighted_pred_flag &&
                        (currSlice->slice_type == P_SLICE || currSlice->slice_type == SP_SLICE)) ||
                       (p_Vid->active_pps->weighted_bipred_idc && currSlice->slice_type == B_SLICE)) &&
                      p_Inp->UseWeightedReferenceME;
  return p_Inp->MEErrorMetric[F_PEL] != 0 || apply_weights || mv_block->ChromaMEEnable;
}

/* ---- speculative batching of full-search calls ----------------------------
 * JM issues IntPelME one partition at a time, each with the predictor its
 * neighbours' final vectors give, so the inputs of later searches are not known
 * in advance.  They are usually close to ones already seen (smooth motion:
 * every partition of a macroblock, and the next macroblocks, get the same
 * predictor and centre, or the ones the same partition of a neighbour got), so
 * on a miss the adapter searches, in ONE batched call (jmme_search_mbs), all 41
 * partitions of the next `g_batch` macroblocks under up to KHYP distinct
 * guesses (spec_hyp) and caches (inputs -> result) per guess.
 * A later call is answered from the cache only when its inputs are identical
 * to the guessed ones -- a search is a pure function of (block, centre,
 * predictor, lambda, range, check_for_00) on the uploaded planes -- so the
 * encoder's output is unchanged; a miss re-batches from the missing
 * macroblock.  The batch length adapts: it doubles when the cache ran out
 * and halves when a guess failed.  Fast full search is batched the same way
 * (its key adds the macroblock's surface centre and range).  JMME_SPECULATE=0
 * sends every call on its own (jmme_full_search_block /
 * jmme_fast_full_search_block). */
typedef struct spec_ent {
  int16_t cx, cy, px, py, sr, chk;       /* FS: centre, predictor, range, check_for_00 */
  int16_t fcx, fcy, frange, mode;        /* FFS: search_center, surface range; mode 0 FS, 1 FFS */
  int16_t mvx, mvy;
  int32_t lambda;
  uint32_t valid;                        /* the g_slot_gen it was cached in (0: none) */
  int64_t cost;
} spec_ent;                              /* 40 B, packed */

#define KHYP 4                     /* guesses per (macroblock, partition) */
#define KWAYS (KHYP + 1)           /* cache ways: the KHYP guesses + the chained search's answer (way KHYP) */
/* Entry (macroblock mb, slot s, way k).  Way-major within a macroblock: JM's
 * calls of one macroblock mostly hit way 0, whose 41 entries (1.6 KB) are
 * contiguous, and the next macroblock's way 0 is prefetched while JM works on
 * this one.  (Slot-major, 5 ways of 48 B per slot, the table's first touch per
 * call was a cache miss: 12.5 ms of a 1080p FS P picture's 82 ms ME time in a
 * JMME_SAMPLE profile.) */
static inline size_t spec_idx(int mb, int s, int k) { return ((size_t)mb * KWAYS + k) * JMME_NSLOT + s; }
static spec_ent *g_spec[2][32];    /* KHYP cached (inputs -> result) per (macroblock, slot) */
static spec_ent *g_seen[2][32];    /* the inputs each (macroblock, slot) was really searched with */
static unsigned g_spec_gen[2][32]; /* g_slot_gen the cached guesses belong to */
static int g_spec_end[2][32];      /* first macroblock past the last batch */
#define MAX_BATCH 2048             /* macroblocks per speculative batch, at most */
static int g_batch = 64, g_speculate = -1, g_mbs_x = 0, g_n_mb = 0;
static long long g_hits = 0, g_batches = 0;
static jmme_mb_req *g_req = NULL;
static jmme_block_res *g_res = NULL;
static spec_ent *g_hyp = NULL;     /* the upper-neighbour guesses (per macroblock) */
static const spec_ent **g_req_row = NULL;   /* the inputs behind each request's 41 slots */
static int *g_req_mb = NULL;
static int g_req_cap = 0;

/* where a frame's batches come from and what they cost (reported at exit):
 * misses past the batch's end vs inside it (a guess failed), per slot */
static long long g_miss_past = 0, g_miss_guess = 0, g_miss_slot[JMME_NSLOT], g_units = 0;
static double g_t_build = 0, g_t_call = 0, g_t_wrap = 0;

/* the adapter's timers read the TSC (a few ns; clock_gettime per EPZS call cost
 * tens of ms per 1080p picture), scaled by a rate measured against
 * CLOCK_MONOTONIC when the encoder starts (calibrate_clock) */
static double g_us_per_tick = 0;
static double mono_us(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}
static void calibrate_clock(void)
{
  double t0, t1;
  unsigned long long c0, c1;
  if (g_us_per_tick > 0) return;
  t0 = mono_us();
  c0 = __rdtsc();
  do t1 = mono_us(); while (t1 - t0 < 2000.0);
  c1 = __rdtsc();
  g_us_per_tick = (t1 - t0) / (double)(c1 - c0);
}
static double now_us(void)
{
  if (g_us_per_tick <= 0) calibrate_clock();
  return (double)__rdtsc() * g_us_per_tick;
}

static spec_ent *spec_table(VideoParameters *p_Vid, int list, int ref)
{
  if (!g_n_mb) {
    g_mbs_x = p_Vid->width / 16;
    g_n_mb = g_mbs_x * (p_Vid->height / 16);
  }
  if (!g_spec[list][ref]) {
    g_spec[list][ref] = (spec_ent *)calloc((size_t)g_n_mb * JMME_NSLOT * KWAYS, sizeof(spec_ent));
    g_seen[list][ref] = (spec_ent *)calloc((size_t)g_n_mb * JMME_NSLOT, sizeof(spec_ent));
    if (!g_spec[list][ref] || !g_seen[list][ref]) error("jm_gpu_me: out of memory", 500);
    g_spec_gen[list][ref] = 0;
  }
  if (g_spec_gen[list][ref] != g_slot_gen[list][ref]) {   /* other planes: every guess is stale (its stamp) */
    g_spec_gen[list][ref] = g_slot_gen[list][ref];
    g_spec_end[list][ref] = 0;
  }
  return g_spec[list][ref];
}

static int spec_key_eq(const spec_ent *e, const spec_ent *w)
{
  return e->mode == w->mode && e->cx == w->cx && e->cy == w->cy && e->px == w->px && e->py == w->py &&
         e->sr == w->sr && e->chk == w->chk && e->fcx == w->fcx && e->fcy == w->fcy && e->frange == w->frange &&
         e->lambda == w->lambda;
}

static int spec_same(const spec_ent *e, const spec_ent *w, unsigned gen) { return e->valid == gen && spec_key_eq(e, w); }

/* Guess h for the 41 partitions of macroblock mb, the search having missed at
 * macroblock mb0 (mb >= mb0) with inputs `want`:
 *   0  every partition gets `want` (uniform motion);
 *   1  each partition gets what the same partition of mb0's left neighbour was searched with;
 *   2  ... of mb's upper neighbour (when that row is done);
 *   3  ... of mb0 itself, so far (the next macroblocks move like this one).
 * Partitions without a known source take `want`.  Returns 0 when the guess has
 * no source at all.  Only inputs are guessed: a cached result is used only for
 * a call whose inputs equal them. */
static int spec_hyp(int list, int ref, int h, int mb0, int mb, const spec_ent *want, int chk00_slot0, spec_ent *out)
{
  const spec_ent *seen = g_seen[list][ref], *src = NULL;
  int s, any = (h == 0), fmb = -1;
  if (h == 1 && mb0 > 0) fmb = mb0 - 1;
  if (h == 2 && mb - g_mbs_x >= 0 && mb - g_mbs_x < mb0) fmb = mb - g_mbs_x;
  if (h == 3 && mb > mb0) fmb = mb0;
  for (s = 0; s < JMME_NSLOT; s++) {
    src = fmb >= 0 ? &seen[(size_t)fmb * JMME_NSLOT + s] : NULL;
    if (src && src->valid == g_slot_gen[list][ref] && src->mode == want->mode) {
      out[s] = *src;
      any = 1;
    } else {
      out[s] = *want;
    }
    out[s].chk = (int16_t)(!want->mode && s == 0 && chk00_slot0);
    out[s].valid = 0;
  }
  if (want->mode)                         /* FFS: one surface centre per macroblock */
    for (s = 1; s < JMME_NSLOT; s++) {
      out[s].fcx = out[0].fcx;
      out[s].fcy = out[0].fcy;
      out[s].frange = out[0].frange;
    }
  return any;
}

/* ---- chained guesses inside the missing macroblock ---------------------------
 * A partition's predictor reads the vectors JM just gave its neighbours inside
 * the macroblock (set_me_parameters after each search, mv_search.c:1614,1720),
 * so a guess taken from other macroblocks fails wherever the vectors of one
 * macroblock differ (the padding rows of a 1080-line picture; any non-uniform
 * motion).  On a miss the adapter therefore also sends the partitions of the
 * same macroblock whose neighbours are decided by now as chains
 * (jmme_search_mbs_chains): the rest of the missing partition's group (a
 * 16x8 / 8x16 pair, or one sub-mode of one 8x8 quadrant) and the groups JM
 * searches after it before the next mode decision -- the other pairs and
 * quadrant 0 after a 16x16 / 16x8 / 8x16 miss, the quadrant's later sub-modes
 * after a quadrant miss.  Each neighbour is taken from JM's get_neighbors and
 * is either a vector JM's mv_info already holds for good (neighbouring
 * macroblocks, earlier quadrants, read now) or an earlier step of the chain;
 * the GPU derives predictor and centre from them as BlockMotionSearch does and
 * searches.  The answers land in cache way KHYP and, like every guess, are used
 * only when JM's real call carries the derived inputs.  Single reference, P
 * slices, integer-pel results only (sub-pel refinement would change the
 * neighbours' vectors), no 8x8 transform (its second pass over the quadrants),
 * JMME_CHAINS=0 turns it off. */
static jmme_chain g_chains[8];
static jmme_chain_res g_chres[8 * JMME_CHAIN_MAX_STEPS];
/* sub-pel on (DisableSubpelME = 0): the chains run SubPelME after every step
 * (jmme_search_mbs_chains_sp), so the later steps read refined vectors as JM's
 * do; g_chain_sp is the SubPelME template of this miss's chains and the
 * refinements land in the sub-pel cache's chain way */
static jmme_subpel_req g_chain_sp[8];
static jmme_block_res g_chspres[8 * JMME_CHAIN_MAX_STEPS];
static int g_chain_sp_on = 0;
static long long g_chain_sp_steps = 0, g_chain_sp_hits = 0, g_chain_sp_nolam = 0;
static int chain_subpel_template(Macroblock *currMB, MEBlock *mv_block, int list, int ref, int lambda_f);
static void store_chain_subpel(int list, int ref, int mb, int sl, const jmme_chain_res *r, const jmme_block_res *f);
static int g_n_chains = 0, g_chain_on = -1, g_chain_head = -1;
static int8_t g_slot_bt[JMME_NSLOT], g_slot_bx[JMME_NSLOT], g_slot_by[JMME_NSLOT];   /* slot_geometry() */
static void slot_geometry(void);
static long long g_chain_sent = 0, g_chain_steps = 0, g_chain_hits = 0, g_chain_head_bad = 0;
static long long g_chain_calls = 0, g_chain_call_fail = 0;
static double g_t_chain = 0, g_t_sp = 0;   /* ms in chain-only calls / sub-pel batches (reported at exit) */
static double g_t_sp_part[3];               /* sub-pel batches: building, the library call, storing (us) */
static int g_chain_only = -1;   /* JMME_CHAIN_ONLY=0: a failed guess always re-batches */
static int8_t g_grp[19][4], g_grp_n[19], g_slot_grp[JMME_NSLOT], g_slot_idx[JMME_NSLOT];

/* JM's search order of a macroblock's partitions as groups whose members chain:
 * 16x16; 16x8; 8x16; then per quadrant q: 8x8, 8x4, 4x8, 4x4 (md_low.c:185-304,
 * mode_decision_P8x8.c:101-135, mv_search.c:1686-1760) */
static void chain_groups(void)
{
  int g = 0, q, i;
  g_grp[g][0] = 0; g_grp_n[g++] = 1;
  g_grp[g][0] = 1; g_grp[g][1] = 2; g_grp_n[g++] = 2;
  g_grp[g][0] = 3; g_grp[g][1] = 4; g_grp_n[g++] = 2;
  for (q = 0; q < 4; q++) {
    const int bx = 2 * (q & 1), by = 2 * (q >> 1);
    g_grp[g][0] = (int8_t)jmme_slot(4, bx, by); g_grp_n[g++] = 1;
    g_grp[g][0] = (int8_t)jmme_slot(5, bx, by); g_grp[g][1] = (int8_t)jmme_slot(5, bx, by + 1); g_grp_n[g++] = 2;
    g_grp[g][0] = (int8_t)jmme_slot(6, bx, by); g_grp[g][1] = (int8_t)jmme_slot(6, bx + 1, by); g_grp_n[g++] = 2;
    g_grp[g][0] = (int8_t)jmme_slot(7, bx, by); g_grp[g][1] = (int8_t)jmme_slot(7, bx + 1, by);
    g_grp[g][2] = (int8_t)jmme_slot(7, bx, by + 1); g_grp[g][3] = (int8_t)jmme_slot(7, bx + 1, by + 1);
    g_grp_n[g++] = 4;
  }
  for (g = 0; g < 19; g++)
    for (i = 0; i < g_grp_n[g]; i++) { g_slot_grp[g_grp[g][i]] = (int8_t)g; g_slot_idx[g_grp[g][i]] = (int8_t)i; }
}

static int chains_on(Macroblock *currMB, int list, int ref)
{
  VideoParameters *p_Vid = currMB->p_Vid;
  InputParameters *p_Inp = currMB->p_Inp;
  Slice *currSlice = currMB->p_Slice;
  if (g_chain_on < 0) {
    const char *e = getenv("JMME_CHAINS");
    g_chain_on = !(e && e[0] == '0');
    chain_groups();
    if (!g_slot_bt[0]) slot_geometry();
  }
  (void)p_Vid;
  return g_chain_on && currSlice->slice_type == P_SLICE && currSlice->structure == FRAME &&
         currMB->list_offset == 0 && list == 0 && ref == 0 && currSlice->listXsize[0] == 1 &&
         !p_Inp->Transform8x8Mode;
}

/* chains for this miss: integer-pel, or with SubPelME when it is on and its
 * template (every step's SubPelME parameters but the step's own block,
 * predictor and answer) is known */
static int chains_ready(Macroblock *currMB, MEBlock *mv_block, int list, int ref, const spec_ent *want)
{
  if (!chains_on(currMB, list, ref)) return 0;
  g_chain_sp_on = !currMB->p_Inp->DisableSubpelME[currMB->p_Vid->view_id];
  return !g_chain_sp_on || chain_subpel_template(currMB, mv_block, list, ref, want->lambda);
}

/* one chain: group g's partitions from index i0, in JM's order */
static void chain_fill(jmme_chain *c, Macroblock *currMB, int list, int ref, int g, int i0, const spec_ent *want)
{
  static const int bw[8] = {0, 16, 16, 8, 8, 8, 4, 4}, bh[8] = {0, 16, 8, 16, 8, 4, 8, 4};
  VideoParameters *p_Vid = currMB->p_Vid;
  InputParameters *p_Inp = currMB->p_Inp;
  PicMotionParams **mvi = p_Vid->enc_picture->mv_info;
  MEFullFast *ff = p_Vid->p_ffast_me;
  MEBlock tmp;
  int k, j, kk;
  memset(c, 0, sizeof *c);
  c->mb_x = (int16_t)currMB->pix_x;
  c->mb_y = (int16_t)currMB->pix_y;
  c->list = (int16_t)list;
  c->ref_idx = (int16_t)ref;
  c->rdopt = (int16_t)p_Inp->rdopt;
  c->lambda = want->lambda;
  c->mv_lim_x0 = (int16_t)p_Vid->MaxHmvR[4]; c->mv_lim_x1 = (int16_t)p_Vid->MaxHmvR[5];
  c->mv_lim_y0 = (int16_t)p_Vid->MaxVmvR[4]; c->mv_lim_y1 = (int16_t)p_Vid->MaxVmvR[5];
  if (want->mode) {
    c->ffs_center_x = ff->search_center[list][ref].mv_x;
    c->ffs_center_y = ff->search_center[list][ref].mv_y;
    c->ffs_range = (int16_t)ff->max_search_range[list][ref];
    c->ffs_pos00_valid = (int16_t)(p_Inp->rdopt == 0);
  }
  memset(&tmp, 0, sizeof tmp);
  tmp.p_Vid = p_Vid;
  for (k = 0; k < g_grp_n[g] - i0; k++) {
    const int sl = g_grp[g][i0 + k], bt = g_slot_bt[sl];
    jmme_chain_step *st = &c->steps[k];
    PixelPos block[4];
    st->slot = (int16_t)sl;
    /* check_for_00 as me_fullsearch.c:61 (chains: P slices, reference 0) */
    st->flags = (int16_t)(!want->mode && sl == 0 && !p_Inp->rdopt ? JMME_CHAIN_CHECK00 : 0);
    get_neighbors(currMB, block, g_slot_bx[sl], g_slot_by[sl], bw[bt]);
    for (j = 0; j < 3; j++) {
      jmme_chain_nb *nb = &st->nb[j];
      const int lx = block[j].pos_x - currMB->block_x, ly = block[j].pos_y - currMB->block_y;
      nb->src = JMME_NB_UNAVAILABLE;
      if (!block[j].available) continue;
      if (lx >= 0 && lx < 4 && ly >= 0 && ly < 4)   /* inside: an earlier step of this chain? */
        for (kk = 0; kk < k; kk++) {
          const int o = c->steps[kk].slot, ox = g_slot_bx[o] >> 2, oy = g_slot_by[o] >> 2;
          if (lx >= ox && lx < ox + (bw[g_slot_bt[o]] >> 2) && ly >= oy && ly < oy + (bh[g_slot_bt[o]] >> 2))
            nb->src = (int16_t)kk;
        }
      if (nb->src == JMME_NB_UNAVAILABLE) {       /* decided by now: JM's mv_info */
        nb->src = JMME_NB_FIXED;
        nb->ref_idx = mvi[block[j].pos_y][block[j].pos_x].ref_idx[list];
        nb->mv_x = mvi[block[j].pos_y][block[j].pos_x].mv[list].mv_x;
        nb->mv_y = mvi[block[j].pos_y][block[j].pos_x].mv[list].mv_y;
      }
    }
    get_search_range(&tmp, p_Inp, (short)ref, bt);
    st->sr_min_x = (int16_t)tmp.searchRange.min_x; st->sr_max_x = (int16_t)tmp.searchRange.max_x;
    st->sr_min_y = (int16_t)tmp.searchRange.min_y; st->sr_max_y = (int16_t)tmp.searchRange.max_y;
  }
  c->n_steps = (int16_t)k;
}

/* the chains that are decided at a miss of slot s of macroblock mb (the current one) */
static int build_chains(Macroblock *currMB, int list, int ref, int mb, int s, const spec_ent *want, int with_s)
{
  const int g0 = g_slot_grp[s], i0 = g_slot_idx[s];
  int n = 0, g, g1;
  (void)mb;
  g_chain_head = -1;
  if (with_s || i0 + 1 < g_grp_n[g0]) {             /* the rest of s's group, s first */
    chain_fill(&g_chains[n++], currMB, list, ref, g0, i0, want);
    g_chain_head = s;
  }
  g1 = g0 <= 2 ? 6 : 3 + 4 * ((g0 - 3) / 4) + 3;   /* through quadrant 0 / through s's quadrant */
  for (g = g0 + 1; g <= g1 && n < 8; g++)
    if (g_grp_n[g] > 1 || g0 <= 2) chain_fill(&g_chains[n++], currMB, list, ref, g, 0, want);
  for (g = 1; g_chain_sp_on && g < n; g++) g_chain_sp[g] = g_chain_sp[0];
  return n;
}

/* the chains' answers -> way KHYP of their (macroblock, slot) */
static void store_chains(int list, int ref, const spec_ent *want)
{
  spec_ent *tab = g_spec[list][ref];
  int i, k;
  for (i = 0; i < g_n_chains; i++) {
    const jmme_chain *c = &g_chains[i];
    const int mb = (c->mb_y >> 4) * g_mbs_x + (c->mb_x >> 4);
    ++g_chain_sent;
    for (k = 0; k < c->n_steps; k++) {
      const jmme_chain_res *r = &g_chres[i * JMME_CHAIN_MAX_STEPS + k];
      const int sl = c->steps[k].slot;
      spec_ent *e = &tab[spec_idx(mb, sl, KHYP)];
      if (r->cost < 0) break;
      memset(e, 0, sizeof *e);
      e->mode = want->mode;
      e->px = r->pred_x; e->py = r->pred_y;
      e->lambda = want->lambda;
      if (want->mode) {
        e->sr = r->range_max;
        e->fcx = c->ffs_center_x; e->fcy = c->ffs_center_y; e->frange = c->ffs_range;
      } else {
        e->cx = r->center_x; e->cy = r->center_y;
        e->sr = r->range_min;
        e->chk = (int16_t)((c->steps[k].flags & JMME_CHAIN_CHECK00) != 0);
      }
      e->mvx = r->mv_x; e->mvy = r->mv_y; e->cost = r->cost;
      e->valid = g_slot_gen[list][ref];
      ++g_chain_steps;
      if (g_chain_sp_on) store_chain_subpel(list, ref, mb, sl, r, &g_chspres[i * JMME_CHAIN_MAX_STEPS + k]);
      /* the chain's first step is the missing call itself: its derived inputs must be the real ones */
      if (i == 0 && k == 0 && sl == g_chain_head && !spec_key_eq(e, want)) ++g_chain_head_bad;
    }
  }
  g_n_chains = 0;
}

/* the engine's buffers for the largest batch, sized at start-up */
static void reserve_batches(void)
{
  if (jmme_reserve(g_me, MAX_BATCH * KHYP)) fail_jm("jmme_reserve");
}

/* one batched search: all 41 partitions of macroblocks mb0.., under every distinct guess */
static int rows_eq(const spec_ent *a, const spec_ent *b)
{
  int s;
  for (s = 0; s < JMME_NSLOT; s++)
    if (!spec_key_eq(&a[s], &b[s])) return 0;
  return 1;
}

static void spec_batch(int list, int ref, int mb0, const spec_ent *want, int chk00_slot0, int rdopt)
{
  static spec_ent hc[4][JMME_NSLOT];
  int ok[4] = {0, 0, 0, 0};
  spec_ent *tab = g_spec[list][ref];
  int n = imin(g_batch, g_n_mb - mb0), nreq = 0, i, s, k, mb;
  double t0 = now_us(), t1, t2;
  if (n * KHYP > g_req_cap) {
    free(g_req);
    free(g_res);
    free(g_hyp);
    free(g_req_mb);
    free(g_req_row);
    g_req_cap = n * KHYP;
    g_req = (jmme_mb_req *)malloc((size_t)g_req_cap * sizeof(jmme_mb_req));
    g_res = (jmme_block_res *)malloc((size_t)g_req_cap * JMME_NSLOT * sizeof(jmme_block_res));
    g_hyp = (spec_ent *)malloc((size_t)g_req_cap * JMME_NSLOT * sizeof(spec_ent));
    g_req_mb = (int *)malloc((size_t)g_req_cap * sizeof(int));
    g_req_row = (const spec_ent **)malloc((size_t)g_req_cap * sizeof(*g_req_row));
    if (!g_req || !g_res || !g_hyp || !g_req_mb || !g_req_row) error("jm_gpu_me: out of memory", 500);
  }
  /* guesses 0, 1 and 3 are the same rows for every macroblock of the batch
   * (want; mb0's left neighbour; mb0 itself): built and compared once */
  ok[0] = spec_hyp(list, ref, 0, mb0, mb0, want, chk00_slot0, hc[0]);
  ok[1] = spec_hyp(list, ref, 1, mb0, mb0, want, chk00_slot0, hc[1]);
  ok[3] = mb0 + 1 < g_n_mb && spec_hyp(list, ref, 3, mb0, mb0 + 1, want, chk00_slot0, hc[3]);
  ok[1] = ok[1] && !rows_eq(hc[1], hc[0]);
  ok[3] = ok[3] && !rows_eq(hc[3], hc[0]) && !(ok[1] && rows_eq(hc[3], hc[1]));
  for (mb = mb0; mb < mb0 + n; mb++) {
    const spec_ent *rows[KHYP];
    spec_ent *h2 = &g_hyp[(size_t)(mb - mb0) * JMME_NSLOT];
    int nr = 0, j;
    rows[nr++] = hc[0];
    if (ok[1]) rows[nr++] = hc[1];
    if (spec_hyp(list, ref, 2, mb0, mb, want, chk00_slot0, h2)) {
      int dup = 0;
      for (j = 0; j < nr && !dup; j++) dup = rows_eq(rows[j], h2);
      if (!dup) rows[nr++] = h2;
    }
    if (mb > mb0 && ok[3] && !(nr > 1 && rows[nr - 1] == h2 && rows_eq(hc[3], h2))) rows[nr++] = hc[3];
    for (j = 0; j < nr; j++) {
      const spec_ent *hy = rows[j];
      jmme_mb_req *r = &g_req[nreq];
      memset(r, 0, sizeof *r);
      r->mb_x = (int16_t)((mb % g_mbs_x) * 16);
      r->mb_y = (int16_t)((mb / g_mbs_x) * 16);
      r->list = (int16_t)list;
      r->ref_idx = (int16_t)ref;
      r->slot_mask = (1ull << JMME_NSLOT) - 1;
      if (want->mode) {                  /* FFS: the MB's surface (setup_fast_full_search) */
        r->ffs_center_x = hy[0].fcx;
        r->ffs_center_y = hy[0].fcy;
        r->ffs_range = hy[0].frange;
        r->ffs_pos00_valid = (int16_t)(rdopt == 0);
      }
      for (s = 0; s < JMME_NSLOT; s++) {
        jmme_block_req *b = &r->blk[s];
        b->pred_x = hy[s].px;
        b->pred_y = hy[s].py;
        b->center_x = hy[s].cx;
        b->center_y = hy[s].cy;
        b->search_range = hy[s].sr;
        b->flags = (int16_t)(hy[s].chk ? JMME_BLK_CHECK00 : 0);
        b->lambda = hy[s].lambda;
      }
      g_req_row[nreq] = hy;
      g_req_mb[nreq++] = mb;
    }
  }
  t1 = now_us();
  if (jmme_search_mbs_chains_sp(g_me, want->mode ? JMME_FAST_FULL_SEARCH : JMME_FULL_SEARCH, g_req, nreq, g_res,
                                g_chains, g_n_chains, g_chain_sp_on ? g_chain_sp : NULL, g_chres, g_chspres))
    fail_jm("jmme_search_mbs_chains_sp");
  t2 = now_us();
  g_t_build += t1 - t0;
  g_t_call += t2 - t1;
  g_units += nreq;
  if (g_trace) fprintf(g_trace, "%d %d %d %.1f %.1f\n", mb0, n, nreq, t1 - t0, t2 - t1);
  for (i = 0; i < nreq; i++) {
    mb = g_req_mb[i];
    k = (i == 0 || g_req_mb[i - 1] != mb) ? 0 : k + 1;       /* guesses of one MB are consecutive */
    /* (older guesses in the ways above k stay: a cached answer is exact for its
     * inputs on these planes, whichever batch searched it) */
    for (s = 0; s < JMME_NSLOT; s++) {
      spec_ent *e = &tab[spec_idx(mb, s, k)];
      *e = g_req_row[i][s];
      e->mvx = g_res[i * JMME_NSLOT + s].mv_x;
      e->mvy = g_res[i * JMME_NSLOT + s].mv_y;
      e->cost = g_res[i * JMME_NSLOT + s].cost;
      e->valid = g_slot_gen[list][ref];
    }
  }
  g_spec_end[list][ref] = mb0 + n;
  ++g_batches;
  store_chains(list, ref, want);
}

static int speculating(void)
{
  if (g_speculate < 0) {
    const char *e = getenv("JMME_SPECULATE"), *t = getenv("JMME_TRACE");
    g_speculate = !(e && e[0] == '0');
    if (t && *t) g_trace = fopen(t, "w");     /* per batch: mb0 n units build_us call_us */
    t = getenv("JMME_TRACE_MISS");
    if (t && *t) g_trace_miss = fopen(t, "w");
  }
  return g_speculate;
}

/* the cached answer for this call, batching on a miss */
/* the sub-pel call that follows an integer answer usually finds its refinement in
 * the matching way of the sub-pel cache (way k for integer way k, way KHYP + 1 for a
 * chain's answer): probed first, and prefetched when the integer answer is found */
static int g_sp_hint_mb = -1, g_sp_hint_s = -1, g_sp_hint_k = 0;
static void sp_hint(int list, int ref, int mb, int s, int k);
static void sp_prefetch_row(int list, int ref, int mb);

static const spec_ent *spec_lookup(Macroblock *currMB, MEBlock *mv_block, int list, int ref, const spec_ent *want,
                                   int chk_rule)
{
  VideoParameters *p_Vid = currMB->p_Vid;
  int mb = (mv_block->pos_y >> 4) * (p_Vid->width / 16) + (mv_block->pos_x >> 4);
  int s = jmme_slot(mv_block->blocktype, (mv_block->pos_x & 15) >> 2, (mv_block->pos_y & 15) >> 2), k;
  spec_ent *tab = spec_table(p_Vid, list, ref), *e;
  if (s < 0 || mb < 0 || mb >= g_n_mb) error("jm_gpu_me: block outside the picture", 500);
  if (s == 0 && mb + 1 < g_n_mb) {   /* a new macroblock: fetch the next one's way 0 and inputs row */
    const char *a = (const char *)&tab[spec_idx(mb + 1, 0, 0)], *b = (const char *)&g_seen[list][ref][(size_t)(mb + 1) * JMME_NSLOT];
    size_t o;
    for (o = 0; o < JMME_NSLOT * sizeof(spec_ent); o += 64) {
      __builtin_prefetch(a + o, 0, 1);
      __builtin_prefetch(b + o, 1, 1);
    }
    sp_prefetch_row(list, ref, mb + 1);
  }
  g_seen[list][ref][(size_t)mb * JMME_NSLOT + s] = *want;
  g_seen[list][ref][(size_t)mb * JMME_NSLOT + s].valid = g_slot_gen[list][ref];
  for (k = 0; k < KWAYS; k++) {
    e = &tab[spec_idx(mb, s, k)];
    if (spec_same(e, want, g_slot_gen[list][ref])) {
      ++g_hits;
      if (k == KHYP) ++g_chain_hits;
      sp_hint(list, ref, mb, s, k);
      return e;
    }
  }
  g_sp_hint_mb = -1;
  const int failed = mb < g_spec_end[list][ref];
  if (failed) {                                                          /* every guess failed */
    ++g_miss_guess;
    ++g_miss_slot[s];
    if (g_trace_miss) {   /* JMME_TRACE_MISS: the inputs that missed and the guesses held for them */
      fprintf(g_trace_miss, "miss mb %d slot %d want c(%d,%d) p(%d,%d) sr %d chk %d lam %d |", mb, s, want->cx, want->cy,
              want->px, want->py, want->sr, want->chk, want->lambda);
      for (k = 0; k < KWAYS; k++) {
        e = &tab[spec_idx(mb, s, k)];
        if (e->valid == g_slot_gen[list][ref])
          fprintf(g_trace_miss, " g%d c(%d,%d) p(%d,%d) sr %d chk %d lam %d", k, e->cx, e->cy, e->px, e->py, e->sr,
                  e->chk, e->lambda);
      }
      fprintf(g_trace_miss, "\n");
    }
  } else {                                                               /* ran past the batch */
    g_batch = imin(MAX_BATCH, g_batch * 2);
    ++g_miss_past;
  }
  if (g_chain_only < 0) {
    const char *c = getenv("JMME_CHAIN_ONLY");
    g_chain_only = !(c && c[0] == '0');
  }
  if (g_chain_only && failed && s != 0 && chains_ready(currMB, mv_block, list, ref, want)) {
    /* a failed guess inside a macroblock whose 16x16 search hit: the
     * macroblock's decided partitions as chains, the missing call first, and no
     * batch (the guesses for the macroblocks after this one stand).  A 16x16
     * miss says the guesses themselves are off: that one re-batches. */
    double tc = now_us();
    g_n_chains = build_chains(currMB, list, ref, mb, s, want, 1);
    if (jmme_search_mbs_chains_sp(g_me, want->mode ? JMME_FAST_FULL_SEARCH : JMME_FULL_SEARCH, g_req, 0, g_res,
                                  g_chains, g_n_chains, g_chain_sp_on ? g_chain_sp : NULL, g_chres, g_chspres))
      fail_jm("jmme_search_mbs_chains_sp");
    ++g_chain_calls;
    store_chains(list, ref, want);
    g_t_chain += now_us() - tc;
    e = &tab[spec_idx(mb, s, KHYP)];
    if (spec_same(e, want, g_slot_gen[list][ref])) return e;
    ++g_chain_call_fail;   /* (the chain stopped before it: a half-way centre or an oversized range) */
  }
  if (failed) g_batch = imax(1, g_batch / 2);   /* a re-batch after a failed guess: shorter */
  g_n_chains = chains_ready(currMB, mv_block, list, ref, want) ? build_chains(currMB, list, ref, mb, s, want, 0) : 0;
  spec_batch(list, ref, mb, want, chk_rule, currMB->p_Inp->rdopt);
  e = &tab[spec_idx(mb, s, 0)];
  if (!spec_same(e, want, g_slot_gen[list][ref])) error("jm_gpu_me: batch lost its own request", 500);
  return e;
}

/* full_search_motion_estimation's contract (me_fullsearch.c:39-103) */
distblk __wrap_full_search_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                             distblk min_mcost, int lambda_factor)
{
  Slice *currSlice = currMB->p_Slice;
  int list = mv_block->list, ref = mv_block->ref_idx;
  /* search_range and check_for_00 as me_fullsearch.c:49,61 derive them */
  int search_range = imin(mv_block->searchRange.max_x, mv_block->searchRange.max_y) >> 2;
  int chk_rule = !currMB->p_Inp->rdopt && currSlice->slice_type != B_SLICE && ref == 0;
  int check_for_00 = mv_block->blocktype == 1 && chk_rule;
  jmme_mv pred = {pred_mv->mv_x, pred_mv->mv_y};
  jmme_mv mv = {mv_block->mv[list].mv_x, mv_block->mv[list].mv_y};   /* centre in */
  distblk cost;
  double t_in;
  if (fs_on_cpu(mv_block)) {
    ++g_cpu_calls;
    return __real_full_search_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
  }
  t_in = (speculating() && g_trace) ? now_us() : 0;
  ensure_planes(currMB, list, ref);
  ++g_calls;
  if (speculating()) {
    spec_ent want;
    const spec_ent *e;
    memset(&want, 0, sizeof want);
    want.cx = mv.mv_x; want.cy = mv.mv_y; want.px = pred.mv_x; want.py = pred.mv_y;
    want.sr = (int16_t)search_range; want.chk = (int16_t)check_for_00; want.lambda = lambda_factor;
    e = spec_lookup(currMB, mv_block, list, ref, &want, chk_rule);
    cost = e->cost;
    if (g_trace) g_t_wrap += now_us() - t_in;
    if (cost >= min_mcost) return min_mcost;
    mv_block->mv[list].mv_x = e->mvx;
    mv_block->mv[list].mv_y = e->mvy;
    return cost;
  }
  cost = jmme_full_search_block(g_me, list, ref, mv_block->pos_x, mv_block->pos_y, mv_block->blocktype, &pred, &mv,
                                min_mcost, lambda_factor, search_range, check_for_00);
  mv_block->mv[list].mv_x = mv.mv_x;                                     /* best out */
  mv_block->mv[list].mv_y = mv.mv_y;
  return cost;
}

/* setup_fast_full_search without the CPU SAD surface: the search centre of
 * me_fullfast.c:312-327 (predictor of the 16x16 block, rounded, clipped so
 * that (0,0) stays inside when RDO is off, then to the level's MV range) */
void __wrap_setup_fast_full_search(Macroblock *currMB, MEBlock *mv_block, int list)
{
  VideoParameters *p_Vid = currMB->p_Vid;
  InputParameters *p_Inp = currMB->p_Inp;
  MEFullFast *ff = p_Vid->p_ffast_me;
  short ref = mv_block->ref_idx;
  int search_range = ff->max_search_range[list][ref] << 2;
  PixelPos block[4];
  MotionVector pmv, *c = &ff->search_center[list][ref];
  if (ffs_on_cpu(currMB, mv_block)) {          /* JM's own surface for JM's own search */
    __real_setup_fast_full_search(currMB, mv_block, list);
    return;
  }
  get_neighbors(currMB, block, 0, 0, 16);
  currMB->GetMVPredictor(currMB, block, &pmv, ref, p_Vid->enc_picture->mv_info, list, 0, 0, 16, 16);
  c->mv_x = (short)(((pmv.mv_x + 2) >> 2) * 4);              /* JM_INT_DIVIDE (defines.h:44) */
  c->mv_y = (short)(((pmv.mv_y + 2) >> 2) * 4);
  if (!p_Inp->rdopt) {
    c->mv_x = (short)iClip3(-search_range, search_range, c->mv_x);
    c->mv_y = (short)iClip3(-search_range, search_range, c->mv_y);
  }
  c->mv_x = (short)iClip3(p_Vid->MaxHmvR[4] + search_range, p_Vid->MaxHmvR[5] - search_range, c->mv_x);
  c->mv_y = (short)iClip3(p_Vid->MaxVmvR[4] + search_range, p_Vid->MaxVmvR[5] - search_range, c->mv_y);
  ff->search_setup_done[list][ref] = 1;
}

/* fast_full_search_motion_estimation's contract (me_fullfast.c:618-689) */
distblk __wrap_fast_full_search_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                                  distblk min_mcost, int lambda_factor)
{
  VideoParameters *p_Vid = currMB->p_Vid;
  MEFullFast *ff = p_Vid->p_ffast_me;
  int list = mv_block->list, ref = mv_block->ref_idx;
  jmme_mv pred = {pred_mv->mv_x, pred_mv->mv_y}, centre, mv;
  distblk cost;
  if (ffs_on_cpu(currMB, mv_block)) {
    ++g_cpu_calls;
    return __real_fast_full_search_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
  }
  if (!ff->search_setup_done[list][ref]) currMB->p_SetupFastFullPelSearch(currMB, mv_block, list);
  centre.mv_x = ff->search_center[list][ref].mv_x;
  centre.mv_y = ff->search_center[list][ref].mv_y;
  ensure_planes(currMB, list, ref);
  ++g_calls;
  if (speculating()) {
    spec_ent want;
    const spec_ent *e;
    memset(&want, 0, sizeof want);
    want.mode = 1;
    want.px = pred.mv_x; want.py = pred.mv_y;
    want.sr = (int16_t)(imax(mv_block->searchRange.max_x, mv_block->searchRange.max_y) >> 2);
    want.fcx = centre.mv_x; want.fcy = centre.mv_y;
    want.frange = (int16_t)ff->max_search_range[list][ref];
    want.lambda = lambda_factor;
    e = spec_lookup(currMB, mv_block, list, ref, &want, 0);
    cost = e->cost;
    if (cost >= min_mcost) {                /* nothing beat the bound: JM keeps the centre */
      mv_block->mv[list].mv_x = centre.mv_x;
      mv_block->mv[list].mv_y = centre.mv_y;
      return min_mcost;
    }
    mv_block->mv[list].mv_x = e->mvx;
    mv_block->mv[list].mv_y = e->mvy;
    return cost;
  }
  cost = jmme_fast_full_search_block(g_me, list, ref, mv_block->pos_x, mv_block->pos_y, mv_block->blocktype, &pred,
                                     &centre, ff->max_search_range[list][ref],
                                     imax(mv_block->searchRange.max_x, mv_block->searchRange.max_y) >> 2,
                                     currMB->p_Inp->rdopt, &mv, min_mcost, lambda_factor);
  mv_block->mv[list].mv_x = mv.mv_x;
  mv_block->mv[list].mv_y = mv.mv_y;
  return cost;
}

/* ---- sub-pel refinement (SubPelME) ------------------------------------------
 * Speculated like the integer search: a sub-pel batch covers the macroblocks
 * whose integer results are cached, each slot guessed with each of that slot's
 * cached integer answers (vector, cost, predictor) and this call's lambdas,
 * metrics and switches; a call uses a cached answer only when every input
 * matches. */
typedef struct sp_ent {
  int16_t px, py, mx, my;
  int64_t min_mcost;
  int32_t lam_h, lam_q;
  uint8_t metric_h, metric_q, start_hp, start_qp, pos2, pos4, flags;
  uint32_t valid;                             /* the g_slot_gen it was cached in (0: none) */
  int16_t omx, omy;
  int64_t cost;
} sp_ent;

static sp_ent *g_sp[2][32];
static unsigned g_sp_gen[2][32];   /* g_slot_gen the cached refinements belong to */
static long long g_sp_calls = 0, g_sp_hits = 0, g_sp_batches = 0, g_sp_cpu = 0;
static jmme_subpel_req *g_sreq = NULL;
static jmme_block_res *g_sres = NULL;
static int g_sreq_cap = 0;
static int8_t g_slot_bt[JMME_NSLOT], g_slot_bx[JMME_NSLOT], g_slot_by[JMME_NSLOT];

static int metric_id(distblk (*f)(StorablePicture *, MEBlock *, distblk, MotionVector *))
{
  if (f == computeSAD) return 0;
  if (f == computeSSE) return 1;
  if (f == computeSATD) return 2;
  return -1;                                  /* weighted / on-the-fly: stays on the CPU */
}

static int sp_same(const sp_ent *e, const sp_ent *w, unsigned gen)
{
  return e->valid == gen && e->px == w->px && e->py == w->py && e->mx == w->mx && e->my == w->my &&
         e->min_mcost == w->min_mcost && e->lam_h == w->lam_h && e->lam_q == w->lam_q &&
         e->metric_h == w->metric_h && e->metric_q == w->metric_q && e->start_hp == w->start_hp &&
         e->start_qp == w->start_qp && e->pos2 == w->pos2 && e->pos4 == w->pos4 && e->flags == w->flags;
}

static void slot_geometry(void)
{
  static const int bw[8] = {0, 16, 16, 8, 8, 8, 4, 4}, bh[8] = {0, 16, 8, 16, 8, 4, 8, 4};
  int bt, x, y, sl;
  for (bt = 1; bt <= 7; bt++)
    for (y = 0; y < 16; y += bh[bt])
      for (x = 0; x < 16; x += bw[bt]) {
        sl = jmme_slot(bt, x >> 2, y >> 2);
        if (sl >= 0) { g_slot_bt[sl] = (int8_t)bt; g_slot_bx[sl] = (int8_t)x; g_slot_by[sl] = (int8_t)y; }
      }
}

#define SPK (KHYP + 2)                  /* sub-pel answers kept per (macroblock, slot): the KHYP guesses,
                                           the real call (way KHYP), the chains' refinement (way KHYP + 1) */
static int *g_sp_dst = NULL;
/* way-major like the integer table: a macroblock's 41 entries of one way are contiguous */
static inline size_t sp_idx(int mb, int s, int k) { return ((size_t)mb * SPK + k) * JMME_NSLOT + s; }

static void sp_prefetch_row(int list, int ref, int mb)   /* the macroblock's way-0 sub-pel entries */
{
  const sp_ent *t = g_sp[list][ref];
  size_t o;
  if (!t) return;
  for (o = 0; o < JMME_NSLOT * sizeof(sp_ent); o += 64) __builtin_prefetch((const char *)&t[sp_idx(mb, 0, 0)] + o, 0, 1);
}

static void sp_hint(int list, int ref, int mb, int s, int k)
{
  const sp_ent *t = g_sp[list][ref];
  g_sp_hint_mb = mb;
  g_sp_hint_s = s;
  g_sp_hint_k = k < KHYP ? k : KHYP + 1;
  if (t) __builtin_prefetch(&t[sp_idx(mb, s, g_sp_hint_k)], 0, 1);
}

static void sp_fill(jmme_subpel_req *q, int mb, int s, int list, int ref, const sp_ent *w)
{
  memset(q, 0, sizeof *q);
  q->pos_x = (int16_t)((mb % g_mbs_x) * 16 + g_slot_bx[s]);
  q->pos_y = (int16_t)((mb / g_mbs_x) * 16 + g_slot_by[s]);
  q->blocktype = (int16_t)g_slot_bt[s];
  q->ref_slot = (int16_t)(list * 32 + ref);
  q->pred_x = w->px;
  q->pred_y = w->py;
  q->mv_x = w->mx;
  q->mv_y = w->my;
  q->lambda_h = w->lam_h;
  q->lambda_q = w->lam_q;
  q->min_mcost = w->min_mcost;
  q->variant = 0;
  q->flags = w->flags;
  q->metric_h = w->metric_h;
  q->metric_q = w->metric_q;
  q->start_hp = w->start_hp;
  q->start_qp = w->start_qp;
  q->search_pos2 = w->pos2;
  q->search_pos4 = w->pos4;
}

/* one batched refinement: the calling block with its real inputs (answer kept
 * in way KHYP) and, for the macroblocks the integer cache covers, every cached
 * integer answer of every slot (way k for integer way k) */
/* the batch buffers for `count` requests (touched: the pages are faulted in here) */
static void sp_reserve(int count)
{
  if (count <= g_sreq_cap) return;
  free(g_sreq);
  free(g_sres);
  free(g_sp_dst);
  g_sreq = (jmme_subpel_req *)malloc((size_t)count * sizeof(jmme_subpel_req));
  g_sres = (jmme_block_res *)malloc((size_t)count * sizeof(jmme_block_res));
  g_sp_dst = (int *)malloc((size_t)count * sizeof(int));
  if (!g_sreq || !g_sres || !g_sp_dst) error("jm_gpu_me: out of memory", 500);
  memset(g_sreq, 0, (size_t)count * sizeof(jmme_subpel_req));
  memset(g_sres, 0, (size_t)count * sizeof(jmme_block_res));
  memset(g_sp_dst, 0, (size_t)count * sizeof(int));
  g_sreq_cap = count;
}

static void sp_batch(int list, int ref, int mb0, int s0, const sp_ent *w, int t8)
{
  const spec_ent *itab = g_spec[list][ref];
  sp_ent *tab = g_sp[list][ref];
  int mb1 = imax(g_spec_end[list][ref], mb0 + 1), n = 0, i, s, k, mb;
  int count = (mb1 - mb0) * JMME_NSLOT * KHYP + 1;
  double t0 = now_us();
  if (!g_slot_bt[0]) slot_geometry();
  sp_reserve(count);
  sp_fill(&g_sreq[n], mb0, s0, list, ref, w);
  g_sp_dst[n++] = (int)sp_idx(mb0, s0, KHYP);
  {
    /* the guesses: this call's request with each cached integer answer's block,
     * predictor, vector and cost (the fields every guess shares filled once) */
    const unsigned gen = g_slot_gen[list][ref];
    jmme_subpel_req tq;
    uint8_t sflags[JMME_NSLOT];
    sp_fill(&tq, mb0, 0, list, ref, w);
    for (s = 0; s < JMME_NSLOT; s++)   /* test8x8 as mv_search.c:1630,1770 set it: Transform8x8Mode on types 1..4 */
      sflags[s] = (uint8_t)((w->flags & JMME_SP_CHECK0) | (t8 && g_slot_bt[s] <= 4 ? JMME_SP_TEST8x8 : 0));
    for (mb = mb0; mb < mb1; mb++) {
      const int16_t bx0 = (int16_t)((mb % g_mbs_x) * 16), by0 = (int16_t)((mb / g_mbs_x) * 16);
      for (k = 0; k < KHYP; k++) {      /* (both tables way-major: slots innermost walk memory in order) */
        const spec_ent *ie = &itab[spec_idx(mb, 0, k)];
        for (s = 0; s < JMME_NSLOT; s++, ie++) {
          jmme_subpel_req *q;
          if (ie->valid != gen) continue;
          q = &g_sreq[n];
          *q = tq;
          q->pos_x = (int16_t)(bx0 + g_slot_bx[s]);
          q->pos_y = (int16_t)(by0 + g_slot_by[s]);
          q->blocktype = (int16_t)g_slot_bt[s];
          q->pred_x = ie->px;
          q->pred_y = ie->py;
          q->mv_x = ie->mvx;
          q->mv_y = ie->mvy;
          q->min_mcost = w->start_hp ? ie->cost : JMME_DISTBLK_MAX;
          q->flags = sflags[s];
          g_sp_dst[n++] = (int)sp_idx(mb, s, k);
        }
      }
    }
  }
  {
    const double t1 = now_us();
    g_t_sp_part[0] += t1 - t0;
    if (jmme_subpel_refine(g_me, g_sreq, n, g_sres)) fail_jm("jmme_subpel_refine");
    g_t_sp_part[1] += now_us() - t1;
  }
  const double t2 = now_us();
  {
    /* every request of the batch shares the call's lambdas, metrics and switches */
    sp_ent te = *w;
    te.valid = g_slot_gen[list][ref];
    for (i = 0; i < n; i++) {
      const jmme_subpel_req *q = &g_sreq[i];
      sp_ent *e = &tab[g_sp_dst[i]];
      *e = te;
      e->px = q->pred_x; e->py = q->pred_y; e->mx = q->mv_x; e->my = q->mv_y;
      e->min_mcost = q->min_mcost; e->flags = q->flags;
      e->omx = g_sres[i].mv_x; e->omy = g_sres[i].mv_y; e->cost = g_sres[i].cost;
    }
  }
  ++g_sp_batches;
  g_t_sp_part[2] += now_us() - t2;
  g_t_sp += now_us() - t0;
}

static sp_ent *sp_table(VideoParameters *p_Vid, int list, int ref)
{
  spec_table(p_Vid, list, ref);                       /* sizes and per-picture reset of the integer table */
  if (!g_sp[list][ref]) {
    size_t n = (size_t)g_n_mb * JMME_NSLOT * SPK;
    g_sp[list][ref] = (sp_ent *)malloc(n * sizeof(sp_ent));
    if (!g_sp[list][ref]) error("jm_gpu_me: out of memory", 500);
    memset(g_sp[list][ref], 0, n * sizeof(sp_ent));
    g_sp_gen[list][ref] = 0;
  }
  if (g_sp_gen[list][ref] != g_slot_gen[list][ref])   /* other planes: every entry is stale (its stamp) */
    g_sp_gen[list][ref] = g_slot_gen[list][ref];
  return g_sp[list][ref];
}

/* The speculative caches of (list 0, ref 0) -- tens of MB at 1080p -- are
 * allocated and touched at encoder start-up, so the first P picture does not
 * pay their page faults inside JM's ME timer. */
static void prefault_tables(VideoParameters *p_Vid, InputParameters *p_Inp)
{
  if (p_Vid->width <= 0 || p_Vid->height <= 0) return;
  spec_table(p_Vid, 0, 0);
  memset(g_spec[0][0], 0, (size_t)g_n_mb * JMME_NSLOT * KWAYS * sizeof(spec_ent));
  memset(g_seen[0][0], 0, (size_t)g_n_mb * JMME_NSLOT * sizeof(spec_ent));
  if (!p_Inp->DisableSubpelME[0]) {
    sp_table(p_Vid, 0, 0);
    sp_reserve(g_n_mb * JMME_NSLOT * KHYP + 1);   /* a sub-pel batch over the whole picture at most */
  }
}

/* lambda_factor[H_PEL] / [Q_PEL] of the F_PEL lambdas seen in sub-pel calls
 * (the integer search receives only lambda_factor[F_PEL]; its caller's array,
 * md_low.c:130 / mode_decision_P8x8.c:63, holds the other two) */
#define NLAM 8
static int g_lam[NLAM][3], g_n_lam = 0;

static void note_lambdas(const int *lambda_factor)
{
  int i;
  for (i = 0; i < g_n_lam; i++)
    if (g_lam[i][0] == lambda_factor[F_PEL]) {
      g_lam[i][1] = lambda_factor[H_PEL];
      g_lam[i][2] = lambda_factor[Q_PEL];
      return;
    }
  i = g_n_lam < NLAM ? g_n_lam++ : (int)(g_sp_calls % NLAM);
  g_lam[i][0] = lambda_factor[F_PEL];
  g_lam[i][1] = lambda_factor[H_PEL];
  g_lam[i][2] = lambda_factor[Q_PEL];
}

/* the SubPelME template of the chains of this miss (g_chain_sp[0]): what
 * __wrap_sub_pel_motion_estimation will hand the GPU for the macroblock's
 * partitions, from the integer call's MEBlock (metrics, search_pos2 / 4 --
 * init_mv_block, mv_search.c:700-769), p_Vid's refinement starts and the sub-pel
 * lambdas last seen with this F_PEL lambda.  0 when JM's sub-pel calls would
 * not be served on the GPU, or the lambdas are not known yet.  (A wrong
 * template only costs hits: every answer is used for identical inputs only.) */
static int chain_subpel_template(Macroblock *currMB, MEBlock *mv_block, int list, int ref, int lambda_f)
{
  VideoParameters *p_Vid = currMB->p_Vid;
  Slice *currSlice = currMB->p_Slice;
  int mode = currMB->p_Inp->SearchMode[p_Vid->view_id];
  int mh = metric_id(mv_block->computePredHPel), mq = metric_id(mv_block->computePredQPel), i;
  jmme_subpel_req *q = &g_chain_sp[0];
  if ((mode != FULL_SEARCH && mode != FAST_FULL_SEARCH) || mh < 0 || mq < 0 || (g_bits > 11 && (mh == 1 || mq == 1)) ||
      mv_block->ChromaMEEnable || mv_block->search_pos2 > 9 || mv_block->search_pos4 > 9)
    return 0;
  for (i = 0; i < g_n_lam && g_lam[i][0] != lambda_f; i++) {}
  if (i == g_n_lam) {
    ++g_chain_sp_nolam;
    return 0;
  }
  memset(q, 0, sizeof *q);
  q->lambda_h = g_lam[i][1];
  q->lambda_q = g_lam[i][2];
  q->metric_h = (uint8_t)mh;
  q->metric_q = (uint8_t)mq;
  q->start_hp = (uint8_t)(p_Vid->start_me_refinement_hp != 0);
  q->start_qp = (uint8_t)(p_Vid->start_me_refinement_qp != 0);
  q->search_pos2 = (uint8_t)mv_block->search_pos2;
  q->search_pos4 = (uint8_t)mv_block->search_pos4;
  q->flags = (uint8_t)((!currMB->p_Inp->rdopt && currSlice->slice_type != B_SLICE) ? JMME_SP_CHECK0 : 0);
  sp_table(p_Vid, list, ref);
  return 1;
}

/* a chain step's refinement -> way KHYP + 1 of its (macroblock, slot), keyed by
 * the inputs BlockMotionSearch hands SubPelME after that step's answer */
static void store_chain_subpel(int list, int ref, int mb, int sl, const jmme_chain_res *r, const jmme_block_res *f)
{
  const jmme_subpel_req *q = &g_chain_sp[0];
  sp_ent *e = &g_sp[list][ref][sp_idx(mb, sl, KHYP + 1)];
  memset(e, 0, sizeof *e);
  e->px = r->pred_x; e->py = r->pred_y; e->mx = r->mv_x; e->my = r->mv_y;
  e->min_mcost = q->start_hp ? r->cost : JMME_DISTBLK_MAX;
  e->lam_h = q->lambda_h; e->lam_q = q->lambda_q;
  e->metric_h = q->metric_h; e->metric_q = q->metric_q; e->start_hp = q->start_hp; e->start_qp = q->start_qp;
  e->pos2 = q->search_pos2; e->pos4 = q->search_pos4; e->flags = q->flags;
  e->omx = f->mv_x; e->omy = f->mv_y; e->cost = f->cost;
  e->valid = g_slot_gen[list][ref];
  ++g_chain_sp_steps;
}

/* sub_pel_motion_estimation's contract (me_fullsearch.c:186-289) */
distblk __wrap_sub_pel_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                         distblk min_mcost, int *lambda_factor)
{
  VideoParameters *p_Vid = currMB->p_Vid;
  Slice *currSlice = currMB->p_Slice;
  int list = mv_block->list, ref = mv_block->ref_idx;
  int mh = metric_id(mv_block->computePredHPel), mq = metric_id(mv_block->computePredQPel);
  int mb, s, i;
  sp_ent want, *e, *tab;
  ++g_sp_calls;
  int mode = currMB->p_Inp->SearchMode[p_Vid->view_id];
  /* GPU sub-pel follows a GPU integer search (FS / FFS); UMHEX's direct calls,
   * weighted / chroma metrics and SSE above 11 bits (libjmme refuses it: JM's int
   * sum can wrap) stay on the CPU */
  if (!speculating() || (mode != FULL_SEARCH && mode != FAST_FULL_SEARCH) || mh < 0 || mq < 0 ||
      (g_bits > 11 && (mh == 1 || mq == 1)) ||
      mv_block->ChromaMEEnable || mv_block->search_pos2 > 9 || mv_block->search_pos4 > 9 ||
      (mv_block->test8x8 && mv_block->blocktype > 4)) {
    ++g_sp_cpu;
    return __real_sub_pel_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
  }
  ensure_planes(currMB, list, ref);
  note_lambdas(lambda_factor);
  memset(&want, 0, sizeof want);
  want.px = pred_mv->mv_x; want.py = pred_mv->mv_y;
  want.mx = mv_block->mv[list].mv_x; want.my = mv_block->mv[list].mv_y;
  want.min_mcost = (int64_t)min_mcost;
  want.lam_h = lambda_factor[H_PEL]; want.lam_q = lambda_factor[Q_PEL];
  want.metric_h = (uint8_t)mh; want.metric_q = (uint8_t)mq;
  want.start_hp = (uint8_t)(p_Vid->start_me_refinement_hp != 0);
  want.start_qp = (uint8_t)(p_Vid->start_me_refinement_qp != 0);
  want.pos2 = (uint8_t)mv_block->search_pos2; want.pos4 = (uint8_t)mv_block->search_pos4;
  want.flags = (uint8_t)((mv_block->test8x8 ? JMME_SP_TEST8x8 : 0) |
                         ((!currMB->p_Inp->rdopt && currSlice->slice_type != B_SLICE) ? JMME_SP_CHECK0 : 0));
  tab = sp_table(p_Vid, list, ref);
  mb = (mv_block->pos_y >> 4) * g_mbs_x + (mv_block->pos_x >> 4);
  s = jmme_slot(mv_block->blocktype, (mv_block->pos_x & 15) >> 2, (mv_block->pos_y & 15) >> 2);
  if (s < 0 || mb < 0 || mb >= g_n_mb) error("jm_gpu_me: block outside the picture", 500);
  i = SPK;
  if (mb == g_sp_hint_mb && s == g_sp_hint_s && sp_same(&tab[sp_idx(mb, s, g_sp_hint_k)], &want, g_slot_gen[list][ref]))
    i = g_sp_hint_k;
  else
    for (i = 0; i < SPK && !sp_same(&tab[sp_idx(mb, s, i)], &want, g_slot_gen[list][ref]); i++) {}
  if (i < SPK) {
    ++g_sp_hits;
    if (i == KHYP + 1) ++g_chain_sp_hits;
    e = &tab[sp_idx(mb, s, i)];
  } else {
    sp_batch(list, ref, mb, s, &want, currMB->p_Inp->Transform8x8Mode != 0);
    e = &tab[sp_idx(mb, s, KHYP)];
    if (!sp_same(e, &want, g_slot_gen[list][ref])) error("jm_gpu_me: sub-pel batch lost its own request", 500);
  }
  mv_block->mv[list].mv_x = e->omx;
  mv_block->mv[list].mv_y = e->omy;
  return (distblk)e->cost;
}

/* ---- EPZS (SearchMode = 3) ---------------------------------------------------
 * JM's four EPZS integer searches (me_epzs.c:54-407, 417-780; EPZSSubPelGrid:
 * me_epzs_int.c:41-420, 431-780) and EPZS_sub_pel_motion_estimation
 * (me_epzs_sub.c:30-222), one GPU call per search.  The caller's half stays
 * JM's: the predictor list is built here with JM's own routines
 * (EPZS_spatial_predictors, _spatial_memory_, _temporal_, EPZSWindowPredictors,
 * EPZSBlockTypePredictors(MB), me_epzs_common.c:1224-1764) and its stop
 * criterion with EPZSDetermineStopCriterion (:1764).  The parts JM generates
 * only when the centre's cost passes a bound are tagged with that bound
 * (JMME_EPZS_PRED_*) -- the GPU computes the centre's cost and keeps the entries
 * whose bound holds, so the list it searches is JM's.
 *
 * JM's state around a search is kept exactly:
 *   BlkCount   ++, skipping 0 (me_epzs.c:92-94);
 *   EPZSMap    never cleared: every cell the search stamps (the GPU returns
 *              them) gets this BlkCount, and the cells that already hold the
 *              new BlkCount (stamped 65535 searches ago, uint16 wrap) are
 *              passed in as visited.  They are found through a ring of
 *              per-BlkCount cell lists (g_ring[c]: every cell holding c), so no
 *              search scans the map.  A search JM ran itself (a metric the GPU
 *              does not serve, or the bipred searches that share the map) leaves
 *              stamps the ring does not know: from then to the next slice the
 *              cells are found by scanning the search window instead;
 *   prevSad    p_EPZS->distortion[...] (the value the GPU returns);
 *   p_motion   EPZSSpatialMem's memory (EPZSREF = 1, defines.h:56): JM's tmp at
 *              every return;
 *   mv         mv_block->mv[list]. */
extern distblk __real_EPZS_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int);
extern distblk __real_EPZS_subMB_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int);
extern distblk __real_EPZS_integer_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int);
extern distblk __real_EPZS_integer_subMB_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int);
extern distblk __real_EPZS_sub_pel_motion_estimation(Macroblock *, MotionVector *, MEBlock *, distblk, int *);

typedef struct cell_list {
  uint32_t *c;
  int n, cap;
} cell_list;

static cell_list *g_ring = NULL;                 /* [65536]: the map cells holding each BlkCount */
static EPZSParameters *g_ring_owner = NULL;
static int g_ring_count = -1, g_ring_foreign = 0, g_ring_side = 0, g_epzs_check = -1;
static long long g_epzs_calls = 0, g_epzs_cpu = 0, g_epzs_foreign = 0, g_epzs_stale = 0, g_epzs_preds = 0;
static long long g_epzs_sp_calls = 0, g_epzs_sp_cpu = 0;
static double g_t_epzs = 0, g_t_epzs_gpu = 0;
static int16_t *g_ep_pred = NULL, *g_ep_stale = NULL, *g_ep_vis = NULL;
static uint8_t *g_ep_cond = NULL;
static int g_ep_pred_cap = 0, g_ep_stale_cap = 0, g_ep_vis_cap = 0;

static void cell_push(cell_list *l, uint32_t c)
{
  if (l->n == l->cap) {
    int cap = l->cap ? 2 * l->cap : 16;
    uint32_t *p = (uint32_t *)realloc(l->c, (size_t)cap * sizeof(uint32_t));
    if (!p) error("jm_gpu_me: out of memory", 500);
    l->c = p;
    l->cap = cap;
  }
  l->c[l->n++] = c;
}

static void grow16(int16_t **p, int *cap, int need)
{
  if (need <= *cap) return;
  *cap = imax(need, 2 * *cap);
  free(*p);
  *p = (int16_t *)malloc((size_t)*cap * 2 * sizeof(int16_t));
  if (!*p) error("jm_gpu_me: out of memory", 500);
}

/* EPZSMap's side (searcharray, me_epzs_common.c:428-431) */
static int epzs_map_side(Macroblock *currMB)
{
  InputParameters *p_Inp = currMB->p_Inp;
  VideoParameters *p_Vid = currMB->p_Vid;
  int sr = p_Inp->search_range[p_Vid->view_id];
  if (p_Inp->BiPredMotionEstimation && p_Inp->BiPredMESearchRange[p_Vid->view_id] > sr)
    sr = p_Inp->BiPredMESearchRange[p_Vid->view_id];
  return (2 * sr + 1) << 2;
}

/* Is the ring still the whole truth about the map?  A fresh EPZS structure
 * (EPZSStructInit per slice, slice.c:1661-1665: BlkCount 1, a zeroed map)
 * restarts it; a BlkCount that moved without us means JM searched itself. */
static void epzs_ring_sync(EPZSParameters *p_EPZS, int side)
{
  int i, j, fresh;
  if (!g_ring) {
    g_ring = (cell_list *)calloc(65536, sizeof(cell_list));
    if (!g_ring) error("jm_gpu_me: out of memory", 500);
  }
  if (p_EPZS == g_ring_owner && (int)p_EPZS->BlkCount == g_ring_count && side == g_ring_side) return;
  fresh = p_EPZS->BlkCount == 1;
  for (i = 0; i < side && fresh; i++)
    for (j = 0; j < side && fresh; j++) fresh = p_EPZS->EPZSMap[i][j] == 0;
  if (fresh) {
    for (i = 0; i < 65536; i++) g_ring[i].n = 0;
    g_ring_foreign = 0;
  } else if (!g_ring_foreign) {
    g_ring_foreign = 1;
    ++g_epzs_foreign;
  }
  g_ring_owner = p_EPZS;
  g_ring_side = side;
  g_ring_count = (int)p_EPZS->BlkCount;
}

/* the last list's layout: where its block-type predictors start (EPZSBlockTypePredictors*), low 16 bits,
 * and where its spatial-memory predictors end (EPZS_spatial_memory_predictors), high 16 bits */
static int g_ep_bt_start = 0, g_ep_mem_end = 0;

/* the predictor list JM would build for this search, every conditional part
 * included and tagged; returns the count (pool: g_ep_pred / g_ep_cond) */
static int epzs_predictors(int variant, Macroblock *currMB, MEBlock *mv_block, distblk stop)
{
  Slice *currSlice = currMB->p_Slice;
  VideoParameters *p_Vid = currMB->p_Vid;
  InputParameters *p_Inp = currMB->p_Inp;
  EPZSParameters *p_EPZS = currSlice->p_EPZS;
  SPoint *pt = p_EPZS->predictor->point;
  int list = mv_block->list, cur_list = list + currMB->list_offset, ref = mv_block->ref_idx;
  int bt = mv_block->blocktype, sub = variant & 1, grid = variant >= 2;
  int field_or_mbaff = currSlice->structure != FRAME || currMB->list_offset;
  StorablePicture *ref_picture = currSlice->listX[cur_list][ref];
  int n = 5, n1, i, w;
  uint8_t cond[2048];
  short invalid_refs;
  (void)stop;
  invalid_refs = EPZS_spatial_predictors(p_EPZS, mv_block, list, currMB->list_offset, (short)ref,
                                         p_Vid->enc_picture->mv_info);
  if (p_Inp->EPZSSpatialMem) EPZS_spatial_memory_predictors(p_EPZS, mv_block, cur_list, &n, ref_picture->size_x >> 2);
  g_ep_mem_end = n;
  for (i = 0; i < n; i++) cond[i] = JMME_EPZS_PRED_ALWAYS;
#if (MVC_EXTENSION_ENABLE)
  if (!sub && p_Inp->EPZSTemporal[currSlice->view_id] && (grid || bt < 5))
#else
  if (!sub && p_Inp->EPZSTemporal && (grid || bt < 5))
#endif
  {
    /* the co-located vector always; its neighbours when min_mcost > stop (me_epzs_common.c:1550) */
    int start = n;
    EPZS_temporal_predictors(currMB, ref_picture, p_EPZS, mv_block, &n, 1, 0);
    n1 = n;
    n = start;
    EPZS_temporal_predictors(currMB, ref_picture, p_EPZS, mv_block, &n, 0, 1);
    for (i = start; i < n; i++) cond[i] = (uint8_t)(i < n1 ? JMME_EPZS_PRED_ALWAYS : JMME_EPZS_PRED_GT_STOP);
  }
  if (!sub) {   /* window predictors (me_epzs.c:181-191, me_epzs_int.c:181-191) */
    int always = p_Inp->EPZSFixed == 3 && (currMB->mb_x == 0 || currMB->mb_y == 0);
    int gated = ((ref < 2 && bt < 4) || (ref < 1 && bt == 4) || (field_or_mbaff && ref < 3)) &&
                (p_Inp->EPZSFixed > 1 || (p_Inp->EPZSFixed && currSlice->slice_type == P_SLICE));
    if (always || gated) {
      int ext = (grid || bt < 5) && invalid_refs > 2 && ref < 1 + field_or_mbaff;
      int start = n;
      EPZSWindowPredictors(&mv_block->mv[list], p_EPZS->predictor, &n,
                           ext ? p_EPZS->window_predictor_ext : p_EPZS->window_predictor);
      if (n > (int)sizeof cond) error("jm_gpu_me: EPZS predictor list too long", 500);
      for (i = start; i < n; i++) cond[i] = (uint8_t)(always ? JMME_EPZS_PRED_ALWAYS : JMME_EPZS_PRED_GT_3STOP);
    }
  }
  g_ep_bt_start = n | (g_ep_mem_end << 16);
  if (currMB->mbAddrX != 0 && p_Inp->EPZSBlockType) {   /* ref == 0 || min_mcost > 2 * stop */
    int start = n;
    if (sub)
      EPZSBlockTypePredictors(currSlice, mv_block, pt, &n);
    else
      EPZSBlockTypePredictorsMB(currSlice, mv_block, pt, &n);
    for (i = start; i < n; i++) cond[i] = (uint8_t)(ref == 0 ? JMME_EPZS_PRED_ALWAYS : JMME_EPZS_PRED_GT_2STOP);
  }
  if (n > (int)sizeof cond) error("jm_gpu_me: EPZS predictor list too long", 500);
  if (n > g_ep_pred_cap) {
    g_ep_pred_cap = imax(n, 2 * g_ep_pred_cap);
    free(g_ep_pred);
    free(g_ep_cond);
    g_ep_pred = (int16_t *)malloc((size_t)g_ep_pred_cap * 2 * sizeof(int16_t));
    g_ep_cond = (uint8_t *)malloc((size_t)g_ep_pred_cap);
    if (!g_ep_pred || !g_ep_cond) error("jm_gpu_me: out of memory", 500);
  }
  for (w = 0; w < n; w++) {
    g_ep_pred[2 * w] = pt[w].motion.mv_x;
    g_ep_pred[2 * w + 1] = pt[w].motion.mv_y;
    g_ep_cond[w] = cond[w];
  }
  return n;
}

static distblk real_epzs(int variant, Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block, distblk min_mcost,
                         int lambda_factor)
{
  switch (variant) {
    case 0: return __real_EPZS_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
    case 1: return __real_EPZS_subMB_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
    case 2: return __real_EPZS_integer_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
    default: return __real_EPZS_integer_subMB_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
  }
}

/* ---- speculative EPZS batches ---------------------------------------------
 * JM's EPZS calls depend on each other (the predictor list holds the final
 * vectors of the neighbours and of the macroblock's other block types, the stop
 * criterion the neighbours' SADs), so one call cannot wait for a GPU round trip
 * each.  Instead a batch searches, in one launch, every partition of the next
 * macroblocks under the inputs the same partition had in already-searched
 * macroblocks (left of the batch, and the row above), and JM's real call is
 * answered from the batch when its inputs equal a guess:
 *   - block, centre, predictor, lambda, range, variant, pattern, thresholds and
 *     the predictor list with its conditions: equal;
 *   - the stop criterion and *prevSad: inside the intervals the search reports
 *     (jmme_epzs_bounds: each comparison with them is monotone, so inside the
 *     intervals the search runs exactly as it ran);
 *   - EPZSMap: the guess ran with no pre-stamped cells; JM's cells that already
 *     hold this BlkCount must not include any the search evaluated (it would
 *     have skipped them), which the stamped-cell list it returns tells.
 * Every answer is JM's exactly.  The EPZS sub-pel refinement of each guess is
 * chained on the device in the same launch and answered the same way.  A call
 * no guess fits is searched alone (with its chained refinement), or starts the
 * next batch when it lies past the current one.  JMME_EPZS_SPECULATE=0: one
 * call per search. */
#define EP_MAXP 128                /* predictors of a list the cache keeps (longer lists: one call each) */
#define EP_MAXV 64                 /* stamped cells kept per cached answer */
#define EP_WAYS 6                  /* guesses per (macroblock, partition, reference): the sources' inputs,
                                      then their second-pass forms (ep_pass2) */
#define EP_REFS 4                  /* references speculated (list 0) */
#define EP_BATCH_MAX 512

typedef struct ep_in {             /* one search's inputs */
  jmme_epzs_req q;                 /* pred_off / n_stale / stale_off / reserved: not compared */
  int32_t pred[EP_MAXP];           /* (x, y) pairs as int16 */
  uint8_t cond[EP_MAXP];
  int32_t mb;                      /* the macroblock (seen ring: which one the entry holds) */
  uint32_t gen;                    /* g_slot_gen of its reference when stored (0: empty) */
  int32_t bt_start;                /* layout (not compared): block-type predictors from (bt_start & 0xffff),
                                      spatial-memory predictors pred[5 .. bt_start >> 16) */
} ep_in;

typedef struct ep_ans {            /* a searched guess: inputs, result, validity, chained refinement */
  ep_in in;
  jmme_epzs_res res;
  jmme_epzs_bounds bnd;
  int16_t vis[EP_MAXV][2];
  jmme_subpel_req spq;             /* the refinement's inputs (mv / min_mcost from res); blocktype 0: none */
  jmme_block_res sp_res;
} ep_ans;

typedef struct ep_spp {            /* EPZS sub-pel parameters of this encode, from JM's last real call */
  int valid, lam_h, lam_q, metric_h, metric_q, start_hp, start_qp, pos2, pos4, check0, t8;
} ep_spp;

static int g_ep_spec = -1, g_ep_batch = 64, g_ep_ring_n = 0;
static ep_in *g_ep_seen = NULL;    /* [ring of macroblocks][41 slots][EP_REFS]: the inputs JM really searched with */
static ep_ans *g_ep_ans = NULL;    /* the current batch's searched guesses */
static int *g_ep_idx = NULL;       /* [batch macroblock][41][EP_REFS][EP_WAYS] -> g_ep_ans index (-1: none) */
static int g_ep_idx_mbs = 0;       /* macroblocks g_ep_idx holds room for */
static int g_ep_cap = 0, g_ep_n = 0, g_ep_mb0 = 0, g_ep_mb1 = 0;
static unsigned g_ep_gens[EP_REFS];   /* g_slot_gen of each reference when the batch was made (0: none) */
static const ep_ans *g_ep_served = NULL;   /* the answer the last EPZS call was served from (its refinement) */
static ep_spp g_ep_spp;
static jmme_epzs_req *g_ep_q = NULL;
static int16_t *g_ep_ppool = NULL;
static uint8_t *g_ep_cpool = NULL;
static jmme_epzs_res *g_ep_res = NULL;
static jmme_epzs_bounds *g_ep_bnd = NULL;
static int16_t *g_ep_vbuf = NULL;
static jmme_subpel_req *g_ep_spq = NULL;
static jmme_block_res *g_ep_spo = NULL;
static int32_t *g_ep_bts = NULL;   /* [g_ep_cap]: bt_start of each request's list */
static int g_ep_pcap = 0;
static long long g_ep_hits = 0, g_ep_batches = 0, g_ep_singles = 0, g_ep_guesses = 0, g_ep_direct = 0;
static long long g_ep_fail_bounds = 0, g_ep_fail_stale = 0, g_ep_fail_inputs = 0, g_ep_sp_hits = 0, g_ep_overflow = 0;
static double g_t_ep_build = 0;
static double g_t_ep_run = 0, g_t_ep_runlib = 0, g_t_ep_p2 = 0, g_t_ep_lookup = 0;   /* host clocks (reported at exit) */
static long long g_ep_lookups = 0;
static long long g_ep_miss_slot[JMME_NSLOT], g_ep_list_diff[JMME_NSLOT];   /* misses inside a batch, by slot */
/* JMME_EPZS_TRACE: misses inside a batch by kind -- [0] no way with these inputs, [1] the stop criterion
 * outside every equal way's interval, [2] prevSad outside, [3] map cells; and the stop misses by
 * log2 of |real - guessed| (the guess's own stop criterion) */
static long long g_ep_miss_kind[4], g_ep_stop_off[24];
static long long g_ep_stop_side[8][2];   /* stop misses by the nearest way's return path, real below / above */
static int g_ep_trace = 0;   /* JMME_EPZS_TRACE=1: per-slot miss counts at exit */
static int g_ep_two_pass = 1;   /* JMME_EPZS_PASS2=0: no second pass (ep_pass2) */
static int g_ep_dump = 0;       /* JMME_EPZS_DUMP=n: print the first n input misses (measurement) */
static int g_ep_clk = -1;       /* the wrapper's per-call clock (JMME_PHASES=1 or JMME_EPZS_TRACE=1) */

static int ep_speculating(Macroblock *currMB, int cur_list, int ref, int n_pred)
{
  if (g_ep_spec < 0) {
    const char *e = getenv("JMME_EPZS_SPECULATE"), *b = getenv("JMME_EPZS_BATCH"), *tr = getenv("JMME_EPZS_TRACE");
    g_ep_spec = !(e && e[0] == '0');
    g_ep_trace = tr && tr[0] == '1';
    {
      const char *p2 = getenv("JMME_EPZS_PASS2");
      g_ep_two_pass = !(p2 && p2[0] == '0');
      const char *dp = getenv("JMME_EPZS_DUMP");
      g_ep_dump = dp ? atoi(dp) : 0;
    }
    if (b && atoi(b) > 0) g_ep_batch = imin(atoi(b), EP_BATCH_MAX);
  }
  if (!g_n_mb) {
    g_mbs_x = currMB->p_Vid->width / 16;
    g_n_mb = g_mbs_x * (currMB->p_Vid->height / 16);
  }
  if (!g_slot_bt[0]) slot_geometry();
  if (!g_ep_spec || cur_list != 0 || ref >= EP_REFS || n_pred > EP_MAXP ||
      currMB->p_Slice->slice_type != P_SLICE || currMB->p_Slice->structure != FRAME) {
    if (g_ep_spec) ++g_ep_direct;
    return 0;
  }
  return 1;
}

static int ep_slot_of(const jmme_epzs_req *q)
{
  return jmme_slot(q->blocktype, (q->pos_x & 15) >> 2, (q->pos_y & 15) >> 2);
}

/* equal inputs, the stop criterion, prevSad and the pre-stamped cells aside */
static int ep_same(const ep_in *a, const jmme_epzs_req *q, const int16_t *pred, const uint8_t *cond)
{
  const jmme_epzs_req *b = &a->q;
  return b->pos_x == q->pos_x && b->pos_y == q->pos_y && b->blocktype == q->blocktype && b->ref_idx == q->ref_idx &&
         b->pred_x == q->pred_x && b->pred_y == q->pred_y && b->center_x == q->center_x &&
         b->center_y == q->center_y && b->max_x == q->max_x && b->max_y == q->max_y && b->lambda == q->lambda &&
         b->variant == q->variant && b->flags == q->flags && b->pattern == q->pattern && b->dual == q->dual &&
         b->medthres == q->medthres && b->ref_slot == q->ref_slot && b->n_pred == q->n_pred &&
         b->bsx == q->bsx && b->bsy == q->bsy &&
         !memcmp(a->pred, pred, (size_t)q->n_pred * 4) && !memcmp(a->cond, cond, (size_t)q->n_pred);
}

/* the same search at another block position (guess -> guess dedup) */
static int ep_same_moved(const ep_in *a, const ep_in *b)
{
  jmme_epzs_req q = b->q;
  q.pos_x = a->q.pos_x;
  q.pos_y = a->q.pos_y;
  return ep_same(a, &q, (const int16_t *)b->pred, b->cond);
}

static void ep_fill_in(ep_in *e, const jmme_epzs_req *q, const int16_t *pred, const uint8_t *cond, int mb, unsigned gen)
{
  e->q = *q;
  e->q.pred_off = 0;
  e->q.n_stale = 0;
  e->q.stale_off = 0;
  e->q.reserved = 0;
  memcpy(e->pred, pred, (size_t)q->n_pred * 4);
  memcpy(e->cond, cond, (size_t)q->n_pred);
  e->mb = mb;
  e->gen = gen;
}

static ep_in *ep_seen_at(int mb, int slot, int ref)
{
  return &g_ep_seen[((size_t)(mb % g_ep_ring_n) * JMME_NSLOT + slot) * EP_REFS + ref];
}

/* the cached answer for this call, or NULL */
static const ep_ans *ep_lookup(Macroblock *currMB, MEBlock *mv_block, const jmme_epzs_req *q, const int16_t *pred,
                               const uint8_t *cond, const int16_t *stale, int n_stale)
{
  const int mb = (mv_block->pos_y >> 4) * g_mbs_x + (mv_block->pos_x >> 4), slot = ep_slot_of(q), ref = q->ref_idx;
  const unsigned gen = g_slot_gen[0][ref];
  int w, i, j;
  (void)currMB;
  if (!g_ep_seen || g_ep_ring_n != g_mbs_x + 4) {
    free(g_ep_seen);
    g_ep_ring_n = g_mbs_x + 4;
    g_ep_seen = (ep_in *)calloc((size_t)g_ep_ring_n * JMME_NSLOT * EP_REFS, sizeof(ep_in));
    if (!g_ep_seen) error("jm_gpu_me: out of memory", 500);
  }
  ep_fill_in(ep_seen_at(mb, slot, ref), q, pred, cond, mb, gen);
  ep_seen_at(mb, slot, ref)->bt_start = g_ep_bt_start;
  if (!gen || g_ep_gens[ref] != gen || mb < g_ep_mb0 || mb >= g_ep_mb1) return NULL;
  ++g_ep_miss_slot[slot];   /* (taken back below on a hit) */
  int kind = 0, stop_path = 0, stop_above = 0;
  int64_t stop_off = -1;
  for (w = 0; w < EP_WAYS; w++) {
    const int k = g_ep_idx[(((size_t)(mb - g_ep_mb0) * JMME_NSLOT + slot) * EP_REFS + ref) * EP_WAYS + w];
    const ep_ans *a;
    if (k < 0) break;
    a = &g_ep_ans[k];
    if (!ep_same(&a->in, q, pred, cond)) {
      if (g_ep_trace && a->in.q.center_x == q->center_x && a->in.q.center_y == q->center_y &&
          a->in.q.pred_x == q->pred_x && a->in.q.pred_y == q->pred_y) ++g_ep_list_diff[slot];
      continue;
    }
    if (q->stop_crit < a->bnd.stop_lo || q->stop_crit > a->bnd.stop_hi || q->prev_sad < a->bnd.prev_lo ||
        q->prev_sad > a->bnd.prev_hi || a->res.n_visited > EP_MAXV) {
      ++g_ep_fail_bounds;
      if (q->stop_crit < a->bnd.stop_lo || q->stop_crit > a->bnd.stop_hi) {
        const int64_t d = q->stop_crit > a->in.q.stop_crit ? q->stop_crit - a->in.q.stop_crit
                                                           : a->in.q.stop_crit - q->stop_crit;
        if (kind < 1) kind = 1;
        if (stop_off < 0 || d < stop_off) {
          stop_off = d;
          stop_path = a->res.path;
          stop_above = q->stop_crit > a->bnd.stop_hi;
        }
      } else if (q->prev_sad < a->bnd.prev_lo || q->prev_sad > a->bnd.prev_hi) {
        if (kind < 2) kind = 2;
      }
      continue;
    }
    for (i = 0; i < n_stale; i++) {   /* a cell JM already holds at this BlkCount: did the guess evaluate it? */
      if (!stale[2 * i] && !stale[2 * i + 1]) continue;   /* the centre is searched first whatever the map holds */
      for (j = 0; j < a->res.n_visited; j++)
        if (a->vis[j][0] == stale[2 * i] && a->vis[j][1] == stale[2 * i + 1]) break;
      if (j < a->res.n_visited) break;
    }
    if (i < n_stale) {
      ++g_ep_fail_stale;
      kind = 3;
      continue;
    }
    ++g_ep_hits;
    --g_ep_miss_slot[slot];
    return a;
  }
  ++g_ep_fail_inputs;
  ++g_ep_miss_kind[kind];
  if (kind == 0 && g_ep_dump > 0 &&   /* JMME_EPZS_DUMP=n: the first n input misses that had guesses */
      g_ep_idx[(((size_t)(mb - g_ep_mb0) * JMME_NSLOT + slot) * EP_REFS + ref) * EP_WAYS] >= 0) {
    --g_ep_dump;
    fprintf(stderr, "epzs-miss mb %d slot %d: c(%d,%d) p(%d,%d) n %d:", mb, slot, q->center_x, q->center_y, q->pred_x,
            q->pred_y, q->n_pred);
    for (i = 0; i < q->n_pred; i++) fprintf(stderr, " %d,%d/%d", pred[2 * i], pred[2 * i + 1], cond[i]);
    fprintf(stderr, "\n");
    {   /* the macroblock's first-guess answers by slot (integer / after SubPelME) */
      int sl;
      fprintf(stderr, "  answers:");
      for (sl = 0; sl < JMME_NSLOT; sl++) {
        const int k0 = g_ep_idx[(((size_t)(mb - g_ep_mb0) * JMME_NSLOT + sl) * EP_REFS + ref) * EP_WAYS];
        if (k0 < 0) fprintf(stderr, " %d:-", sl);
        else fprintf(stderr, " %d:%d,%d/%d,%d", sl, g_ep_ans[k0].res.mv_x, g_ep_ans[k0].res.mv_y, g_ep_ans[k0].sp_res.mv_x,
                     g_ep_ans[k0].sp_res.mv_y);
      }
      fprintf(stderr, "\n");
    }
    for (w = 0; w < EP_WAYS; w++) {
      const int k = g_ep_idx[(((size_t)(mb - g_ep_mb0) * JMME_NSLOT + slot) * EP_REFS + ref) * EP_WAYS + w];
      const ep_in *a;
      if (k < 0) break;
      a = &g_ep_ans[k].in;
      fprintf(stderr, "  way %d: c(%d,%d) p(%d,%d) n %d lam %d:", w, a->q.center_x, a->q.center_y, a->q.pred_x,
              a->q.pred_y, a->q.n_pred, a->q.lambda);
      for (i = 0; i < a->q.n_pred; i++) {
        const int16_t *ap = (const int16_t *)a->pred;
        const int same = i < q->n_pred && ap[2 * i] == pred[2 * i] && ap[2 * i + 1] == pred[2 * i + 1] && a->cond[i] == cond[i];
        fprintf(stderr, same ? " ." : " %d,%d/%d", ap[2 * i], ap[2 * i + 1], a->cond[i]);
      }
      fprintf(stderr, "\n");
    }
  }
  if (kind == 1) {
    int b = 0;
    while (b < 23 && (stop_off >> b) > 0) ++b;
    ++g_ep_stop_off[b];
    ++g_ep_stop_side[stop_path >= 0 && stop_path < 8 ? stop_path : 0][stop_above];
  }
  return NULL;
}

static void ep_grow(int n, int n_pred)
{
  if (n > g_ep_cap) {
    g_ep_cap = imax(n, 2 * g_ep_cap);
    free(g_ep_ans); free(g_ep_q); free(g_ep_res); free(g_ep_bnd); free(g_ep_vbuf); free(g_ep_spq); free(g_ep_spo);
    free(g_ep_bts);
    g_ep_bts = (int32_t *)malloc((size_t)g_ep_cap * sizeof(int32_t));
    g_ep_ans = (ep_ans *)malloc((size_t)g_ep_cap * sizeof(ep_ans));
    g_ep_q = (jmme_epzs_req *)malloc((size_t)g_ep_cap * sizeof(jmme_epzs_req));
    g_ep_res = (jmme_epzs_res *)malloc((size_t)g_ep_cap * sizeof(jmme_epzs_res));
    g_ep_bnd = (jmme_epzs_bounds *)malloc((size_t)g_ep_cap * sizeof(jmme_epzs_bounds));
    g_ep_vbuf = (int16_t *)malloc((size_t)g_ep_cap * EP_MAXV * 4);
    g_ep_spq = (jmme_subpel_req *)malloc((size_t)g_ep_cap * sizeof(jmme_subpel_req));
    g_ep_spo = (jmme_block_res *)malloc((size_t)g_ep_cap * sizeof(jmme_block_res));
    if (!g_ep_ans || !g_ep_q || !g_ep_res || !g_ep_bnd || !g_ep_vbuf || !g_ep_spq || !g_ep_spo || !g_ep_bts)
      error("jm_gpu_me: out of memory", 500);
  }
  if (n_pred > g_ep_pcap) {
    g_ep_pcap = imax(n_pred, 2 * g_ep_pcap);
    free(g_ep_ppool); free(g_ep_cpool);
    g_ep_ppool = (int16_t *)malloc((size_t)g_ep_pcap * 4);
    g_ep_cpool = (uint8_t *)malloc((size_t)g_ep_pcap);
    if (!g_ep_ppool || !g_ep_cpool) error("jm_gpu_me: out of memory", 500);
  }
}

/* request k of the batch: the search with inputs e at its own block; its refinement */
static int g_ep_np = 0;
static void ep_add(int k, const ep_in *e, int pos_x, int pos_y, EPZSParameters *p_EPZS)
{
  jmme_epzs_req *q = &g_ep_q[k];
  jmme_subpel_req *sp = &g_ep_spq[k];
  *q = e->q;
  q->pos_x = (int16_t)pos_x;
  q->pos_y = (int16_t)pos_y;
  q->pred_off = g_ep_np;
  q->n_stale = 0;
  q->stale_off = 0;
  memcpy(g_ep_ppool + 2 * (size_t)g_ep_np, e->pred, (size_t)e->q.n_pred * 4);
  memcpy(g_ep_cpool + g_ep_np, e->cond, (size_t)e->q.n_pred);
  g_ep_np += e->q.n_pred;
  g_ep_bts[k] = e->bt_start;
  memset(sp, 0, sizeof *sp);
  if (g_ep_spp.valid) {   /* EPZS_sub_pel_motion_estimation of the result (mv_search.c:966-976) */
    sp->pos_x = (int16_t)pos_x;
    sp->pos_y = (int16_t)pos_y;
    sp->blocktype = q->blocktype;
    sp->ref_slot = (int16_t)q->ref_slot;
    sp->pred_x = q->pred_x;
    sp->pred_y = q->pred_y;
    sp->lambda_h = g_ep_spp.lam_h;
    sp->lambda_q = g_ep_spp.lam_q;
    sp->subthres = (int64_t)p_EPZS->subthres[q->blocktype];
    sp->variant = 1;
    sp->flags = (uint8_t)((g_ep_spp.t8 && q->blocktype <= 4 ? JMME_SP_TEST8x8 : 0) | (g_ep_spp.check0 ? JMME_SP_CHECK0 : 0));
    sp->metric_h = (uint8_t)g_ep_spp.metric_h;
    sp->metric_q = (uint8_t)g_ep_spp.metric_q;
    sp->start_hp = (uint8_t)g_ep_spp.start_hp;
    sp->start_qp = (uint8_t)g_ep_spp.start_qp;
    sp->search_pos2 = (uint8_t)g_ep_spp.pos2;
    sp->search_pos4 = (uint8_t)g_ep_spp.pos4;
  }
}

/* search requests k0..n-1 (request 0, the real call, with its pre-stamped cells) and keep the answers */
static void ep_run_from(int k0, int n, const int16_t *stale, int n_stale, unsigned gen)
{
  int k;
  double t0 = now_us(), t1;
  if (k0 >= n) return;
  g_ep_q[k0].n_stale = k0 == 0 ? n_stale : 0;
  for (k = k0; k < n; k++) g_ep_spo[k].mv_x = g_ep_spo[k].mv_y = 0, g_ep_spo[k].cost = 0, g_ep_spo[k].reserved = 0;
  if (jmme_epzs_speculate(g_me, g_ep_q + k0, n - k0, g_ep_ppool, g_ep_cpool, g_ep_np, stale, k0 == 0 ? n_stale : 0,
                          g_ep_res + k0, g_ep_bnd + k0, g_ep_vbuf + 2 * (size_t)EP_MAXV * k0, EP_MAXV, g_ep_spq + k0,
                          g_ep_spo + k0))
    fail_jm("jmme_epzs_speculate");
  t1 = now_us();
  g_t_ep_runlib += t1 - t0;
  for (k = k0; k < n; k++) {
    ep_ans *a = &g_ep_ans[k];
    const int16_t *pp = g_ep_ppool + 2 * (size_t)g_ep_q[k].pred_off;
    ep_fill_in(&a->in, &g_ep_q[k], pp, g_ep_cpool + g_ep_q[k].pred_off, -1, gen);
    a->in.bt_start = g_ep_bts[k];
    a->res = g_ep_res[k];
    a->bnd = g_ep_bnd[k];
    memcpy(a->vis, g_ep_vbuf + 2 * (size_t)EP_MAXV * k, (size_t)imin(a->res.n_visited, EP_MAXV) * 4);
    a->spq = g_ep_spq[k];
    if (a->spq.blocktype) {   /* what the chained refinement was handed */
      a->spq.mv_x = a->res.mv_x;
      a->spq.mv_y = a->res.mv_y;
      a->spq.min_mcost = a->spq.start_hp ? a->res.cost : JMME_DISTBLK_MAX;
    }
    a->sp_res = g_ep_spo[k];
  }
  g_t_ep_run += now_us() - t0;
}

static void ep_run(int n, const int16_t *stale, int n_stale, unsigned gen) { ep_run_from(0, n, stale, n_stale, gen); }

/* ---- second pass: the stop criterion and prevSad the batch's own answers imply
 * A guess copies its stop criterion and prevSad from the call it was taken from,
 * but JM derives them from the distortion row of its own neighbours
 * (EPZSDetermineStopCriterion, me_epzs_common.c:1764-1780: the left, upper and
 * upper-right 4x4 columns of p_EPZS->distortion[list][blocktype - 1], which
 * every search writes at its own column when it updates prevSad).  After the
 * first launch the adapter replays the batch in JM's order on a copy of that
 * row -- JM's row as it stands, then each partition's first guess's answer --
 * and searches again every guess whose intervals do not hold the replayed pair
 * (one more launch).  Single slice, one reference, no 8x8 transform (JM's
 * order of the partitions is then the chains' order, chain_groups). */
static int64_t *g_ep_vrow = NULL;   /* [7][columns]: the replayed distortion rows */
static int g_ep_vcols = 0;
static long long g_ep_pass2 = 0, g_ep_pass2_batches = 0;
static long long g_ep_list_fixes = 0;   /* second-pass guesses whose list was rebuilt from this batch's answers */
static ep_in g_ep_fix;                  /* (a guess's inputs with its tail replaced) */

/* *d = *e, the list only as far as it goes (a whole ep_in is ~0.7 KB: the passes copy one per way) */
static void ep_copy_in(ep_in *d, const ep_in *e)
{
  d->q = e->q;
  memcpy(d->pred, e->pred, (size_t)e->q.n_pred * 4);
  memcpy(d->cond, e->cond, (size_t)e->q.n_pred);
  d->mb = e->mb;
  d->gen = e->gen;
  d->bt_start = e->bt_start;
}

static int ep_avail_c(int bx, int by, int bsx)   /* get_neighbors' upper-right rule inside the MB (mv_search.c:283-301) */
{
  if (by > 0) {
    if (bx < 8) {
      if (by == 8) return bsx != 16;
      return bx + bsx != 8;
    }
    return bx + bsx != 16;
  }
  return 1;
}

/* The answer JM is assumed to get for (macroblock mb0 + xr, slot): its first guess.  (A third pass
 * repeating the rebuild on the second pass's answers saved ~600 searches alone per 1080p P picture
 * for ~36 ms more host work: measured slower, removed.) */
static int ep_assumed(int xr, int slot)
{
  return g_ep_idx[(((size_t)xr * JMME_NSLOT + slot) * EP_REFS + 0) * EP_WAYS];
}

/* A partition's spatial predictors 1..4 as the batch assumes them (sp_on 0: keep the guess's own)
 * and the MV predictor they imply */
typedef struct ep_hyp {
  int16_t sp[5][2];
  int sp_on[5], pv_on;
  int16_t pv[2];
} ep_hyp;

static const int kEpW4[8] = {0, 4, 4, 2, 2, 2, 1, 1}, kEpH4[8] = {0, 4, 2, 4, 2, 1, 2, 1};

/* the refined answer the batch assumes for (macroblock mb0 + xr, block type m at 4x4 position (x4, y4)),
 * or 0 when it has none */
static int ep_refined_at(int xr, int m, int x4, int y4, int16_t v[2])
{
  const int pk = ep_assumed(xr, jmme_slot(m, x4 - x4 % kEpW4[m], y4 - y4 % kEpH4[m]));
  const ep_ans *pa = pk >= 0 ? &g_ep_ans[pk] : NULL;
  if (!pa || !pa->spq.blocktype) return 0;
  v[0] = pa->sp_res.mv_x;
  v[1] = pa->sp_res.mv_y;
  return 1;
}

/* the neighbours of the partition of block type bt at (bx, by) of macroblock x: inside this macroblock
 * the refined answer of the same block type's partition there (set_me_parameters after each search),
 * in a macroblock JM has decided its mv_info, in the left macroblock when it lies in this batch unknown */
static void ep_neighbours(ep_hyp *H, int x, int mb0, int bt, int bx, int by, VideoParameters *p_Vid)
{
  static const int16_t kNone[5][2] = {{0, 0}, {12, 0}, {0, 12}, {-12, 0}, {0, -12}};   /* unavailable */
  const int x4 = bx >> 2, y4 = by >> 2, w4 = kEpW4[bt];
  const int mbx4 = (x % g_mbs_x) * 4, mby4 = (x / g_mbs_x) * 4, W4 = p_Vid->width >> 2;
  PicMotionParams **mvi = p_Vid->enc_picture->mv_info;
  const int nx[5] = {0, x4 - 1, x4, x4 + w4, x4 - 1}, ny[5] = {0, y4, y4 - 1, y4 - 1, y4 - 1};
  int st[5] = {0, 0, 0, 0, 0}, nref[5] = {0, 0, 0, 0, 0};   /* 1 known, 0 not known, -1 unavailable; refs */
  int j;
  memset(H, 0, sizeof *H);
  for (j = 1; j <= 4; j++) {
    const int px4 = mbx4 + nx[j], py4 = mby4 + ny[j];
    if (px4 < 0 || py4 < 0 || px4 >= W4) { st[j] = -1; continue; }
    if (j == 3 && !ep_avail_c(bx, by, 4 * w4)) { st[j] = -1; continue; }
    if (nx[j] >= 0 && nx[j] <= 3 && ny[j] >= 0) {   /* inside this macroblock */
      if (ep_refined_at(x - mb0, bt, nx[j], ny[j], H->sp[j])) st[j] = 1;
    } else if (ny[j] < 0 || x - 1 < mb0) {   /* a macroblock JM has decided: its mv_info */
      const PicMotionParams *mp = &mvi[py4][px4];
      if (mp->ref_idx[0] == 0 || (mp->mv[0].mv_x == 0 && mp->mv[0].mv_y == 0)) {
        H->sp[j][0] = mp->mv[0].mv_x;
        H->sp[j][1] = mp->mv[0].mv_y;
        nref[j] = mp->ref_idx[0];
        st[j] = 1;
      }
    }
  }
  if (st[3] < 0) {   /* get_neighbors: an unavailable up-right is the up-left (mv_search.c:303-306) */
    st[3] = st[4];
    nref[3] = nref[4];
    H->sp[3][0] = H->sp[4][0];
    H->sp[3][1] = H->sp[4][1];
  }
  for (j = 1; j <= 4; j++) {
    if (st[j] < 0) { H->sp[j][0] = kNone[j][0]; H->sp[j][1] = kNone[j][1]; }
    if (st[j] == 0) { H->sp[j][0] = H->sp[j][1] = 0; }
    H->sp_on[j] = st[j] != 0;
  }
  /* the block's MV predictor from the same neighbours (GetMotionVectorPredictorNormal,
   * lcommon/src/mv_prediction.c:192-300: one matching reference, the 8x16 / 16x8 directions, else
   * the median), ref 0; unknown when a neighbour is */
  if (st[1] && st[2] && st[3]) {
    const int aL = st[1] > 0, aU = st[2] > 0, aR = st[3] > 0;
    const int rL = aL ? nref[1] : -1, rU = aU ? nref[2] : -1, rR = aR ? nref[3] : -1;
    const int bsx = (bt <= 2) ? 16 : (bt <= 5) ? 8 : 4;
    const int bsy = (bt == 1 || bt == 3) ? 16 : (bt == 2 || bt == 4 || bt == 6) ? 8 : 4;
    int type = 0;   /* 0 median, 1 left, 2 up, 3 up-right */
    if (rL == 0 && rU != 0 && rR != 0) type = 1;
    else if (rL != 0 && rU == 0 && rR != 0) type = 2;
    else if (rL != 0 && rU != 0 && rR == 0) type = 3;
    if (bsx == 8 && bsy == 16) {
      if (bx == 0) { if (rL == 0) type = 1; } else if (rR == 0) type = 3;
    } else if (bsx == 16 && bsy == 8) {
      if (by == 0) { if (rU == 0) type = 2; } else if (rL == 0) type = 1;
    }
    if (type == 0) {
      if (!(aU || aR)) {
        H->pv[0] = aL ? H->sp[1][0] : 0;
        H->pv[1] = aL ? H->sp[1][1] : 0;
      } else {
        int k2;
        for (k2 = 0; k2 < 2; k2++) {
          const int va = aL ? H->sp[1][k2] : 0, vb = aU ? H->sp[2][k2] : 0, vc = aR ? H->sp[3][k2] : 0;
          H->pv[k2] = (int16_t)(va + vb + vc - imin(va, imin(vb, vc)) - imax(va, imax(vb, vc)));
        }
      }
    } else {
      const int jn = type, av = jn == 1 ? aL : jn == 2 ? aU : aR;
      H->pv[0] = av ? H->sp[jn][0] : 0;
      H->pv[1] = av ? H->sp[jn][1] : 0;
    }
    H->pv_on = 1;
  }
}

static void ep_pass2(Macroblock *currMB, int mb0, int s0, int nmb, unsigned gen, int *n_io)
{
  VideoParameters *p_Vid = currMB->p_Vid;
  InputParameters *p_Inp = currMB->p_Inp;
  Slice *currSlice = currMB->p_Slice;
  EPZSParameters *p_EPZS = currSlice->p_EPZS;
  const int cols = p_Vid->width >> 2, n0 = *n_io;
  int n = n0, x, g, i, bt, started = 0;
  if (p_Inp->slice_mode || p_Inp->Transform8x8Mode || currSlice->listXsize[0] != 1) return;
  if (!g_grp_n[0]) chain_groups();
  if (cols > g_ep_vcols) {
    free(g_ep_vrow);
    g_ep_vrow = (int64_t *)malloc((size_t)7 * cols * sizeof(int64_t));
    if (!g_ep_vrow) error("jm_gpu_me: out of memory", 500);
    g_ep_vcols = cols;
  }
  for (bt = 1; bt <= 7; bt++)
    for (i = 0; i < cols; i++) g_ep_vrow[(size_t)(bt - 1) * cols + i] = (int64_t)p_EPZS->distortion[0][bt - 1][i];
  for (x = mb0; x < mb0 + nmb; x++) {
    const int mbx = (x % g_mbs_x) * 16, mby = (x / g_mbs_x) * 16;
    for (g = 0; g < 19; g++)
      for (i = 0; i < g_grp_n[g]; i++) {
        const int t = g_grp[g][i];
        int *idx = &g_ep_idx[(((size_t)(x - mb0) * JMME_NSLOT + t) * EP_REFS + 0) * EP_WAYS];
        const int bx = g_slot_bx[t], by = g_slot_by[t];
        const int bsx = (g_slot_bt[t] <= 2) ? 16 : (g_slot_bt[t] <= 5) ? 8 : 4;
        const int px = mbx + bx, py = mby + by, c = px >> 2, bs4 = bsx >> 2;
        int64_t *row, sadA, sadB, sadC, stop, ld, prev;
        int w, nw, k;
        if (x == mb0 && !started) {   /* the slots before the missing one are JM's by now */
          if (t != s0) continue;
          started = 1;
        }
        bt = g_slot_bt[t];
        row = &g_ep_vrow[(size_t)(bt - 1) * cols];
        if (idx[0] < 0) continue;
        {
          const jmme_epzs_req *q0 = &g_ep_ans[idx[0]].in.q;
          const int availA = px > 0, availB = py > 0;
          const int avail2 = (py > 0 && px + bsx < p_Vid->width && ep_avail_c(bx, by, bsx)) || (px > 0 && py > 0);
          ld = (int64_t)q0->lambda * ((q0->variant & 1) ? 3 : 2);
          sadA = availA ? row[c - bs4] : JMME_DISTBLK_MAX;
          sadB = availB ? row[c] : JMME_DISTBLK_MAX;
          sadC = avail2 && c + bs4 < cols ? row[c + bs4] : JMME_DISTBLK_MAX;
          stop = sadA < sadB ? sadA : sadB;
          stop = sadC < stop ? sadC : stop;
          stop = stop > (int64_t)p_EPZS->minthres[bt] ? stop : (int64_t)p_EPZS->minthres[bt];
          stop = stop < (int64_t)p_EPZS->maxthres[bt] + ld ? stop : (int64_t)p_EPZS->maxthres[bt] + ld;
          stop = (9 * ((int64_t)p_EPZS->medthres[bt] + ld > stop ? (int64_t)p_EPZS->medthres[bt] + ld : stop) +
                  2 * (int64_t)p_EPZS->medthres[bt]) >> 3;
          stop += ld;
          prev = row[c];
        }
        for (nw = 0; nw < EP_WAYS && idx[nw] >= 0; nw++) {}
        const int nw0 = nw;   /* the first pass's ways (the ones added here are searched after the loop) */
        /* the block-type predictors JM will append (EPZSBlockTypePredictors(MB), me_epzs_common.c:1224-1266,
         * 1608-1645; ref 0, frame): this macroblock's final vectors of the parent block type and of the
         * 16x16 at this position (all_mv, set after SubPelME), as the batch's first guesses answered them */
        int16_t tail[2][2];
        int n_tail = -1;
        if (p_Inp->EPZSBlockType && x != 0 && bt != 1) {
          /* BLOCK_PARENT (me_epzs_common.c:32) and each block type's size in 4x4 units */
          static const int kParent[8] = {1, 1, 1, 1, 2, 4, 4, 5}, kW4[8] = {0, 4, 4, 2, 2, 2, 1, 1},
                           kH4[8] = {0, 4, 2, 4, 2, 1, 2, 1};
          const int sub = g_ep_ans[idx[0]].in.q.variant & 1, P = kParent[bt];
          const int x4 = bx >> 2, y4 = by >> 2;
          const int ps[2] = {jmme_slot(P, x4 - x4 % kW4[P], y4 - y4 % kH4[P]), (sub || P != 1) ? 0 : -1};
          int j;
          n_tail = 0;
          for (j = 0; j < 2 && ps[j] >= 0 && n_tail >= 0; j++) {
            const int pk = ep_assumed(x - mb0, ps[j]);
            const ep_ans *pa = pk >= 0 ? &g_ep_ans[pk] : NULL;
            if (!pa || !pa->spq.blocktype) { n_tail = -1; break; }   /* (no chained refinement: final vector unknown) */
            if (pa->sp_res.mv_x | pa->sp_res.mv_y) {
              tail[n_tail][0] = pa->sp_res.mv_x;
              tail[n_tail][1] = pa->sp_res.mv_y;
              ++n_tail;
            }
          }
        }
        /* the spatial predictors of neighbours inside this macroblock (EPZS_spatial_predictors,
         * me_epzs_common.c:1276-1370) and the MV predictor they imply: ep_neighbours.  (Round 6 also
         * branched the guesses over the rate-distortion decisions those neighbours hang on -- the
         * sub-mode chosen for an earlier 8x8 block, the left macroblock's final mode: 1,115 fewer
         * searches alone per 1080p P picture for 28,928 more guesses, and the second pass's added
         * host time ate the gain (JM ME 0.449 vs 0.456 s); not kept: profiles/round6/epzs_hyp/.) */
        ep_hyp hyp0;
        ep_neighbours(&hyp0, x, mb0, bt, bx, by, p_Vid);
        /* the spatial-memory predictors (EPZS_spatial_memory_predictors, me_epzs_common.c:1675-1718,
         * EPZSREF): p_motion[ref][blocktype - 1][block row][picture column] at the left, up and up-right
         * block, i.e. the `tmp` of the same block type's search there -- this batch's answer where JM
         * will have searched it before this call (this macroblock, or one left of it in the batch),
         * otherwise JM's memory as it stands (the row above, or macroblocks JM has done) */
        int16_t mem[3][2];
        int n_mem = -1;
        if (p_Inp->EPZSSpatialMem && p_EPZS->p_motion) {
          static const int kW4[8] = {0, 4, 4, 2, 2, 2, 1, 1}, kH4[8] = {0, 4, 2, 4, 2, 1, 2, 1};
          const int w4 = kW4[bt], h4 = kH4[bt], x4 = bx >> 2, y4 = by >> 2, xc = x % g_mbs_x, w4pic = p_Vid->width >> 2;
          const int pic_x = xc * 4 + x4, up = y4 > 0 ? y4 - h4 : 4 - h4;
          const int rk_t = g_slot_grp[t] * 4 + g_slot_idx[t], rk_s0 = g_slot_grp[s0] * 4 + g_slot_idx[s0];
          int rc[3][2], nrc = 0, j;
          MotionVector **pm = p_EPZS->p_motion[0][0][bt - 1];
          if (pic_x > 0) { rc[nrc][0] = y4; rc[nrc++][1] = pic_x - w4; }
          rc[nrc][0] = up; rc[nrc++][1] = pic_x;
          if (pic_x + w4 < w4pic) { rc[nrc][0] = up; rc[nrc++][1] = pic_x + w4; }
          n_mem = 0;
          for (j = 0; j < nrc && n_mem >= 0; j++) {
            const int row = rc[j][0], col = rc[j][1], cm = col >> 2, xr = x - (xc - cm);
            const int sl = jmme_slot(bt, (col & 3) - (col & 3) % w4, row - row % h4);
            const int rk = g_slot_grp[sl] * 4 + g_slot_idx[sl];
            int16_t vx, vy;
            /* searched in this batch before this call, and not yet by JM when the batch was made */
            const int batch = (cm == xc && rk < rk_t) || (cm < xc && xr >= mb0);
            if (batch && !(xr == mb0 && rk < rk_s0)) {
              const int pk = ep_assumed(xr - mb0, sl);
              if (pk < 0) { n_mem = -1; break; }
              vx = g_ep_ans[pk].res.motion_x;
              vy = g_ep_ans[pk].res.motion_y;
            } else {
              vx = pm[row][col].mv_x;
              vy = pm[row][col].mv_y;
            }
            if (vx | vy) { mem[n_mem][0] = vx; mem[n_mem][1] = vy; ++n_mem; }
          }
        }
        for (w = 0; w < nw0 && nw < EP_WAYS; w++) {
          const ep_ans *a = &g_ep_ans[idx[w]];
          const ep_in *in = &a->in;
          const int16_t (*sp)[2] = hyp0.sp;
          const int *sp_on = hyp0.sp_on, pv_on = hyp0.pv_on;
          const int16_t *pv = hyp0.pv;
          const int np = a->in.q.n_pred, bs = a->in.bt_start & 0xffff, me = a->in.bt_start >> 16;
          const int16_t *ap = (const int16_t *)a->in.pred;
          int fixed = 0, j, o;
          int16_t *tp;
          if (idx[w] == 0 && x == mb0 && t == s0) continue;   /* the real call */
          const int shaped = np >= 5 && me >= 5 && me <= bs && bs <= np;   /* (else: only the stop replay) */
          /* rebuild: spatial [0, 5) | spatial memory [5, me) | temporal + window [me, bs) | block type [bs, np) */
          if (shaped) ep_copy_in(&g_ep_fix, &a->in);
          tp = (int16_t *)g_ep_fix.pred;
          o = 5;
          if (shaped) {
          for (j = 1; j <= 4; j++)
            if (sp_on[j]) { tp[2 * j] = sp[j][0]; tp[2 * j + 1] = sp[j][1]; }
          if (n_mem >= 0) {
            for (j = 0; j < n_mem; j++, o++) { tp[2 * o] = mem[j][0]; tp[2 * o + 1] = mem[j][1]; g_ep_fix.cond[o] = 0; }
          } else {
            for (j = 5; j < me; j++, o++) { tp[2 * o] = ap[2 * j]; tp[2 * o + 1] = ap[2 * j + 1]; g_ep_fix.cond[o] = a->in.cond[j]; }
          }
          if (o + (bs - me) + (n_tail >= 0 ? n_tail : np - bs) > EP_MAXP) goto no_fix;
          for (j = me; j < bs; j++, o++) { tp[2 * o] = ap[2 * j]; tp[2 * o + 1] = ap[2 * j + 1]; g_ep_fix.cond[o] = a->in.cond[j]; }
          if (n_tail >= 0) {
            for (j = 0; j < n_tail; j++, o++) { tp[2 * o] = tail[j][0]; tp[2 * o + 1] = tail[j][1]; g_ep_fix.cond[o] = 0; }
          } else {
            for (j = bs; j < np; j++, o++) { tp[2 * o] = ap[2 * j]; tp[2 * o + 1] = ap[2 * j + 1]; g_ep_fix.cond[o] = a->in.cond[j]; }
          }
          g_ep_fix.q.n_pred = o;
          /* the predictor, and the centre when the guess's centre was its predictor and no list part
           * hangs on the centre (window predictors: the sub-block searches have none) */
          if (pv_on && (pv[0] != a->in.q.pred_x || pv[1] != a->in.q.pred_y) && a->in.q.center_x == a->in.q.pred_x &&
              a->in.q.center_y == a->in.q.pred_y && me == bs &&
              (a->in.q.variant >= 2 || !((pv[0] | pv[1]) & 3))) {   /* (integer grid: the centre is whole-pel) */
            g_ep_fix.q.pred_x = g_ep_fix.q.center_x = pv[0];
            g_ep_fix.q.pred_y = g_ep_fix.q.center_y = pv[1];
          }
          fixed = o != np || memcmp(g_ep_fix.pred, a->in.pred, (size_t)np * 4) || memcmp(g_ep_fix.cond, a->in.cond, (size_t)np) ||
                  g_ep_fix.q.pred_x != a->in.q.pred_x || g_ep_fix.q.pred_y != a->in.q.pred_y;
          if (fixed) {
            ++g_ep_list_fixes;
            in = &g_ep_fix;
          }
          }
        no_fix:
          if (in == &a->in && stop >= a->bnd.stop_lo && stop <= a->bnd.stop_hi && prev >= a->bnd.prev_lo &&
              prev <= a->bnd.prev_hi)
            continue;
          for (k = 0; k < nw0; k++) {   /* a way with these inputs that already holds the pair */
            const ep_ans *o = &g_ep_ans[idx[k]];
            if ((k != w || in != &a->in) && stop >= o->bnd.stop_lo && stop <= o->bnd.stop_hi &&
                prev >= o->bnd.prev_lo && prev <= o->bnd.prev_hi &&
                ep_same(&o->in, &in->q, (const int16_t *)in->pred, in->cond))
              break;
          }
          if (k < nw0) continue;
          ep_add(n, in, px, py, p_EPZS);
          g_ep_q[n].stop_crit = stop;
          g_ep_q[n].prev_sad = prev;
          idx[nw++] = n++;
        }
        {   /* the row after this partition: its first guess's answer (the real call's for the missing one) */
          const ep_ans *a = &g_ep_ans[ep_assumed(x - mb0, t)];
          if (a->bnd.prev_written) row[c] = a->res.cost;
        }
      }
  }
  if (n > n0) {
    ep_run_from(n0, n, NULL, 0, gen);
    g_ep_pass2 += n - n0;
    ++g_ep_pass2_batches;
  }
  *n_io = n;
}

/* no guess fits: search the call alone, or start the next batch when it lies past the current one */
static const ep_ans *ep_miss(Macroblock *currMB, MEBlock *mv_block, const jmme_epzs_req *q, const int16_t *pred,
                             const uint8_t *cond, const int16_t *stale, int n_stale)
{
  EPZSParameters *p_EPZS = currMB->p_Slice->p_EPZS;
  const int mb = (mv_block->pos_y >> 4) * g_mbs_x + (mv_block->pos_x >> 4), ref = q->ref_idx;
  const unsigned gen = g_slot_gen[0][ref];
  const int inside = gen && g_ep_gens[ref] == gen && mb >= g_ep_mb0 && mb < g_ep_mb1;
  ep_in want;
  int n = 1, x, t, r, w, nmb;
  double t0 = now_us();
  ep_fill_in(&want, q, pred, cond, mb, gen);
  want.bt_start = g_ep_bt_start;
  if (inside) {   /* a guess failed: this call alone; the batch's other guesses stand */
    ep_grow(1, q->n_pred);
    g_ep_np = 0;
    ep_add(0, &want, q->pos_x, q->pos_y, p_EPZS);
    g_t_ep_build += now_us() - t0;
    ep_run(1, stale, n_stale, gen);
    ++g_ep_singles;
    /* (request 0 of the batch was a call already served: the batch's other guesses stand) */
    return &g_ep_ans[0];
  }
  /* a new batch from this macroblock: the call itself (way 0 of its slot), and
   * for every partition of the next macroblocks the inputs the same partition
   * had left of the batch and in the row above (distinct ones only) */
  nmb = imin(g_ep_batch, g_n_mb - mb);
  {
    int need = 1 + nmb * JMME_NSLOT * EP_REFS * EP_WAYS;   /* at most EP_WAYS guesses per partition and reference */
    ep_grow(need + 1, (need + 1) * EP_MAXP);
    if (nmb > g_ep_idx_mbs) {   /* (kept across batches: a fresh 250 KB block per batch was malloc / page churn) */
      free(g_ep_idx);
      g_ep_idx_mbs = nmb;
      g_ep_idx = (int *)malloc((size_t)nmb * JMME_NSLOT * EP_REFS * EP_WAYS * sizeof(int));
      if (!g_ep_idx) error("jm_gpu_me: out of memory", 500);
    }
    memset(g_ep_idx, 0xff, (size_t)nmb * JMME_NSLOT * EP_REFS * EP_WAYS * sizeof(int));
  }
  g_ep_np = 0;
  ep_add(0, &want, q->pos_x, q->pos_y, p_EPZS);
  g_ep_idx[(((size_t)0 * JMME_NSLOT + ep_slot_of(q)) * EP_REFS + ref) * EP_WAYS] = 0;
  for (x = mb; x < mb + nmb; x++) {
    const int col = x % g_mbs_x;
    int src[4], ns = 0, i;
    if (mb % g_mbs_x) src[ns++] = mb - 1;                         /* left of the batch, this row */
    if (x - g_mbs_x >= 0 && x - g_mbs_x < mb) src[ns++] = x - g_mbs_x;
    if (col + 1 < g_mbs_x && x - g_mbs_x + 1 >= 0 && x - g_mbs_x + 1 < mb) src[ns++] = x - g_mbs_x + 1;
    if (col > 0 && x - g_mbs_x - 1 >= 0 && x - g_mbs_x - 1 < mb) src[ns++] = x - g_mbs_x - 1;
    for (t = 0; t < JMME_NSLOT; t++) {
      const int px = col * 16 + g_slot_bx[t], py = (x / g_mbs_x) * 16 + g_slot_by[t];
      for (r = 0; r < EP_REFS; r++) {
        int *idx = &g_ep_idx[(((size_t)(x - mb) * JMME_NSLOT + t) * EP_REFS + r) * EP_WAYS];
        if (!g_slot_gen[0][r]) continue;   /* a reference not in use: nothing seen for it */
        w = 0;
        while (w < EP_WAYS && idx[w] >= 0) w++;
        for (i = 0; i < ns && w < EP_WAYS; i++) {
          const ep_in *e = ep_seen_at(src[i], t, r);
          int d;
          if (!g_slot_gen[0][r] || e->mb != src[i] || e->gen != g_slot_gen[0][r]) continue;
          for (d = 0; d < w; d++) {   /* a guess already made for this partition */
            const ep_in *o = idx[d] == 0 ? &want : &g_ep_ans[idx[d]].in;
            if (ep_same_moved(o, e) && o->q.pos_x == px && o->q.pos_y == py) break;
          }
          if (d < w) continue;
          ep_add(n, e, px, py, p_EPZS);
          g_ep_ans[n].in.q = g_ep_q[n];   /* (dedup reads the guess's inputs before the run) */
          g_ep_ans[n].in.bt_start = e->bt_start;
          g_ep_ans[n].in.q.pos_x = (int16_t)px;
          g_ep_ans[n].in.q.pos_y = (int16_t)py;
          memcpy(g_ep_ans[n].in.pred, e->pred, (size_t)e->q.n_pred * 4);
          memcpy(g_ep_ans[n].in.cond, e->cond, (size_t)e->q.n_pred);
          idx[w++] = n++;
        }
      }
    }
  }
  g_t_ep_build += now_us() - t0;
  ep_run(n, stale, n_stale, gen);
  if (g_ep_two_pass) {
    t0 = now_us();
    ep_pass2(currMB, mb, ep_slot_of(q), nmb, gen, &n);
    g_t_ep_p2 += now_us() - t0;
  }
  g_ep_n = n;
  g_ep_mb0 = mb;
  g_ep_mb1 = mb + nmb;
  for (r = 0; r < EP_REFS; r++) g_ep_gens[r] = g_slot_gen[0][r];   /* (a call for another reference stays inside) */
  g_ep_guesses += n - 1;
  ++g_ep_batches;
  return &g_ep_ans[0];
}

/* JM's EPZSMap after the search: every cell it stamped gets BlkCount cnt */
static void ep_apply(EPZSParameters *p_EPZS, const int16_t *vis, int n_vis, uint16 cnt, int side, int max_x, int max_y)
{
  int i;
  for (i = 0; i < n_vis; i++) {
    int r = max_y + vis[2 * i + 1], col = max_x + vis[2 * i];
    if (p_EPZS->EPZSMap[r][col] != cnt) {
      p_EPZS->EPZSMap[r][col] = cnt;
      if (!g_ring_foreign) cell_push(&g_ring[cnt], (uint32_t)(r * side + col));
    }
  }
}

static distblk epzs_gpu(int variant, Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block, distblk min_mcost,
                        int lambda_factor)
{
  Slice *currSlice = currMB->p_Slice;
  InputParameters *p_Inp = currMB->p_Inp;
  EPZSParameters *p_EPZS = currSlice->p_EPZS;
  int list = mv_block->list, cur_list = list + currMB->list_offset, ref = mv_block->ref_idx;
  int bt = mv_block->blocktype, grid = variant >= 2;
  int max_x = mv_block->searchRange.max_x, max_y = mv_block->searchRange.max_y;
  MotionVector *mv = &mv_block->mv[list];
  distblk lambda_dist = weighted_cost(lambda_factor, (variant & 1) ? 3 : 2);
  distblk *prevSad = &p_EPZS->distortion[cur_list][bt - 1][mv_block->pos_x2];
  int side = epzs_map_side(currMB), n_pred, n_stale = 0, i, max_vis;
  uint16 cnt;
  jmme_epzs_req q;
  jmme_epzs_res res;
  double t0, t1;
  init_once(currMB->p_Vid, p_Inp);
  if (fs_on_cpu(mv_block) || 2 * max_x + 1 > side || 2 * max_y + 1 > side) {
    ++g_epzs_cpu;
    return real_epzs(variant, currMB, pred_mv, mv_block, min_mcost, lambda_factor);
  }
  if (g_ep_clk < 0) {   /* per-call clocks only when asked for (two TSC reads a call were ~13 ms per 1080p picture) */
    const char *ph = getenv("JMME_PHASES"), *tr = getenv("JMME_EPZS_TRACE");
    g_ep_clk = (ph && ph[0] == '1') || (tr && tr[0] == '1');
  }
  t0 = g_ep_clk ? now_us() : 0.0;
  ensure_planes(currMB, list, ref);
  ++g_epzs_calls;
  epzs_ring_sync(p_EPZS, side);
  cnt = (uint16)(p_EPZS->BlkCount + 1);
  if (cnt == 0) cnt = 1;

  /* cells already holding cnt inside this search's window, (dx, dy) from the centre */
  if (!g_ring_foreign) {
    cell_list *l = &g_ring[cnt];
    int k = 0;
    grow16(&g_ep_stale, &g_ep_stale_cap, l->n + 1);
    for (i = 0; i < l->n; i++) {
      uint32_t c = l->c[i];
      int r = (int)(c / (uint32_t)side), col = (int)(c % (uint32_t)side);
      if (p_EPZS->EPZSMap[r][col] != cnt) continue;       /* overwritten since */
      l->c[k++] = c;
      if (r <= 2 * max_y && col <= 2 * max_x) {
        g_ep_stale[2 * n_stale] = (int16_t)(col - max_x);
        g_ep_stale[2 * n_stale + 1] = (int16_t)(r - max_y);
        ++n_stale;
      }
    }
    l->n = k;
  } else {
    int step = grid ? 1 : 4, r, col;
    for (r = 0; r <= 2 * max_y; r += step)
      for (col = 0; col <= 2 * max_x; col += step)
        if (p_EPZS->EPZSMap[r][col] == cnt) {
          grow16(&g_ep_stale, &g_ep_stale_cap, n_stale + 1);
          g_ep_stale[2 * n_stale] = (int16_t)(col - max_x);
          g_ep_stale[2 * n_stale + 1] = (int16_t)(r - max_y);
          ++n_stale;
        }
  }
  g_epzs_stale += n_stale;
  if (g_epzs_check < 0) {
    const char *e = getenv("JMME_EPZS_CHECK");
    g_epzs_check = e && e[0] == '1';
  }
  if (g_epzs_check && !g_ring_foreign) {   /* the ring against a scan of the window */
    int step = grid ? 1 : 4, r, col, found = 0, k;
    for (r = 0; r <= 2 * max_y; r += step)
      for (col = 0; col <= 2 * max_x; col += step)
        if (p_EPZS->EPZSMap[r][col] == cnt) {
          for (k = 0; k < n_stale; k++)
            if (g_ep_stale[2 * k] == col - max_x && g_ep_stale[2 * k + 1] == r - max_y) break;
          if (k == n_stale) error("jm_gpu_me: JMME_EPZS_CHECK: a map cell holding the next BlkCount is not in the ring", 500);
          ++found;
        }
    if (found != n_stale) error("jm_gpu_me: JMME_EPZS_CHECK: the ring lists cells the window scan does not find", 500);
  }

  memset(&q, 0, sizeof q);
  q.stop_crit = (int64_t)EPZSDetermineStopCriterion(p_EPZS, prevSad, mv_block, lambda_dist);
  n_pred = epzs_predictors(variant, currMB, mv_block, (distblk)q.stop_crit);
  g_epzs_preds += n_pred;
  q.pos_x = mv_block->pos_x;
  q.pos_y = mv_block->pos_y;
  q.bsx = mv_block->blocksize_x;
  q.bsy = mv_block->blocksize_y;
  q.blocktype = (int16_t)bt;
  q.ref_idx = (int16_t)ref;
  q.pred_x = pred_mv->mv_x;
  q.pred_y = pred_mv->mv_y;
  q.center_x = mv->mv_x;
  q.center_y = mv->mv_y;
  q.max_x = (int16_t)max_x;
  q.max_y = (int16_t)max_y;
  q.lambda = lambda_factor;
  q.variant = (uint8_t)variant;
  q.flags = (uint8_t)((currSlice->structure == FRAME ? JMME_EPZS_FRAME : 0) |
                      (currSlice->slice_type == P_SLICE ? JMME_EPZS_PSLICE : 0));
  q.pattern = (uint8_t)p_Inp->EPZSPattern;
  q.dual = (uint8_t)p_Inp->EPZSDual;
  q.n_pred = n_pred;
  q.n_stale = n_stale;
  q.ref_slot = list * 32 + ref;
  q.prev_sad = (int64_t)*prevSad;
  q.medthres = (int64_t)p_EPZS->medthres[bt];

  const ep_ans *a = NULL;
  if (ep_speculating(currMB, cur_list, ref, n_pred)) {
    /* the speculative path: a cached answer whose inputs are this call's, or a batch */
    t1 = g_ep_trace ? now_us() : 0.0;
    a = ep_lookup(currMB, mv_block, &q, g_ep_pred, g_ep_cond, g_ep_stale, n_stale);
    if (g_ep_trace) { g_t_ep_lookup += now_us() - t1; ++g_ep_lookups; }
    if (!a) {   /* (hits are not timed: two clock reads per call were a tenth of the hits' cost) */
      t1 = now_us();
      a = ep_miss(currMB, mv_block, &q, g_ep_pred, g_ep_cond, g_ep_stale, n_stale);
      g_t_epzs_gpu += now_us() - t1;
    }
    if (a->res.n_visited > EP_MAXV) {   /* (the call itself stamped more cells than a batch keeps: searched again) */
      ++g_ep_overflow;
      a = NULL;
    }
  }
  if (a) {
    res = a->res;
    ep_apply(p_EPZS, &a->vis[0][0], res.n_visited, cnt, side, max_x, max_y);
    g_ep_served = a;
    if (a->bnd.prev_written) *prevSad = (distblk)res.cost;
  } else {
    /* one search per call: its whole window can be stamped */
    max_vis = grid ? (2 * max_x + 1) * (2 * max_y + 1) : ((max_x >> 1) + 1) * ((max_y >> 1) + 1);
    grow16(&g_ep_vis, &g_ep_vis_cap, max_vis);
    t1 = now_us();
    if (jmme_epzs_search_ex(g_me, &q, 1, g_ep_pred, g_ep_cond, n_pred, g_ep_stale, n_stale, &res, g_ep_vis, max_vis))
      fail_jm("jmme_epzs_search_ex");
    g_t_epzs_gpu += now_us() - t1;
    ep_apply(p_EPZS, g_ep_vis, res.n_visited, cnt, side, max_x, max_y);
    g_ep_served = NULL;
    *prevSad = (distblk)res.prev_sad;
  }

  /* JM's side effects */
  p_EPZS->BlkCount = cnt;
  g_ring_count = cnt;
  if (p_Inp->EPZSSpatialMem) {
    MotionVector *m = &p_EPZS->p_motion[cur_list][ref][bt - 1][mv_block->block_y][mv_block->pos_x2];
    m->mv_x = res.motion_x;
    m->mv_y = res.motion_y;
  }
  mv->mv_x = res.mv_x;
  mv->mv_y = res.mv_y;
  if (g_ep_clk) g_t_epzs += now_us() - t0;
  return (distblk)res.cost;
}

distblk __wrap_EPZS_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block, distblk min_mcost,
                                      int lambda_factor)
{
  return epzs_gpu(0, currMB, pred_mv, mv_block, min_mcost, lambda_factor);
}

distblk __wrap_EPZS_subMB_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                            distblk min_mcost, int lambda_factor)
{
  return epzs_gpu(1, currMB, pred_mv, mv_block, min_mcost, lambda_factor);
}

distblk __wrap_EPZS_integer_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                              distblk min_mcost, int lambda_factor)
{
  return epzs_gpu(2, currMB, pred_mv, mv_block, min_mcost, lambda_factor);
}

distblk __wrap_EPZS_integer_subMB_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                                    distblk min_mcost, int lambda_factor)
{
  return epzs_gpu(3, currMB, pred_mv, mv_block, min_mcost, lambda_factor);
}

/* EPZS_sub_pel_motion_estimation's contract (me_epzs_sub.c:30-222): variant 1
 * of jmme_subpel_refine, its early-exit threshold p_EPZS->subthres[blocktype] */
distblk __wrap_EPZS_sub_pel_motion_estimation(Macroblock *currMB, MotionVector *pred_mv, MEBlock *mv_block,
                                              distblk min_mcost, int *lambda_factor)
{
  VideoParameters *p_Vid = currMB->p_Vid;
  Slice *currSlice = currMB->p_Slice;
  int list = mv_block->list, ref = mv_block->ref_idx;
  int mh = metric_id(mv_block->computePredHPel), mq = metric_id(mv_block->computePredQPel);
  jmme_subpel_req q;
  jmme_block_res r;
  init_once(p_Vid, currMB->p_Inp);
  if (mh < 0 || mq < 0 || (g_bits > 11 && (mh == 1 || mq == 1)) || mv_block->ChromaMEEnable ||
      mv_block->search_pos2 > 9 || mv_block->search_pos4 > 9 ||
      (mv_block->test8x8 && mv_block->blocktype > 4)) {
    ++g_epzs_sp_cpu;
    return __real_EPZS_sub_pel_motion_estimation(currMB, pred_mv, mv_block, min_mcost, lambda_factor);
  }
  ++g_epzs_sp_calls;
  ensure_planes(currMB, list, ref);
  memset(&q, 0, sizeof q);
  q.pos_x = mv_block->pos_x;
  q.pos_y = mv_block->pos_y;
  q.blocktype = (int16_t)mv_block->blocktype;
  q.ref_slot = (int16_t)(list * 32 + ref);
  q.pred_x = pred_mv->mv_x;
  q.pred_y = pred_mv->mv_y;
  q.mv_x = mv_block->mv[list].mv_x;
  q.mv_y = mv_block->mv[list].mv_y;
  q.lambda_h = lambda_factor[H_PEL];
  q.lambda_q = lambda_factor[Q_PEL];
  q.min_mcost = (int64_t)min_mcost;
  q.subthres = (int64_t)currSlice->p_EPZS->subthres[mv_block->blocktype];
  q.variant = 1;
  q.flags = (uint8_t)((mv_block->test8x8 ? JMME_SP_TEST8x8 : 0) |
                      ((!currMB->p_Inp->rdopt && currSlice->slice_type != B_SLICE) ? JMME_SP_CHECK0 : 0));
  q.metric_h = (uint8_t)mh;
  q.metric_q = (uint8_t)mq;
  q.start_hp = (uint8_t)(p_Vid->start_me_refinement_hp != 0);
  q.start_qp = (uint8_t)(p_Vid->start_me_refinement_qp != 0);
  q.search_pos2 = (uint8_t)mv_block->search_pos2;
  q.search_pos4 = (uint8_t)mv_block->search_pos4;
  /* the parameters the next batches chain their refinements with */
  g_ep_spp.lam_h = q.lambda_h;
  g_ep_spp.lam_q = q.lambda_q;
  g_ep_spp.metric_h = q.metric_h;
  g_ep_spp.metric_q = q.metric_q;
  g_ep_spp.start_hp = q.start_hp;
  g_ep_spp.start_qp = q.start_qp;
  g_ep_spp.pos2 = q.search_pos2;
  g_ep_spp.pos4 = q.search_pos4;
  g_ep_spp.check0 = (q.flags & JMME_SP_CHECK0) != 0;
  g_ep_spp.t8 = currMB->p_Inp->Transform8x8Mode != 0;
  g_ep_spp.valid = 1;
  if (g_ep_served && g_ep_served->spq.blocktype && !memcmp(&g_ep_served->spq, &q, sizeof q)) {
    /* refined on the device right after the integer search this call follows */
    r = g_ep_served->sp_res;
    ++g_ep_sp_hits;
  } else if (jmme_subpel_refine(g_me, &q, 1, &r)) {
    fail_jm("jmme_subpel_refine");
  }
  g_ep_served = NULL;
  mv_block->mv[list].mv_x = r.mv_x;
  mv_block->mv[list].mv_y = r.mv_y;
  return (distblk)r.cost;
}

/* reported at exit, so a run shows the searches really went to the GPU */
static void report(void) __attribute__((destructor));
static void report(void)
{
  if (g_me || g_cpu_calls || g_epzs_cpu) {
    fprintf(stderr, "jm_gpu_me: %lld integer-pel searches on the GPU (libjmme): %lld from %lld speculative "
                    "batches, the rest one call each; %lld on the CPU (non-SAD or weighted metric)\n",
            g_calls, g_hits + g_batches + g_chain_calls - g_chain_call_fail, g_batches, g_cpu_calls);
    fprintf(stderr, "jm_gpu_me: %lld sub-pel refinements: %lld cached, %lld batches, %lld on the CPU; "
                    "%.1f ms in sub-pel batches (building %.1f, in the library %.1f, storing %.1f)\n", g_sp_calls,
              g_sp_hits, g_sp_batches, g_sp_cpu, g_t_sp * 1e-3, g_t_sp_part[0] * 1e-3, g_t_sp_part[1] * 1e-3,
              g_t_sp_part[2] * 1e-3);
    if (g_batches) {
      int s;
      fprintf(stderr, "jm_gpu_me: integer batches: %lld past the batch, %lld failed guesses; %lld units; "
                      "%.1f ms building, %.1f ms in jmme_search_mbs; failed guesses by slot:",
              g_miss_past, g_miss_guess, g_units, g_t_build * 1e-3, g_t_call * 1e-3);
      if (g_trace)
        fprintf(stderr, " [%.1f ms inside the FS wrapper, %.1f ms uploading %lld planes (longest %.1f ms)]",
                g_t_wrap * 1e-3, g_t_planes * 1e-3, g_n_uploads, g_t_plane_max * 1e-3);
      for (s = 0; s < JMME_NSLOT; s++) fprintf(stderr, " %lld", g_miss_slot[s]);
      fprintf(stderr, "\n");
    }
    if (g_chain_sent)
      fprintf(stderr, "jm_gpu_me: chained guesses: %lld chains, %lld steps, %lld calls answered, %lld head mismatches; "
                      "%lld chain-only calls (%lld fell back to a batch); %.1f ms in chain-only calls\n",
              g_chain_sent, g_chain_steps, g_chain_hits, g_chain_head_bad, g_chain_calls, g_chain_call_fail,
              g_t_chain * 1e-3);
    if (g_chain_sp_steps || g_chain_sp_nolam)
      fprintf(stderr, "jm_gpu_me: chained sub-pel: %lld refinements, %lld calls answered; %lld misses without "
                      "known sub-pel lambdas\n", g_chain_sp_steps, g_chain_sp_hits, g_chain_sp_nolam);
    if (g_epzs_calls || g_epzs_cpu)
      fprintf(stderr, "jm_gpu_me: %lld EPZS searches on the GPU (libjmme); %lld on the CPU; "
                      "%lld predictors, %lld pre-stamped map cells, %lld switches to window scans; "
                      "%.1f ms in the EPZS wrapper, %.1f ms in the engine\n",
              g_epzs_calls, g_epzs_cpu, g_epzs_preds, g_epzs_stale, g_epzs_foreign, g_t_epzs * 1e-3,
              g_t_epzs_gpu * 1e-3);
    if (g_epzs_calls && g_ep_spec > 0)
      fprintf(stderr, "jm_gpu_me: EPZS speculation: %lld searches answered from %lld batches (%lld guesses), "
                      "%lld searched alone; %lld not speculated; guesses refused: %lld inputs, %lld bounds, "
                      "%lld map cells; %.1f ms building batches; %lld searched again (more stamped cells than kept); "
                      "%lld second-pass guesses in %lld launches (%lld with lists rebuilt from the batch's answers)\n",
              g_ep_hits, g_ep_batches, g_ep_guesses, g_ep_singles, g_ep_direct, g_ep_fail_inputs, g_ep_fail_bounds,
              g_ep_fail_stale, g_t_ep_build * 1e-3, g_ep_overflow, g_ep_pass2, g_ep_pass2_batches, g_ep_list_fixes);
    if (g_epzs_calls && g_ep_batches)
      fprintf(stderr, "jm_gpu_me: EPZS host clocks: %.1f ms running guesses (%.1f ms of it in the library), %.1f ms in the "
                      "second pass (with its runs), %.1f ms in %lld lookups (JMME_EPZS_TRACE=1 only)\n",
              g_t_ep_run * 1e-3, g_t_ep_runlib * 1e-3, g_t_ep_p2 * 1e-3, g_t_ep_lookup * 1e-3, g_ep_lookups);
    if (g_ep_trace) {
      int sl;
      fprintf(stderr, "jm_gpu_me: EPZS misses inside batches by slot (list-only differences):");
      for (sl = 0; sl < JMME_NSLOT; sl++) fprintf(stderr, " %d:%lld(%lld)", sl, g_ep_miss_slot[sl], g_ep_list_diff[sl]);
      fprintf(stderr, "\njm_gpu_me: EPZS misses inside batches by kind: %lld inputs, %lld stop criterion, %lld prevSad, "
                      "%lld map cells; stop misses by bits of |real - guessed|:",
              g_ep_miss_kind[0], g_ep_miss_kind[1], g_ep_miss_kind[2], g_ep_miss_kind[3]);
      for (sl = 0; sl < 24; sl++) fprintf(stderr, " %lld", g_ep_stop_off[sl]);
      fprintf(stderr, "\njm_gpu_me: EPZS stop misses by the nearest way's return path (real below / above its interval):");
      for (sl = 0; sl < 8; sl++) fprintf(stderr, " %d:%lld/%lld", sl, g_ep_stop_side[sl][0], g_ep_stop_side[sl][1]);
      fprintf(stderr, "\n");
    }
    if (g_epzs_sp_calls || g_epzs_sp_cpu)
      fprintf(stderr, "jm_gpu_me: %lld EPZS sub-pel refinements on the GPU (%lld chained in the search's launch), "
                      "%lld on the CPU\n", g_epzs_sp_calls, g_ep_sp_hits, g_epzs_sp_cpu);
    if (g_trace) fclose(g_trace);
    if (g_trace_miss) fclose(g_trace_miss);
    if (g_me) jmme_destroy(g_me);
  }
}
