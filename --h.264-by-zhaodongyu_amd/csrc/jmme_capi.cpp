// jmme_capi.cpp -- host side of libjmme.so: configuration (JM .cfg keys),
// frame-buffer upload from JM's get_mem2Dpel layout, request validation and
// kernel launch.  See include/jmme.h for the reference interfaces replaced.
#include <hip/hip_runtime.h>

#include <cctype>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "jmme.h"
#include "jmme_common.h"
#include "jmme_internal.h"
#include "jmme_tq_internal.h"
#include "jmme_epzs_internal.h"
#include "jmme_fractal_internal.h"
#include "jmme_subpel_internal.h"

using namespace jmme;

namespace {

thread_local std::string g_err;

int fail(const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return -1;
}

#define HIPCHK(x)                                                                 \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) return fail("%s: %s", #x, hipGetErrorString(e_));      \
  } while (0)


// Every entry point that takes a context runs on the context's device and
// restores the caller's current device on return, so contexts on several GPUs
// (or a caller such as torch that switches devices) never mix pointers.
struct DevGuard {
  int prev = -1;
  // keep_server: the caller may hand a request to a running EPZS server; every
  // other entry point stops it first (it may write what the server reads)
  explicit DevGuard(const jmme_ctx *c, bool keep_server = false);
  ~DevGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
  DevGuard(const DevGuard &) = delete;
  DevGuard &operator=(const DevGuard &) = delete;
};

}  // namespace

#ifndef JMME_CHUNK_STRIPES
#define JMME_CHUNK_STRIPES 8
#endif
// Items dealt to an XCD at a time (the item kernel's chunks, c % 8 -> XCD c).
// JMME_CHUNK_STRIPES=1: a picture row of macroblocks / 8 when that divides, so
// that a full frame's chunk c is column stripe c % 8 of its row -- each XCD
// then serves one stripe of columns top to bottom and its L2 holds the windows
// of vertical as well as horizontal neighbours; else 16.
inline int item_chunk(int width, int *rot) {
  static const int stripes = [] { const char *e = getenv("JMME_CHUNK_STRIPES"); return e ? atoi(e) : JMME_CHUNK_STRIPES; }();
  const int mbs_x = width / 16;
  const bool on = stripes && mbs_x >= 8 && mbs_x % 8 == 0;
  *rot = on && stripes > 1 ? stripes : 0;
  return on ? mbs_x / 8 : 16;
}

struct jmme_ctx {
  jmme_config cfg;
  int device = 0;
  int max_mvd = 0;
  int width = 0, height = 0, pitch = 0;      // pitch in pels
  bool hbd = false;                          // SourceBitDepthLuma > 8: 16-bit planes, small-kernel search only
  int max_pel = 255;
  uint8_t *d_cur = nullptr;
  uint8_t *d_refs[kMaxLists * kMaxRefs] = {};
  const uint8_t **d_ref_table = nullptr;     // device copy of d_refs
  bool ref_table_dirty = true;
  uint8_t *h_stage = nullptr;                // u16 -> u8 conversion buffer (pinned: one DMA per plane)
  size_t cap_stage = 0;
  jmme_mb_req *d_req = nullptr;
  jmme_block_res *d_out = nullptr;
  size_t cap_units = 0;
  unsigned long long *d_stamps = nullptr;    // diagnostic builds only
  void *d_tree = nullptr;                    // fractal quadtree scratch (lists + per-level results)
  size_t cap_tree = 0;
  void *d_pool = nullptr;                    // fractal pool images (7 sizes) + flags + survivor counter
  size_t cap_pool = 0;
  int pool_min_range = 80;                   // jmme_fractal_search: pruned pool search from this radius up
  int pool_mfma = 1;                         // 4x4 full pool: matrix-core bound test (0: VALU)
  size_t cap_stamps = 0;
  unsigned *d_counts = nullptr;              // 2 x kCountWords: [0] further groups, [2] status, [8..15] XCD tickets
  int counts_half = 0;                       // the set the next launch uses (the plan kernel zeroes the other)
  unsigned *last_counts = nullptr;           // the set of the last launch (status)
  Item *d_items = nullptr;                   // work items (one per unit x partition group)
  size_t cap_items = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  // quarter-pel sub-images per reference slot (getSubImagesLuma), built lazily
  uint8_t *d_subs[kMaxLists * kMaxRefs] = {};
  bool sub_stale[kMaxLists * kMaxRefs] = {};
  const uint8_t **d_sub_table = nullptr;     // device copy of d_subs
  bool sub_table_dirty = true;
  // synchronous calls: pinned host staging + a device scratch for sub-pel requests,
  // kept across calls (one DMA each way and one stream sync per call)
  uint8_t *h_pin = nullptr;
  size_t cap_pin = 0;
  uint8_t *d_sp = nullptr;
  size_t cap_sp = 0;
  // low-latency small batches (launch_search_small): host-built items and the
  // results in mapped pinned memory, the keys and completion counter on the device
  int small_max_wg = 4096;                   // largest grid sent down the small path (0: never)
  SmallItem *h_sitems = nullptr;
  size_t cap_sitems = 0;
  jmme_block_res *h_sout = nullptr;
  size_t cap_sout = 0;
  jmme_chain_res *h_chres = nullptr;         // jmme_search_mbs_chains results (mapped pinned)
  jmme_block_res *h_chsp = nullptr;          // jmme_search_mbs_chains_sp refinements (mapped pinned)
  uint32_t *h_chdone = nullptr;              // per chain: the launch's number behind its results (mapped, coherent)
  void *dv_chdone = nullptr;
  uint32_t chain_seq = 0;
  void *dv_chsp = nullptr;
  unsigned long long *h_hkeys = nullptr;    // small latency form: per-tile keys (mapped pinned)
  size_t cap_hkeys = 0;
  uint8_t *h_emap = nullptr;                 // jmme_epzs_search_ex: mapped pinned request / result block
  size_t cap_emap = 0;
  unsigned long long *d_skeys = nullptr;     // per (item, tile) keys, cap_skeys * JMME_NSLOT
  size_t cap_skeys = 0;
  hipStream_t chain_stream = nullptr;        // chains run beside the batch of the same call (non-blocking)
  // EPZS searches alone (JMME_SINGLE_MODE: 0 null stream + sync, 1 own stream + sync,
  // 2 own stream + the kernel's completion word polled in mapped memory, 3 (default)
  // the resident server below)
  int single_mode = -1;
  hipStream_t single_stream = nullptr;
  uint32_t *h_done = nullptr;
  void *dv_done = nullptr;
  uint32_t done_seq = 0;
  // JMME_SINGLE_MODE 3: the resident EPZS server (jmme_epzs.hip
  // epzs_server_kernel) and its mailbox in mapped pinned memory
  EpzsBox *h_box = nullptr;
  EpzsBox *d_box = nullptr;
  hipStream_t srv_stream = nullptr;
  bool srv_running = false;
  int srv_grid = -1, srv_hbd = -1, srv_map_words = 0;
  uint32_t srv_seq = 0;
  uint32_t srv_idle_ticks = 200000;          // 2 ms at s_memrealtime's 100 MHz (JMME_EPZS_SERVER_IDLE_US)
  long long srv_launches = 0, srv_served = 0;
  long long srv_fallbacks = 0;   // requests the server left unserved (2 s without it), launched instead
  double srv_service_us = 0;                 // JMME_PHASES: the server's own time per request, summed
  double srv_host_us[4] = {};                // JMME_PHASES: a search alone on the host -- call entry to the
                                             // server hand-off, hand-off to posted, posted to done, done to return
  double srv_t_call = 0, srv_t_post = 0, srv_t_done = 0;
  double srv_cycles = 0;
  double ep_batch_us[3] = {};                // JMME_PHASES: batches -- copies in, launches + wait, copies out
  double srv_rph_us[6] = {};                 // JMME_PHASES: the refinement's phase ends and passes (from its window)                     // JMME_PHASES: s_memtime ticks over the requests' service, summed
  double srv_copy_us = 0, srv_search_us = 0; // (to the request's copy in LDS, to the search's end)
  double srv_ph_us[10] = {};                  // (the search's phases: set-up, centre, predictors, walk, visited
                                             //  (its word list); the refinement's window and phases)
  bool srv_check = false;                    // JMME_EPZS_SERVER_CHECK: every served search again by the fused kernel
  uint8_t *h_chk = nullptr;                  // (its outputs, mapped pinned)
  long long srv_mismatch = 0;
  std::vector<SmallItem> small_scratch;      // search_small's items (kept: no allocation per call)
  void *dv_hkeys = nullptr, *dv_chres = nullptr, *dv_sitems = nullptr, *dv_sout = nullptr;   // device views
  std::vector<uint8_t *> spare_planes;       // jmme_reserve: plane buffers the first uploads take
  size_t spare_bytes = 0;                    // their size (taken only by uploads of that size)
  // JMME_PHASES=1: host-side phase times of the latency calls, printed at jmme_destroy
  bool phases = false;
  double ph_us[12] = {};
  double ep_us[2] = {};                      // JMME_PHASES: jmme_epzs_speculate time, searches alone / batches
  long long ep_n[2] = {};
  long long ph_calls = 0, ph_big = 0;
  // jmme_residual4x4: parameter sets, requests and results in one mapped pinned
  // block the kernel reads and writes across PCIe (a few blocks per call)
  uint8_t *h_rq = nullptr;
  void *dv_rq = nullptr;
  size_t cap_rq = 0;
  hipStream_t rq_stream = nullptr;
};

namespace {
double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// adds the time since *t to ctx->ph_us[i] and restarts *t (JMME_PHASES only)
inline void phase(jmme_ctx *ctx, int i, double *t) {
  if (!ctx->phases) return;
  const double n = now_us();
  ctx->ph_us[i] += n - *t;
  *t = n;
}

// the resident EPZS server exits at its next poll; returns once its stream is idle
int server_stop(jmme_ctx *ctx) {
  if (!ctx->srv_running) return 0;
  ctx->srv_running = false;
  __atomic_store_n(&ctx->h_box->quit, 1u, __ATOMIC_RELEASE);
  const hipError_t e = hipStreamSynchronize(ctx->srv_stream);
  __atomic_store_n(&ctx->h_box->quit, 0u, __ATOMIC_RELEASE);
  if (e != hipSuccess) return fail("EPZS server: %s", hipGetErrorString(e));
  return 0;
}
}  // namespace

DevGuard::DevGuard(const jmme_ctx *c, bool keep_server) {
  int cur = 0;
  if (c && hipGetDevice(&cur) == hipSuccess && cur != c->device && hipSetDevice(c->device) == hipSuccess) prev = cur;
  if (c && !keep_server) (void)server_stop(const_cast<jmme_ctx *>(c));
}

// ----------------------------------------------------------------- config --
extern "C" int jmme_config_default(jmme_config *c) {
  if (!c) return fail("null config");
  // defaults of JM's Map[] (JM/lencod/inc/configfile.h, column 4)
  c->SourceWidth = 176;
  c->SourceHeight = 144;
  c->SearchMode = 0;
  c->SearchRange = 16;
  c->NumberReferenceFrames = 1;
  c->DisableSubpelME = 0;
  c->RDOptimization = 0;
  c->MEDistortionFPel = 0;
  c->MDDistortion = 2;
  c->EPZSSubPelGrid = 0;
  c->RestrictSearchRange = 2;
  c->UseMVLimits = 0;
  c->SetMVXLimit = 0;
  c->SetMVYLimit = 0;
  c->ChromaMEEnable = 0;
  c->SourceBitDepthLuma = 8;
  return 0;
}

namespace {

int *cfg_field(jmme_config *c, const std::string &k) {
  struct { const char *name; size_t off; } tab[] = {
#define F(n) {#n, offsetof(jmme_config, n)}
      F(SourceWidth), F(SourceHeight), F(SearchMode), F(SearchRange), F(NumberReferenceFrames),
      F(DisableSubpelME), F(RDOptimization), F(MEDistortionFPel), F(MDDistortion), F(EPZSSubPelGrid),
      F(RestrictSearchRange), F(UseMVLimits), F(SetMVXLimit), F(SetMVYLimit), F(ChromaMEEnable),
      F(SourceBitDepthLuma),
#undef F
  };
  for (auto &t : tab)
    if (k == t.name) return reinterpret_cast<int *>(reinterpret_cast<char *>(c) + t.off);
  return nullptr;
}

// One "Key = Value" assignment, JM syntax (ParseContent, configfile.c):
// '#' starts a comment; values are numbers (ints, or doubles truncated by JM
// for int params) or quoted strings (ignored here).
int apply_assign(jmme_config *c, const std::string &key, const std::string &val) {
  int *f = cfg_field(c, key);
  if (!f) return 0;  // not an ME key: JM's Map has it, we do not need it
  const char *s = val.c_str();
  char *end = nullptr;
  double d = strtod(s, &end);
  if (end == s) return fail("config: bad value '%s' for %s", s, key.c_str());
  *f = (int)d;
  return 0;
}

int parse_text(jmme_config *c, const std::string &text) {
  size_t i = 0, n = text.size();
  std::vector<std::string> tok;
  while (i < n) {
    char ch = text[i];
    if (ch == '#') {
      while (i < n && text[i] != '\n') ++i;
    } else if (isspace((unsigned char)ch)) {
      ++i;
    } else if (ch == '=') {
      tok.push_back("=");
      ++i;
    } else if (ch == '"') {
      size_t j = text.find('"', i + 1);
      if (j == std::string::npos) return fail("config: unterminated string");
      tok.push_back(text.substr(i, j - i + 1));
      i = j + 1;
    } else {
      size_t j = i;
      while (j < n && !isspace((unsigned char)text[j]) && text[j] != '=' && text[j] != '#') ++j;
      tok.push_back(text.substr(i, j - i));
      i = j;
    }
  }
  for (size_t k = 0; k < tok.size();) {
    if (k + 2 < tok.size() + 0 && tok[k + 1] == "=") {
      if (apply_assign(c, tok[k], tok[k + 2])) return -1;
      k += 3;
    } else if (k + 1 < tok.size() && tok[k + 1] == "=") {
      return fail("config: missing value for %s", tok[k].c_str());
    } else {
      ++k;
    }
  }
  return 0;
}

}  // namespace

extern "C" int jmme_config_parse(jmme_config *c, const char *path, int argc, const char *const *argv) {
  if (!c) return fail("null config");
  if (path) {
    FILE *fp = fopen(path, "rb");
    if (!fp) return fail("config: cannot open %s", path);
    std::string text;
    char buf[4096];
    size_t r;
    while ((r = fread(buf, 1, sizeof buf, fp)) > 0) text.append(buf, r);
    fclose(fp);
    if (parse_text(c, text)) return -1;
  }
  for (int i = 0; i < argc; ++i)
    if (argv[i] && parse_text(c, argv[i])) return -1;
  // JM clears EPZSSubPelGrid unless SearchMode is EPZS (PatchInp, configfile.c:1330-1335)
  if (c->SearchMode != JMME_EPZS) c->EPZSSubPelGrid = 0;
  return 0;
}

extern "C" int jmme_max_mvd(const jmme_config *c) {
  // init_motion_search_module, JM/lencod/src/mv_search.c:321-328
  int sr = c->SearchRange;
  int nsp = 4 * (2 * sr + 3);
  int max_mv_bits = 3 + 2 * (int)ceil(log((double)(nsp + 1)) / log(2.0) + 1e-10);
  int base = (1 << (max_mv_bits >> 1)) - 1;
  if (c->UseMVLimits) {
    int lim = 4 * (c->SetMVXLimit > c->SetMVYLimit ? c->SetMVXLimit : c->SetMVYLimit);
    return lim > base ? lim : base;
  }
  return base;
}

// ---------------------------------------------------------------- context --
extern "C" const char *jmme_last_error(void) { return g_err.c_str(); }
extern "C" const char *jmme_version(void) { return "jmme 0.1 (gfx950)"; }

extern "C" jmme_ctx *jmme_create(const jmme_config *cfg, int device) {
  if (!cfg) { fail("null config"); return nullptr; }
  if (cfg->ChromaMEEnable) { fail("ChromaMEEnable != 0 is not supported"); return nullptr; }
  // JM's imgpel holds 8..14-bit luma (defines.h:37, configfile.h SourceBitDepthLuma)
  if (cfg->SourceBitDepthLuma < 8 || cfg->SourceBitDepthLuma > 14) {
    fail("SourceBitDepthLuma %d outside 8..14", cfg->SourceBitDepthLuma);
    return nullptr;
  }
  // the integer-pel kernels compute JM's computeSAD (me_distortion.c:349); SSE /
  // SATD full-pel metrics (MEDistortionFPel 1/2, lencod.c:782-796) would give
  // different vectors, so they are refused rather than silently searched with SAD
  if (cfg->MEDistortionFPel != 0) {
    fail("MEDistortionFPel %d: only SAD (0) integer-pel search is supported", cfg->MEDistortionFPel);
    return nullptr;
  }
  if (cfg->SearchRange < 0 || cfg->SearchRange > JMME_MAX_RANGE) {
    fail("SearchRange %d outside [0,%d]", cfg->SearchRange, JMME_MAX_RANGE);
    return nullptr;
  }
  auto *ctx = new jmme_ctx;
  ctx->cfg = *cfg;
  ctx->hbd = cfg->SourceBitDepthLuma > 8;
  ctx->max_pel = (1 << cfg->SourceBitDepthLuma) - 1;
  ctx->max_mvd = jmme_max_mvd(cfg);
  hipError_t e;
  int caller_dev = -1;
  (void)hipGetDevice(&caller_dev);
  if (device >= 0 && device != caller_dev) {
    e = hipSetDevice(device);
    if (e != hipSuccess) { fail("hipSetDevice(%d): %s", device, hipGetErrorString(e)); delete ctx; return nullptr; }
  }
  (void)hipGetDevice(&ctx->device);
  {
    const char *ph = getenv("JMME_PHASES");
    ctx->phases = ph && *ph && *ph != '0';
  }
  // allocations below go to ctx->device; the caller's current device is restored on return
  struct Restore {
    int d, was;
    ~Restore() { if (d >= 0 && d != was) (void)hipSetDevice(d); }
  } restore_{caller_dev, ctx->device};
  if ((e = hipMalloc(&ctx->d_ref_table, sizeof(uint8_t *) * kMaxLists * kMaxRefs)) != hipSuccess ||
      (e = hipMalloc(&ctx->d_counts, 2 * kCountWords * sizeof(unsigned))) != hipSuccess ||
      (e = hipMemset(ctx->d_counts, 0, 2 * kCountWords * sizeof(unsigned))) != hipSuccess ||
      (e = hipMalloc(&ctx->d_sub_table, sizeof(uint8_t *) * kMaxLists * kMaxRefs)) != hipSuccess ||
      (e = hipEventCreate(&ctx->ev0)) != hipSuccess || (e = hipEventCreate(&ctx->ev1)) != hipSuccess) {
    fail("jmme_create: %s", hipGetErrorString(e));
    jmme_destroy(ctx);
    return nullptr;
  }
  return ctx;
}

extern "C" void jmme_destroy(jmme_ctx *ctx) {
  DevGuard dg_(ctx);
  if (!ctx) return;
  if (ctx->phases && ctx->ph_calls) {
    static const char *names[12] = {"chains: validate+launch", "small: items", "small: launch", "small: sync",
                                    "small: host finish", "chains: sync+copy", "big: validate", "big: stage+launch",
                                    "big: sync", "big: scatter", "", ""};
    fprintf(stderr, "jmme phases over %lld chained calls (us per call):", ctx->ph_calls);
    for (int i = 0; i < 6; ++i)
      if (ctx->ph_us[i] > 0) fprintf(stderr, " %s %.2f;", names[i], ctx->ph_us[i] / ctx->ph_calls);
    fprintf(stderr, "\njmme phases over %lld throughput-path calls (us per call):", ctx->ph_big);
    for (int i = 6; i < 10; ++i)
      if (ctx->ph_us[i] > 0) fprintf(stderr, " %s %.2f;", names[i], ctx->ph_us[i] / std::max(1ll, ctx->ph_big));
    fprintf(stderr, "\n");
  }
  (void)hipFree(ctx->d_cur);
  for (auto *p : ctx->d_refs) (void)hipFree(p);
  for (auto *p : ctx->spare_planes) (void)hipFree(p);
  (void)hipFree(ctx->d_ref_table);
  (void)hipFree(ctx->d_req);
  (void)hipFree(ctx->d_out);
  (void)hipFree(ctx->d_counts);
  (void)hipFree(ctx->d_items);
  (void)hipFree(ctx->d_stamps);
  (void)hipFree(ctx->d_tree);
  (void)hipFree(ctx->d_pool);
  for (auto *p : ctx->d_subs) (void)hipFree(p);
  (void)hipFree(ctx->d_sub_table);
  (void)hipFree(ctx->d_sp);
  if (ctx->h_pin) (void)hipHostFree(ctx->h_pin);
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  if (ctx->h_sitems) (void)hipHostFree(ctx->h_sitems);
  if (ctx->h_sout) (void)hipHostFree(ctx->h_sout);
  if (ctx->h_emap) (void)hipHostFree(ctx->h_emap);
  if (ctx->h_hkeys) (void)hipHostFree(ctx->h_hkeys);
  if (ctx->h_chres) (void)hipHostFree(ctx->h_chres);
  if (ctx->h_chsp) (void)hipHostFree(ctx->h_chsp);
  if (ctx->chain_stream) (void)hipStreamDestroy(ctx->chain_stream);
  if (ctx->single_stream) {
    (void)hipStreamSynchronize(ctx->single_stream);
    (void)hipStreamDestroy(ctx->single_stream);
  }
  if (ctx->h_done) (void)hipHostFree(ctx->h_done);
  if (ctx->h_chdone) (void)hipHostFree(ctx->h_chdone);
  if (ctx->srv_fallbacks)   // (always reported: it says the GPU's queues were oversubscribed)
    fprintf(stderr, "jmme EPZS server: %lld requests not taken within 2 s, launched on their own\n", ctx->srv_fallbacks);
  if (ctx->phases && ctx->srv_launches)
    fprintf(stderr, "jmme EPZS server: %lld searches over %lld launches; %.2f us per search in the server "
            "(request copy %.2f, search to %.2f)\n", ctx->srv_served, ctx->srv_launches,
            ctx->srv_service_us / std::max(1ll, ctx->srv_served), ctx->srv_copy_us / std::max(1ll, ctx->srv_served),
            ctx->srv_search_us / std::max(1ll, ctx->srv_served));
  if (ctx->phases && ctx->srv_served)
    fprintf(stderr, "jmme EPZS server search phases (us): set-up %.2f, centre %.2f, predictors %.2f, walk %.2f, "
            "visited %.2f (word list %.2f); refinement: window %.2f, phases %.2f; predictor rounds (summed over all "
            "searches / searches): set-up %.2f, costs %.2f\n",
            ctx->srv_ph_us[0] / ctx->srv_served, ctx->srv_ph_us[1] / ctx->srv_served,
            ctx->srv_ph_us[2] / ctx->srv_served, ctx->srv_ph_us[3] / ctx->srv_served,
            ctx->srv_ph_us[4] / ctx->srv_served, ctx->srv_ph_us[5] / ctx->srv_served,
            ctx->srv_ph_us[6] / ctx->srv_served, ctx->srv_ph_us[7] / ctx->srv_served, ctx->srv_ph_us[8] / ctx->srv_served,
            ctx->srv_ph_us[9] / ctx->srv_served);
  if (ctx->phases && ctx->srv_served)
    fprintf(stderr, "jmme EPZS server host side (us per search): call to hand-off %.2f, hand-off to posted %.2f, "
            "posted to done %.2f, done to return %.2f; shader clock while serving %.0f MHz\n",
            ctx->srv_host_us[0] / ctx->srv_served,
            ctx->srv_host_us[1] / ctx->srv_served, ctx->srv_host_us[2] / ctx->srv_served,
            ctx->srv_host_us[3] / ctx->srv_served, ctx->srv_cycles / std::max(1e-9, ctx->srv_service_us));
  if (ctx->phases && ctx->srv_served)
    fprintf(stderr, "jmme EPZS server refinement (us from its window, mean): phase A ends %.2f, B %.2f, C %.2f, D %.2f; "
            "first pass ends %.2f, second %.2f\n", ctx->srv_rph_us[0] / ctx->srv_served,
            ctx->srv_rph_us[1] / ctx->srv_served, ctx->srv_rph_us[2] / ctx->srv_served,
            ctx->srv_rph_us[3] / ctx->srv_served, ctx->srv_rph_us[4] / ctx->srv_served,
            ctx->srv_rph_us[5] / ctx->srv_served);
  if (ctx->srv_check) fprintf(stderr, "jmme EPZS server check: %lld mismatches\n", ctx->srv_mismatch);
  if (ctx->phases && ctx->ep_n[1])
    fprintf(stderr, "jmme EPZS batches (ms in all): validation and copies in %.1f, launches and wait %.1f, copies "
            "out %.1f\n", ctx->ep_batch_us[0] * 1e-3, ctx->ep_batch_us[1] * 1e-3, ctx->ep_batch_us[2] * 1e-3);
  if (ctx->phases && (ctx->ep_n[0] || ctx->ep_n[1]))
    fprintf(stderr, "jmme EPZS calls: %lld alone, %.1f ms (%.2f us each); %lld batches, %.1f ms\n", ctx->ep_n[0],
            ctx->ep_us[0] / 1e3, ctx->ep_us[0] / std::max(1ll, ctx->ep_n[0]), ctx->ep_n[1], ctx->ep_us[1] / 1e3);
  if (ctx->h_chk) (void)hipHostFree(ctx->h_chk);
  if (ctx->rq_stream) (void)hipStreamDestroy(ctx->rq_stream);
  if (ctx->h_rq) (void)hipHostFree(ctx->h_rq);
  (void)server_stop(ctx);   // (the guard above has stopped it already)
  if (ctx->srv_stream) (void)hipStreamDestroy(ctx->srv_stream);
  if (ctx->h_box) (void)hipHostFree(ctx->h_box);
  (void)hipFree(ctx->d_skeys);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  delete ctx;
}

namespace {

int set_geometry(jmme_ctx *ctx, int w, int h) {
  if (w <= 0 || h <= 0 || (w & 15) || (h & 15))
    return fail("picture %dx%d: width and height must be positive multiples of 16 (JM's coded size)", w, h);
  if (ctx->width == w && ctx->height == h) return 0;
  if (ctx->width) return fail("picture size changed from %dx%d to %dx%d", ctx->width, ctx->height, w, h);
  ctx->width = w;
  ctx->height = h;
  ctx->pitch = (w + 63) & ~63;
  return 0;
}

// JM get_mem2Dpel(_pad) planes: rows[y] equally spaced.  Converted to 8-bit
// (or kept 16-bit when the context is high bit depth).
int upload_plane(jmme_ctx *ctx, uint8_t **dst, const jmme_imgpel *const *rows, int w, int h) {
  if (!rows || !rows[0]) return fail("null plane");
  if (set_geometry(ctx, w, h)) return -1;
  ptrdiff_t stride = h > 1 ? rows[1] - rows[0] : w;
  const size_t es = ctx->hbd ? 2 : 1, bytes = (size_t)ctx->pitch * h * es;
  if (bytes > ctx->cap_stage) {
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    ctx->h_stage = nullptr;
    ctx->cap_stage = 0;
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_stage), bytes, hipHostMallocDefault));
    ctx->cap_stage = bytes;
  }
  for (int y = 0; y < h; ++y) {
    const jmme_imgpel *src = rows[0] + (ptrdiff_t)y * stride;
    if (rows[y] != src) return fail("plane rows are not equally spaced (row %d)", y);
    unsigned m = 0;
    if (ctx->hbd) {
      uint16_t *d = reinterpret_cast<uint16_t *>(ctx->h_stage) + (size_t)y * ctx->pitch;
      for (int x = 0; x < w; ++x) { m |= src[x]; d[x] = src[x]; }
    } else {
      uint8_t *d = ctx->h_stage + (size_t)y * ctx->pitch;
      for (int x = 0; x < w; ++x) { m |= src[x]; d[x] = (uint8_t)src[x]; }
    }
    if (m > (unsigned)ctx->max_pel)
      return fail("sample above %d in row %d (SourceBitDepthLuma %d)", ctx->max_pel, y, ctx->cfg.SourceBitDepthLuma);
  }
  if (!*dst && !ctx->spare_planes.empty() && ctx->spare_bytes == bytes) {   // the size jmme_reserve expected
    *dst = ctx->spare_planes.back();
    ctx->spare_planes.pop_back();
  }
  if (!*dst) HIPCHK(hipMalloc(dst, bytes));
  // complete before the staging buffer is refilled by the next upload
  HIPCHK(hipMemcpyAsync(*dst, ctx->h_stage, bytes, hipMemcpyHostToDevice, nullptr));
  HIPCHK(hipStreamSynchronize(nullptr));
  return 0;
}

}  // namespace

extern "C" int jmme_upload_cur(jmme_ctx *ctx, const jmme_imgpel *const *rows, int w, int h) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  return upload_plane(ctx, &ctx->d_cur, rows, w, h);
}

extern "C" int jmme_upload_ref(jmme_ctx *ctx, int list, int ref_idx, const jmme_imgpel *const *rows, int w, int h) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (list < 0 || list >= kMaxLists || ref_idx < 0 || ref_idx >= kMaxRefs)
    return fail("list/ref_idx (%d,%d) out of range", list, ref_idx);
  uint8_t **slot = &ctx->d_refs[list * kMaxRefs + ref_idx];
  bool fresh = *slot == nullptr;
  if (upload_plane(ctx, slot, rows, w, h)) return -1;
  if (fresh) ctx->ref_table_dirty = true;
  ctx->sub_stale[list * kMaxRefs + ref_idx] = true;
  return 0;
}

// ----------------------------------------------------------------- search --
extern "C" int jmme_slot(int bt, int bx, int by) { return slot_of(bt, bx, by); }
extern "C" int jmme_spiral_index(int ox, int oy) { return spiral_index(ox, oy); }
extern "C" void jmme_spiral_offset(int idx, int *ox, int *oy) { spiral_offset(idx, ox, oy); }
extern "C" int jmme_mvbits(int v) { return mvbits(v); }

namespace {

// host-array convenience: stage through device buffers owned by this call
struct DevBuf {
  void *p = nullptr;
  ~DevBuf() { (void)hipFree(p); }
  hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 4); }
};

int ensure_units(jmme_ctx *ctx, size_t n) {
  if (n <= ctx->cap_units) return 0;
  (void)hipFree(ctx->d_req);
  (void)hipFree(ctx->d_out);
  ctx->d_req = nullptr;
  ctx->d_out = nullptr;
  size_t cap = std::max<size_t>({n, 1024, 2 * ctx->cap_units});   // geometric: few reallocations while batches grow
  HIPCHK(hipMalloc(&ctx->d_req, cap * sizeof(jmme_mb_req)));
  HIPCHK(hipMalloc(&ctx->d_out, cap * JMME_NSLOT * sizeof(jmme_block_res)));
  ctx->cap_units = cap;
  return 0;
}

// every unit yields at most one item per searched partition
int ensure_items(jmme_ctx *ctx, size_t n) {
  if (n <= ctx->cap_items) return 0;
  (void)hipFree(ctx->d_items);
  ctx->d_items = nullptr;
  size_t cap = std::max<size_t>({n, 4096, 2 * ctx->cap_items});
  HIPCHK(hipMalloc(&ctx->d_items, cap * sizeof(Item)));
  ctx->cap_items = cap;
  return 0;
}

int sync_ref_table(jmme_ctx *ctx, hipStream_t s) {
  if (!ctx->ref_table_dirty) return 0;
  HIPCHK(hipMemcpyAsync(ctx->d_ref_table, ctx->d_refs, sizeof(ctx->d_refs), hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  ctx->ref_table_dirty = false;
  return 0;
}

int launch(jmme_ctx *ctx, int mode, const uint8_t *d_cur, const uint8_t *const *d_ref_table, int pitch,
           int w, int h, const jmme_mb_req *d_req, int n, jmme_block_res *d_out, hipStream_t s,
           uint32_t *debug_words = nullptr, bool planes_8bit = false) {
  // high bit depth: the context's 16-bit planes go to the 64-bit-key v_sad_u16
  // instance of the item kernel; explicitly 8-bit planes to the 8-bit one
  const bool hbd = ctx->hbd && !planes_8bit;
  if (mode != JMME_FULL_SEARCH && mode != JMME_FAST_FULL_SEARCH)
    return fail("search mode %d not supported by the batched engine (FS=-1, FFS=0)", mode);
  if (n < 0) return fail("negative unit count");
  if (n == 0) return 0;
  if (ensure_items(ctx, (size_t)n * JMME_NSLOT)) return -1;
  KParams p{};
  p.cur = d_cur;
  p.refs = d_ref_table;
  p.pitch = pitch;
  p.width = w;
  p.height = h;
  p.req = d_req;
  p.out = d_out;
  p.n = n;
  p.mode = mode;
  p.max_mvd = ctx->max_mvd;
  p.lds_range = ctx->cfg.SearchRange;
  // 32-bit keys: 8-bit planes, or 16-bit ones up to 10 bits (a 4x4 SAD < 2^14: its
  // key SAD << 16 + K stays exact; larger partitions saturate into the exact
  // re-search); JMME_HBD_KEY32=0 keeps 16-bit planes on the 64-bit keys (A/B)
  static const bool hbd_key32 = [] { const char *e = getenv("JMME_HBD_KEY32"); return !(e && e[0] == '0'); }();
  p.key32 = (!hbd || (hbd_key32 && ctx->cfg.SourceBitDepthLuma <= 10)) && p.lds_range <= kKey32MaxRange;
  p.hbd = hbd ? 1 : 0;
  p.items = ctx->d_items;
  p.item_cap = (unsigned)ctx->cap_items;
  p.counts = ctx->d_counts + ctx->counts_half * kCountWords;
  p.counts_next = ctx->d_counts + (ctx->counts_half ^ 1) * kCountWords;
  p.debug_words = debug_words;
  p.chunk = item_chunk(w, &p.rot);
#ifdef JMME_STAMPS
  // n units x 8 words, then 4 words per workgroup (up to kStampWGs)
  const size_t words = (size_t)n * 8 + (size_t)kStampWGs * 4;
  if (words > ctx->cap_stamps) {
    (void)hipFree(ctx->d_stamps);
    HIPCHK(hipMalloc(&ctx->d_stamps, words * sizeof(unsigned long long)));
    ctx->cap_stamps = words;
  }
  p.stamps = ctx->d_stamps;
  HIPCHK(hipMemsetAsync(ctx->d_stamps, 0, words * sizeof(unsigned long long), s));
#endif
  // jmme_last_kernel_ms: the main item kernel alone (ev0 .. ev1)
  if (launch_search(p, s, ctx->ev0, ctx->ev1) != hipSuccess) {
    // the plan kernel may have launched and counted into this set (and zeroed
    // only the other one): leave both clean for the next launch
    (void)hipMemsetAsync(ctx->d_counts, 0, 2 * kCountWords * sizeof(*ctx->d_counts), s);
    ctx->counts_half = 0;
    return fail("launch_search: the item-kernel launch failed");
  }
  ctx->last_counts = p.counts;
  ctx->counts_half ^= 1;
  ctx->timed = true;
  return 0;
}

int ensure_pin(jmme_ctx *ctx, size_t bytes) {
  if (bytes <= ctx->cap_pin) return 0;
  if (ctx->h_pin) (void)hipHostFree(ctx->h_pin);
  ctx->h_pin = nullptr;
  ctx->cap_pin = 0;
  size_t cap = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 2;
  HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_pin), cap, hipHostMallocDefault));
  ctx->cap_pin = cap;
  return 0;
}

int ensure_sp(jmme_ctx *ctx, size_t bytes) {
  if (bytes <= ctx->cap_sp) return 0;
  (void)hipFree(ctx->d_sp);
  ctx->d_sp = nullptr;
  ctx->cap_sp = 0;
  size_t cap = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 2;
  HIPCHK(hipMalloc(&ctx->d_sp, cap));
  ctx->cap_sp = cap;
  return 0;
}

constexpr size_t align64(size_t v) { return (v + 63) & ~size_t(63); }

int status_words(const unsigned *st, const jmme_ctx *ctx) {
  if (st[2] & 8u) return fail("internal (JMME_DBG_CHECKS): the waves of a workgroup computed different saturated-slot masks");
  if (st[2] & 16u) return fail("internal (JMME_DBG_CHECKS): the waves of a workgroup disagree on the item");
  if (st[2] & 4u) return fail("internal: the refine pass lost a winner");
  if (st[2] & 1u) return fail("a request's search range exceeds the configured SearchRange %d (or an FFS block range its surface's)", ctx->cfg.SearchRange);
  if (st[2] & 2u) return fail("a full-search centre is not on the integer grid (EPZSSubPelGrid sub-pel centres are not supported)");
  return 0;
}

int check_status(jmme_ctx *ctx, hipStream_t s) {
  unsigned st[3] = {0, 0, 0};
  if (!ctx->last_counts) return 0;   // no batched launch yet
  HIPCHK(hipMemcpyAsync(st, ctx->last_counts, sizeof st, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return status_words(st, ctx);
}

int validate(const jmme_ctx *ctx, int mode, const jmme_mb_req *req, int n) {
  for (int i = 0; i < n; ++i) {
    const jmme_mb_req &r = req[i];
    if (r.mb_x < 0 || r.mb_y < 0 || (r.mb_x & 15) || (r.mb_y & 15) || r.mb_x + 16 > ctx->width ||
        r.mb_y + 16 > ctx->height)
      return fail("unit %d: macroblock (%d,%d) outside the %dx%d picture", i, r.mb_x, r.mb_y, ctx->width, ctx->height);
    if (r.list < 0 || r.list >= kMaxLists || r.ref_idx < 0 || r.ref_idx >= kMaxRefs ||
        !ctx->d_refs[r.list * kMaxRefs + r.ref_idx])
      return fail("unit %d: reference (%d,%d) not uploaded", i, r.list, r.ref_idx);
    if (r.slot_mask >> JMME_NSLOT) return fail("unit %d: slot mask has bits above %d", i, JMME_NSLOT - 1);
    if (mode == JMME_FAST_FULL_SEARCH) {
      if (r.ffs_range < 0 || r.ffs_range > ctx->cfg.SearchRange)
        return fail("unit %d: FFS range %d outside [0,%d]", i, r.ffs_range, ctx->cfg.SearchRange);
      if ((r.ffs_center_x | r.ffs_center_y) & 3) return fail("unit %d: FFS centre not integer", i);
    }
    for (int s = 0; s < JMME_NSLOT; ++s) {
      if (!((r.slot_mask >> s) & 1)) continue;
      const jmme_block_req &b = r.blk[s];
      if (b.lambda < 0) return fail("unit %d slot %d: negative lambda", i, s);
      if (mode == JMME_FULL_SEARCH) {
        if (b.search_range < 0 || b.search_range > ctx->cfg.SearchRange)
          return fail("unit %d slot %d: range %d outside [0,%d]", i, s, b.search_range, ctx->cfg.SearchRange);
        if ((b.center_x | b.center_y) & 3)
          return fail("unit %d slot %d: sub-pel search centre (EPZSSubPelGrid) not supported", i, s);
      } else if (b.search_range < 0 || b.search_range > r.ffs_range) {
        return fail("unit %d slot %d: block range %d outside the FFS surface range %d", i, s, b.search_range, r.ffs_range);
      }
    }
  }
  return 0;
}

// ---- small batches (launch_search_small) -----------------------------------
// The partitions of a unit that share a window and a predictor/lambda form one
// item, as the plan kernel groups them (FS: centre, range, predictor, lambda;
// FFS: the unit's surface + predictor, lambda and own range).
void small_items(const jmme_ctx *ctx, int mode, const jmme_mb_req *req, int n, std::vector<SmallItem> &items,
                 int *max_range) {
  const bool ffs = mode == JMME_FAST_FULL_SEARCH;
  items.clear();
  *max_range = 0;
  for (int u = 0; u < n; ++u) {
    const jmme_mb_req &r = req[u];
    uint64_t rem = r.slot_mask & ((1ull << JMME_NSLOT) - 1);
    while (rem) {
      const int lead = __builtin_ctzll(rem);
      const jmme_block_req &a = r.blk[lead];
      uint64_t gm = 0;
      for (uint64_t m = rem; m; m &= m - 1) {
        const int sl = __builtin_ctzll(m);
        const jmme_block_req &b = r.blk[sl];
        if (b.pred_x == a.pred_x && b.pred_y == a.pred_y && b.lambda == a.lambda && b.search_range == a.search_range &&
            (ffs || (b.center_x == a.center_x && b.center_y == a.center_y)))
          gm |= 1ull << sl;
      }
      rem &= ~gm;
      SmallItem it{};
      it.ref = ctx->d_refs[r.list * kMaxRefs + r.ref_idx];
      it.gmask = gm;
      it.u = u;
      it.mb_x = r.mb_x;
      it.mb_y = r.mb_y;
      it.cqx = ffs ? r.ffs_center_x : a.center_x;
      it.cqy = ffs ? r.ffs_center_y : a.center_y;
      it.R = ffs ? r.ffs_range : a.search_range;
      it.rs = a.search_range;
      it.px = a.pred_x;
      it.py = a.pred_y;
      it.lam = a.lambda;
      it.flags = (int16_t)(((!ffs && (gm & 1) && (r.blk[0].flags & JMME_BLK_CHECK00)) ? kItemChk00 : 0) |
                           ((ffs && r.ffs_pos00_valid) ? kItemPreseed : 0));
      it.bmask = 0;
      for (uint64_t m = gm; m; m &= m - 1) {
        const SlotGeom sg = slot_geom(__builtin_ctzll(m));
        for (int y = 0; y < sg.h; ++y)
          for (int x = 0; x < sg.w; ++x) it.bmask |= (uint16_t)(1u << ((sg.by + y) * 4 + sg.bx + x));
      }
      *max_range = std::max(*max_range, (int)it.R);
      items.push_back(it);
    }
  }
}

// 1 = served (results in out), 0 = too large for the small path, -1 = error
int search_small(jmme_ctx *ctx, int mode, const jmme_mb_req *req, int n, jmme_block_res *out, hipStream_t s,
                 bool force = false) {
  if (ctx->small_max_wg <= 0 && !force) return 0;
  // the latency form is for a few units (the drop-in's re-batches): larger
  // batches go to the throughput path without building their items here
  constexpr int kSmallMaxUnits = 32;
  if (n > kSmallMaxUnits && !force) return 0;
  double t_ph = ctx->phases ? now_us() : 0;
  std::vector<SmallItem> &items = ctx->small_scratch;
  int max_r = 0;
  small_items(ctx, mode, req, n, items, &max_r);
  const int tiles = (2 * max_r + 1 + kSmallTile - 1) / kSmallTile;
  const long long wgs = (long long)items.size() * tiles * tiles;
  if (items.empty() || (wgs > ctx->small_max_wg && !force)) return items.empty() ? 1 : 0;
  // 32-bit costs: (SAD << 5) + lambda * mvbits must not wrap.  A batch with
  // such a lambda (8-bit or 16-bit planes) falls through to the item kernel,
  // whose 64-bit keys serve it exactly.
  for (const SmallItem &it : items)
    if ((uint64_t)it.lam * 64u + ((uint64_t)256 * ctx->max_pel << 5) >= (1ull << 32)) {
      return 0;
    }
  if (items.size() > ctx->cap_sitems) {
    if (ctx->h_sitems) (void)hipHostFree(ctx->h_sitems);
    ctx->h_sitems = nullptr;
    ctx->cap_sitems = 0;
    const size_t cap = std::max<size_t>(256, items.size());
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_sitems), cap * sizeof(SmallItem), hipHostMallocMapped));
    HIPCHK(hipHostGetDevicePointer(&ctx->dv_sitems, ctx->h_sitems, 0));
    ctx->cap_sitems = cap;
  }
  if ((size_t)wgs > ctx->cap_skeys) {              // one key per (item, tile, partition)
    (void)hipFree(ctx->d_skeys);
    ctx->d_skeys = nullptr;
    ctx->cap_skeys = 0;
    const size_t cap = std::max<size_t>(4096, (size_t)wgs);
    HIPCHK(hipMalloc(&ctx->d_skeys, cap * JMME_NSLOT * sizeof(unsigned long long) + cap * sizeof(int4)));
    ctx->cap_skeys = cap;
  }
  if ((size_t)n * JMME_NSLOT > ctx->cap_sout) {
    if (ctx->h_sout) (void)hipHostFree(ctx->h_sout);
    ctx->h_sout = nullptr;
    ctx->cap_sout = 0;
    const size_t cap = std::max<size_t>(64 * JMME_NSLOT, (size_t)n * JMME_NSLOT);
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_sout), cap * sizeof(jmme_block_res), hipHostMallocMapped));
    HIPCHK(hipHostGetDevicePointer(&ctx->dv_sout, ctx->h_sout, 0));
    ctx->cap_sout = cap;
  }
  SmallParams p{};
  p.cur = ctx->d_cur;
  p.pitch = ctx->pitch;
  p.width = ctx->width;
  p.height = ctx->height;
  p.mode = mode;
  p.max_mvd = ctx->max_mvd;
  p.hbd = ctx->hbd ? 1 : 0;
  p.n_items = (int)items.size();
  p.tiles = tiles;
  const int tpi = tiles * tiles;
  // Up to kSmallInline items travel in the kernel arguments (no read of host
  // memory before the first load).  Latency form for a few items: the per-tile
  // keys go to mapped host memory and the minimum over tiles is taken here (one
  // launch); past kHostFinishItems the host's reads of those keys cost more
  // than the finish launch (tools/ubench_small.py: 1 unit 35.1 -> 30.2 us,
  // 8 units 37.6 -> 48.6 us).
  constexpr size_t kHostFinishItems = 4;
  const bool lat = items.size() <= kHostFinishItems;
  p.n_inline = (int)std::min(items.size(), (size_t)kSmallInline);
  std::memcpy(p.inl, items.data(), (size_t)p.n_inline * sizeof(SmallItem));
  void *d_items = nullptr, *d_sout = nullptr, *d_hkeys = nullptr;
  if (lat) {
    const size_t nk = (size_t)wgs * JMME_NSLOT;
    if (nk > ctx->cap_hkeys) {
      if (ctx->h_hkeys) (void)hipHostFree(ctx->h_hkeys);
      ctx->h_hkeys = nullptr;
      ctx->cap_hkeys = 0;
      const size_t cap = std::max<size_t>(64 * 1024, nk);
      HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_hkeys), cap * sizeof(unsigned long long),
                           hipHostMallocMapped));
      HIPCHK(hipHostGetDevicePointer(&ctx->dv_hkeys, ctx->h_hkeys, 0));
      ctx->cap_hkeys = cap;
    }
    d_hkeys = ctx->dv_hkeys;
    p.host_finish = 1;
    p.keys = static_cast<unsigned long long *>(d_hkeys);
    phase(ctx, 1, &t_ph);
    HIPCHK(launch_search_small(p, s));
    phase(ctx, 2, &t_ph);
    HIPCHK(hipStreamSynchronize(s));
    phase(ctx, 3, &t_ph);
    ctx->timed = false;
    const bool ffs = mode == JMME_FAST_FULL_SEARCH;
    for (size_t ii = 0; ii < items.size(); ++ii) {
      const SmallItem &it = items[ii];
      const unsigned long long *k0 = ctx->h_hkeys + ii * tpi * JMME_NSLOT;
      for (uint64_t m = it.gmask; m; m &= m - 1) {
        const int sl = __builtin_ctzll(m);
        unsigned long long k = ~0ull;
        for (int t = 0; t < tpi; ++t) k = std::min(k, k0[(size_t)t * JMME_NSLOT + sl]);
        // block_result (jmme_search.hip): the winning spiral rank -> vector
        jmme_block_res &r = out[(size_t)it.u * JMME_NSLOT + sl];
        r.reserved = 0;
        if (k == ~0ull) {
          r.mv_x = it.cqx; r.mv_y = it.cqy; r.cost = JMME_DISTBLK_MAX;
          continue;
        }
        const int rank = (int)(uint32_t)(k & 0xffffffffu);
        int ox, oy;
        if (ffs && rank == 0) { ox = -(it.cqx >> 2); oy = -(it.cqy >> 2); }   // the pre-seeded (0,0)
        else spiral_offset(ffs ? rank - 1 : rank, &ox, &oy);
        r.mv_x = (int16_t)(it.cqx + 4 * ox);
        r.mv_y = (int16_t)(it.cqy + 4 * oy);
        r.cost = (int64_t)(k >> 32);
      }
    }
    phase(ctx, 4, &t_ph);
    return 1;
  }
  std::memcpy(ctx->h_sitems, items.data(), items.size() * sizeof(SmallItem));
  d_items = ctx->dv_sitems;
  d_sout = ctx->dv_sout;
  p.items = static_cast<const SmallItem *>(d_items);
  p.keys = ctx->d_skeys;
  p.info = reinterpret_cast<int4 *>(ctx->d_skeys + ctx->cap_skeys * JMME_NSLOT);   // items <= workgroups <= cap
  p.out = static_cast<jmme_block_res *>(d_sout);
  phase(ctx, 1, &t_ph);
  HIPCHK(launch_search_small(p, s));
  phase(ctx, 2, &t_ph);
  HIPCHK(hipStreamSynchronize(s));
  phase(ctx, 3, &t_ph);
  ctx->timed = false;
  for (int i = 0; i < n; ++i)
    for (int sl = 0; sl < JMME_NSLOT; ++sl)
      if ((req[i].slot_mask >> sl) & 1) out[(size_t)i * JMME_NSLOT + sl] = ctx->h_sout[(size_t)i * JMME_NSLOT + sl];
  phase(ctx, 4, &t_ph);
  return 1;
}

}  // namespace

extern "C" int jmme_set_small_batch_limit(jmme_ctx *ctx, int max_workgroups) {
  if (!ctx) return fail("null ctx");
  ctx->small_max_wg = max_workgroups < 0 ? 0 : max_workgroups;
  return 0;
}

extern "C" int jmme_search_mbs(jmme_ctx *ctx, int mode, const jmme_mb_req *req, int n, jmme_block_res *out) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (!ctx->d_cur) return fail("current picture not uploaded");
  if (n == 0) return 0;
  if (!req || !out) return fail("null request/result array");
  double t_ph = ctx->phases ? now_us() : 0;
  if (validate(ctx, mode, req, n)) return -1;
  hipStream_t s = nullptr;
  // a batch of a few units: the low-latency path (one launch, no copies)
  if (mode == JMME_FULL_SEARCH || mode == JMME_FAST_FULL_SEARCH) {
    // (high bit depth too: small batches on the 16-bit small kernel, the rest on
    // the 16-bit item kernel)
    const int r = search_small(ctx, mode, req, n, out, s);
    if (r != 0) return r < 0 ? -1 : 0;
  }
  if (ctx->phases) ++ctx->ph_big;
  phase(ctx, 6, &t_ph);
  if (ensure_units(ctx, (size_t)n)) return -1;
  if (sync_ref_table(ctx, s)) return -1;
  // pinned staging: [requests | results | status words]
  const size_t rq = align64((size_t)n * sizeof(jmme_mb_req)), rs = align64((size_t)n * JMME_NSLOT * sizeof(jmme_block_res));
  if (ensure_pin(ctx, rq + rs + 64)) return -1;
  std::memcpy(ctx->h_pin, req, (size_t)n * sizeof(jmme_mb_req));
  HIPCHK(hipMemcpyAsync(ctx->d_req, ctx->h_pin, (size_t)n * sizeof(jmme_mb_req), hipMemcpyHostToDevice, s));
  if (launch(ctx, mode, ctx->d_cur, ctx->d_ref_table, ctx->pitch, ctx->width, ctx->height, ctx->d_req, n,
             ctx->d_out, s))
    return -1;
  // results for searched slots only: copy the whole block, then merge
  const jmme_block_res *tmp = reinterpret_cast<const jmme_block_res *>(ctx->h_pin + rq);
  const unsigned *st = reinterpret_cast<const unsigned *>(ctx->h_pin + rq + rs);
  HIPCHK(hipMemcpyAsync(ctx->h_pin + rq, ctx->d_out, (size_t)n * JMME_NSLOT * sizeof(jmme_block_res),
                        hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(ctx->h_pin + rq + rs, ctx->last_counts, 3 * sizeof(unsigned), hipMemcpyDeviceToHost, s));
  phase(ctx, 7, &t_ph);
  HIPCHK(hipStreamSynchronize(s));
  phase(ctx, 8, &t_ph);
  if (status_words(st, ctx)) return -1;
  constexpr uint64_t kAll = (1ull << JMME_NSLOT) - 1;
  for (int i = 0; i < n; ++i) {
    if ((req[i].slot_mask & kAll) == kAll) {
      std::memcpy(&out[(size_t)i * JMME_NSLOT], &tmp[(size_t)i * JMME_NSLOT], JMME_NSLOT * sizeof(jmme_block_res));
      continue;
    }
    for (int sl = 0; sl < JMME_NSLOT; ++sl)
      if ((req[i].slot_mask >> sl) & 1) out[(size_t)i * JMME_NSLOT + sl] = tmp[(size_t)i * JMME_NSLOT + sl];
  }
  phase(ctx, 9, &t_ph);
  return 0;
}

// chained searches: validated and launched (asynchronously, on stream s)
// before the batch of the same call, so the batch's stream sync covers them
namespace {
int prepare_subs(jmme_ctx *ctx, hipStream_t s);

// an in-chain SubPelME template (jmme_search_mbs_chains_sp): what
// jmme_subpel_validate checks of a request's parameters, variant 0, no test8x8
int check_chain_sp(const jmme_ctx *ctx, int i, const jmme_subpel_req &q) {
  if (q.variant != 0) return fail("chain %d: sub-pel variant %d (chains run sub_pel_motion_estimation)", i, q.variant);
  if (q.flags & ~JMME_SP_CHECK0) return fail("chain %d: sub-pel flags %d (no test8x8 in chains)", i, q.flags);
  if (q.metric_h > 2 || q.metric_q > 2) return fail("chain %d: sub-pel metric %d/%d", i, q.metric_h, q.metric_q);
  if ((q.metric_h == 1 || q.metric_q == 1) && ctx->cfg.SourceBitDepthLuma > 11)
    return fail("chain %d: SSE sub-pel metric at SourceBitDepthLuma %d (int sums may wrap)", i,
                ctx->cfg.SourceBitDepthLuma);
  if (q.start_hp > 1 || q.start_qp > 1) return fail("chain %d: start_hp/qp", i);
  if (q.search_pos2 > 9 || q.search_pos4 > 9)
    return fail("chain %d: search_pos2/4 %d/%d beyond JM's 9-point rings", i, q.search_pos2, q.search_pos4);
  if (q.lambda_h < 0 || q.lambda_q < 0) return fail("chain %d: negative sub-pel lambda", i);
  return 0;
}

int launch_chains(jmme_ctx *ctx, int mode, const jmme_chain *chains, int n, hipStream_t s,
                  const jmme_subpel_req *sp = nullptr) {
  if (n <= 0) return 0;
  if (n > kChainInline) return fail("%d chains in one call (at most %d)", n, kChainInline);
  if (mode != JMME_FULL_SEARCH && mode != JMME_FAST_FULL_SEARCH) return fail("chains: mode %d", mode);
  ChainParams p{};
  int max_r = 0;
  for (int i = 0; i < n; ++i) {
    const jmme_chain &c = chains[i];
    if (c.n_steps < 1 || c.n_steps > JMME_CHAIN_MAX_STEPS) return fail("chain %d: %d steps", i, c.n_steps);
    if (c.mb_x < 0 || c.mb_y < 0 || (c.mb_x & 15) || (c.mb_y & 15) || c.mb_x + 16 > ctx->width ||
        c.mb_y + 16 > ctx->height)
      return fail("chain %d: macroblock (%d,%d) outside the picture", i, c.mb_x, c.mb_y);
    if (c.list < 0 || c.list >= kMaxLists || c.ref_idx < 0 || c.ref_idx >= kMaxRefs ||
        !ctx->d_refs[c.list * kMaxRefs + c.ref_idx])
      return fail("chain %d: reference (%d,%d) not uploaded", i, c.list, c.ref_idx);
    if (c.lambda < 0) return fail("chain %d: negative lambda", i);
    // 32-bit costs: (SAD << 5) + lambda * mvbits must not wrap (16-bit planes: SAD up to 256 * max_pel)
    if ((uint64_t)c.lambda * 64u + ((uint64_t)256 * ctx->max_pel << 5) >= (1ull << 32))
      return fail("chain %d: lambda %d too large for 32-bit costs", i, c.lambda);
    if (mode == JMME_FAST_FULL_SEARCH && (c.ffs_range < 0 || c.ffs_range > kChainMaxR || (c.ffs_center_x & 3) ||
                                          (c.ffs_center_y & 3)))
      return fail("chain %d: FFS surface range %d / centre", i, c.ffs_range);
    for (int k = 0; k < c.n_steps; ++k) {
      const jmme_chain_step &st = c.steps[k];
      if (st.slot < 0 || st.slot >= JMME_NSLOT) return fail("chain %d step %d: slot %d", i, k, st.slot);
      if ((st.flags & ~JMME_CHAIN_CHECK00) || ((st.flags & JMME_CHAIN_CHECK00) && st.slot != 0))
        return fail("chain %d step %d: flags %d (check_for_00 is a 16x16 step's)", i, k, st.flags);
      for (int j = 0; j < 3; ++j)
        if (st.nb[j].src < JMME_NB_FIXED || st.nb[j].src >= k)
          return fail("chain %d step %d: neighbour source %d", i, k, st.nb[j].src);
      if (st.sr_min_x > 0 || st.sr_max_x < 0 || st.sr_min_y > 0 || st.sr_max_y < 0)
        return fail("chain %d step %d: search window", i, k);
    }
  }
  max_r = kChainMaxR;
  const size_t nres = (size_t)n * JMME_CHAIN_MAX_STEPS;
  if (!ctx->h_chres) {
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_chres), kChainInline * JMME_CHAIN_MAX_STEPS *
                                                                      sizeof(jmme_chain_res), hipHostMallocMapped));
    HIPCHK(hipHostGetDevicePointer(&ctx->dv_chres, ctx->h_chres, 0));
  }
  std::memset(ctx->h_chres, 0, nres * sizeof(jmme_chain_res));
  void *d_res = ctx->dv_chres;
  if (sync_ref_table(ctx, s)) return -1;
  if (sp) {
    for (int i = 0; i < n; ++i)
      if (check_chain_sp(ctx, i, sp[i])) return -1;
    if (!ctx->h_chsp) {
      HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_chsp), kChainInline * JMME_CHAIN_MAX_STEPS *
                                                                       sizeof(jmme_block_res), hipHostMallocMapped));
      HIPCHK(hipHostGetDevicePointer(&ctx->dv_chsp, ctx->h_chsp, 0));
    }
    std::memset(ctx->h_chsp, 0, nres * sizeof(jmme_block_res));
    if (prepare_subs(ctx, s)) return -1;
    const SubGeom g = sub_geom(ctx->width, ctx->height);
    p.subs = ctx->d_sub_table;
    p.sub_pitch = g.pitch;
    p.plane_stride = g.plane_stride;
    p.sp_res = static_cast<jmme_block_res *>(ctx->dv_chsp);
    std::memcpy(p.sp, sp, (size_t)n * sizeof(jmme_subpel_req));
  }
  p.cur = ctx->d_cur;
  p.refs = ctx->d_ref_table;
  p.pitch = ctx->pitch;
  p.width = ctx->width;
  p.height = ctx->height;
  p.mode = mode;
  p.max_mvd = ctx->max_mvd;
  p.n = n;
  p.max_r = max_r;
  p.hbd = ctx->hbd ? 1 : 0;
  p.res = static_cast<jmme_chain_res *>(d_res);
  if (!ctx->h_chdone) {
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_chdone), kChainInline * sizeof(uint32_t),
                         hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer(&ctx->dv_chdone, ctx->h_chdone, 0));
    std::memset(ctx->h_chdone, 0, kChainInline * sizeof(uint32_t));
  }
  p.done = static_cast<uint32_t *>(ctx->dv_chdone);
  p.seq = ++ctx->chain_seq;
  std::memcpy(p.chains, chains, (size_t)n * sizeof(jmme_chain));
  HIPCHK(launch_search_chains(p, s));
  return 0;
}

// the chains of the last launch have stored their completion words (polled:
// a stream synchronisation costs more than the words' PCIe write); 2 s
// without them, the stream is synchronised instead (surfacing a fault)
int wait_chains(jmme_ctx *ctx, int n, hipStream_t s) {
  const uint32_t seq = ctx->chain_seq;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i)
    for (unsigned spin = 1; __atomic_load_n(&ctx->h_chdone[i], __ATOMIC_ACQUIRE) != seq; ++spin) {
      if ((spin & 4095u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        HIPCHK(hipStreamSynchronize(s));
        if (__atomic_load_n(&ctx->h_chdone[i], __ATOMIC_ACQUIRE) != seq) return fail("chains: no completion word");
      }
      __builtin_ia32_pause();
    }
  return 0;
}
}  // namespace

extern "C" int jmme_search_mbs_chains_sp(jmme_ctx *ctx, int mode, const jmme_mb_req *req, int n,
                                         jmme_block_res *out, const jmme_chain *chains, int n_chains,
                                         const jmme_subpel_req *sp, jmme_chain_res *res, jmme_block_res *sp_res) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (!ctx->d_cur) return fail("current picture not uploaded");
  if (n_chains < 0 || (n_chains && (!chains || !res))) return fail("null chain array");
  if (sp && n_chains && !sp_res) return fail("null sub-pel result array");
  if (n_chains == 0) return jmme_search_mbs(ctx, mode, req, n, out);
  if (!ctx->chain_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->chain_stream, hipStreamNonBlocking));
  double t_ph = ctx->phases ? now_us() : 0;
  if (ctx->phases) ++ctx->ph_calls;
  // the chains run on their own stream beside the batch (which syncs the null
  // stream).  On one stream, one after the other, the call took longer
  // (JMME_PHASES, 1080p drop-in: 51 us waiting, against 29 + 12 on two streams)
  if (launch_chains(ctx, mode, chains, n_chains, ctx->chain_stream, sp)) return -1;
  phase(ctx, 0, &t_ph);
  const int rc = n ? jmme_search_mbs(ctx, mode, req, n, out) : 0;
  if (ctx->phases) t_ph = now_us();
  if (rc) {
    (void)hipStreamSynchronize(ctx->chain_stream);
    return rc;
  }
  if (wait_chains(ctx, n_chains, ctx->chain_stream)) return -1;
  std::memcpy(res, ctx->h_chres, (size_t)n_chains * JMME_CHAIN_MAX_STEPS * sizeof(jmme_chain_res));
  if (sp) std::memcpy(sp_res, ctx->h_chsp, (size_t)n_chains * JMME_CHAIN_MAX_STEPS * sizeof(jmme_block_res));
  phase(ctx, 5, &t_ph);
  return 0;
}

extern "C" int jmme_search_mbs_chains(jmme_ctx *ctx, int mode, const jmme_mb_req *req, int n, jmme_block_res *out,
                                      const jmme_chain *chains, int n_chains, jmme_chain_res *res) {
  return jmme_search_mbs_chains_sp(ctx, mode, req, n, out, chains, n_chains, nullptr, res, nullptr);
}

extern "C" int jmme_search_mbs_async(jmme_ctx *ctx, int mode, const jmme_mb_req *d_req, int n,
                                     jmme_block_res *d_out, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (!ctx->d_cur) return fail("current picture not uploaded");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (sync_ref_table(ctx, s)) return -1;
  return launch(ctx, mode, ctx->d_cur, ctx->d_ref_table, ctx->pitch, ctx->width, ctx->height, d_req, n, d_out, s);
}

extern "C" int jmme_search_mbs_planes_async(jmme_ctx *ctx, int mode, const uint8_t *d_cur, const uint8_t *d_ref,
                                            int pitch, int w, int h, const jmme_mb_req *d_req, int n,
                                            jmme_block_res *d_out, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (!d_cur || !d_ref) return fail("null plane");
  if (pitch < w || (pitch & 3) || (w & 15) || (h & 15)) return fail("bad plane geometry %dx%d pitch %d", w, h, pitch);
  // the item kernel reads MB rows with scalar loads, which ignore the low
  // address bits: a plane base off a dword boundary would read shifted pels
  if (((uintptr_t)d_cur | (uintptr_t)d_ref) & 3) return fail("plane base not 4-byte aligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // every (list, ref) of this call reads the one given plane
  std::vector<const uint8_t *> tab(kMaxLists * kMaxRefs, d_ref);
  HIPCHK(hipMemcpyAsync(ctx->d_ref_table, tab.data(), tab.size() * sizeof(void *), hipMemcpyHostToDevice, s));
  ctx->ref_table_dirty = true;
  return launch(ctx, mode, d_cur, ctx->d_ref_table, pitch, w, h, d_req, n, d_out, s, nullptr, true);
}

extern "C" int jmme_search_status(jmme_ctx *ctx, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  // the device-request paths skip validate(): the plan kernel refuses what
  // would overrun the launch (ranges, sub-pel centres) and flags it here
  return check_status(ctx, reinterpret_cast<hipStream_t>(stream));
}

extern "C" float jmme_last_kernel_ms(jmme_ctx *ctx) {
  DevGuard dg_(ctx);
  if (!ctx || !ctx->timed) return -1.0f;
  float ms = -1.0f;
  if (hipEventSynchronize(ctx->ev1) != hipSuccess) return -1.0f;
  if (hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) != hipSuccess) return -1.0f;
  return ms;
}

extern "C" jmme_distblk jmme_full_search_block(jmme_ctx *ctx, int list, int ref_idx, int pos_x, int pos_y,
                                               int blocktype, const jmme_mv *pred_mv, jmme_mv *mv_inout,
                                               jmme_distblk min_mcost, int lambda_factor, int search_range,
                                               int check_for_00) {
  DevGuard dg_(ctx);
  // IntPelME-signature drop-in: one partition as a one-slot unit.  JM's
  // error() semantics on failure (print, exit 500).
  int mb_x = pos_x & ~15, mb_y = pos_y & ~15;
  int s = slot_of(blocktype, (pos_x - mb_x) >> 2, (pos_y - mb_y) >> 2);
  jmme_mb_req r;
  memset(&r, 0, sizeof r);
  r.mb_x = (int16_t)mb_x;
  r.mb_y = (int16_t)mb_y;
  r.list = (int16_t)list;
  r.ref_idx = (int16_t)ref_idx;
  if (s < 0) { fprintf(stderr, "jmme_full_search_block: bad block\n"); exit(500); }
  r.slot_mask = 1ull << s;
  r.blk[s].pred_x = pred_mv->mv_x;
  r.blk[s].pred_y = pred_mv->mv_y;
  r.blk[s].center_x = mv_inout->mv_x;
  r.blk[s].center_y = mv_inout->mv_y;
  r.blk[s].search_range = (int16_t)search_range;
  r.blk[s].flags = (int16_t)(check_for_00 ? JMME_BLK_CHECK00 : 0);
  r.blk[s].lambda = lambda_factor;
  jmme_block_res out[JMME_NSLOT];
  if (jmme_search_mbs(ctx, JMME_FULL_SEARCH, &r, 1, out)) {
    fprintf(stderr, "jmme_full_search_block: %s\n", jmme_last_error());
    exit(500);
  }
  // JM's min_mcost argument is DISTBLK_MAX from BlockMotionSearch (mv_search.c:878);
  // a smaller incoming bound only matters when nothing beats it.
  if (out[s].cost >= min_mcost) return min_mcost;
  mv_inout->mv_x = out[s].mv_x;
  mv_inout->mv_y = out[s].mv_y;
  return out[s].cost;
}

// ------------------------------------------------- transforms / quant / SATD --

extern "C" int jmme_transform_async(jmme_ctx *ctx, int op, const int32_t *d_in, int32_t *d_out, int n, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (n < 0) return fail("negative block count");
  if (!transform_elems(op)) return fail("unknown transform op %d", op);
  if (n == 0) return 0;
  if (!d_in || !d_out) return fail("null block array");
  HIPCHK(launch_transform(op, d_in, d_out, n, reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

extern "C" int jmme_transform(jmme_ctx *ctx, int op, const int32_t *in, int32_t *out, int n) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  const int e = transform_elems(op);
  if (!e) return fail("unknown transform op %d", op);
  if (n <= 0) return n < 0 ? fail("negative block count") : 0;
  if (!in || !out) return fail("null block array");
  const size_t bytes = (size_t)n * e * 4;
  DevBuf a, b;
  HIPCHK(a.alloc(bytes));
  HIPCHK(b.alloc(bytes));
  HIPCHK(hipMemcpy(a.p, in, bytes, hipMemcpyHostToDevice));
  HIPCHK(launch_transform(op, (const int32_t *)a.p, (int32_t *)b.p, n, nullptr));
  HIPCHK(hipMemcpy(out, b.p, bytes, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int jmme_satd_async(jmme_ctx *ctx, int size, const int16_t *d_diff, int32_t *d_out, int n, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (size != 4 && size != 8) return fail("SATD block size %d (4 or 8)", size);
  if (n < 0) return fail("negative block count");
  if (n == 0) return 0;
  if (!d_diff || !d_out) return fail("null array");
  HIPCHK(launch_satd(size, d_diff, d_out, n, reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

extern "C" int jmme_satd(jmme_ctx *ctx, int size, const int16_t *diff, int32_t *out, int n) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (size != 4 && size != 8) return fail("SATD block size %d (4 or 8)", size);
  if (n <= 0) return n < 0 ? fail("negative block count") : 0;
  if (!diff || !out) return fail("null array");
  const size_t in_b = (size_t)n * size * size * 2, out_b = (size_t)n * 4;
  DevBuf a, b;
  HIPCHK(a.alloc(in_b));
  HIPCHK(b.alloc(out_b));
  HIPCHK(hipMemcpy(a.p, diff, in_b, hipMemcpyHostToDevice));
  HIPCHK(launch_satd(size, (const int16_t *)a.p, (int32_t *)b.p, n, nullptr));
  HIPCHK(hipMemcpy(out, b.p, out_b, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int jmme_quant4x4_async(jmme_ctx *ctx, const jmme_quant4x4_params *d_params, const int32_t *d_param_idx,
                                   int32_t *d_coef, int32_t *d_levels, int32_t *d_runs, int32_t *d_coeff_cost,
                                   int32_t *d_nonzero, int n, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (n < 0) return fail("negative block count");
  if (n == 0) return 0;
  if (!d_params || !d_coef || !d_levels || !d_runs || !d_coeff_cost || !d_nonzero) return fail("null array");
  HIPCHK(launch_quant4x4(d_params, d_param_idx, d_coef, d_levels, d_runs, d_coeff_cost, d_nonzero, n,
                         reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

extern "C" int jmme_quant4x4(jmme_ctx *ctx, const jmme_quant4x4_params *params, int n_params, const int32_t *param_idx,
                             int32_t *coef, int32_t *levels, int32_t *runs, int32_t *coeff_cost, int32_t *nonzero,
                             int n) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (n <= 0) return n < 0 ? fail("negative block count") : 0;
  if (!params || n_params <= 0 || !coef || !levels || !runs || !coeff_cost || !nonzero) return fail("null array");
  for (int p = 0; p < n_params; ++p) {
    const jmme_quant4x4_params &q = params[p];
    if (q.qp_per < 0 || q.qp_per > 16) return fail("quant set %d: qp_per %d out of range", p, q.qp_per);
    for (int k = 0; k < 16; ++k)
      if (q.scan[k][0] > 3 || q.scan[k][1] > 3) return fail("quant set %d: scan entry %d outside 4x4", p, k);
  }
  if (param_idx)
    for (int b = 0; b < n; ++b)
      if (param_idx[b] < 0 || param_idx[b] >= n_params) return fail("block %d: parameter set %d of %d", b, param_idx[b], n_params);
  DevBuf dp, di, dc, dl, dr, dk, dn;
  HIPCHK(dp.alloc(sizeof(jmme_quant4x4_params) * n_params));
  HIPCHK(dc.alloc((size_t)n * 64));
  HIPCHK(dl.alloc((size_t)n * 68));
  HIPCHK(dr.alloc((size_t)n * 64));
  HIPCHK(dk.alloc((size_t)n * 4));
  HIPCHK(dn.alloc((size_t)n * 4));
  HIPCHK(hipMemcpy(dp.p, params, sizeof(jmme_quant4x4_params) * n_params, hipMemcpyHostToDevice));
  if (param_idx) {
    HIPCHK(di.alloc((size_t)n * 4));
    HIPCHK(hipMemcpy(di.p, param_idx, (size_t)n * 4, hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemcpy(dc.p, coef, (size_t)n * 64, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dk.p, coeff_cost, (size_t)n * 4, hipMemcpyHostToDevice));
  HIPCHK(launch_quant4x4((const jmme_quant4x4_params *)dp.p, (const int32_t *)di.p, (int32_t *)dc.p, (int32_t *)dl.p,
                         (int32_t *)dr.p, (int32_t *)dk.p, (int32_t *)dn.p, n, nullptr));
  HIPCHK(hipMemcpy(coef, dc.p, (size_t)n * 64, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(levels, dl.p, (size_t)n * 68, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(runs, dr.p, (size_t)n * 64, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(coeff_cost, dk.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(nonzero, dn.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int jmme_residual4x4(jmme_ctx *ctx, const jmme_quant4x4_params *params, int n_params,
                                const jmme_resid4x4_req *req, jmme_resid4x4_res *res, int n) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (n <= 0) return n < 0 ? fail("negative block count") : 0;
  if (!params || n_params <= 0 || !req || !res) return fail("null array");
  for (int p = 0; p < n_params; ++p) {
    const jmme_quant4x4_params &q = params[p];
    if (q.qp_per < 0 || q.qp_per > 16) return fail("quant set %d: qp_per %d out of range", p, q.qp_per);
    for (int k = 0; k < 16; ++k)
      if (q.scan[k][0] > 3 || q.scan[k][1] > 3) return fail("quant set %d: scan entry %d outside 4x4", p, k);
  }
  for (int b = 0; b < n; ++b) {
    if (req[b].param < 0 || req[b].param >= n_params) return fail("block %d: parameter set %d of %d", b, req[b].param, n_params);
    if (req[b].max_pel <= 0 || req[b].max_pel > 0xffff) return fail("block %d: max_pel %d", b, req[b].max_pel);
  }
  const size_t pb = (sizeof(jmme_quant4x4_params) * n_params + 255) & ~(size_t)255;
  const size_t qb = (sizeof(jmme_resid4x4_req) * n + 255) & ~(size_t)255, rb = sizeof(jmme_resid4x4_res) * n;
  if (pb + qb + rb > ctx->cap_rq) {
    if (ctx->h_rq) HIPCHK(hipHostFree(ctx->h_rq));
    ctx->h_rq = nullptr;
    ctx->cap_rq = std::max(pb + qb + rb, (size_t)1 << 16);
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_rq), ctx->cap_rq, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer(&ctx->dv_rq, ctx->h_rq, 0));
  }
  if (!ctx->rq_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->rq_stream, hipStreamNonBlocking));
  std::memcpy(ctx->h_rq, params, sizeof(jmme_quant4x4_params) * n_params);
  std::memcpy(ctx->h_rq + pb, req, sizeof(jmme_resid4x4_req) * n);
  uint8_t *dv = static_cast<uint8_t *>(ctx->dv_rq);
  HIPCHK(launch_residual4x4(reinterpret_cast<const jmme_quant4x4_params *>(dv),
                            reinterpret_cast<const jmme_resid4x4_req *>(dv + pb),
                            reinterpret_cast<jmme_resid4x4_res *>(dv + pb + qb), n, ctx->rq_stream));
  HIPCHK(hipStreamSynchronize(ctx->rq_stream));
  std::memcpy(res, ctx->h_rq + pb + qb, rb);
  return 0;
}

// ------------------------------------------------------------------ fractal --
namespace {

bool fractal_block_ok(int bsx, int bsy) {
  return (bsx == 16 && (bsy == 16 || bsy == 8)) || (bsx == 8 && (bsy == 16 || bsy == 8 || bsy == 4)) ||
         (bsx == 4 && (bsy == 8 || bsy == 4));
}

int fractal_geom_ok(int pitch, int w, int h) {
  if (w < 16 || h < 16 || pitch < w || (pitch & 3)) return fail("fractal plane %dx%d pitch %d: need >= 16x16, pitch %% 4 == 0", w, h, pitch);
  return 0;
}

}  // namespace

extern "C" int jmme_fractal_words_async(jmme_ctx *ctx, const uint8_t *d_ref, int pitch, int width, int height,
                                        uint32_t *d_words, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (fractal_geom_ok(pitch, width, height)) return -1;
  if (!d_ref || !d_words) return fail("null plane");
  HIPCHK(launch_fractal_words(d_ref, pitch, width, height, d_words, width, reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

extern "C" int jmme_fractal_search_async(jmme_ctx *ctx, const uint8_t *d_org, int pitch, const uint32_t *d_words,
                                         int width, int height, int search_range, const jmme_fractal_req *d_req,
                                         int n, jmme_fractal_res *d_out, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (fractal_geom_ok(pitch, width, height)) return -1;
  if (search_range < 0) return fail("negative search range");
  if (n < 0) return fail("negative request count");
  if (n == 0) return 0;
  if (!d_org || !d_words || !d_req || !d_out) return fail("null array");
  FractalParams p{};
  p.org = d_org;
  p.pitch = pitch;
  p.words = d_words;
  p.wpitch = width;
  p.width = width;
  p.height = height;
  // beyond max(W, H) every window is the whole picture: same candidates, same ranks
  p.range = std::min(search_range, std::max(width, height));
  p.req = d_req;
  p.out = d_out;
  p.n = n;
  if (p.range < ctx->pool_min_range) {
    HIPCHK(launch_fractal_search(p, reinterpret_cast<hipStream_t>(stream)));
    return 0;
  }
  // pruned pool search: scratch = 7 pool images + flags + counter
  const size_t img = ((size_t)width * height * sizeof(float) * 2 + 255) & ~(size_t)255;
  const size_t bytes = 8 * img + 256;
  if (bytes > ctx->cap_pool) {
    (void)hipFree(ctx->d_pool);
    ctx->d_pool = nullptr;
    ctx->cap_pool = 0;
    HIPCHK(hipMalloc(&ctx->d_pool, bytes));
    HIPCHK(hipMemset(ctx->d_pool, 0, bytes));
    ctx->cap_pool = bytes;
  }
  char *base = static_cast<char *>(ctx->d_pool);
  FractalPoolParams pp{};
  pp.base = p;
  // [0, 256): flags, counter (fixed offsets: the buffer outlives a smaller frame); then the images
  pp.flags = reinterpret_cast<int *>(base);
  pp.stats = reinterpret_cast<unsigned long long *>(base + 64);
  for (int s = 0; s < 7; ++s) pp.pool[s] = base + 256 + (size_t)s * img;
  pp.bw = base + 256 + (size_t)7 * img;
  pp.use_mfma = ctx->pool_mfma;
  pp.seed_range = 4;
  HIPCHK(launch_fractal_pool(pp, reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

extern "C" int jmme_fractal_set_pool_min_range(jmme_ctx *ctx, int min_range) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (min_range < 0) return fail("negative pool radius");
  ctx->pool_min_range = min_range;
  return 0;
}

extern "C" int jmme_fractal_set_pool_mfma(jmme_ctx *ctx, int on) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  ctx->pool_mfma = on != 0;
  return 0;
}

extern "C" int jmme_fractal_pool_survivors(jmme_ctx *ctx, unsigned long long *survivors) {
  DevGuard dg_(ctx);
  if (!ctx || !survivors) return fail("null argument");
  *survivors = 0;
  if (!ctx->d_pool) return 0;
  unsigned long long *d = reinterpret_cast<unsigned long long *>(static_cast<char *>(ctx->d_pool) + 64);
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(survivors, d, sizeof *survivors, hipMemcpyDeviceToHost));
  HIPCHK(hipMemset(d, 0, sizeof *survivors));
  return 0;
}

extern "C" int jmme_fractal_search(jmme_ctx *ctx, const uint8_t *org, const uint8_t *ref, int pitch, int width,
                                   int height, int search_range, const jmme_fractal_req *req, int n,
                                   jmme_fractal_res *out) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (fractal_geom_ok(pitch, width, height)) return -1;
  if (search_range < 0) return fail("negative search range");
  if (n <= 0) return n < 0 ? fail("negative request count") : 0;
  if (!org || !ref || !req || !out) return fail("null array");
  for (int i = 0; i < n; ++i) {
    const jmme_fractal_req &q = req[i];
    if (!fractal_block_ok(q.bsx, q.bsy)) return fail("request %d: block %dx%d not a thesis block size", i, q.bsx, q.bsy);
    if (q.block_x < 0 || q.block_y < 0 || q.block_x % q.bsx || q.block_y % q.bsy || q.block_x + q.bsx > width ||
        q.block_y + q.bsy > height)
      return fail("request %d: range block (%d,%d) %dx%d not aligned inside %dx%d", i, q.block_x, q.block_y, q.bsx,
                  q.bsy, width, height);
  }
  const size_t plane = (size_t)pitch * height;
  DevBuf o, r, w, dq, dout;
  HIPCHK(o.alloc(plane));
  HIPCHK(r.alloc(plane));
  HIPCHK(w.alloc((size_t)width * height * 4));
  HIPCHK(dq.alloc((size_t)n * sizeof(jmme_fractal_req)));
  HIPCHK(dout.alloc((size_t)n * sizeof(jmme_fractal_res)));
  HIPCHK(hipMemcpy(o.p, org, plane, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(r.p, ref, plane, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dq.p, req, (size_t)n * sizeof(jmme_fractal_req), hipMemcpyHostToDevice));
  if (jmme_fractal_words_async(ctx, (const uint8_t *)r.p, pitch, width, height, (uint32_t *)w.p, nullptr)) return -1;
  if (jmme_fractal_search_async(ctx, (const uint8_t *)o.p, pitch, (const uint32_t *)w.p, width, height,
                                search_range, (const jmme_fractal_req *)dq.p, n, (jmme_fractal_res *)dout.p,
                                nullptr))
    return -1;
  HIPCHK(hipMemcpy(out, dout.p, (size_t)n * sizeof(jmme_fractal_res), hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int jmme_fractal_box_sums(jmme_ctx *ctx, const uint8_t *plane, int pitch, int width, int height, int bsx,
                                     int bsy, double *sum, double *sum2) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (fractal_geom_ok(pitch, width, height)) return -1;
  if (bsx < 1 || bsy < 1 || bsx > 16 || bsy > 16 || bsx > width || bsy > height) return fail("box %dx%d", bsx, bsy);
  if (!plane || !sum || !sum2) return fail("null array");
  const int w = width - bsx + 1, h = height - bsy + 1;
  DevBuf dp, hs, hs2, ds, ds2;
  HIPCHK(dp.alloc((size_t)pitch * height));
  HIPCHK(hs.alloc((size_t)w * height * 4));
  HIPCHK(hs2.alloc((size_t)w * height * 4));
  HIPCHK(ds.alloc((size_t)w * h * 8));
  HIPCHK(ds2.alloc((size_t)w * h * 8));
  HIPCHK(hipMemcpy(dp.p, plane, (size_t)pitch * height, hipMemcpyHostToDevice));
  HIPCHK(launch_box_sums((const uint8_t *)dp.p, pitch, width, height, bsx, bsy, (uint32_t *)hs.p, (uint32_t *)hs2.p,
                         (double *)ds.p, (double *)ds2.p, nullptr));
  HIPCHK(hipMemcpy(sum, ds.p, (size_t)w * h * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(sum2, ds2.p, (size_t)w * h * 8, hipMemcpyDeviceToHost));
  return 0;
}

// -------------------------------------------------------------------- EPZS --
static_assert(sizeof(jmme_epzs_req) == 80 && sizeof(jmme_epzs_res) == 32, "EPZS ABI layout");
static_assert(sizeof(jmme_chain) == 176 && sizeof(jmme_chain_step) == 36 && sizeof(jmme_chain_res) == 24,
              "chain ABI layout");

namespace {
int prepare_subs(jmme_ctx *ctx, hipStream_t s);   // sub-pel section below
}  // namespace

namespace {
int build_epzs_params(jmme_ctx *ctx, EpzsParams &p, const jmme_epzs_req *d_req, int n, const int16_t *d_preds,
                      const uint8_t *d_cond, const int16_t *d_stale, jmme_epzs_res *d_out, int16_t *d_vis,
                      int max_visited, hipStream_t s, jmme_epzs_bounds *d_bounds = nullptr,
                      jmme_block_res *d_int = nullptr, const EpzsOne *one = nullptr,
                      jmme_block_res *d_fused_out = nullptr, uint32_t *d_done = nullptr, uint32_t done_seq = 0) {
  if (sync_ref_table(ctx, s)) return -1;
  std::memset(&p, 0, sizeof p);
  p.cur = ctx->d_cur;
  p.hbd = ctx->hbd ? 1 : 0;   // 16-bit planes / sub-images: the v_sad_u16 instantiation
  p.refs = ctx->d_ref_table;
  p.pitch = ctx->pitch;
  p.width = ctx->width;
  p.height = ctx->height;
  p.req = d_req;
  p.preds = d_preds;
  p.stale = d_stale;
  p.out = d_out;
  p.n = n;
  p.grid = ctx->cfg.EPZSSubPelGrid ? 1 : 0;
  if (p.grid) {   // EPZS_integer_(subMB_)motion_estimation: candidates on the quarter-pel sub-images
    if (ctx->cfg.SearchRange > 64) return fail("EPZSSubPelGrid: SearchRange %d > 64", ctx->cfg.SearchRange);
    if (prepare_subs(ctx, s)) return -1;
    const SubGeom g = sub_geom(ctx->width, ctx->height);
    p.subs = ctx->d_sub_table;
    p.sub_pitch = g.pitch;
    p.plane_stride = g.plane_stride;
    p.max_qpel = 4 * ctx->cfg.SearchRange;
  } else {
    p.max_qpel = kEpzsMaxQpel;
  }
  p.map_words = (int)epzs_map_words(p.grid, p.max_qpel);
  p.pred_cond = d_cond;
  p.visited = d_vis;
  p.max_visited = max_visited;
  p.bounds = d_bounds;
  p.int_out = d_int;
  if (one) {   // a search alone, in the kernel arguments; its wave refines its own answer
    if (prepare_subs(ctx, s)) return -1;
    const SubGeom g = sub_geom(ctx->width, ctx->height);
    p.fused = 1;
    p.fused_sp.cur = ctx->d_cur;
    p.fused_sp.cur_pitch = ctx->pitch;
    p.fused_sp.width = ctx->width;
    p.fused_sp.height = ctx->height;
    p.fused_sp.hbd = ctx->hbd ? 1 : 0;
    p.fused_sp.subs = ctx->d_sub_table;
    p.fused_sp.sub_pitch = g.pitch;
    p.fused_sp.plane_stride = g.plane_stride;
    p.fused_sp.req = nullptr;
    p.fused_sp.int_res = nullptr;
    p.fused_sp.out = d_fused_out;
    p.fused_sp.n = 1;
    p.fused_sp.per_wave = 1;
    p.one = *one;
    p.done = d_done;
    p.done_seq = done_seq;
  }
  return 0;
}

// the request built in box->p, posted as box->req's chunks: three dwords of it
// and the request number in each 16-byte store (one x86 store each), so a chunk
// the server reads is never half old, half new
static void post_request(EpzsBox *box, uint32_t seq) {
  typedef uint32_t v4u __attribute__((vector_size(16)));
  const uint32_t *src = reinterpret_cast<const uint32_t *>(&box->p);
  constexpr int kDw = (int)(sizeof(EpzsParams) / 4);
  for (int i = 0; i < kEpzsReqChunks; ++i) {
    v4u c;
    for (int k = 0; k < 3; ++k) c[k] = 3 * i + k < kDw ? src[3 * i + k] : 0u;
    c[3] = seq;
    *reinterpret_cast<volatile v4u *>(&box->req[i]) = c;
  }
  __atomic_store_n(&box->seq, seq, __ATOMIC_RELEASE);
}

// JMME_SINGLE_MODE 3: a fused search alone handed to the resident server.
// (Re)launches it when it is not running -- first use, stopped by another
// entry point, or gone after its idle time -- and waits for the request's
// number in the completion word.
int epzs_serve(jmme_ctx *ctx, const jmme_epzs_req *d_req, const int16_t *d_preds, const uint8_t *d_cond,
               const int16_t *d_stale, jmme_epzs_res *d_out, int16_t *d_vis, int max_visited,
               jmme_epzs_bounds *d_bnd, jmme_block_res *d_int, const EpzsOne &one, jmme_block_res *d_spo) {
  const double t_in = ctx->phases ? now_us() : 0.0;
  if (!ctx->h_box) {
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_box), sizeof(EpzsBox), hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(static_cast<void *>(ctx->h_box), 0, sizeof(EpzsBox));
    void *dv = nullptr;
    HIPCHK(hipHostGetDevicePointer(&dv, ctx->h_box, 0));
    ctx->d_box = static_cast<EpzsBox *>(dv);
  }
  if (!ctx->srv_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->srv_stream, hipStreamNonBlocking));
  // a reference table or sub-images still to build are writes the server would not see: stop it first
  bool prep = ctx->ref_table_dirty || ctx->sub_table_dirty;
  for (int k = 0; k < kMaxLists * kMaxRefs && !prep; ++k) prep = ctx->d_refs[k] && (ctx->sub_stale[k] || !ctx->d_subs[k]);
  if (prep && server_stop(ctx)) return -1;
  EpzsBox *box = ctx->h_box;
  // the server is idle between requests (the last one's number is in `done`), so
  // the request is built in place
  if (build_epzs_params(ctx, box->p, d_req, 1, d_preds, d_cond, d_stale, d_out, d_vis, max_visited, ctx->srv_stream,
                        d_bnd, d_int, &one, d_spo, nullptr, 0))
    return -1;
  const EpzsParams &p = box->p;
  if (ctx->srv_running && (ctx->srv_grid != p.grid || ctx->srv_hbd != p.hbd || ctx->srv_map_words < p.map_words) &&
      server_stop(ctx))
    return -1;
  const uint32_t seq = ++ctx->srv_seq;
  auto start = [&]() -> int {
    __atomic_store_n(&box->alive, 1u, __ATOMIC_RELEASE);
    HIPCHK(launch_epzs_server(ctx->d_box, p.grid != 0, p.hbd != 0, p.map_words, seq - 1, ctx->srv_idle_ticks,
                              1000000000ull /* 10 s */, ctx->srv_stream));
    ctx->srv_running = true;
    ctx->srv_grid = p.grid;
    ctx->srv_hbd = p.hbd;
    ctx->srv_map_words = p.map_words;
    ++ctx->srv_launches;
    return 0;
  };
  if (!ctx->srv_running && start()) return -1;
  post_request(box, seq);
  const double t_post = ctx->phases ? now_us() : 0.0;
  auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 1; __atomic_load_n(&box->done, __ATOMIC_ACQUIRE) != seq; ++spin) {
    if ((spin & 63u) == 0 && __atomic_load_n(&box->alive, __ATOMIC_ACQUIRE) == 0) {
      // it left (idle or life time) without this request, or served it just before
      if (__atomic_load_n(&box->done, __ATOMIC_ACQUIRE) == seq) break;
      ctx->srv_running = false;
      HIPCHK(hipStreamSynchronize(ctx->srv_stream));
      if (start()) return -1;
    }
    if ((spin & 4095u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      // 2 s without it: on a GPU whose mapped queues are oversubscribed (more
      // processes' queues than the hardware maps) the server's queue can stay
      // unmapped that long.  Stop it (surfacing a fault) and, when it left
      // without the request, hand the request back for an ordinary launch.
      const int r = server_stop(ctx);
      if (r) return -1;
      if (__atomic_load_n(&box->done, __ATOMIC_ACQUIRE) == seq) break;
      ++ctx->srv_fallbacks;
      return 1;
    }
    __builtin_ia32_pause();
  }
  ++ctx->srv_served;
  if (ctx->phases) {
    ctx->srv_t_done = now_us();
    ctx->srv_host_us[0] += t_in - ctx->srv_t_call;
    ctx->srv_host_us[1] += t_post - t_in;
    ctx->srv_host_us[2] += ctx->srv_t_done - t_post;
    ctx->srv_service_us += 0.01 * box->service;
    ctx->srv_cycles += box->cycles;
    for (int i = 0; i < 6; ++i) ctx->srv_rph_us[i] += 0.01 * box->rph[i];
    ctx->srv_copy_us += 0.01 * box->copy;
    ctx->srv_search_us += 0.01 * box->search;
    for (int i = 0; i < 10; ++i) ctx->srv_ph_us[i] += 0.01 * box->ph[i];
  }
  return 0;
}

// JMME_EPZS_SERVER_CHECK (diagnostic): the request the server just served, run
// again by the fused launch into a block of its own; any difference is printed
int epzs_serve_check(jmme_ctx *ctx, const jmme_epzs_res *h_out, const jmme_epzs_bounds *h_bnd, const int16_t *h_vis,
                     const jmme_block_res *h_spo, jmme_block_res spo0, int max_visited) {
  const size_t b_out = 64, b_bnd = 64, b_int = 64, b_spo = 64, b_vis = align64((size_t)max_visited * 4);
  if (!ctx->h_chk) HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_chk), 256 + 4 * 65536, hipHostMallocMapped));
  if (b_vis > 4 * 65536) return fail("server check: max_visited %d", max_visited);
  void *dv = nullptr;
  HIPCHK(hipHostGetDevicePointer(&dv, ctx->h_chk, 0));
  uint8_t *h = ctx->h_chk, *d = static_cast<uint8_t *>(dv);
  std::memset(h, 0, 256 + b_vis);
  std::memcpy(h + b_out + b_bnd + b_int, &spo0, sizeof spo0);
  EpzsParams pc = ctx->h_box->p;
  pc.out = reinterpret_cast<jmme_epzs_res *>(d);
  pc.bounds = reinterpret_cast<jmme_epzs_bounds *>(d + b_out);
  pc.int_out = pc.int_out ? reinterpret_cast<jmme_block_res *>(d + b_out + b_bnd) : nullptr;
  pc.fused_sp.out = reinterpret_cast<jmme_block_res *>(d + b_out + b_bnd + b_int);
  pc.visited = reinterpret_cast<int16_t *>(d + b_out + b_bnd + b_int + b_spo);
  pc.done = nullptr;
  if (!ctx->single_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->single_stream, hipStreamNonBlocking));
  HIPCHK(launch_epzs(pc, ctx->single_stream));
  HIPCHK(hipStreamSynchronize(ctx->single_stream));
  const jmme_epzs_res *o = reinterpret_cast<const jmme_epzs_res *>(h);
  const jmme_epzs_bounds *b = reinterpret_cast<const jmme_epzs_bounds *>(h + b_out);
  const jmme_block_res *sp = reinterpret_cast<const jmme_block_res *>(h + b_out + b_bnd + b_int);
  const int16_t *v = reinterpret_cast<const int16_t *>(h + b_out + b_bnd + b_int + b_spo);
  const int nv = std::min(o->n_visited, max_visited);
  const bool same = !std::memcmp(o, h_out, sizeof *o) && !std::memcmp(b, h_bnd, sizeof *b) &&
                    !std::memcmp(sp, h_spo, sizeof *sp) && !std::memcmp(v, h_vis, (size_t)nv * 4);
  if (!same && ctx->srv_mismatch++ < 20) {
    const jmme_epzs_req &q = pc.one.q;
    fprintf(stderr, "jmme EPZS server check: request %u (%d,%d) %dx%d bt %d var %d n_pred %d n_stale %d | server mv (%d,%d) "
            "cost %lld path %d nv %d sp (%d,%d) %lld | fused mv (%d,%d) cost %lld path %d nv %d sp (%d,%d) %lld | bounds %s "
            "visited %s\n", ctx->srv_seq, q.pos_x, q.pos_y, q.bsx, q.bsy, q.blocktype, q.variant, q.n_pred, q.n_stale,
            h_out->mv_x, h_out->mv_y, (long long)h_out->cost, h_out->path, h_out->n_visited, h_spo->mv_x, h_spo->mv_y,
            (long long)h_spo->cost, o->mv_x, o->mv_y, (long long)o->cost, o->path, o->n_visited, sp->mv_x, sp->mv_y,
            (long long)sp->cost, std::memcmp(b, h_bnd, sizeof *b) ? "differ" : "same",
            std::memcmp(v, h_vis, (size_t)nv * 4) ? "differ" : "same");
  }
  return 0;
}

int launch_epzs_ex(jmme_ctx *ctx, const jmme_epzs_req *d_req, int n, const int16_t *d_preds, const uint8_t *d_cond,
                   const int16_t *d_stale, jmme_epzs_res *d_out, int16_t *d_vis, int max_visited, hipStream_t s,
                   jmme_epzs_bounds *d_bounds = nullptr, jmme_block_res *d_int = nullptr,
                   const EpzsOne *one = nullptr, jmme_block_res *d_fused_out = nullptr,
                   uint32_t *d_done = nullptr, uint32_t done_seq = 0) {
  EpzsParams p;
  if (build_epzs_params(ctx, p, d_req, n, d_preds, d_cond, d_stale, d_out, d_vis, max_visited, s, d_bounds, d_int, one,
                        d_fused_out, d_done, done_seq))
    return -1;
  HIPCHK(launch_epzs(p, s));
  return 0;
}
}  // namespace

extern "C" int jmme_epzs_search_async(jmme_ctx *ctx, const jmme_epzs_req *d_req, int n, const int16_t *d_preds,
                                      const int16_t *d_stale, jmme_epzs_res *d_out, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (n < 0) return fail("negative request count");
  if (n == 0) return 0;
  if (!ctx->d_cur) return fail("no current frame uploaded");
  if (!d_req || !d_out || !d_preds || !d_stale) return fail("null array");
  return launch_epzs_ex(ctx, d_req, n, d_preds, nullptr, d_stale, d_out, nullptr, 0,
                        reinterpret_cast<hipStream_t>(stream));
}

namespace {
// the checks of the host-array EPZS entry points
int epzs_validate(const jmme_ctx *ctx, const jmme_epzs_req *req, int n, int n_preds, int n_stale) {
  for (int i = 0; i < n; ++i) {
    const jmme_epzs_req &q = req[i];
    const bool size_ok = (q.bsx == 16 || q.bsx == 8 || q.bsx == 4) && (q.bsy == 16 || q.bsy == 8 || q.bsy == 4) &&
                         !(q.bsx == 16 && q.bsy == 4) && !(q.bsx == 4 && q.bsy == 16);
    if (!size_ok) return fail("request %d: block %dx%d", i, q.bsx, q.bsy);
    if (q.pos_x < 0 || q.pos_y < 0 || (q.pos_x & 3) || (q.pos_y & 3) || q.pos_x + q.bsx > ctx->width ||
        q.pos_y + q.bsy > ctx->height)
      return fail("request %d: block (%d,%d) %dx%d outside the %dx%d picture", i, q.pos_x, q.pos_y, q.bsx, q.bsy,
                  ctx->width, ctx->height);
    const bool grid = ctx->cfg.EPZSSubPelGrid != 0;
    if (grid ? q.variant < 2 : q.variant > 1)
      return fail("request %d: variant %d does not match EPZSSubPelGrid %d (0/1: integer grid, 2/3: quarter-pel grid)",
                  i, q.variant, ctx->cfg.EPZSSubPelGrid);
    if (!grid && ((q.center_x & 3) || (q.center_y & 3)))
      return fail("request %d: centre (%d,%d) is not integer-pel", i, q.center_x, q.center_y);
    if (grid && (q.max_x > 4 * ctx->cfg.SearchRange || q.max_y > 4 * ctx->cfg.SearchRange))
      return fail("request %d: search range (%d,%d) qpel beyond 4 x SearchRange", i, q.max_x, q.max_y);
    if (q.max_x < 0 || q.max_y < 0 || q.max_x > kEpzsMaxQpel || q.max_y > kEpzsMaxQpel)
      return fail("request %d: search range (%d,%d) qpel outside 0..%d", i, q.max_x, q.max_y, kEpzsMaxQpel);
    if (q.variant > 3 || q.pattern > 5 || q.dual > 6) return fail("request %d: variant/pattern/dual", i);
    if (!grid && (q.pattern == 4 || q.dual == 5))
      return fail("request %d: the SBP large diamond refines on half-pel points (needs EPZSSubPelGrid 1)", i);
    if (q.blocktype < 1 || q.blocktype > 7) return fail("request %d: blocktype %d", i, q.blocktype);
    if (q.n_pred < 0 || q.pred_off < 0 || (int64_t)q.pred_off + q.n_pred > n_preds)
      return fail("request %d: predictors [%d, +%d) outside the pool of %d", i, q.pred_off, q.n_pred, n_preds);
    if (q.n_stale < 0 || q.stale_off < 0 || (int64_t)q.stale_off + q.n_stale > n_stale)
      return fail("request %d: map cells [%d, +%d) outside the pool of %d", i, q.stale_off, q.n_stale, n_stale);
    if (q.ref_slot < 0 || q.ref_slot >= kMaxLists * kMaxRefs || !ctx->d_refs[q.ref_slot])
      return fail("request %d: reference slot %d not uploaded", i, q.ref_slot);
  }
  return 0;
}
}  // namespace

extern "C" int jmme_epzs_search(jmme_ctx *ctx, const jmme_epzs_req *req, int n, const int16_t *preds, int n_preds,
                                const int16_t *stale, int n_stale, jmme_epzs_res *out) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (n <= 0) return n < 0 ? fail("negative request count") : 0;
  if (!req || !out || (n_preds && !preds) || (n_stale && !stale)) return fail("null array");
  if (!ctx->d_cur) return fail("no current frame uploaded");
  if (epzs_validate(ctx, req, n, n_preds, n_stale)) return -1;
  DevBuf dq, dp, ds, dout;
  HIPCHK(dq.alloc((size_t)n * sizeof(jmme_epzs_req)));
  HIPCHK(dp.alloc((size_t)(n_preds ? n_preds : 1) * 4));
  HIPCHK(ds.alloc((size_t)(n_stale ? n_stale : 1) * 4));
  HIPCHK(dout.alloc((size_t)n * sizeof(jmme_epzs_res)));
  HIPCHK(hipMemcpy(dq.p, req, (size_t)n * sizeof(jmme_epzs_req), hipMemcpyHostToDevice));
  if (n_preds) HIPCHK(hipMemcpy(dp.p, preds, (size_t)n_preds * 4, hipMemcpyHostToDevice));
  if (n_stale) HIPCHK(hipMemcpy(ds.p, stale, (size_t)n_stale * 4, hipMemcpyHostToDevice));
  if (jmme_epzs_search_async(ctx, (const jmme_epzs_req *)dq.p, n, (const int16_t *)dp.p, (const int16_t *)ds.p,
                             (jmme_epzs_res *)dout.p, nullptr))
    return -1;
  HIPCHK(hipMemcpy(out, dout.p, (size_t)n * sizeof(jmme_epzs_res), hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int jmme_epzs_search_ex(jmme_ctx *ctx, const jmme_epzs_req *req, int n, const int16_t *preds,
                                   const uint8_t *pred_cond, int n_preds, const int16_t *stale, int n_stale,
                                   jmme_epzs_res *out, int16_t *visited, int max_visited) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (n <= 0) return n < 0 ? fail("negative request count") : 0;
  if (!req || !out || (n_preds && !preds) || (n_stale && !stale)) return fail("null array");
  if (!ctx->d_cur) return fail("no current frame uploaded");
  if (visited && max_visited <= 0) return fail("max_visited must be positive");
  if (epzs_validate(ctx, req, n, n_preds, n_stale)) return -1;
  if (pred_cond)
    for (int i = 0; i < n_preds; ++i)
      if (pred_cond[i] > JMME_EPZS_PRED_GT_3STOP) return fail("predictor %d: condition %d", i, pred_cond[i]);
  // one mapped pinned block: [req | preds | stale | cond | out | visited]
  const size_t b_req = align64((size_t)n * sizeof(jmme_epzs_req)), b_pred = align64((size_t)n_preds * 4 + 4);
  const size_t b_stale = align64((size_t)n_stale * 4 + 4), b_cond = align64((size_t)n_preds + 1);
  const size_t b_out = align64((size_t)n * sizeof(jmme_epzs_res));
  const size_t b_vis = visited ? align64((size_t)n * max_visited * 4) : 0;
  const size_t need = b_req + b_pred + b_stale + b_cond + b_out + b_vis;
  if (need > ctx->cap_emap) {
    if (ctx->h_emap) (void)hipHostFree(ctx->h_emap);
    ctx->h_emap = nullptr;
    ctx->cap_emap = 0;
    const size_t cap = std::max<size_t>(1u << 20, need + need / 2);
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_emap), cap, hipHostMallocMapped));
    ctx->cap_emap = cap;
  }
  uint8_t *h = ctx->h_emap;
  void *dh = nullptr;
  HIPCHK(hipHostGetDevicePointer(&dh, h, 0));
  uint8_t *d = static_cast<uint8_t *>(dh);
  size_t o = 0;
  std::memcpy(h + o, req, (size_t)n * sizeof(jmme_epzs_req));
  const jmme_epzs_req *d_req = reinterpret_cast<const jmme_epzs_req *>(d + o);
  o += b_req;
  if (n_preds) std::memcpy(h + o, preds, (size_t)n_preds * 4);
  const int16_t *d_preds = reinterpret_cast<const int16_t *>(d + o);
  o += b_pred;
  if (n_stale) std::memcpy(h + o, stale, (size_t)n_stale * 4);
  const int16_t *d_stale = reinterpret_cast<const int16_t *>(d + o);
  o += b_stale;
  if (pred_cond && n_preds) std::memcpy(h + o, pred_cond, (size_t)n_preds);
  const uint8_t *d_cond = pred_cond ? d + o : nullptr;
  o += b_cond;
  jmme_epzs_res *h_out = reinterpret_cast<jmme_epzs_res *>(h + o), *d_out = reinterpret_cast<jmme_epzs_res *>(d + o);
  o += b_out;
  int16_t *h_vis = visited ? reinterpret_cast<int16_t *>(h + o) : nullptr;
  int16_t *d_vis = visited ? reinterpret_cast<int16_t *>(d + o) : nullptr;
  hipStream_t s = nullptr;
  if (launch_epzs_ex(ctx, d_req, n, d_preds, d_cond, d_stale, d_out, d_vis, max_visited, s)) return -1;
  HIPCHK(hipStreamSynchronize(s));
  std::memcpy(out, h_out, (size_t)n * sizeof(jmme_epzs_res));
  for (int i = 0; i < n; ++i)
    if (visited && out[i].n_visited > max_visited)
      return fail("request %d: the search stamped %d map cells, more than max_visited %d", i, out[i].n_visited,
                  max_visited);
  if (visited)   // only the pairs each search wrote
    for (int i = 0; i < n; ++i)
      std::memcpy(visited + 2 * (size_t)max_visited * i, h_vis + 2 * (size_t)max_visited * i,
                  (size_t)out[i].n_visited * 4);
  return 0;
}

static_assert(sizeof(jmme_epzs_bounds) == 40, "EPZS bounds ABI layout");

extern "C" int jmme_epzs_speculate(jmme_ctx *ctx, const jmme_epzs_req *req, int n, const int16_t *preds,
                                   const uint8_t *pred_cond, int n_preds, const int16_t *stale, int n_stale,
                                   jmme_epzs_res *out, jmme_epzs_bounds *bounds, int16_t *visited, int max_visited,
                                   const jmme_subpel_req *sp_req, jmme_block_res *sp_out) {
  DevGuard dg_(ctx, true);   // a search alone may go to the running server (below)
  if (!ctx) return fail("null ctx");
  struct EpTimer {   // JMME_PHASES: the call's time, by kind
    jmme_ctx *c; int k; double t0;
    ~EpTimer() { if (c->phases) { c->ep_us[k] += now_us() - t0; ++c->ep_n[k]; } }
  } ep_timer_{ctx, n > 1, ctx->phases ? now_us() : 0.0};
  if (n <= 0) return n < 0 ? fail("negative request count") : 0;
  if (!req || !out || !bounds || !visited || (n_preds && !preds) || (n_stale && !stale)) return fail("null array");
  if (sp_req && !sp_out) return fail("sub-pel requests without an output array");
  if (!ctx->d_cur) return fail("no current frame uploaded");
  if (max_visited <= 0) return fail("max_visited must be positive");
  if (epzs_validate(ctx, req, n, n_preds, n_stale)) return -1;
  if (pred_cond)
    for (int i = 0; i < n_preds; ++i)
      if (pred_cond[i] > JMME_EPZS_PRED_GT_3STOP) return fail("predictor %d: condition %d", i, pred_cond[i]);
  if (sp_req && jmme_subpel_validate(ctx, sp_req, n)) return -1;
  // one mapped pinned block: [req | preds | stale | cond | out | bounds | visited | sp_req | int | sp_out]
  const size_t b_req = align64((size_t)n * sizeof(jmme_epzs_req)), b_pred = align64((size_t)n_preds * 4 + 4);
  const size_t b_stale = align64((size_t)n_stale * 4 + 4), b_cond = align64((size_t)n_preds + 1);
  const size_t b_out = align64((size_t)n * sizeof(jmme_epzs_res)), b_bnd = align64((size_t)n * sizeof(jmme_epzs_bounds));
  const size_t b_vis = align64((size_t)n * max_visited * 4);
  const size_t b_sp = sp_req ? align64((size_t)n * sizeof(jmme_subpel_req)) : 0;
  const size_t b_res = sp_req ? align64((size_t)n * sizeof(jmme_block_res)) : 0;
  const size_t need = b_req + b_pred + b_stale + b_cond + b_out + b_bnd + b_vis + b_sp + 2 * b_res;
  if (need > ctx->cap_emap) {
    if (server_stop(ctx)) return -1;   // (its next request lands in the new block)
    if (ctx->h_emap) (void)hipHostFree(ctx->h_emap);
    ctx->h_emap = nullptr;
    ctx->cap_emap = 0;
    const size_t cap = std::max<size_t>(1u << 20, need + need / 2);
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_emap), cap, hipHostMallocMapped));
    ctx->cap_emap = cap;
  }
  uint8_t *h = ctx->h_emap;
  void *dh = nullptr;
  HIPCHK(hipHostGetDevicePointer(&dh, h, 0));
  uint8_t *d = static_cast<uint8_t *>(dh);
  size_t o = 0;
  std::memcpy(h + o, req, (size_t)n * sizeof(jmme_epzs_req));
  const jmme_epzs_req *d_req = reinterpret_cast<const jmme_epzs_req *>(d + o);
  o += b_req;
  if (n_preds) std::memcpy(h + o, preds, (size_t)n_preds * 4);
  const int16_t *d_preds = reinterpret_cast<const int16_t *>(d + o);
  o += b_pred;
  if (n_stale) std::memcpy(h + o, stale, (size_t)n_stale * 4);
  const int16_t *d_stale = reinterpret_cast<const int16_t *>(d + o);
  o += b_stale;
  if (pred_cond && n_preds) std::memcpy(h + o, pred_cond, (size_t)n_preds);
  const uint8_t *d_cond = pred_cond ? d + o : nullptr;
  o += b_cond;
  jmme_epzs_res *h_out = reinterpret_cast<jmme_epzs_res *>(h + o), *d_out = reinterpret_cast<jmme_epzs_res *>(d + o);
  o += b_out;
  jmme_epzs_bounds *h_bnd = reinterpret_cast<jmme_epzs_bounds *>(h + o);
  jmme_epzs_bounds *d_bnd = reinterpret_cast<jmme_epzs_bounds *>(d + o);
  o += b_bnd;
  int16_t *h_vis = reinterpret_cast<int16_t *>(h + o), *d_vis = reinterpret_cast<int16_t *>(d + o);
  o += b_vis;
  const jmme_subpel_req *d_spq = nullptr;
  jmme_block_res *d_int = nullptr, *d_spo = nullptr, *h_spo = nullptr;
  if (sp_req) {
    std::memcpy(h + o, sp_req, (size_t)n * sizeof(jmme_subpel_req));
    d_spq = reinterpret_cast<const jmme_subpel_req *>(d + o);
    o += b_sp;
    d_int = reinterpret_cast<jmme_block_res *>(d + o);
    o += b_res;
    std::memcpy(h + o, sp_out, (size_t)n * sizeof(jmme_block_res));   // blocktype-0 entries keep theirs
    d_spo = reinterpret_cast<jmme_block_res *>(d + o);
    h_spo = reinterpret_cast<jmme_block_res *>(h + o);
  }
  // a search alone (the drop-in's misses) travels in the kernel arguments and its
  // wave refines its own answer in the same launch; batches: the
  // 16-refinements-per-wave kernel after it
  const bool fuse = sp_req && n == 1 && req[0].n_pred <= kEpzsStageP && req[0].n_stale <= kEpzsStageS;
  EpzsOne one{};
  if (fuse) {
    one.q = req[0];
    one.q.pred_off = 0;
    one.q.stale_off = 0;
    one.spq = sp_req[0];
    if (req[0].n_pred) std::memcpy(one.preds, preds + 2 * (size_t)req[0].pred_off, (size_t)req[0].n_pred * 4);
    if (pred_cond && req[0].n_pred) std::memcpy(one.cond, pred_cond + req[0].pred_off, (size_t)req[0].n_pred);
    if (req[0].n_stale) std::memcpy(one.stale, stale + 2 * (size_t)req[0].stale_off, (size_t)req[0].n_stale * 4);
  }
  if (ctx->single_mode < 0) {
    const char *e = std::getenv("JMME_SINGLE_MODE");
    ctx->single_mode = e ? std::max(0, std::min(3, std::atoi(e))) : 3;
    ctx->srv_check = std::getenv("JMME_EPZS_SERVER_CHECK") != nullptr;
    const char *ie = std::getenv("JMME_EPZS_SERVER_IDLE_US");
    if (ie) ctx->srv_idle_ticks = (uint32_t)std::max(1, std::min(1000000, std::atoi(ie))) * 100u;
  }
  int mode = fuse ? ctx->single_mode : 0;
  const double t_staged = ctx->phases && n > 1 ? now_us() : 0.0;   // (batches: the copies in are done)
  if (mode != 3 && server_stop(ctx)) return -1;
  int served = 1;
  const jmme_block_res spo0 = h_spo ? *h_spo : jmme_block_res{};   // (the server check's input)
  if (mode == 3) {   // the resident server: no launch on the search's path
    ctx->srv_t_call = ep_timer_.t0;
    const int r = epzs_serve(ctx, d_req, d_preds, d_cond, d_stale, d_out, d_vis, max_visited, d_bnd, d_int, one, d_spo);
    if (r < 0) return -1;
    served = r == 0;
    if (!served) mode = 1;   // (not taken: the fused launch below)
  }
  if (mode == 3 && served) {
    if (ctx->srv_check && epzs_serve_check(ctx, h_out, h_bnd, h_vis, h_spo, spo0, max_visited)) return -1;
    std::memcpy(out, h_out, sizeof(jmme_epzs_res));
    std::memcpy(bounds, h_bnd, sizeof(jmme_epzs_bounds));
    std::memcpy(visited, h_vis, (size_t)std::min(out[0].n_visited, max_visited) * 4);
    std::memcpy(sp_out, h_spo, sizeof(jmme_block_res));
    if (ctx->phases) ctx->srv_host_us[3] += now_us() - ctx->srv_t_done;
    return 0;
  }
  if (mode >= 1 && !ctx->single_stream) HIPCHK(hipStreamCreateWithFlags(&ctx->single_stream, hipStreamNonBlocking));
  if (mode == 2 && !ctx->h_done) {
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_done), 64, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer(&ctx->dv_done, ctx->h_done, 0));
    __atomic_store_n(ctx->h_done, 0u, __ATOMIC_RELEASE);
  }
  hipStream_t s = mode >= 1 ? ctx->single_stream : nullptr;
  const uint32_t seq = mode == 2 ? ++ctx->done_seq : 0;
  if (launch_epzs_ex(ctx, d_req, n, d_preds, d_cond, d_stale, d_out, d_vis, max_visited, s, d_bnd, d_int,
                     fuse ? &one : nullptr, fuse ? d_spo : nullptr,
                     mode == 2 ? static_cast<uint32_t *>(ctx->dv_done) : nullptr, seq))
    return -1;
  if (sp_req && !fuse && jmme_subpel_refine_async(ctx, d_spq, n, d_int, d_spo, s)) return -1;
  if (mode == 2) {   // the kernel stores seq after a system-scope fence behind its last result
    auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 1; __atomic_load_n(ctx->h_done, __ATOMIC_ACQUIRE) != seq; ++spin) {
      if ((spin & 4095u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        HIPCHK(hipStreamSynchronize(s));   // (surfaces a fault; a finished kernel has stored seq)
        if (__atomic_load_n(ctx->h_done, __ATOMIC_ACQUIRE) != seq) return fail("EPZS search alone: no completion word");
      }
      __builtin_ia32_pause();
    }
  } else {
    HIPCHK(hipStreamSynchronize(s));
  }
  const double t_synced = ctx->phases && n > 1 ? now_us() : 0.0;
  std::memcpy(out, h_out, (size_t)n * sizeof(jmme_epzs_res));
  std::memcpy(bounds, h_bnd, (size_t)n * sizeof(jmme_epzs_bounds));
  for (int i = 0; i < n; ++i)   // only the pairs each search wrote
    std::memcpy(visited + 2 * (size_t)max_visited * i, h_vis + 2 * (size_t)max_visited * i,
                (size_t)std::min(out[i].n_visited, max_visited) * 4);
  if (sp_req) std::memcpy(sp_out, h_spo, (size_t)n * sizeof(jmme_block_res));
  if (ctx->phases && n > 1) {
    ctx->ep_batch_us[0] += t_staged - ep_timer_.t0;   // validation and copies in
    ctx->ep_batch_us[1] += t_synced - t_staged;       // launches and the wait
    ctx->ep_batch_us[2] += now_us() - t_synced;       // copies out
  }
  return 0;
}

// fractal quadtree (encode_one_macroblock): scratch carved from
// one ctx buffer -- counts, the three id lists, the four levels' results
extern "C" int jmme_fractal_encode_mb_rows_async(jmme_ctx *ctx, const uint8_t *d_org, const uint8_t *d_ref0,
                                                 int pitch, const uint32_t *const *d_words, int n_refs, int width,
                                                 int height, int mb_row0, int mb_row1, int search_range, double tol_16,
                                                 double tol_8, jmme_fractal_mb *d_out, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (fractal_geom_ok(pitch, width, height)) return -1;
  if (width % 16 || height % 16) return fail("fractal macroblock plane %dx%d: need multiples of 16", width, height);
  if (n_refs < 1 || n_refs > JMME_FRACTAL_MAX_VIEWS) return fail("n_refs %d not in 1..%d", n_refs, JMME_FRACTAL_MAX_VIEWS);
  if (search_range < 0) return fail("negative search range");
  if (mb_row0 < 0 || mb_row1 > height / 16 || mb_row0 > mb_row1)
    return fail("macroblock rows [%d,%d) outside [0,%d)", mb_row0, mb_row1, height / 16);
  if (!d_org || !d_ref0 || !d_words || !d_out) return fail("null array");
  for (int k = 0; k < n_refs; ++k)
    if (!d_words[k]) return fail("null words image for view %d", k);
  const int mbs_x = width / 16, n_mb = mbs_x * (mb_row1 - mb_row0);
  if (n_mb == 0) return 0;
  const size_t res = sizeof(jmme_fractal_res);
  const size_t off_list1 = 256, off_list2 = off_list1 + (size_t)n_mb * 4, off_list3 = off_list2 + (size_t)n_mb * 16;
  const size_t off_res0 = (off_list3 + (size_t)n_mb * 16 + 255) & ~(size_t)255;
  const size_t off_res1 = off_res0 + (size_t)n_mb * n_refs * res;
  const size_t off_res2 = off_res1 + (size_t)n_mb * 4 * n_refs * res;
  const size_t off_res3 = off_res2 + (size_t)n_mb * 16 * n_refs * res;
  const size_t bytes = off_res3 + (size_t)n_mb * 16 * n_refs * res;
  if (bytes > ctx->cap_tree) {
    (void)hipFree(ctx->d_tree);
    ctx->d_tree = nullptr;
    ctx->cap_tree = 0;
    HIPCHK(hipMalloc(&ctx->d_tree, bytes));
    ctx->cap_tree = bytes;
  }
  char *base = static_cast<char *>(ctx->d_tree);
  FractalTreeParams p{};
  p.org = d_org;
  p.ref0 = d_ref0;
  p.pitch = pitch;
  for (int k = 0; k < n_refs; ++k) p.words[k] = d_words[k];
  p.n_refs = n_refs;
  p.wpitch = width;
  p.width = width;
  p.height = height;
  p.range = search_range;
  p.mbs_x = mbs_x;
  p.n_mb = n_mb;
  p.mb0 = mb_row0 * mbs_x;
  // `tol*tol*no` as the thesis writes it (block_enc.c:797, 1328, 1584)
  p.thr16 = tol_16 * tol_16 * 256;
  p.thr8 = tol_8 * tol_8 * 64;
  p.thr_pair = tol_8 * tol_8 * 32;
  p.out = d_out;
  p.count = reinterpret_cast<int *>(base);
  p.list[1] = reinterpret_cast<int *>(base + off_list1);
  p.list[2] = reinterpret_cast<int *>(base + off_list2);
  p.list[3] = reinterpret_cast<int *>(base + off_list3);
  p.res[0] = reinterpret_cast<jmme_fractal_res *>(base + off_res0);
  p.res[1] = reinterpret_cast<jmme_fractal_res *>(base + off_res1);
  p.res[2] = reinterpret_cast<jmme_fractal_res *>(base + off_res2);
  p.res[3] = reinterpret_cast<jmme_fractal_res *>(base + off_res3);
  HIPCHK(launch_fractal_tree(p, reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

extern "C" int jmme_fractal_encode_mbs_async(jmme_ctx *ctx, const uint8_t *d_org, const uint8_t *d_ref0, int pitch,
                                             const uint32_t *const *d_words, int n_refs, int width, int height,
                                             int search_range, double tol_16, double tol_8, jmme_fractal_mb *d_out,
                                             void *stream) {
  return jmme_fractal_encode_mb_rows_async(ctx, d_org, d_ref0, pitch, d_words, n_refs, width, height, 0,
                                           height > 0 ? height / 16 : 0, search_range, tol_16, tol_8, d_out, stream);
}

extern "C" int jmme_fractal_encode_mbs(jmme_ctx *ctx, const uint8_t *org, const uint8_t *const *refs, int n_refs,
                                       int pitch, int width, int height, int search_range, double tol_16,
                                       double tol_8, jmme_fractal_mb *out) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (fractal_geom_ok(pitch, width, height)) return -1;
  if (width % 16 || height % 16) return fail("fractal macroblock plane %dx%d: need multiples of 16", width, height);
  if (n_refs < 1 || n_refs > JMME_FRACTAL_MAX_VIEWS) return fail("n_refs %d not in 1..%d", n_refs, JMME_FRACTAL_MAX_VIEWS);
  if (!org || !refs || !out) return fail("null array");
  for (int k = 0; k < n_refs; ++k)
    if (!refs[k]) return fail("null reference view %d", k);
  const size_t plane = (size_t)pitch * height;
  const int n_mb = (width / 16) * (height / 16);
  DevBuf o, r[JMME_FRACTAL_MAX_VIEWS], w[JMME_FRACTAL_MAX_VIEWS], dout;
  const uint32_t *words[JMME_FRACTAL_MAX_VIEWS] = {};
  HIPCHK(o.alloc(plane));
  HIPCHK(hipMemcpy(o.p, org, plane, hipMemcpyHostToDevice));
  for (int k = 0; k < n_refs; ++k) {
    HIPCHK(r[k].alloc(plane));
    HIPCHK(w[k].alloc((size_t)width * height * 4));
    HIPCHK(hipMemcpy(r[k].p, refs[k], plane, hipMemcpyHostToDevice));
    if (jmme_fractal_words_async(ctx, (const uint8_t *)r[k].p, pitch, width, height, (uint32_t *)w[k].p, nullptr))
      return -1;
    words[k] = (const uint32_t *)w[k].p;
  }
  HIPCHK(dout.alloc((size_t)n_mb * sizeof(jmme_fractal_mb)));
  if (jmme_fractal_encode_mbs_async(ctx, (const uint8_t *)o.p, (const uint8_t *)r[0].p, pitch, words, n_refs, width,
                                    height, search_range, tol_16, tol_8, (jmme_fractal_mb *)dout.p, nullptr))
    return -1;
  HIPCHK(hipMemcpy(out, dout.p, (size_t)n_mb * sizeof(jmme_fractal_mb), hipMemcpyDeviceToHost));
  return 0;
}

// fractal decoder (block_dec.c:20-1160): views are device planes
extern "C" int jmme_fractal_decode_mbs_async(jmme_ctx *ctx, const jmme_fractal_mb *d_mbs,
                                             const uint8_t *const *d_views, int n_views, int pitch, int width,
                                             int height, int component, uint8_t *d_rec, int *d_status,
                                             void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (fractal_geom_ok(pitch, width, height)) return -1;
  if (width % 16 || height % 16) return fail("fractal macroblock plane %dx%d: need multiples of 16", width, height);
  if (n_views < 1 || n_views > JMME_FRACTAL_MAX_VIEWS) return fail("n_views %d not in 1..%d", n_views, JMME_FRACTAL_MAX_VIEWS);
  if (component < 1 || component > 3) return fail("component %d not 1 (Y), 2 (U) or 3 (V)", component);
  if (!d_mbs || !d_views || !d_rec) return fail("null array");
  FractalDecodeParams p{};
  p.mbs = d_mbs;
  for (int k = 0; k < n_views; ++k) {
    if (!d_views[k]) return fail("null view %d", k);
    p.views[k] = d_views[k];
  }
  p.n_views = n_views;
  p.pitch = pitch;
  p.width = width;
  p.height = height;
  p.component = component;
  p.mbs_x = width / 16;
  p.n_mb = (width / 16) * (height / 16);
  p.rec = d_rec;
  p.status = d_status;
  HIPCHK(launch_fractal_decode(p, reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

extern "C" int jmme_fractal_decode_mbs(jmme_ctx *ctx, const jmme_fractal_mb *mbs, const uint8_t *const *views,
                                       int n_views, int pitch, int width, int height, int component, uint8_t *rec) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (fractal_geom_ok(pitch, width, height)) return -1;
  if (width % 16 || height % 16) return fail("fractal macroblock plane %dx%d: need multiples of 16", width, height);
  if (n_views < 1 || n_views > JMME_FRACTAL_MAX_VIEWS) return fail("n_views %d not in 1..%d", n_views, JMME_FRACTAL_MAX_VIEWS);
  if (!mbs || !views || !rec) return fail("null array");
  const size_t plane = (size_t)pitch * height;
  const int n_mb = (width / 16) * (height / 16);
  DevBuf dm, v[JMME_FRACTAL_MAX_VIEWS], dr, ds;
  const uint8_t *dv[JMME_FRACTAL_MAX_VIEWS] = {};
  HIPCHK(dm.alloc((size_t)n_mb * sizeof(jmme_fractal_mb)));
  HIPCHK(hipMemcpy(dm.p, mbs, (size_t)n_mb * sizeof(jmme_fractal_mb), hipMemcpyHostToDevice));
  for (int k = 0; k < n_views; ++k) {
    if (!views[k]) return fail("null view %d", k);
    HIPCHK(v[k].alloc(plane));
    HIPCHK(hipMemcpy(v[k].p, views[k], plane, hipMemcpyHostToDevice));
    dv[k] = (const uint8_t *)v[k].p;
  }
  HIPCHK(dr.alloc(plane));
  HIPCHK(hipMemset(dr.p, 0, plane));
  HIPCHK(ds.alloc(sizeof(int)));
  HIPCHK(hipMemset(ds.p, 0, sizeof(int)));
  if (jmme_fractal_decode_mbs_async(ctx, (const jmme_fractal_mb *)dm.p, dv, n_views, pitch, width, height, component,
                                    (uint8_t *)dr.p, (int *)ds.p, nullptr))
    return -1;
  int status = 0;
  HIPCHK(hipMemcpy(&status, ds.p, sizeof(int), hipMemcpyDeviceToHost));
  if (status) return fail("fractal decode: a leaf maps to a view >= %d or its domain block leaves the plane", n_views);
  // rows beyond `width` in a pitched plane are not the decoder's
  std::vector<uint8_t> tmp(plane);
  HIPCHK(hipMemcpy(tmp.data(), dr.p, plane, hipMemcpyDeviceToHost));
  for (int y = 0; y < height; ++y) memcpy(rec + (size_t)y * pitch, tmp.data() + (size_t)y * pitch, width);
  return 0;
}

extern "C" jmme_distblk jmme_fast_full_search_block(jmme_ctx *ctx, int list, int ref_idx, int pos_x, int pos_y,
                                                    int blocktype, const jmme_mv *pred_mv,
                                                    const jmme_mv *search_center, int surface_range,
                                                    int block_range, int rdopt, jmme_mv *mv_out,
                                                    jmme_distblk min_mcost, int lambda_factor) {
  DevGuard dg_(ctx);
  // fast_full_search_motion_estimation's contract for one partition, as a
  // one-slot FFS unit (the surface of setup_fast_full_search is the unit's
  // window).  JM's error() semantics on failure (print, exit 500).
  int mb_x = pos_x & ~15, mb_y = pos_y & ~15;
  int s = slot_of(blocktype, (pos_x - mb_x) >> 2, (pos_y - mb_y) >> 2);
  if (s < 0 || !pred_mv || !search_center || !mv_out) {
    fprintf(stderr, "jmme_fast_full_search_block: bad block or null argument\n");
    exit(500);
  }
  jmme_mb_req r;
  memset(&r, 0, sizeof r);
  r.mb_x = (int16_t)mb_x;
  r.mb_y = (int16_t)mb_y;
  r.list = (int16_t)list;
  r.ref_idx = (int16_t)ref_idx;
  r.slot_mask = 1ull << s;
  r.ffs_center_x = search_center->mv_x;
  r.ffs_center_y = search_center->mv_y;
  r.ffs_range = (int16_t)surface_range;
  r.ffs_pos00_valid = (int16_t)(rdopt == 0);
  r.blk[s].pred_x = pred_mv->mv_x;
  r.blk[s].pred_y = pred_mv->mv_y;
  r.blk[s].search_range = (int16_t)block_range;
  r.blk[s].lambda = lambda_factor;
  jmme_block_res out[JMME_NSLOT];
  if (jmme_search_mbs(ctx, JMME_FAST_FULL_SEARCH, &r, 1, out)) {
    fprintf(stderr, "jmme_fast_full_search_block: %s\n", jmme_last_error());
    exit(500);
  }
  // nothing beat the incoming bound: JM keeps best_pos = 0, i.e. the centre
  if (out[s].cost >= min_mcost) {
    *mv_out = *search_center;
    return min_mcost;
  }
  mv_out->mv_x = out[s].mv_x;
  mv_out->mv_y = out[s].mv_y;
  return out[s].cost;
}

extern "C" int jmme_debug_window(jmme_ctx *ctx, int mode, const jmme_mb_req *req, uint32_t *out, int max_words) {
  DevGuard dg_(ctx);
  // Test hook: run unit `req` (one unit) and return the first reference
  // window it staged in LDS (rows x (2R+13) words, word[y][x] = pels x..x+3).
  if (!ctx) return fail("null ctx");
  if (validate(ctx, mode, req, 1)) return -1;
  if (ensure_units(ctx, 1)) return -1;
  const int R = ctx->cfg.SearchRange;
  const int words = (2 * R + 16) * (2 * R + 13);
  if (max_words < words) return fail("debug buffer needs %d words", words);
  uint32_t *d = nullptr;
  HIPCHK(hipMalloc(&d, (size_t)words * 4));
  hipStream_t s = nullptr;
  if (sync_ref_table(ctx, s)) return -1;
  HIPCHK(hipMemcpy(ctx->d_req, req, sizeof(jmme_mb_req), hipMemcpyHostToDevice));
  int rc = launch(ctx, mode, ctx->d_cur, ctx->d_ref_table, ctx->pitch, ctx->width, ctx->height, ctx->d_req, 1,
                  ctx->d_out, s, d);
  if (rc == 0) HIPCHK(hipMemcpy(out, d, (size_t)words * 4, hipMemcpyDeviceToHost));
  (void)hipFree(d);
  return rc;
}

extern "C" int jmme_debug_stamps(jmme_ctx *ctx, uint64_t *out, int max_units) {
  DevGuard dg_(ctx);
  // Diagnostic builds (-DJMME_STAMPS): per-unit s_memtime phase sums of the
  // last launch: [wait, expand, sweep, reduce, refine, output, nslots, items].
  if (!ctx) return fail("null ctx");
  if (!ctx->d_stamps) return fail("library built without JMME_STAMPS");
  // Rows of 8 words; the first n rows are the units, the rest per-workgroup
  // records (4 words each: start, end, HW_ID, XCC_ID << 32 | items).
  size_t n = (size_t)max_units < ctx->cap_stamps / 8 ? (size_t)max_units : ctx->cap_stamps / 8;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, ctx->d_stamps, n * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return (int)n;
}

// ------------------------------------------------------------- sub-pel ME --
// getSubImagesLuma (img_luma.c:611-680) + sub_pel_motion_estimation /
// EPZS_sub_pel_motion_estimation (me_fullsearch.c:186-289, me_epzs_sub.c:30-222)
namespace {

// high bit depth: 16-bit sub-images clipped to max_imgpel_value (the same
// sample type as the context's planes)
int build_sub_images(jmme_ctx *ctx, int slot, hipStream_t s) {
  if (!ctx->d_refs[slot]) return fail("reference slot %d not uploaded", slot);
  const SubGeom g = sub_geom(ctx->width, ctx->height);
  if (!ctx->d_subs[slot]) {
    HIPCHK(hipMalloc(&ctx->d_subs[slot], 16 * g.plane_stride * (ctx->hbd ? 2 : 1)));
    ctx->sub_table_dirty = true;
  }
  HIPCHK(launch_sub_images(ctx->d_refs[slot], ctx->pitch, ctx->width, ctx->height, ctx->d_subs[slot], g.pitch,
                           g.plane_stride, s, ctx->hbd ? ctx->cfg.SourceBitDepthLuma : 8));
  ctx->sub_stale[slot] = false;
  return 0;
}

// build every stale uploaded slot, then publish the table
int prepare_subs(jmme_ctx *ctx, hipStream_t s) {
  for (int k = 0; k < kMaxLists * kMaxRefs; ++k)
    if (ctx->d_refs[k] && (ctx->sub_stale[k] || !ctx->d_subs[k]))
      if (build_sub_images(ctx, k, s)) return -1;
  if (ctx->sub_table_dirty) {
    HIPCHK(hipMemcpyAsync(ctx->d_sub_table, ctx->d_subs, sizeof(ctx->d_subs), hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    ctx->sub_table_dirty = false;
  }
  return 0;
}

}  // namespace

extern "C" int jmme_interpolate_ref(jmme_ctx *ctx, int list, int ref_idx, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (list < 0 || list >= kMaxLists || ref_idx < 0 || ref_idx >= kMaxRefs)
    return fail("list/ref_idx (%d,%d) out of range", list, ref_idx);
  return build_sub_images(ctx, list * kMaxRefs + ref_idx, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int jmme_get_sub_images(jmme_ctx *ctx, int list, int ref_idx, jmme_imgpel ****sub) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (!sub) return fail("null sub-image array");
  if (list < 0 || list >= kMaxLists || ref_idx < 0 || ref_idx >= kMaxRefs)
    return fail("list/ref_idx (%d,%d) out of range", list, ref_idx);
  const int slot = list * kMaxRefs + ref_idx;
  if (!ctx->d_refs[slot]) return fail("reference slot %d not uploaded", slot);
  if ((ctx->sub_stale[slot] || !ctx->d_subs[slot]) && build_sub_images(ctx, slot, nullptr)) return -1;
  const SubGeom g = sub_geom(ctx->width, ctx->height);
  const size_t es = ctx->hbd ? 2 : 1;
  std::vector<uint8_t> h(16 * g.plane_stride * es);
  HIPCHK(hipMemcpy(h.data(), ctx->d_subs[slot], h.size(), hipMemcpyDeviceToHost));
  for (int k = 0; k < 16; ++k) {
    jmme_imgpel **rows = sub[k >> 2][k & 3];
    if (!rows) return fail("null row array for sub-image [%d][%d]", k >> 2, k & 3);
    for (int j = 0; j < g.ph; ++j) {
      jmme_imgpel *d = rows[j - JMME_SUBPEL_PAD_Y];
      if (!d) return fail("null row %d of sub-image [%d][%d]", j - JMME_SUBPEL_PAD_Y, k >> 2, k & 3);
      d -= JMME_SUBPEL_PAD_X;
      const size_t o = (size_t)k * g.plane_stride + (size_t)j * g.pitch;
      if (ctx->hbd) {
        const uint16_t *srow = reinterpret_cast<const uint16_t *>(h.data()) + o;
        for (int i = 0; i < g.pw; ++i) d[i] = srow[i];
      } else {
        const uint8_t *srow = &h[o];
        for (int i = 0; i < g.pw; ++i) d[i] = srow[i];
      }
    }
  }
  return 0;
}

extern "C" int jmme_sub_images_async(jmme_ctx *ctx, const uint8_t *d_src, int src_pitch, int width, int height,
                                     uint8_t *d_dst, int dst_pitch, size_t plane_stride, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (!d_src || !d_dst) return fail("null plane");
  if (width <= 0 || height <= 0 || src_pitch < width) return fail("bad source plane %dx%d pitch %d", width, height,
                                                                    src_pitch);
  const int pw = width + 2 * JMME_SUBPEL_PAD_X, ph = height + 2 * JMME_SUBPEL_PAD_Y;
  if (dst_pitch < ((pw + 3) & ~3) || (dst_pitch & 3) || (reinterpret_cast<uintptr_t>(d_dst) & 3))
    return fail("sub-image pitch %d: need a multiple of 4 >= %d and a 4-byte aligned buffer", dst_pitch, pw);
  if (plane_stride < (size_t)ph * dst_pitch || (plane_stride & 3)) return fail("sub-image plane stride too small");
  if (15 * plane_stride + (size_t)ph * dst_pitch >= ((size_t)1 << 32))
    return fail("sub-image planes span %zu bytes: the 16 planes must lie within 4 GiB", 16 * plane_stride);
  HIPCHK(launch_sub_images(d_src, src_pitch, width, height, d_dst, dst_pitch, plane_stride,
                           reinterpret_cast<hipStream_t>(stream)));
  return 0;
}

extern "C" int jmme_subpel_validate(jmme_ctx *ctx, const jmme_subpel_req *req, int n) {
  DevGuard dg_(ctx, true);   // (host-side checks only: a running EPZS server may stay)
  if (!ctx) return fail("null ctx");
  if (n < 0) return fail("negative request count");
  if (n && !req) return fail("null request array");
  if (!ctx->d_cur) return fail("no current frame uploaded");
  for (int i = 0; i < n; ++i) {
    const jmme_subpel_req &q = req[i];
    if (q.blocktype == 0) continue;
    if (q.blocktype < 1 || q.blocktype > 7) return fail("request %d: blocktype %d", i, q.blocktype);
    const int bsx = (q.blocktype <= 2) ? 16 : (q.blocktype <= 5) ? 8 : 4;
    const int bsy = (q.blocktype == 1 || q.blocktype == 3) ? 16 : (q.blocktype == 2 || q.blocktype == 4 ||
                                                                   q.blocktype == 6) ? 8 : 4;
    if (q.pos_x < 0 || q.pos_y < 0 || (q.pos_x & 3) || (q.pos_y & 3) || q.pos_x + bsx > ctx->width ||
        q.pos_y + bsy > ctx->height)
      return fail("request %d: block (%d,%d) %dx%d outside the %dx%d picture", i, q.pos_x, q.pos_y, bsx, bsy,
                  ctx->width, ctx->height);
    if (q.ref_slot < 0 || q.ref_slot >= kMaxLists * kMaxRefs || !ctx->d_refs[q.ref_slot])
      return fail("request %d: reference slot %d not uploaded", i, q.ref_slot);
    if (q.variant > 1) return fail("request %d: variant %d", i, q.variant);
    if (q.metric_h > 2 || q.metric_q > 2) return fail("request %d: metric %d/%d", i, q.metric_h, q.metric_q);
    // computeSSE sums into an int (me_distortion.c:1197): above 11 bits a 16x16
    // block's sum can pass 2^31, where JM's row-wise early exit meets a wrapped sum
    if ((q.metric_h == 1 || q.metric_q == 1) && ctx->cfg.SourceBitDepthLuma > 11)
      return fail("request %d: SSE sub-pel metric at SourceBitDepthLuma %d (int sums may wrap)", i,
                  ctx->cfg.SourceBitDepthLuma);
    if (q.start_hp > 1 || q.start_qp > 1) return fail("request %d: start_hp/qp", i);
    if (q.search_pos2 > 9 || q.search_pos4 > 9)
      return fail("request %d: search_pos2/4 %d/%d beyond JM's 9-point rings", i, q.search_pos2, q.search_pos4);
    if ((q.flags & JMME_SP_TEST8x8) && (bsx < 8 || bsy < 8))
      return fail("request %d: test8x8 on a %dx%d block", i, bsx, bsy);
    if (q.min_mcost < 0 || q.min_mcost > JMME_DISTBLK_MAX) return fail("request %d: min_mcost out of range", i);
    if (q.lambda_h < 0 || q.lambda_q < 0) return fail("request %d: negative lambda", i);
    // the refined vector stays within +-(3/4 pel) of mv; mvbits is closed-form for any difference
    if (std::abs(q.mv_x) > 8192 || std::abs(q.mv_y) > 8192) return fail("request %d: mv out of range", i);
  }
  return 0;
}

extern "C" int jmme_subpel_refine_async(jmme_ctx *ctx, const jmme_subpel_req *d_req, int n,
                                        const jmme_block_res *d_int, jmme_block_res *d_out, void *stream) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (n < 0) return fail("negative request count");
  if (n == 0) return 0;
  if (!d_req || !d_out) return fail("null array");
  if (!ctx->d_cur) return fail("no current frame uploaded");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (prepare_subs(ctx, s)) return -1;
  const SubGeom g = sub_geom(ctx->width, ctx->height);
  SubpelParams p{};
  p.cur = ctx->d_cur;
  p.cur_pitch = ctx->pitch;
  p.width = ctx->width;
  p.height = ctx->height;
  p.hbd = ctx->hbd ? 1 : 0;
  p.subs = ctx->d_sub_table;
  p.sub_pitch = g.pitch;
  p.plane_stride = g.plane_stride;
  p.req = d_req;
  p.int_res = d_int;
  p.out = d_out;
  p.n = n;
  HIPCHK(launch_subpel(p, s));
  return 0;
}

extern "C" int jmme_subpel_refine(jmme_ctx *ctx, const jmme_subpel_req *req, int n, jmme_block_res *out) {
  DevGuard dg_(ctx);
  if (jmme_subpel_validate(ctx, req, n)) return -1;
  if (n == 0) return 0;
  if (!out) return fail("null output array");
  // one H2D of [requests | entry outputs] (blocktype-0 entries keep theirs), one D2H, one sync
  const size_t rq = align64((size_t)n * sizeof(jmme_subpel_req)), ro = (size_t)n * sizeof(jmme_block_res);
  if (ensure_pin(ctx, rq + ro) || ensure_sp(ctx, rq + ro)) return -1;
  std::memcpy(ctx->h_pin, req, (size_t)n * sizeof(jmme_subpel_req));
  std::memcpy(ctx->h_pin + rq, out, ro);
  hipStream_t s = nullptr;
  HIPCHK(hipMemcpyAsync(ctx->d_sp, ctx->h_pin, rq + ro, hipMemcpyHostToDevice, s));
  if (jmme_subpel_refine_async(ctx, reinterpret_cast<const jmme_subpel_req *>(ctx->d_sp), n, nullptr,
                               reinterpret_cast<jmme_block_res *>(ctx->d_sp + rq), s))
    return -1;
  HIPCHK(hipMemcpyAsync(ctx->h_pin + rq, ctx->d_sp + rq, ro, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  std::memcpy(out, ctx->h_pin + rq, ro);
  return 0;
}
static_assert(sizeof(jmme_subpel_req) == 48, "sub-pel ABI layout");

// One-time start-up work out of the first search: HIP loads a translation
// unit's kernels at their first launch and the item kernel's occupancy query is
// cached on first use, so a tiny search through both search paths (and one
// sub-image interpolation) on a dummy 64 x 64 plane pays for it here.
extern "C" int jmme_prepare(jmme_ctx *ctx) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  constexpr int kW = 64, kH = 64;
  const auto g = sub_geom(kW, kH);
  DevBuf plane, table, dreq, dout, subs;
  HIPCHK(plane.alloc((size_t)kW * kH * 2));   // 16-bit pels for a high-bit-depth context
  HIPCHK(hipMemset(plane.p, 0, (size_t)kW * kH * 2));
  std::vector<const uint8_t *> tab(kMaxLists * kMaxRefs, static_cast<const uint8_t *>(plane.p));
  HIPCHK(table.alloc(tab.size() * sizeof(void *)));
  HIPCHK(hipMemcpy(table.p, tab.data(), tab.size() * sizeof(void *), hipMemcpyHostToDevice));
  jmme_mb_req r;
  std::memset(&r, 0, sizeof r);
  r.mb_x = 16;
  r.mb_y = 16;
  r.slot_mask = 1;
  r.blk[0].search_range = (int16_t)std::min(1, ctx->cfg.SearchRange);
  r.ffs_range = r.blk[0].search_range;
  HIPCHK(dreq.alloc(sizeof r));
  HIPCHK(hipMemcpy(dreq.p, &r, sizeof r, hipMemcpyHostToDevice));
  HIPCHK(dout.alloc(JMME_NSLOT * sizeof(jmme_block_res)));
  for (int mode : {JMME_FULL_SEARCH, JMME_FAST_FULL_SEARCH})
    if (launch(ctx, mode, static_cast<const uint8_t *>(plane.p), static_cast<const uint8_t *const *>(table.p), kW, kW,
               kH, static_cast<const jmme_mb_req *>(dreq.p), 1, static_cast<jmme_block_res *>(dout.p), nullptr, nullptr,
               true))
      return -1;
  // the small path reads the context's planes: borrow the dummy for one call
  uint8_t *cur = ctx->d_cur, *ref0 = ctx->d_refs[0];
  const int w = ctx->width, h = ctx->height, pitch = ctx->pitch;
  ctx->d_cur = ctx->d_refs[0] = static_cast<uint8_t *>(plane.p);
  ctx->width = kW;
  ctx->height = kH;
  ctx->pitch = kW;
  jmme_block_res res[JMME_NSLOT];
  int rc = 0;
  for (int mode : {JMME_FULL_SEARCH, JMME_FAST_FULL_SEARCH})
    if (rc >= 0) rc = search_small(ctx, mode, &r, 1, res, nullptr, true);
  // the chain kernels, their stream and result block (jmme_search_mbs_chains)
  if (rc >= 0) {   // (16-bit contexts: the v_sad_u16 instantiation on the 16-bit dummy plane)
    jmme_chain c;
    std::memset(&c, 0, sizeof c);
    c.mb_x = c.mb_y = 16;
    c.n_steps = 1;
    c.mv_lim_x0 = c.mv_lim_y0 = -512;
    c.mv_lim_x1 = c.mv_lim_y1 = 511;
    c.ffs_range = 1;
    c.steps[0].slot = 0;
    for (int j = 0; j < 3; ++j) c.steps[0].nb[j].src = JMME_NB_UNAVAILABLE;
    c.steps[0].sr_min_x = c.steps[0].sr_min_y = -4;
    c.steps[0].sr_max_x = c.steps[0].sr_max_y = 4;
    const bool dirty = ctx->ref_table_dirty;
    const uint8_t **rt = ctx->d_ref_table;
    ctx->d_ref_table = static_cast<const uint8_t **>(table.p);
    ctx->ref_table_dirty = false;
    jmme_chain_res cres[JMME_CHAIN_MAX_STEPS];
    for (int mode : {JMME_FULL_SEARCH, JMME_FAST_FULL_SEARCH})
      if (rc >= 0 && jmme_search_mbs_chains(ctx, mode, &r, 0, res, &c, 1, cres)) rc = -1;
    ctx->d_ref_table = rt;
    ctx->ref_table_dirty = dirty;
  }
  ctx->d_cur = cur;
  ctx->d_refs[0] = ref0;
  ctx->width = w;
  ctx->height = h;
  ctx->pitch = pitch;
  if (rc < 0) return -1;
  HIPCHK(subs.alloc(16 * g.plane_stride * 2));
  HIPCHK(launch_sub_images(static_cast<const uint8_t *>(plane.p), kW, kW, kH, static_cast<uint8_t *>(subs.p), g.pitch,
                           g.plane_stride, nullptr, ctx->hbd ? ctx->cfg.SourceBitDepthLuma : 8));
  HIPCHK(hipDeviceSynchronize());
  return 0;
}

extern "C" int jmme_reserve(jmme_ctx *ctx, int max_units) {
  DevGuard dg_(ctx);
  if (!ctx) return fail("null ctx");
  if (max_units < 0) return fail("negative unit count");
  const size_t n = (size_t)max_units;
  if (ensure_units(ctx, n) || ensure_items(ctx, n * JMME_NSLOT)) return -1;
  const size_t rq = align64(n * sizeof(jmme_mb_req)), rs = align64(n * JMME_NSLOT * sizeof(jmme_block_res));
  size_t pin = rq + rs + 64;
  if (!ctx->cfg.DisableSubpelME) {   // jmme_subpel_refine's [requests | outputs] for n * JMME_NSLOT refinements
    const size_t nsp = n * JMME_NSLOT, sp = align64(nsp * sizeof(jmme_subpel_req)) + nsp * sizeof(jmme_block_res);
    if (ensure_sp(ctx, sp)) return -1;
    pin = std::max(pin, sp);
  }
  if (ensure_pin(ctx, pin)) return -1;
  // the configured picture's planes: the staging buffer and device planes for
  // the current picture and every reference of list 0, taken by the first uploads
  const int w = ctx->cfg.SourceWidth, h = ctx->cfg.SourceHeight;
  if (w > 0 && h > 0 && !(w & 15) && !(h & 15) && (!ctx->width || (ctx->width == w && ctx->height == h))) {
    const size_t bytes = (size_t)((w + 63) & ~63) * h * (ctx->hbd ? 2 : 1);   // set_geometry's pitch
    if (bytes > ctx->cap_stage) {
      if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
      ctx->h_stage = nullptr;
      ctx->cap_stage = 0;
      HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_stage), bytes, hipHostMallocDefault));
      ctx->cap_stage = bytes;
    }
    const int planes = 1 + std::min(std::max(ctx->cfg.NumberReferenceFrames, 1), kMaxRefs);
    if (ctx->spare_bytes != bytes) {
      for (auto *p : ctx->spare_planes) (void)hipFree(p);
      ctx->spare_planes.clear();
      ctx->spare_bytes = bytes;
    }
    while ((int)ctx->spare_planes.size() < planes) {
      uint8_t *d = nullptr;
      HIPCHK(hipMalloc(&d, bytes));
      ctx->spare_planes.push_back(d);
    }
    // one plane-sized copy: the first large host-to-device copy of a process
    // sets up its DMA path (~8 ms measured inside the first P picture's ME time)
    std::memset(ctx->h_stage, 0, bytes);
    HIPCHK(hipMemcpyAsync(ctx->spare_planes.back(), ctx->h_stage, bytes, hipMemcpyHostToDevice, nullptr));
    HIPCHK(hipStreamSynchronize(nullptr));
  }
  return 0;
}
