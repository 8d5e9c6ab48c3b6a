// jmme_epzs_internal.h -- launcher of the EPZS kernel (csrc/jmme_epzs.hip);
// not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "jmme.h"
#include "jmme_subpel_internal.h"

namespace jmme {

constexpr int kEpzsMaxQpel = 4 * JMME_MAX_RANGE;   // largest searchRange.max_x / max_y (qpel)

// a search alone (jmme_epzs_speculate with n = 1, the drop-in's misses) travels
// whole in the kernel arguments: no host-mapped read on its path
constexpr int kEpzsStageP = 128, kEpzsStageS = 64;
struct EpzsOne {
  jmme_epzs_req q;                 // pred_off = stale_off = 0
  jmme_subpel_req spq;             // its refinement (blocktype 0: none)
  uint32_t preds[kEpzsStageP];     // (x, y) int16 pairs
  uint32_t stale[kEpzsStageS];
  uint8_t cond[kEpzsStageP];
};

struct alignas(16) EpzsParams {   // (whole uint4s: the server copies it so)
  const uint8_t *cur;                  // current frame: 8-bit, or 16-bit when hbd
  const uint8_t *const *refs;          // device table of reference planes (list * 32 + ref_idx)
  int pitch, width, height;            // pitch in samples
  int hbd;                             // 16-bit planes and sub-images (SourceBitDepthLuma 9..14)
  const jmme_epzs_req *req;
  const int16_t *preds, *stale;        // (x, y) pools
  jmme_epzs_res *out;
  int n;
  // EPZSSubPelGrid = 1 (variants 2 / 3): candidates on the quarter-pel sub-images
  int grid;
  const uint8_t *const *subs;          // device table of sub-image sets (list * 32 + ref_idx)
  int sub_pitch;
  size_t plane_stride;
  int max_qpel;                        // largest searchRange.max_x / max_y the map is sized for
  int map_words;                       // epzs_map_words(grid, max_qpel)
  // drop-in extras (jmme_epzs_search_ex): predictor conditions parallel to
  // preds (JMME_EPZS_PRED_*; null: all unconditional) and the visited cells of
  // each search, (dx, dy) qpel from the centre, max_visited per search (null: not written)
  const uint8_t *pred_cond;
  int16_t *visited;
  int max_visited;
  // speculative batches (jmme_epzs_speculate): each search's validity
  // intervals, and its result as a jmme_block_res for the chained sub-pel
  // refinement (null: not written)
  jmme_epzs_bounds *bounds;
  jmme_block_res *int_out;
  // fused refinement (a search alone): the wave that searched the request in
  // `one` runs its EPZS sub-pel refinement one.spq itself, from its own
  // answer, into fused_sp.out[0] (fused = 0: none; the caller chains the
  // refinement kernel instead)
  int fused;
  SubpelParams fused_sp;
  EpzsOne one;                     // fused = 1: the one request, its lists and its refinement
  uint32_t *done;                  // fused: done_seq is stored here (mapped memory) after everything else
  uint32_t done_seq;
};

// A wave's EPZSMap area: the bitmap (one bit per cell of the largest window,
// whole quads), then one flag bit per bitmap word that a search stamped (whole
// quads): the next search clears only the flagged words, and the visited cells
// are read back from them, not from a scan of the whole bitmap
__host__ __device__ inline int epzs_bitmap_words(bool grid, int max_qpel) {
  const int side = grid ? 2 * max_qpel + 1 : 2 * (max_qpel >> 2) + 1;
  return ((side * side + 31) / 32 + 3) & ~3;
}
__host__ __device__ inline int epzs_flag_words(int bitmap_words) { return ((bitmap_words + 31) / 32 + 3) & ~3; }
size_t epzs_map_words(bool grid, int max_qpel);   // bitmap + flags
hipError_t launch_epzs(const EpzsParams &p, hipStream_t s);
// The resident server's mailbox (JMME_SINGLE_MODE 3), in mapped pinned host
// memory; each word the two sides exchange has a cache line to itself
struct alignas(64) EpzsBox {
  uint32_t seq, pad0[15];     // host: the request number (the server reads it from req[])
  uint32_t quit, pad1[15];    // host: 1 = the server exits at its next poll
  uint32_t done, pad2[15];    // server: the number it served, after its results and a system fence
  uint32_t alive, pad3[15];   // host: 1 before a launch; server: 0 as its last store
  uint32_t service, copy, search, ph[10], cycles, pad4[2];
  uint32_t rph[6], pad5[10];  // server: the refinement's phase ends A, B, C, D and its two passes (from its window)   // server: the request's time from its number seen to its
                                              // results stored, to its copy in LDS, to the search's end, and
                                              // the search's phases and the refinement's window
                                              // load and phases (10 ns ticks)
  EpzsParams p;               // host: the request is built here (a fused search alone: fused = 1, one = its
                              // lists), then written to req[] -- the server reads req[] only
  uint4 req[(sizeof(EpzsParams) / 4 + 2) / 3];   // host: p as chunks (three dwords of p, then the request number)
};
constexpr int kEpzsReqChunks = (int)((sizeof(EpzsParams) / 4 + 2) / 3);
hipError_t launch_epzs_server(EpzsBox *d_box, bool grid, bool hbd, int map_words, uint32_t last, uint32_t idle_ticks,
                              unsigned long long life_ticks, hipStream_t s);

}  // namespace jmme
