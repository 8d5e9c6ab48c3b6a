// jmme_fractal_internal.h -- launchers of the fractal kernels
// (csrc/jmme_fractal.hip); not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "jmme.h"

namespace jmme {

struct FractalParams {
  const uint8_t *org;          // range (current) plane, 8-bit
  int pitch;                   // bytes per row of org
  const uint32_t *words;       // reference words image: word[y][x] = pels x..x+3
  int wpitch;                  // words per row of the words image
  int width, height;           // picture size (bound_chk)
  int range;                   // search range R
  const jmme_fractal_req *req;
  jmme_fractal_res *out;
  int n;
};

// quadtree encoder (encode_one_macroblock): level 0 = 16x16 of
// every macroblock, 1 = the four 8x8 of split macroblocks, 2 = the 8x4 / 4x8
// pairs of unmatched 8x8, 3 = the four 4x4 of 8x8 whose pairs failed.  Level
// L >= 1 works on the ids in list[L] (count[L] of them), appended on the device
// by the gate of level L-1; res[L] holds one search result per (node, block,
// view) in that order.
struct FractalTreeParams {
  const uint8_t *org, *ref0;   // range plane, view 0 (the gate's co-located block)
  int pitch;
  const uint32_t *words[JMME_FRACTAL_MAX_VIEWS];
  int n_refs, wpitch;
  int width, height, range, mbs_x, n_mb;
  int mb0;                        // raster index of out[0] (an MB-row band starts there; 0 = whole plane)
  double thr16, thr8, thr_pair;   // tol_16^2*256, tol_8^2*64, tol_8^2*32 (thesis operand order)
  jmme_fractal_mb *out;
  jmme_fractal_res *res[4];
  int *list[4];                   // list[1..3]
  int *count;                     // count[1..3] (count[0] unused)
};

// pruned domain-pool search (jmme_fractal_pool.hip): the windowed kernel at
// radius seed_range seeds out[], then per block size present in req[] a pool
// image (pool[s]: float2 {Σd, n·Σd² − (Σd)²} per domain position, wpitch x
// height) and the pruned search over the full window
struct FractalPoolParams {
  FractalParams base;
  void *pool[7];                  // 16x16, 16x8, 8x16, 8x8, 8x4, 4x8, 4x4
  int *flags;                     // [8] sizes present (zeroed by the launcher)
  unsigned long long *stats;      // [0] += exactly evaluated survivors
  int seed_range;
  void *bw;                       // 4x4 full pool on the matrix cores: bf16 words image (uint2, wpitch x height)
  int use_mfma;
};

hipError_t launch_fractal_pool(const FractalPoolParams &p, hipStream_t s);

hipError_t launch_fractal_tree(const FractalTreeParams &p, hipStream_t s);

// decoder (decode_one_macroblock and the block decoders, block_dec.c:20-1160)
struct FractalDecodeParams {
  const jmme_fractal_mb *mbs;
  const uint8_t *views[JMME_FRACTAL_MAX_VIEWS];
  int n_views, pitch, width, height, component, mbs_x, n_mb;
  uint8_t *rec;
  int *status;                    // |= 1 when a leaf's view or domain block is out of range (nullable)
};

hipError_t launch_fractal_decode(const FractalDecodeParams &p, hipStream_t s);

hipError_t launch_fractal_words(const uint8_t *ref, int pitch, int W, int H, uint32_t *words, int wpitch,
                                hipStream_t s);
hipError_t launch_fractal_search(const FractalParams &p, hipStream_t s);
hipError_t launch_box_sums(const uint8_t *p, int pitch, int W, int H, int bsx, int bsy, uint32_t *hs, uint32_t *hs2,
                           double *sum, double *sum2, hipStream_t s);

}  // namespace jmme
