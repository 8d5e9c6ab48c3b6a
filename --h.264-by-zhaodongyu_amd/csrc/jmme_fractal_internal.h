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

hipError_t launch_fractal_words(const uint8_t *ref, int pitch, int W, int H, uint32_t *words, int wpitch,
                                hipStream_t s);
hipError_t launch_fractal_search(const FractalParams &p, hipStream_t s);
hipError_t launch_box_sums(const uint8_t *p, int pitch, int W, int H, int bsx, int bsy, uint32_t *hs, uint32_t *hs2,
                           double *sum, double *sum2, hipStream_t s);

}  // namespace jmme
