// jmme_subpel_internal.h -- launchers of the quarter-pel interpolation and
// sub-pel refinement kernels (csrc/jmme_subpel.hip); not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "jmme.h"

namespace jmme {

// padded sub-image geometry of a W x H picture (get_mem4Dpel_pad, memalloc.c:881-904)
struct SubGeom {
  int pw, ph;            // W + 64, H + 40
  int pitch;             // samples per padded row (>= pw, multiple of 64)
  size_t plane_stride;   // samples per sub-image (ph * pitch + read slack); bytes = samples * (hbd ? 2 : 1)
};
inline SubGeom sub_geom(int w, int h) {
  SubGeom g;
  g.pw = w + 2 * JMME_SUBPEL_PAD_X;
  g.ph = h + 2 * JMME_SUBPEL_PAD_Y;
  g.pitch = (g.pw + 63) & ~63;
  g.plane_stride = (size_t)g.ph * g.pitch + 256;
  return g;
}

// bits = SourceBitDepthLuma: 8 -> 8-bit planes; 9..14 -> 16-bit planes and
// samples clipped to (1 << bits) - 1.  Pitches and the plane stride in samples.
hipError_t launch_sub_images(const uint8_t *src, int src_pitch, int w, int h, uint8_t *dst, int dst_pitch,
                             size_t plane_stride, hipStream_t s, int bits = 8);

struct SubpelParams {
  const uint8_t *cur;                  // current picture: 8-bit, or 16-bit when hbd (pitch in samples)
  int cur_pitch, width, height;
  int hbd;                             // 16-bit planes (SourceBitDepthLuma 9..14)
  const uint8_t *const *subs;          // device table [list*32 + ref]: 16 sub-images each
  int sub_pitch;
  size_t plane_stride;
  const jmme_subpel_req *req;
  const jmme_block_res *int_res;       // optional integer-pel results aligned with req
  jmme_block_res *out;
  int n;
  int per_wave;                        // refinements per wave (1..16), set by launch_subpel
};

hipError_t launch_subpel(const SubpelParams &p, hipStream_t s);

}  // namespace jmme
