// jmme_epzs.hip -- launchers of the EPZS kernels (jmme_epzs_impl.inc, one
// translation unit per (grid, sample width): jmme_epzs_g*h*.hip), SURVEY.md §8 a11
#include <hip/hip_runtime.h>

#include "jmme_epzs_internal.h"

namespace jmme {

namespace {
constexpr int kWG = 256;
constexpr int kWaves = kWG / 64;
}  // namespace

#define JMME_EPZS_DECL(g, h)                                                                                        \
  hipError_t launch_epzs_g##g##h(const EpzsParams &p, hipStream_t s, int grid, size_t lds);                        \
  hipError_t launch_epzs_server_g##g##h(EpzsBox *d_box, size_t lds, uint32_t last, uint32_t idle_ticks,           \
                                         unsigned long long life_ticks, hipStream_t s);
JMME_EPZS_DECL(0, 0)
JMME_EPZS_DECL(0, 1)
JMME_EPZS_DECL(1, 0)
JMME_EPZS_DECL(1, 1)

hipError_t launch_epzs_server(EpzsBox *d_box, bool grid, bool hbd, int map_words, uint32_t last, uint32_t idle_ticks,
                              unsigned long long life_ticks, hipStream_t s) {
  const size_t lds = (size_t)map_words * sizeof(uint32_t);
  auto f = grid ? (hbd ? launch_epzs_server_g11 : launch_epzs_server_g10)
                : (hbd ? launch_epzs_server_g01 : launch_epzs_server_g00);
  return f(d_box, lds, last, idle_ticks, life_ticks, s);
}

size_t epzs_map_words(bool grid, int max_qpel) {   // bitmap + flags, whole quads
  const int bw = epzs_bitmap_words(grid, max_qpel);
  return (size_t)bw + (size_t)epzs_flag_words(bw);
}

hipError_t launch_epzs(const EpzsParams &p, hipStream_t s) {
  int grid = (p.n + kWaves - 1) / kWaves;
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  const size_t lds = (size_t)kWaves * p.map_words * sizeof(uint32_t);
  auto f = p.grid ? (p.hbd ? launch_epzs_g11 : launch_epzs_g10) : (p.hbd ? launch_epzs_g01 : launch_epzs_g00);
  return f(p, s, grid, lds);
}

}  // namespace jmme
