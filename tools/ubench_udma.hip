// Does an LDS-DMA dword load (global_load_lds_dword) from a byte address that is
// not dword aligned deliver the 4 bytes at that address?  The item kernel's
// window staging could then fetch its "word[y][x] = pels x..x+3" layout directly
// (one DMA dword per word) instead of expanding aligned dwords in LDS.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/ubench_udma tools/ubench_udma.hip
// Prints one JSON line: mismatches per byte shift (0..3) and the timing of both forms.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

__global__ void udma_kernel(const uint8_t *src, int shift, uint32_t *out, int rows) {
  extern __shared__ uint32_t lds[];
  const int lane = threadIdx.x;
  for (int r = 0; r < rows; ++r) {
    const uint8_t *g = src + (size_t)r * 4096 + shift + 4 * lane;   // unaligned when shift != 0
    const uint32_t dst = (uint32_t)(uintptr_t)(lds + r * 64);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g), "s"(dst) : "memory", "m0");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int r = 0; r < rows; ++r) out[(size_t)r * 64 + lane] = lds[r * 64 + lane];
}

int main() {
  const int rows = 16;
  std::vector<uint8_t> h(rows * 4096 + 64);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)(i * 131 + 7 + (i >> 8));
  uint8_t *d = nullptr;
  uint32_t *o = nullptr;
  if (hipMalloc(&d, h.size()) != hipSuccess || hipMalloc(&o, rows * 64 * 4) != hipSuccess) return 1;
  hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice);
  int bad[4] = {0, 0, 0, 0};
  for (int s = 0; s < 4; ++s) {
    hipMemset(o, 0, rows * 64 * 4);
    hipLaunchKernelGGL(udma_kernel, dim3(1), dim3(64), rows * 64 * 4, 0, d, s, o, rows);
    if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"kernel failed at shift %d\"}\n", s); return 2; }
    std::vector<uint32_t> got(rows * 64);
    hipMemcpy(got.data(), o, got.size() * 4, hipMemcpyDeviceToHost);
    for (int r = 0; r < rows; ++r)
      for (int l = 0; l < 64; ++l) {
        uint32_t want;
        std::memcpy(&want, &h[(size_t)r * 4096 + s + 4 * l], 4);
        if (got[r * 64 + l] != want) ++bad[s];
      }
  }
  printf("{\"mismatches_by_shift\": [%d, %d, %d, %d], \"dwords_per_shift\": %d}\n", bad[0], bad[1], bad[2], bad[3],
         rows * 64);
  return 0;
}
