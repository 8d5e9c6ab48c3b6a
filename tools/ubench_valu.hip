// ubench_valu.hip -- measured VALU throughput of the instructions the ME
// kernel is built from (v_sad_u8, v_add/v_lshl_add/v_min u32, 64-bit
// compare+select), so roofline fractions use a measured ceiling.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int kIters = 4096;
constexpr int kChains = 8;   // independent dependency chains per lane

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned *out, unsigned seed) {
  unsigned a[kChains], b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x;
  unsigned long long q[kChains];
#pragma unroll
  for (int i = 0; i < kChains; ++i) { a[i] = seed + i * 7919u + threadIdx.x; q[i] = a[i]; }
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < kChains; ++i) {
      if (OP == 0) a[i] = __builtin_amdgcn_sad_u8(b, c, a[i]);
      if (OP == 1) a[i] = a[i] + b;
      if (OP == 2) a[i] = (b << 18) + a[i];                 // v_lshl_add_u32
      if (OP == 3) a[i] = min(a[i], b + (unsigned)i);        // v_min_u32 (+ folded add)
      if (OP == 4) { unsigned long long kk = ((unsigned long long)b << 32) | a[i]; q[i] = q[i] < kk ? q[i] : kk; a[i] += 1; }
    }
    asm volatile("" : "+v"(b));
  }
  unsigned r = 0;
#pragma unroll
  for (int i = 0; i < kChains; ++i) r += a[i] + (unsigned)q[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
float run(unsigned *d, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u + r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  const int blocks = 256 * 8;   // 8 workgroups (32 waves) per CU
  unsigned *d;
  CHK(hipMalloc(&d, blocks * 256 * 4));
  const double lane_ops = (double)blocks * 256 * kIters * kChains;
  const char *names[] = {"v_sad_u8", "v_add_u32", "v_lshl_add_u32", "v_min_u32", "u64 key min"};
  float t[5] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks), run<4>(d, blocks)};
  for (int i = 0; i < 5; ++i)
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"G_lane_ops_per_s\": %.1f}\n", names[i], t[i], lane_ops / (t[i] * 1e-3) / 1e9);
  return 0;
}
