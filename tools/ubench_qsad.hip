// ubench_qsad.hip -- throughput of the gfx950 SAD family: v_sad_u8 (4 abs-diffs
// per lane), v_qsad_pk_u16_u8 (4 sliding positions x 4 = 16 abs-diffs per lane,
// 4 x u16 accumulators) and v_mqsad_u32_u8 (masked, 4 x u32), each as 8
// independent chains per lane at 8 workgroups (32 waves) per CU.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_qsad.hip -o tools/ubench_qsad
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int kIters = 2048;
constexpr int kChains = 8;
typedef unsigned u4 __attribute__((ext_vector_type(4)));

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned *out, unsigned seed) {
  unsigned b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x;
  unsigned long long w = ((unsigned long long)(c * 7u) << 32) | b;
  unsigned a[kChains];
  unsigned long long q[kChains];
  u4 m[kChains];
#pragma unroll
  for (int i = 0; i < kChains; ++i) {
    a[i] = seed + i * 7919u + threadIdx.x;
    q[i] = a[i];
    m[i] = u4{a[i], a[i] + 1, a[i] + 2, a[i] + 3};
  }
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < kChains; ++i) {
      if (OP == 0) a[i] = __builtin_amdgcn_sad_u8(b, c, a[i]);
      if (OP == 1) q[i] = __builtin_amdgcn_qsad_pk_u16_u8(w, c, q[i]);
      if (OP == 2) m[i] = __builtin_amdgcn_mqsad_u32_u8(w, c, m[i]);
      if (OP == 3) a[i] = __builtin_amdgcn_sad_hi_u8(b, c, a[i]);
    }
    asm volatile("" : "+v"(b), "+v"(c), "+v"(w));
  }
  unsigned r = 0;
#pragma unroll
  for (int i = 0; i < kChains; ++i) r += a[i] + (unsigned)q[i] + (unsigned)(q[i] >> 32) + m[i].x + m[i].y + m[i].z + m[i].w;
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
  unsigned *d;
  const int blocks_max = 256 * 8;
  CHK(hipMalloc(&d, blocks_max * 256 * 4));
  const char *names[] = {"v_sad_u8", "v_qsad_pk_u16_u8", "v_mqsad_u32_u8", "v_sad_hi_u8"};
  const int absdiff[] = {4, 16, 16, 4};
  for (int wpc : {4, 8}) {   // workgroups per CU: 4 = 4 waves/SIMD, 8 = 8 waves/SIMD
    const int blocks = 256 * wpc;
    const double lane_ops = (double)blocks * 256 * kIters * kChains;
    float t[4] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks)};
    for (int i = 0; i < 4; ++i)
      printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"G_lane_ops_per_s\": %.1f, \"T_absdiff_per_s\": %.2f}\n",
             names[i], wpc, t[i], lane_ops / (t[i] * 1e-3) / 1e9, lane_ops * absdiff[i] / (t[i] * 1e-3) / 1e12);
  }
  return 0;
}
