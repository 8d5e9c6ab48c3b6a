// ubench_occ.hip -- VALU issue rate of the full-search sweep's instruction mix
// against the number of waves resident per SIMD (1, 2, 3, 4, 6, 8): tells
// whether the item kernel (4 waves per SIMD) is held back by per-wave issue
// (a wave alone issues one VALU instruction per ~4 cycles; the SIMD-32 pipe
// takes a full-rate one every 2) or by the pipe itself.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_occ.hip -o tools/ubench_occ
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int kIters = 1024;

// OP 0: v_sad_hi_u8 (SGPR operand), 12 chains
// OP 1: v_add3_u32, 12 chains
// OP 2: v_min_u32, 12 chains
// OP 3: v_min3_u32, 12 chains
// OP 4: the sweep's mix per row: 12 v_sad_hi_u8 + 5 v_add3_u32 + 5 v_min_u32 + 4 v_add_u32
// OP 5: v_add_u32 (VOP2), 6: v_add_f32, 7: v_min_f32, 8: v_pk_add_f32 (2 lanes' worth), 9: v_fma_f32,
// 10: v_pk_min_u16, all 12 chains
template <int OP>
__global__ __launch_bounds__(256) void k(unsigned *out, unsigned seed) {
  unsigned a[12], m[5];
  const unsigned s0 = __builtin_amdgcn_readfirstlane(seed * 7u + 1u);
  unsigned b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x;
#pragma unroll
  for (int i = 0; i < 12; ++i) a[i] = seed + i * 7919u + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 5; ++i) m[i] = ~0u - i;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      if (OP == 0 || OP == 4) {
        unsigned r;
        asm volatile("v_sad_hi_u8 %0, %1, %2, %3" : "=v"(r) : "v"(b), "s"(s0), "v"(a[i]));
        a[i] = r;
      }
      if (OP == 1) { unsigned r; asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a[i]), "v"(b), "v"(c)); a[i] = r; }
      if (OP == 2) { unsigned r; asm volatile("v_min_u32 %0, %1, %2" : "=v"(r) : "v"(a[i]), "v"(b)); a[i] = r; }
      if (OP == 3) { unsigned r; asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a[i]), "v"(b), "v"(c)); a[i] = r; }
      if (OP == 5) { unsigned r; asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a[i]), "v"(b)); a[i] = r; }
      if (OP == 6) { unsigned r; asm volatile("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a[i]), "v"(b)); a[i] = r; }
      if (OP == 7) { unsigned r; asm volatile("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a[i]), "v"(b)); a[i] = r; }
      if (OP == 8 && i < 6) {
        unsigned long long r, x = ((unsigned long long)a[2 * i + 1] << 32) | a[2 * i], y = ((unsigned long long)c << 32) | b;
        asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
        a[2 * i] = (unsigned)r; a[2 * i + 1] = (unsigned)(r >> 32);
      }
      if (OP == 9) { unsigned r; asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a[i]), "v"(b), "v"(c)); a[i] = r; }
      if (OP == 10) { unsigned r; asm volatile("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a[i]), "v"(b)); a[i] = r; }
    }
    if (OP == 4) {
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        unsigned r, q;
        asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a[i]), "v"(a[i + 5]), "v"(c));
        asm volatile("v_min_u32 %0, %1, %2" : "=v"(q) : "v"(m[i]), "v"(r));
        m[i] = q;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) { unsigned r; asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a[i + 8]), "v"(b)); a[i + 8] = r; }
    }
    asm volatile("" : "+v"(b), "+v"(c));
  }
  unsigned r = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) r += a[i];
#pragma unroll
  for (int i = 0; i < 5; ++i) r += m[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
float run(unsigned *d, int blocks) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u + r);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
  return ms / 5;
}

// shader clock: s_memtime (core clock) against s_memrealtime (100 MHz)
__global__ void clk(unsigned long long *o) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  unsigned a = threadIdx.x;
  for (int i = 0; i < 200000; ++i) asm volatile("v_add_u32 %0, %0, 1" : "+v"(a));
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) { o[0] = t1 - t0; o[1] = r1 - r0; o[2] = a; }
}

int main() {
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned *d;
  CHK(hipMalloc(&d, (size_t)cus * 8 * 256 * 4));
  const char *names[] = {"v_sad_hi_u8 (sgpr)", "v_add3_u32", "v_min_u32", "v_min3_u32", "sweep mix 12 sad:5 add3:5 min:4 add",
                         "v_add_u32", "v_add_f32", "v_min_f32", "v_pk_add_f32", "v_fma_f32", "v_pk_min_u16"};
  const int per_iter[] = {12, 12, 12, 12, 26, 12, 12, 12, 6, 12, 12};
  const int occ[] = {1, 2, 3, 4, 6, 8};
  for (int o : occ) {
    const int blocks = cus * o;   // o workgroups of 4 waves per CU = o waves per SIMD
    float t[11] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks), run<4>(d, blocks),
                   run<5>(d, blocks), run<6>(d, blocks), run<7>(d, blocks), run<8>(d, blocks), run<9>(d, blocks),
                   run<10>(d, blocks)};
    for (int i = 0; i < 11; ++i) {
      // wave-instructions issued per SIMD, and the SIMD's rate of them
      const double per_simd = (double)o * kIters * per_iter[i];
      printf("{\"waves_per_simd\": %d, \"op\": \"%s\", \"ms\": %.4f, \"ns_per_wave_inst_per_simd\": %.3f}\n", o, names[i],
             t[i], t[i] * 1e6 / per_simd);
    }
  }
  unsigned long long *dc, hc[3];
  CHK(hipMalloc(&dc, 24));
  hipLaunchKernelGGL(clk, dim3(cus * 4), dim3(256), 0, 0, dc);
  CHK(hipMemcpy(hc, dc, 24, hipMemcpyDeviceToHost));
  printf("{\"shader_clock_mhz\": %.1f, \"memtime_ticks\": %llu, \"realtime_ticks\": %llu}\n",
         (double)hc[0] / ((double)hc[1] * 10.0) * 1000.0, hc[0], hc[1]);
  return 0;
}
