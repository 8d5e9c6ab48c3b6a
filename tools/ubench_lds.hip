// ubench_lds.hip -- facts the v5 full-search sweep is built on, measured on the
// box rather than assumed:
//   * v_sad_hi_u8 semantics (D = (SAD(S0,S1) << 16) + S2, modulo 2^32) and
//     throughput, and v_sad_u8 with its current-block operand in an SGPR;
//   * the unsigned saturating add (uadd.sat -> v_add_u32 ... clamp);
//   * LDS: ds_read_b32 at byte addresses that are not 4-aligned (result and
//     rate), ds_read2_b32 (the v4 window read) and a broadcast ds_read_b128
//     (the v4 current-MB read), in wave-instructions per CU per clock.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_lds.hip -o tools/ubench_lds
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int kIters = 2048;
constexpr int kChains = 8;

// ---------------------------------------------------------------- semantics
__global__ void sem(const unsigned *a, const unsigned *b, const unsigned *c, unsigned *o_hi, unsigned *o_sat,
                    unsigned *o_lds, int n) {
  __shared__ unsigned char buf[1024 + 64];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  // LDS image: byte k = (k * 37 + 11) & 255
  for (int k = threadIdx.x; k < 1024 + 64; k += blockDim.x) buf[k] = (unsigned char)((k * 37 + 11) & 255);
  __syncthreads();
  if (i >= n) return;
  o_hi[i] = __builtin_amdgcn_sad_hi_u8(a[i], b[i], c[i]);
  o_sat[i] = __builtin_elementwise_add_sat(a[i], c[i]);
  const unsigned addr = (unsigned)(uintptr_t)(buf) + (unsigned)(i & 1023);
  unsigned v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  o_lds[i] = v;
}

// ---------------------------------------------------------------- VALU rates
// OP 0: v_sad_hi_u8, 1: v_sad_u8 with an SGPR current operand, 2: v_sad_u8 (VGPRs),
//    3: uadd.sat, 4: v_add_u32
template <int OP>
__global__ __launch_bounds__(256) void tput(unsigned *out, unsigned seed) {
  unsigned a[kChains];
  unsigned b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x;
  const unsigned su = __builtin_amdgcn_readfirstlane(seed * 7u + blockIdx.x);
#pragma unroll
  for (int i = 0; i < kChains; ++i) a[i] = seed + i * 7919u + threadIdx.x;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < kChains; ++i) {
      if (OP == 0) a[i] = __builtin_amdgcn_sad_hi_u8(b, c, a[i]);
      if (OP == 1) { unsigned r; asm volatile("v_sad_u8 %0, %1, %2, %3" : "=v"(r) : "v"(b), "s"(su), "v"(a[i])); a[i] = r; }
      if (OP == 2) a[i] = __builtin_amdgcn_sad_u8(b, c, a[i]);
      if (OP == 3) a[i] = __builtin_elementwise_add_sat(a[i], b);
      if (OP == 4) a[i] = a[i] + b;
    }
    asm volatile("" : "+v"(b), "+v"(c));
  }
  unsigned r = 0;
#pragma unroll
  for (int i = 0; i < kChains; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// ---------------------------------------------------------------- LDS rates
// MODE 0: ds_read2_b32 offsets 0/16 B at lane*4 (+row)  -- the v4 window read
//      1: ds_read_b32 at byte address lane + k (unaligned, consecutive bytes per lane)
//      2: ds_read_b128 broadcast (every lane the same address) -- the v4 current-MB read
//      3: ds_read_b32 at lane*4 (aligned baseline)
//      4: ds_read_b64 at byte address lane + k (unaligned)
constexpr int kLdsIters = 512;
template <int MODE>
__global__ __launch_bounds__(256) void lds_tput(unsigned *out, int seed) {
  __shared__ __attribute__((aligned(16))) unsigned buf[4096];
  for (int k = threadIdx.x; k < 4096; k += 256) buf[k] = k * 2654435761u + seed;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const unsigned base = (unsigned)(uintptr_t)buf;
  unsigned acc = 0;
  unsigned row = ((threadIdx.x >> 6) * 1024) & 8191;
  for (int it = 0; it < kLdsIters; ++it) {
    unsigned v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (MODE == 0) {
        const unsigned ad = base + row + 4u * lane + 320u * k;
        unsigned long long t;
        asm volatile("ds_read2_b32 %0, %1 offset1:4" : "=v"(t) : "v"(ad));
        v[k] = (unsigned)t ^ (unsigned)(t >> 32);
      }
      if (MODE == 1) {
        const unsigned ad = base + row + lane + 1u + 80u * k;
        asm volatile("ds_read_b32 %0, %1" : "=v"(v[k]) : "v"(ad));
      }
      if (MODE == 2) {
        const unsigned ad = base + row + 16u * k;
        typedef unsigned u4v __attribute__((ext_vector_type(4)));
        u4v t;
        asm volatile("ds_read_b128 %0, %1" : "=v"(t) : "v"(ad));
        v[k] = t.x ^ t.w;
      }
      if (MODE == 3) {
        const unsigned ad = base + row + 4u * lane + 320u * k;
        asm volatile("ds_read_b32 %0, %1" : "=v"(v[k]) : "v"(ad));
      }
      if (MODE == 4) {
        const unsigned ad = base + row + lane + 1u + 80u * k;
        unsigned long long t;
        asm volatile("ds_read_b64 %0, %1" : "=v"(t) : "v"(ad));
        v[k] = (unsigned)t ^ (unsigned)(t >> 32);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];
    row = (row + 512u) & 8191u;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <typename F>
float timeit(F f) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  f(0);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) f(r + 1);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  const int n = 1 << 16;
  std::vector<unsigned> a(n), b(n), c(n), ohi(n), osat(n), olds(n);
  srand(4242);
  auto r32 = [] { return ((unsigned)rand() << 16) ^ (unsigned)rand(); };
  for (int i = 0; i < n; ++i) { a[i] = r32(); b[i] = r32(); c[i] = (i & 1) ? r32() : (0xffffffffu - (r32() & 0xfffff)); }
  unsigned *da, *db, *dc, *dhi, *dsat, *dlds;
  CHK(hipMalloc(&da, n * 4)); CHK(hipMalloc(&db, n * 4)); CHK(hipMalloc(&dc, n * 4));
  CHK(hipMalloc(&dhi, n * 4)); CHK(hipMalloc(&dsat, n * 4)); CHK(hipMalloc(&dlds, n * 4));
  CHK(hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dc, c.data(), n * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(sem, dim3(n / 256), dim3(256), 0, 0, da, db, dc, dhi, dsat, dlds, n);
  CHK(hipDeviceSynchronize());
  CHK(hipMemcpy(ohi.data(), dhi, n * 4, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(osat.data(), dsat, n * 4, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(olds.data(), dlds, n * 4, hipMemcpyDeviceToHost));
  long bad_hi = 0, bad_sat = 0, bad_lds = 0;
  for (int i = 0; i < n; ++i) {
    unsigned s = 0;
    for (int k = 0; k < 4; ++k) s += (unsigned)abs((int)((a[i] >> (8 * k)) & 255) - (int)((b[i] >> (8 * k)) & 255));
    bad_hi += ohi[i] != (unsigned)((s << 16) + c[i]);
    const unsigned long long t = (unsigned long long)a[i] + c[i];
    bad_sat += osat[i] != (t > 0xffffffffull ? 0xffffffffu : (unsigned)t);
    const int k0 = i & 1023;
    unsigned e = 0;
    for (int k = 0; k < 4; ++k) e |= (unsigned)(((k0 + k) * 37 + 11) & 255) << (8 * k);
    bad_lds += olds[i] != e;
  }
  printf("{\"semantics\": {\"n\": %d, \"sad_hi_u8_bad\": %ld, \"uadd_sat_bad\": %ld, \"ds_read_b32_unaligned_bad\": %ld}}\n", n,
         bad_hi, bad_sat, bad_lds);

  const int blocks = 256 * 8;
  unsigned *d;
  CHK(hipMalloc(&d, blocks * 256 * 4));
  const double lane_ops = (double)blocks * 256 * kIters * kChains;
  const char *vn[] = {"v_sad_hi_u8", "v_sad_u8 (sgpr cur)", "v_sad_u8", "v_add_u32 clamp (uadd.sat)", "v_add_u32"};
  float tv[5] = {
      timeit([&](int r) { hipLaunchKernelGGL(tput<0>, dim3(blocks), dim3(256), 0, 0, d, 1u + r); }),
      timeit([&](int r) { hipLaunchKernelGGL(tput<1>, dim3(blocks), dim3(256), 0, 0, d, 1u + r); }),
      timeit([&](int r) { hipLaunchKernelGGL(tput<2>, dim3(blocks), dim3(256), 0, 0, d, 1u + r); }),
      timeit([&](int r) { hipLaunchKernelGGL(tput<3>, dim3(blocks), dim3(256), 0, 0, d, 1u + r); }),
      timeit([&](int r) { hipLaunchKernelGGL(tput<4>, dim3(blocks), dim3(256), 0, 0, d, 1u + r); })};
  for (int i = 0; i < 5; ++i)
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"G_lane_ops_per_s\": %.1f}\n", vn[i], tv[i], lane_ops / (tv[i] * 1e-3) / 1e9);

  int dev = 0, clk_khz = 0, cus = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const double winst = (double)blocks * 4 * kLdsIters * 8;   // wave-instructions
  const char *ln[] = {"ds_read2_b32 (lane*4, +16 B)", "ds_read_b32 unaligned (lane+1+k)", "ds_read_b128 broadcast",
                      "ds_read_b32 aligned (lane*4)", "ds_read_b64 unaligned (lane+1+k)"};
  float tl[5] = {
      timeit([&](int r) { hipLaunchKernelGGL(lds_tput<0>, dim3(blocks), dim3(256), 0, 0, d, r); }),
      timeit([&](int r) { hipLaunchKernelGGL(lds_tput<1>, dim3(blocks), dim3(256), 0, 0, d, r); }),
      timeit([&](int r) { hipLaunchKernelGGL(lds_tput<2>, dim3(blocks), dim3(256), 0, 0, d, r); }),
      timeit([&](int r) { hipLaunchKernelGGL(lds_tput<3>, dim3(blocks), dim3(256), 0, 0, d, r); }),
      timeit([&](int r) { hipLaunchKernelGGL(lds_tput<4>, dim3(blocks), dim3(256), 0, 0, d, r); })};
  for (int i = 0; i < 5; ++i) {
    // CU-clocks per wave-instruction at the nominal clock
    const double cyc = (tl[i] * 1e-3) * (clk_khz * 1e3) * cus / winst;
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"cu_clk_per_wave_inst\": %.2f, \"clock_mhz\": %d}\n", ln[i], tl[i], cyc,
           clk_khz / 1000);
  }
  return 0;
}
