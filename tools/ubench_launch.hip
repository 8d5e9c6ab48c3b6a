// ubench_launch.hip -- round-trip latency floor of one launch + stream sync on
// MI355X, for the drop-in's one-batch-per-miss pattern: what an empty kernel
// costs, and what each ingredient of the small-batch search kernel adds
// (grid size, a read of host-mapped memory, device-scope atomics, a fence).
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_launch.hip -o tools/ubench_launch
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_empty() {}

__global__ void k_hostread(const int *h, int *sink) {
  if (threadIdx.x == 0 && h[blockIdx.x & 63] == 12345) sink[0] = 1;
}

__global__ void k_atomics(unsigned long long *keys, int fence) {
  if ((threadIdx.x & 63) == 0) atomicMin(keys + blockIdx.x * 41 + (threadIdx.x >> 6), (unsigned long long)blockIdx.x);
  if (fence) __threadfence();
}

__global__ void k_spin(int iters, int *sink) {
  int v = threadIdx.x;
  for (int i = 0; i < iters; ++i) v = v * 1664525 + 1013904223;
  if (v == 42) sink[0] = v;
}

template <typename F>
double round_trip_us(F launch, hipStream_t s, int reps) {
  for (int i = 0; i < 20; ++i) { launch(); (void)hipStreamSynchronize(s); }
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; ++i) { launch(); (void)hipStreamSynchronize(s); }
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

template <typename F>
double gpu_us(F launch, hipStream_t s, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  double tot = 0;
  for (int i = 0; i < reps; ++i) {
    (void)hipEventRecord(a, s);
    launch();
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    tot += ms * 1e3;
  }
  return tot / reps;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  int *h, *sink;
  unsigned long long *keys;
  CK(hipHostMalloc(&h, 4096, hipHostMallocMapped));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&keys, 4096 * 41 * 8));
  int *dh = nullptr;
  CK(hipHostGetDevicePointer((void **)&dh, h, 0));
  const int reps = 500;
  auto line = [&](const char *what, double rt, double g) { printf("{\"case\": \"%s\", \"round_trip_us\": %.2f, \"event_us\": %.2f}\n", what, rt, g); };
  for (int grid : {1, 8, 64, 512, 4096}) {
    auto f = [&] { hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s); };
    char n[64]; snprintf(n, sizeof n, "empty grid %d", grid);
    line(n, round_trip_us(f, s, reps), gpu_us(f, s, reps));
  }
  for (int grid : {8, 64, 512}) {
    auto f = [&] { hipLaunchKernelGGL(k_hostread, dim3(grid), dim3(256), 0, s, dh, sink); };
    char n[64]; snprintf(n, sizeof n, "host-mapped read grid %d", grid);
    line(n, round_trip_us(f, s, reps), gpu_us(f, s, reps));
  }
  for (int fence : {0, 1})
    for (int grid : {8, 64, 512}) {
      auto f = [&] { hipLaunchKernelGGL(k_atomics, dim3(grid), dim3(256), 0, s, keys, fence); };
      char n[64]; snprintf(n, sizeof n, "atomics grid %d fence %d", grid, fence);
      line(n, round_trip_us(f, s, reps), gpu_us(f, s, reps));
    }
  for (int iters : {1000, 10000}) {
    auto f = [&] { hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s, iters, sink); };
    char n[64]; snprintf(n, sizeof n, "spin %d grid 64", iters);
    line(n, round_trip_us(f, s, reps), gpu_us(f, s, reps));
  }
  // back to back: 4 empty launches then one sync (the cost of a launch alone)
  {
    auto f = [&] { for (int i = 0; i < 4; ++i) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, s); };
    line("4 empty launches grid 64 then sync", round_trip_us(f, s, reps), gpu_us(f, s, reps));
  }
  return 0;
}
