// ubench_sad.hip -- semantics and measured throughput of the gfx950 byte-SAD
// instruction family (v_sad_u8, v_qsad_pk_u16_u8, v_mqsad_pk_u16_u8,
// v_mqsad_u32_u8, v_sad_u16) and of the packed/3-operand integer ops a
// SAD-surface kernel is built from.  The semantic check compares each
// instruction with a host model on random operands, so the search kernels can
// rely on the exact behaviour measured here.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_sad.hip -o tools/ubench_sad
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef unsigned short us2 __attribute__((ext_vector_type(2)));

constexpr int kIters = 2048;
constexpr int kChains = 8;

// OP: 0 sad_u8, 1 qsad_pk, 2 mqsad_pk, 3 mqsad_u32, 4 sad_u16, 5 add_u32,
//     6 pk_add_u16, 7 pk_min_u16, 8 min3_u32, 9 add3_u32, 10 mad_u32_u16 (op_sel hi),
//     11 lshl_add_u32, 12 alignbyte
template <int OP>
__global__ __launch_bounds__(256) void tput(unsigned *out, unsigned seed) {
  unsigned a[kChains];
  unsigned long long q[kChains];
  u4 w[kChains];
  unsigned b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x;
  unsigned long long s0 = ((unsigned long long)c << 32) | b;
#pragma unroll
  for (int i = 0; i < kChains; ++i) {
    a[i] = seed + i * 7919u + threadIdx.x;
    q[i] = a[i];
    w[i] = u4{a[i], a[i] + 1, a[i] + 2, a[i] + 3};
  }
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < kChains; ++i) {
      if (OP == 0) a[i] = __builtin_amdgcn_sad_u8(b, c, a[i]);
      if (OP == 1) q[i] = __builtin_amdgcn_qsad_pk_u16_u8(s0, c, q[i]);
      if (OP == 2) q[i] = __builtin_amdgcn_mqsad_pk_u16_u8(s0, c, q[i]);
      if (OP == 3) w[i] = __builtin_amdgcn_mqsad_u32_u8(s0, c, w[i]);
      if (OP == 4) a[i] = __builtin_amdgcn_sad_u16(b, c, a[i]);
      if (OP == 5) a[i] = a[i] + b;
      if (OP == 6) { us2 x = __builtin_bit_cast(us2, a[i]), y = __builtin_bit_cast(us2, b); a[i] = __builtin_bit_cast(unsigned, x + y); }
      if (OP == 7) { us2 x = __builtin_bit_cast(us2, a[i]), y = __builtin_bit_cast(us2, b); a[i] = __builtin_bit_cast(unsigned, __builtin_elementwise_min(x, y)); }
      if (OP == 8) a[i] = min(min(a[i], b), c);
      if (OP == 9) a[i] = a[i] + b + c;
      if (OP == 10) { unsigned r; asm volatile("v_mad_u32_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"(r) : "v"(b), "v"(c), "v"(a[i])); a[i] = r; }
      if (OP == 11) a[i] = (b << 15) + a[i];
      if (OP == 12) a[i] = __builtin_amdgcn_alignbyte(a[i], b, c);
    }
    asm volatile("" : "+v"(b), "+v"(c));
    s0 = ((unsigned long long)c << 32) | b;
  }
  unsigned r = 0;
#pragma unroll
  for (int i = 0; i < kChains; ++i) r += a[i] + (unsigned)q[i] + (unsigned)(q[i] >> 32) + w[i].x + w[i].y + w[i].z + w[i].w;
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
float run(unsigned *d, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(tput<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(tput<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u + r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

// semantics: one instruction per lane on random operands
__global__ void sem(const unsigned long long *s0, const unsigned *s1, const unsigned long long *acc64,
                    const u4 *acc128, unsigned long long *o_qsad, unsigned long long *o_mqsad, u4 *o_mq32,
                    unsigned *o_sad16, unsigned *o_mad, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  o_qsad[i] = __builtin_amdgcn_qsad_pk_u16_u8(s0[i], s1[i], acc64[i]);
  o_mqsad[i] = __builtin_amdgcn_mqsad_pk_u16_u8(s0[i], s1[i], acc64[i]);
  o_mq32[i] = __builtin_amdgcn_mqsad_u32_u8(s0[i], s1[i], acc128[i]);
  o_sad16[i] = __builtin_amdgcn_sad_u16((unsigned)s0[i], s1[i], (unsigned)acc64[i]);
  unsigned r;
  asm volatile("v_mad_u32_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"(r) : "v"((unsigned)s0[i]), "v"(s1[i]), "v"((unsigned)acc64[i]));
  o_mad[i] = r;
}

static unsigned sad4(unsigned a, unsigned b, bool masked) {
  unsigned s = 0;
  for (int k = 0; k < 4; ++k) {
    int x = (a >> (8 * k)) & 255, y = (b >> (8 * k)) & 255;
    if (masked && y == 0) continue;
    s += (unsigned)abs(x - y);
  }
  return s;
}

int main() {
  // ---- semantics
  const int n = 1 << 16;
  std::vector<unsigned long long> s0(n), acc64(n), oq(n), om(n);
  std::vector<unsigned> s1(n), o16(n), omad(n);
  std::vector<u4> acc128(n), om32(n);
  srand(12345);
  auto r32 = [] { return ((unsigned)rand() << 16) ^ (unsigned)rand(); };
  for (int i = 0; i < n; ++i) {
    s0[i] = ((unsigned long long)r32() << 32) | r32();
    s1[i] = r32();
    if (i % 7 == 0) s1[i] &= 0x00ff00ffu;   // zero bytes (masked variants)
    if (i % 5 == 0) s0[i] &= 0xff00ff00ff00ff00ull;
    // accumulators: small (realistic) and near the 16-bit top (wrap/clamp behaviour)
    unsigned long long a = 0;
    for (int k = 0; k < 4; ++k) a |= (unsigned long long)((i % 3 == 0) ? (65535 - (r32() & 1023)) : (r32() & 4095)) << (16 * k);
    acc64[i] = a;
    acc128[i] = u4{r32() & 0xfffff, r32() & 0xfffff, r32(), r32() & 0xfffff};
  }
  unsigned long long *d_s0, *d_a64, *d_oq, *d_om;
  unsigned *d_s1, *d_o16, *d_mad;
  u4 *d_a128, *d_o32;
  CHK(hipMalloc(&d_s0, n * 8)); CHK(hipMalloc(&d_a64, n * 8)); CHK(hipMalloc(&d_oq, n * 8)); CHK(hipMalloc(&d_om, n * 8));
  CHK(hipMalloc(&d_s1, n * 4)); CHK(hipMalloc(&d_o16, n * 4)); CHK(hipMalloc(&d_mad, n * 4));
  CHK(hipMalloc(&d_a128, n * 16)); CHK(hipMalloc(&d_o32, n * 16));
  CHK(hipMemcpy(d_s0, s0.data(), n * 8, hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_a64, acc64.data(), n * 8, hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_s1, s1.data(), n * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_a128, acc128.data(), n * 16, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(sem, dim3(n / 256), dim3(256), 0, 0, d_s0, d_s1, d_a64, d_a128, d_oq, d_om, d_o32, d_o16, d_mad, n);
  CHK(hipDeviceSynchronize());
  CHK(hipMemcpy(oq.data(), d_oq, n * 8, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(om.data(), d_om, n * 8, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(om32.data(), d_o32, n * 16, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(o16.data(), d_o16, n * 4, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(omad.data(), d_mad, n * 4, hipMemcpyDeviceToHost));
  // model: result lane k = acc lane k + SAD(bytes k..k+3 of src0, src1); 16-bit lanes
  // either wrap (mod 2^16) or clamp -- count both
  long bad_q_wrap = 0, bad_q_clamp = 0, bad_m_wrap = 0, bad_m_clamp = 0, bad_m32 = 0, bad_m32_nomask = 0, bad16 = 0, badmad = 0;
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < 4; ++k) {
      const unsigned win = (unsigned)(s0[i] >> (8 * k));
      const unsigned acc = (unsigned)(acc64[i] >> (16 * k)) & 0xffff;
      const unsigned gq = (unsigned)(oq[i] >> (16 * k)) & 0xffff, gm = (unsigned)(om[i] >> (16 * k)) & 0xffff;
      const unsigned eq = acc + sad4(win, s1[i], false), em = acc + sad4(win, s1[i], true);
      bad_q_wrap += gq != (eq & 0xffff);
      bad_q_clamp += gq != (eq > 0xffff ? 0xffff : eq);
      bad_m_wrap += gm != (em & 0xffff);
      bad_m_clamp += gm != (em > 0xffff ? 0xffff : em);
      const unsigned a32 = acc128[i][k];
      bad_m32 += om32[i][k] != a32 + sad4(win, s1[i], true);
      bad_m32_nomask += om32[i][k] != a32 + sad4(win, s1[i], false);
    }
    unsigned e16 = (unsigned)acc64[i];
    for (int k = 0; k < 2; ++k) e16 += (unsigned)abs((int)(((unsigned)s0[i] >> (16 * k)) & 0xffff) - (int)((s1[i] >> (16 * k)) & 0xffff));
    bad16 += o16[i] != e16;
    badmad += omad[i] != (((unsigned)s0[i] >> 16) * (s1[i] & 0xffff) + (unsigned)acc64[i]);
  }
  printf("{\"semantics\": {\"n\": %d, \"qsad_pk_wrap_bad\": %ld, \"qsad_pk_clamp_bad\": %ld, \"mqsad_pk_wrap_bad\": %ld, "
         "\"mqsad_pk_clamp_bad\": %ld, \"mqsad_u32_masked_bad\": %ld, \"mqsad_u32_unmasked_bad\": %ld, \"sad_u16_bad\": %ld, "
         "\"mad_u32_u16_opsel_hi_bad\": %ld}}\n",
         n, bad_q_wrap, bad_q_clamp, bad_m_wrap, bad_m_clamp, bad_m32, bad_m32_nomask, bad16, badmad);

  // ---- throughput
  const int blocks = 256 * 8;
  unsigned *d;
  CHK(hipMalloc(&d, blocks * 256 * 4));
  const double lane_ops = (double)blocks * 256 * kIters * kChains;
  const char *names[] = {"v_sad_u8", "v_qsad_pk_u16_u8", "v_mqsad_pk_u16_u8", "v_mqsad_u32_u8", "v_sad_u16",
                         "v_add_u32", "v_pk_add_u16", "v_pk_min_u16", "v_min3_u32", "v_add3_u32",
                         "v_mad_u32_u16 op_sel", "v_lshl_add_u32", "v_alignbyte_b32"};
  const int absdiff[] = {4, 16, 16, 16, 2, 0, 0, 0, 0, 0, 0, 0, 0};
  float t[13] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks), run<4>(d, blocks),
                 run<5>(d, blocks), run<6>(d, blocks), run<7>(d, blocks), run<8>(d, blocks), run<9>(d, blocks),
                 run<10>(d, blocks), run<11>(d, blocks), run<12>(d, blocks)};
  for (int i = 0; i < 13; ++i)
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"G_lane_ops_per_s\": %.1f, \"T_absdiff_per_s\": %.2f}\n", names[i], t[i],
           lane_ops / (t[i] * 1e-3) / 1e9, lane_ops * absdiff[i] / (t[i] * 1e-3) / 1e12);
  return 0;
}
