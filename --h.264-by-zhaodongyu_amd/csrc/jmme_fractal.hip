// jmme_fractal.hip -- gfx950 kernels for the thesis codec's fractal
// domain-range block matching, ZL =
// /root/reference/2.论文程序/ZhangLing_Yu_version1/H264Fractal:
//
//   compute_domain_Sum / compute_range_Sum   ZL/src/compute.c:277-~1091   (box sums)
//   compute_rms + compute_rdSum + QUAN_A     ZL/src/compute.c:6-215,
//                                            ZL/inc/defines_enc.h:19-22, 591-601
//   full_search + bound_chk                  ZL/src/block_enc.c:1933-1977, 2894-2919
//
// Exactness.  Every sum the thesis keeps in doubles (Σd, Σd², Σr, Σr², Σrd,
// n·Σd² − (Σd)², n·Σrd − Σr·Σd) is an integer below 2^53, so it is formed in
// integer arithmetic here (v_sad_u8 / v_dot4_u32_u8) and converted: the same
// doubles.  The remaining FP64 steps -- α = num/det, (int)(α·100), a/100 and
// the rms polynomial -- are evaluated with the thesis's operand order and no
// FMA contraction (#pragma clang fp contract(off)), IEEE-rounded division
// included, so every candidate's rms is bit-identical to the thesis's.  The
// search returns the lexicographic minimum of (rms, spiral rank), which is
// what full_search's strict '<' walk over its spiral keeps.
//
// Mapping: one wave per range block (request); the (2R+1)^2 spiral ranks are
// dealt across its 64 lanes; domain rows are read as aligned dwords from a
// "words" image of the reference (word[y][x] = pels x..x+3, built once per
// reference) that stays cache-resident; the range block sits in LDS and is
// read by broadcast.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "jmme.h"
#include "jmme_fractal_device.h"
#include "jmme_fractal_internal.h"

namespace jmme {

namespace {

constexpr int kWG = 256;
constexpr int kWaves = kWG / 64;

// lexicographic (rms, rank) minimum across the wave; lane 0 ends with it
__device__ __forceinline__ void wave_min(double &rms, int &rank, int &a) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double o_rms = __shfl_xor(rms, off, 64);
    const int o_rank = __shfl_xor(rank, off, 64);
    const int o_a = __shfl_xor(a, off, 64);
    if (o_rms < rms || (o_rms == rms && o_rank < rank)) { rms = o_rms; rank = o_rank; a = o_a; }
  }
}

template <int BSX, int BSY>
__device__ __forceinline__ void search_one(const FractalParams &p, const jmme_fractal_req &rq, uint32_t *rng,
                                           int lane, jmme_fractal_res *out) {
  constexpr int NQ = BSX / 4;            // dwords per row
  constexpr int ND = NQ * BSY;           // dwords per block
  constexpr int NO = BSX * BSY;
  const int bx = rq.block_x, by = rq.block_y;
  // range block -> LDS (per wave), and its sums
  unsigned s1 = 0, s2 = 0;
  if (lane < ND) {
    const int r = lane / NQ, q = lane - r * NQ;
    const uint32_t v = *reinterpret_cast<const uint32_t *>(p.org + (size_t)(by + r) * p.pitch + bx + 4 * q);
    rng[lane] = v;
    s1 = __builtin_amdgcn_sad_u8(v, 0u, 0u);
    s2 = __builtin_amdgcn_udot4(v, v, 0u, false);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    s1 += __shfl_xor(s1, off, 64);
    s2 += __shfl_xor(s2, off, 64);
  }
  RangeStats rg;
  rg.rs1 = (double)s1;
  rg.rs2 = (double)s2;
  {
#pragma clang fp contract(off)
    rg.beta = (double)quan_a((int)(rg.rs1 / NO));    // beta = QUAN_A(rsum1 / no), compute.c:161-164
  }
  rg.bad_beta = rg.beta < -60 || rg.beta > 255;
  __builtin_amdgcn_wave_barrier();

  // bound_chk window (block_enc.c:2894-2919)
  const int R = p.range;
  const int ilow = max(bx - R, 0), ihigh = min(bx + R, p.width - BSX);
  const int jlow = max(by - R, 0), jhigh = min(by + R, p.height - BSY);
  const int ncand = (2 * R + 1) * (2 * R + 1);
  double best = 1e30 * 2;   // above any rms, so rank decides among equals
  int best_rank = 0x7fffffff, best_a = 0;
  for (int rank = lane; rank < ncand; rank += 64) {
    int i, j;
    spiral_xy(rank, i, j);
    const int m = bx + i, n = by + j;
    if (rank != 0 && !(m >= ilow && m <= ihigh && n >= jlow && n <= jhigh)) continue;
    unsigned ds1 = 0, ds2 = 0, rd = 0;
    const uint32_t *w = p.words + (size_t)n * p.wpitch + m;
#pragma unroll
    for (int r = 0; r < BSY; ++r)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const uint32_t d = w[(size_t)r * p.wpitch + 4 * q];
        ds1 = __builtin_amdgcn_sad_u8(d, 0u, ds1);
        ds2 = __builtin_amdgcn_udot4(d, d, ds2, false);
        rd = __builtin_amdgcn_udot4(rng[r * NQ + q], d, rd, false);
      }
    int a;
    const double rms = rms_of(ds1, ds2, rd, NO, rg, a);
    if (rms < best || (rms == best && rank < best_rank)) { best = rms; best_rank = rank; best_a = a; }
  }
  wave_min(best, best_rank, best_a);
  if (lane == 0) {
    int i, j;
    spiral_xy(best_rank, i, j);
    jmme_fractal_res res;
    res.rms = best;
    {
#pragma clang fp contract(off)
      res.scale = (double)best_a / 100;
    }
    res.offset = rg.beta;
    res.x = i;                  // (0,0) winner: the thesis leaves the caller's 0, 0
    res.y = j;
    *out = res;
  }
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(kWG) void fractal_search_kernel(FractalParams p) {
  __shared__ uint32_t s_rng[kWaves][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int t = blockIdx.x * kWaves + wave; t < p.n; t += gridDim.x * kWaves) {
    const jmme_fractal_req rq = p.req[t];
    uint32_t *rng = s_rng[wave];
    jmme_fractal_res *o = p.out + t;
    switch ((rq.bsx << 8) | rq.bsy) {
      case (16 << 8) | 16: search_one<16, 16>(p, rq, rng, lane, o); break;
      case (16 << 8) | 8: search_one<16, 8>(p, rq, rng, lane, o); break;
      case (8 << 8) | 16: search_one<8, 16>(p, rq, rng, lane, o); break;
      case (8 << 8) | 8: search_one<8, 8>(p, rq, rng, lane, o); break;
      case (8 << 8) | 4: search_one<8, 4>(p, rq, rng, lane, o); break;
      case (4 << 8) | 8: search_one<4, 8>(p, rq, rng, lane, o); break;
      case (4 << 8) | 4: search_one<4, 4>(p, rq, rng, lane, o); break;
      default: break;   // validated on the host
    }
  }
}

// word[y][x] = pels x..x+3 of the reference (x <= W-4), from two aligned dwords
__global__ __launch_bounds__(kWG) void words_kernel(const uint8_t *__restrict__ ref, int pitch, int W, int H,
                                                    uint32_t *__restrict__ words, int wpitch) {
  const int x = blockIdx.x * kWG + threadIdx.x, y = blockIdx.y;
  if (x > W - 4 || y >= H) return;
  const uint8_t *row = ref + (size_t)y * pitch;
  const int xa = x & ~3;
  const uint32_t lo = *reinterpret_cast<const uint32_t *>(row + xa);
  const uint32_t hi = (xa + 4 < pitch) ? *reinterpret_cast<const uint32_t *>(row + xa + 4) : 0u;
  words[(size_t)y * wpitch + x] = __builtin_amdgcn_alignbyte(hi, lo, x & 3);
}

// compute_domain_Sum for one block size: horizontal then vertical integer box
// sums, stored as doubles (exact)
__global__ __launch_bounds__(kWG) void box_hsum_kernel(const uint8_t *__restrict__ p, int pitch, int W, int H,
                                                       int bsx, uint32_t *__restrict__ hs, uint32_t *__restrict__ hs2) {
  const int x = blockIdx.x * kWG + threadIdx.x, y = blockIdx.y;
  const int w = W - bsx + 1;
  if (x >= w || y >= H) return;
  unsigned s = 0, s2 = 0;
  for (int c = 0; c < bsx; ++c) {
    const unsigned v = p[(size_t)y * pitch + x + c];
    s += v;
    s2 += v * v;
  }
  hs[(size_t)y * w + x] = s;
  hs2[(size_t)y * w + x] = s2;
}

__global__ __launch_bounds__(kWG) void box_vsum_kernel(const uint32_t *__restrict__ hs, const uint32_t *__restrict__ hs2,
                                                       int w, int H, int bsy, double *__restrict__ sum,
                                                       double *__restrict__ sum2) {
  const int x = blockIdx.x * kWG + threadIdx.x, y = blockIdx.y;
  if (x >= w || y > H - bsy) return;
  unsigned s = 0, s2 = 0;
  for (int r = 0; r < bsy; ++r) {
    s += hs[(size_t)(y + r) * w + x];
    s2 += hs2[(size_t)(y + r) * w + x];
  }
  sum[(size_t)y * w + x] = (double)s;
  sum2[(size_t)y * w + x] = (double)s2;
}

// ------------------------------------------------------------------ a17 --
// encode_one_macroblock's quadtree (block_enc.c:508-1932) as four search
// levels, each followed by a gate kernel that reduces over the views, decides
// the split and appends the next level's node ids on the device (no host
// round trip between levels).

// the gate's squared correlation (block_enc.c:760-796).  The thesis sums
// column by column (ii = x*16 + y); sR, sD are exact in any order (every
// (R-r)^2 is a multiple of 2^-16 below 2^16, so all partial sums fit 53
// bits), the 256 correlation terms are formed in parallel and then added in
// ii order by one lane, so mr is bit-identical.
__global__ __launch_bounds__(kWG) void tree_init_kernel(FractalTreeParams p) {
#pragma clang fp contract(off)
  __shared__ double s_t[kWaves][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int mb = blockIdx.x * kWaves + wave;
  if (blockIdx.x == 0 && threadIdx.x < 4) p.count[threadIdx.x] = 0;
  const bool valid = mb < p.n_mb;
  if (valid) {
    uint64_t *rec = reinterpret_cast<uint64_t *>(p.out + mb);
    for (int i = lane; i < (int)(sizeof(jmme_fractal_mb) / 8); i += 64) rec[i] = 0;
    const int bx = ((p.mb0 + mb) % p.mbs_x) * 16, by = ((p.mb0 + mb) / p.mbs_x) * 16;
    const int x = lane >> 2, y0 = (lane & 3) * 4;     // ii = x*16 + y0 + e
    int rv[4], dv[4], sr = 0, sd = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const size_t o = (size_t)(by + y0 + e) * p.pitch + bx + x;
      rv[e] = p.org[o];
      dv[e] = p.ref0[o];
      sr += rv[e];
      sd += dv[e];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      sr += __shfl_xor(sr, off, 64);
      sd += __shfl_xor(sd, off, 64);
    }
    const double r = (double)sr / 256, d = (double)sd / 256;
    double sR = 0, sD = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sR += (rv[e] - r) * (rv[e] - r);
      sD += (dv[e] - d) * (dv[e] - d);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      sR += __shfl_xor(sR, off, 64);
      sD += __shfl_xor(sD, off, 64);
    }
    const double qR = sqrt(sR), qD = sqrt(sD);
#pragma unroll
    for (int e = 0; e < 4; ++e) s_t[wave][lane * 4 + e] = ((rv[e] - r) / qR) * ((dv[e] - d) / qD);
  }
  __syncthreads();
  if (valid && lane == 0) {
    double mr = 0;
    for (int ii = 0; ii < 256; ++ii) mr += s_t[wave][ii];
    p.out[mb].chun = mr * mr;
  }
}

__device__ __forceinline__ const uint32_t *view_words(const FractalTreeParams &p, int k) {
  return k == 0 ? p.words[0] : k == 1 ? p.words[1] : k == 2 ? p.words[2] : p.words[3];
}

template <int LEVEL>
__global__ __launch_bounds__(kWG) void tree_search_kernel(FractalTreeParams p) {
  __shared__ uint32_t s_rng[kWaves][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int S = LEVEL == 0 ? 1 : 4;
  const int K = p.n_refs;
  const int nodes = LEVEL == 0 ? p.n_mb : p.count[LEVEL];
  const int total = nodes * S * K;
  for (int t = blockIdx.x * kWaves + wave; t < total; t += gridDim.x * kWaves) {
    const int k = t % K, s = (t / K) % S, i = t / (K * S);
    const int id = LEVEL == 0 ? i : p.list[LEVEL][i];
    FractalParams fp;
    fp.org = p.org;
    fp.pitch = p.pitch;
    fp.words = view_words(p, k);
    fp.wpitch = p.wpitch;
    fp.width = p.width;
    fp.height = p.height;
    fp.range = p.range;
    jmme_fractal_res *o = p.res[LEVEL] + t;
    const int mb = p.mb0 + (LEVEL <= 1 ? id : id >> 2);   // ids are band-local, the picture is whole
    int bx = (mb % p.mbs_x) * 16, by = (mb / p.mbs_x) * 16;
    jmme_fractal_req rq;
    if (LEVEL == 0) {
      rq = {(int16_t)bx, (int16_t)by, 16, 16};
      search_one<16, 16>(fp, rq, s_rng[wave], lane, o);
    } else if (LEVEL == 1) {
      rq = {(int16_t)(bx + (s & 1) * 8), (int16_t)(by + (s >> 1) * 8), 8, 8};
      search_one<8, 8>(fp, rq, s_rng[wave], lane, o);
    } else {
      bx += (id & 1) * 8;
      by += ((id >> 1) & 1) * 8;
      if (LEVEL == 3) {
        rq = {(int16_t)(bx + (s & 1) * 4), (int16_t)(by + (s >> 1) * 4), 4, 4};
        search_one<4, 4>(fp, rq, s_rng[wave], lane, o);
      } else if (s < 2) {          // 8x4 pair, encode_block_rect mode 1 depth 2
        rq = {(int16_t)bx, (int16_t)(by + 4 * s), 8, 4};
        search_one<8, 4>(fp, rq, s_rng[wave], lane, o);
      } else {                     // 4x8 pair, mode 2
        rq = {(int16_t)(bx + 4 * (s - 2)), (int16_t)by, 4, 8};
        search_one<4, 8>(fp, rq, s_rng[wave], lane, o);
      }
    }
  }
}

// first strict minimum over the views (the thesis's `if (rms_rl < rms)`
// chain); quirk4: encode_block_4 sets partition = reference = 1 when view 1
// wins (block_enc.c:1773)
__device__ __forceinline__ jmme_fractal_node pick_view(const jmme_fractal_res *r, int K, bool quirk4) {
  jmme_fractal_res b = r[0];
  int ref = 0, part = 0;
  for (int k = 1; k < K; ++k) {
    const jmme_fractal_res c = r[k];
    if (c.rms < b.rms) {
      b = c;
      ref = k;
      if (quirk4 && k == 1) part = 1;
    }
  }
  jmme_fractal_node n;
  n.rms = b.rms;
  n.scale = b.scale;
  n.offset = b.offset;
  n.x = b.x;
  n.y = b.y;
  n.reference = ref;
  n.partition = part;
  return n;
}

// wave-aggregated append; every lane of the wave calls it
__device__ __forceinline__ int append(int *count, bool pred) {
  const unsigned long long m = __ballot(pred);
  if (!m) return -1;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(count, __popcll(m));
  base = __shfl(base, leader, 64);
  return base + __popcll(m & ((1ull << lane) - 1));
}

// level 0 -> 1: encode_one_macroblock's gate (block_enc.c:797)
__global__ __launch_bounds__(kWG) void tree_gate0_kernel(FractalTreeParams p) {
  const int mb = blockIdx.x * kWG + threadIdx.x;
  bool split = false;
  if (mb < p.n_mb) {
    jmme_fractal_node n = pick_view(p.res[0] + (size_t)mb * p.n_refs, p.n_refs, false);
    const double chun = p.out[mb].chun;
    split = chun <= 1 && chun >= 0.9 && n.rms > p.thr16;
    if (split) n.partition = 3;
    p.out[mb].mb = n;
  }
  const int idx = append(p.count + 1, split);
  if (split) p.list[1][idx] = mb;
}

// level 1 -> 2: encode_block_8's test (block_enc.c:1584)
__global__ __launch_bounds__(kWG) void tree_gate1_kernel(FractalTreeParams p) {
  const int t = blockIdx.x * kWG + threadIdx.x;
  bool fail = false;
  int b8 = 0;
  if (t < p.count[1] * 4) {
    const int mb = p.list[1][t >> 2], q = t & 3;
    const jmme_fractal_node n = pick_view(p.res[1] + (size_t)t * p.n_refs, p.n_refs, false);
    p.out[mb].b8[q] = n;
    fail = n.rms > p.thr8;
    b8 = mb * 4 + q;
  }
  const int idx = append(p.count + 2, fail);
  if (fail) p.list[2][idx] = b8;
}

// level 2 -> 3: the 8x4 pair, else the 4x8 pair (block_enc.c:1586-1632; a
// pair stops at its first unmatched half, which leaves the same outcome)
__global__ __launch_bounds__(kWG) void tree_gate2_kernel(FractalTreeParams p) {
  const int t = blockIdx.x * kWG + threadIdx.x;
  bool quad = false;
  int b8 = 0;
  if (t < p.count[2]) {
    b8 = p.list[2][t];
    jmme_fractal_mb *m = p.out + (b8 >> 2);
    const int q = b8 & 3;
    jmme_fractal_node h[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) h[s] = pick_view(p.res[2] + ((size_t)t * 4 + s) * p.n_refs, p.n_refs, false);
    const bool m1 = !(h[0].rms > p.thr_pair) && !(h[1].rms > p.thr_pair);
    const bool m2 = !(h[2].rms > p.thr_pair) && !(h[3].rms > p.thr_pair);
    if (m1) {
      m->sub[q][0] = h[0];
      m->sub[q][1] = h[1];
      m->b8[q].partition = 1;
    } else if (m2) {
      m->sub[q][0] = h[2];
      m->sub[q][1] = h[3];
      m->b8[q].partition = 2;
    } else {
      m->b8[q].partition = 3;
      quad = true;
    }
  }
  const int idx = append(p.count + 3, quad);
  if (quad) p.list[3][idx] = b8;
}

// level 3: the four 4x4 (encode_block_4)
__global__ __launch_bounds__(kWG) void tree_gate3_kernel(FractalTreeParams p) {
  const int t = blockIdx.x * kWG + threadIdx.x;
  if (t >= p.count[3] * 4) return;
  const int b8 = p.list[3][t >> 2], s = t & 3;
  p.out[b8 >> 2].sub[b8 & 3][s] = pick_view(p.res[3] + (size_t)t * p.n_refs, p.n_refs, true);
}

// ------------------------------------------------------------ decoder --
// decode_one_macroblock / decode_block_rect / _8 / _4 (ZL/src/block_dec.c:
// 20-1160), num_regions == 1.  The view a leaf reads depends on the level,
// the component and the reference index (the thesis's per-level branches,
// quirks included -- see oracle/fractal_oracle.c fro_leaf_view).
enum { kL16, kL8, kL84, kL48, kL4 };

__device__ __forceinline__ int leaf_view(int kind, int component, int ref) {
  switch (kind) {
    case kL16: return (ref >= 0 && ref <= 3) ? ref : -1;            // :126-209
    case kL8: return ref == 0 ? 0 : 1;                              // :861-904
    case kL84:
    case kL48: return (ref == 0 || ref == 1 || ref == 2) ? ref : 3; // :558-701
    default:                                                        // :1078-1146
      if (component == 3) return ref == 0 ? 0 : ref == 2 ? 2 : 3;   // V repeats `reference==0` (:1135)
      return (ref == 0 || ref == 1 || ref == 2) ? ref : 3;
  }
}

// one workgroup per macroblock, one thread per pel; each leaf's domain box sum
// is accumulated in LDS (exact integers), then every pel evaluates the
// thesis's expression in its operand order
__global__ __launch_bounds__(kWG) void fractal_decode_kernel(FractalDecodeParams p) {
#pragma clang fp contract(off)
  __shared__ int s_sum[16];
  const int m = blockIdx.x, t = threadIdx.x;
  const int px = t & 15, py = t >> 4;
  if (t < 16) s_sum[t] = 0;
  __syncthreads();
  const jmme_fractal_mb &mb = p.mbs[m];
  const int bx = (m % p.mbs_x) * 16, by = (m / p.mbs_x) * 16;
  const jmme_fractal_node *node;
  int kind, lx, ly, bsx, bsy;
  if (mb.mb.partition == 0) {
    node = &mb.mb; kind = kL16; lx = 0; ly = 0; bsx = 16; bsy = 16;
  } else {
    const int q = (py >> 3) * 2 + (px >> 3);
    const int x8 = (px >> 3) * 8, y8 = (py >> 3) * 8;
    const int part = mb.b8[q].partition;
    if (part == 0) {
      node = &mb.b8[q]; kind = kL8; lx = x8; ly = y8; bsx = 8; bsy = 8;
    } else if (part == 1) {
      const int h = (py & 7) >> 2;
      node = &mb.sub[q][h]; kind = kL84; lx = x8; ly = y8 + 4 * h; bsx = 8; bsy = 4;
    } else if (part == 2) {
      const int h = (px & 7) >> 2;
      node = &mb.sub[q][h]; kind = kL48; lx = x8 + 4 * h; ly = y8; bsx = 4; bsy = 8;
    } else {
      const int c = ((py & 7) >> 2) * 2 + ((px & 7) >> 2);
      node = &mb.sub[q][c]; kind = kL4; lx = x8 + (c & 1) * 4; ly = y8 + (c >> 1) * 4; bsx = 4; bsy = 4;
    }
  }
  const int leaf = (ly >> 2) * 4 + (lx >> 2);
  const int v = leaf_view(kind, p.component, node->reference);
  const int dx = bx + lx + node->x, dy = by + ly + node->y;
  const bool ok = v >= 0 && v < p.n_views && dx >= 0 && dy >= 0 && dx + bsx <= p.width && dy + bsy <= p.height;
  int d = 0;
  if (ok) d = p.views[v][(size_t)(dy + py - ly) * p.pitch + dx + px - lx];
  else if (p.status) atomicOr(p.status, 1);
  atomicAdd(&s_sum[leaf], d);
  __syncthreads();
  const double scale = node->scale, offset = node->offset;
  const double average_domain = (double)s_sum[leaf] / (double)(bsx * bsy);
  const double a = 0.5 + scale * d + offset - scale * average_domain;
  p.rec[(size_t)(by + py) * p.pitch + bx + px] = ok ? (uint8_t)(a < 0.0 ? 0 : (a > 255.0 ? 255 : a)) : 0;
}

}  // namespace

hipError_t launch_fractal_decode(const FractalDecodeParams &p, hipStream_t s) {
  if (p.n_mb > 0) hipLaunchKernelGGL(fractal_decode_kernel, dim3(p.n_mb), dim3(kWG), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_fractal_words(const uint8_t *ref, int pitch, int W, int H, uint32_t *words, int wpitch,
                                hipStream_t s) {
  hipLaunchKernelGGL(words_kernel, dim3((W + kWG - 1) / kWG, H), dim3(kWG), 0, s, ref, pitch, W, H, words, wpitch);
  return hipGetLastError();
}

hipError_t launch_fractal_search(const FractalParams &p, hipStream_t s) {
  int grid = (p.n + kWaves - 1) / kWaves;
  if (grid > 65535) grid = 65535;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(fractal_search_kernel, dim3(grid), dim3(kWG), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_box_sums(const uint8_t *p, int pitch, int W, int H, int bsx, int bsy, uint32_t *hs, uint32_t *hs2,
                           double *sum, double *sum2, hipStream_t s) {
  const int w = W - bsx + 1;
  hipLaunchKernelGGL(box_hsum_kernel, dim3((w + kWG - 1) / kWG, H), dim3(kWG), 0, s, p, pitch, W, H, bsx, hs, hs2);
  hipLaunchKernelGGL(box_vsum_kernel, dim3((w + kWG - 1) / kWG, H - bsy + 1), dim3(kWG), 0, s, hs, hs2, w, H, bsy,
                     sum, sum2);
  return hipGetLastError();
}

hipError_t launch_fractal_tree(const FractalTreeParams &p, hipStream_t s) {
  const int n = p.n_mb, K = p.n_refs;
  auto waves = [](long long w) { return (int)std::min<long long>(std::max<long long>((w + kWaves - 1) / kWaves, 1), 4096); };
  auto threads = [](long long t) { return (int)std::max<long long>((t + kWG - 1) / kWG, 1); };
  hipLaunchKernelGGL(tree_init_kernel, dim3((n + kWaves - 1) / kWaves), dim3(kWG), 0, s, p);
  hipLaunchKernelGGL(tree_search_kernel<0>, dim3(waves((long long)n * K)), dim3(kWG), 0, s, p);
  hipLaunchKernelGGL(tree_gate0_kernel, dim3(threads(n)), dim3(kWG), 0, s, p);
  hipLaunchKernelGGL(tree_search_kernel<1>, dim3(waves((long long)n * 4 * K)), dim3(kWG), 0, s, p);
  hipLaunchKernelGGL(tree_gate1_kernel, dim3(threads(4LL * n)), dim3(kWG), 0, s, p);
  hipLaunchKernelGGL(tree_search_kernel<2>, dim3(waves((long long)n * 16 * K)), dim3(kWG), 0, s, p);
  hipLaunchKernelGGL(tree_gate2_kernel, dim3(threads(4LL * n)), dim3(kWG), 0, s, p);
  hipLaunchKernelGGL(tree_search_kernel<3>, dim3(waves((long long)n * 16 * K)), dim3(kWG), 0, s, p);
  hipLaunchKernelGGL(tree_gate3_kernel, dim3(threads(16LL * n)), dim3(kWG), 0, s, p);
  return hipGetLastError();
}

}  // namespace jmme
