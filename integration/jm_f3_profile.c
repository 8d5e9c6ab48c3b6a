/*
 * jm_f3_profile.c -- measurement only (JMME_F3_PROFILE=1): how much of a JM
 * encode the calls a speculative GPU form of SURVEY §8(f)3 would serve take on
 * the CPU, and how often they are made.  Mode decision reaches the 4x4 / 8x8
 * residual coding and the 4x4 / 8x8 distortion through function pointers that
 * JM sets per macroblock (select_transform, block.c:2390-2460) and per encoder
 * (select_distortion, me_distortion.c:148-170); both setters are wrapped
 * (ld --wrap) and, when profiling, the pointers are swapped for timed
 * trampolines that call JM's own function.  The totals are printed at exit.
 *   residual_transform_quant_luma_4x4  block.c:660-745
 *   residual_transform_quant_luma_8x8  block.c:1095-1330 (and its _cavlc form)
 *   distortion4x4 / distortion8x8      me_distortion.c:38-140
 * Without JMME_F3_PROFILE the wrappers only call through.
 */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <x86intrin.h>

#include "global.h"

typedef int (*rq4_fn)(Macroblock *, ColorPlane, int, int, int *, int);
typedef int (*rq8_fn)(Macroblock *, ColorPlane, int, int *, int);
typedef distblk (*dist_fn)(short *, distblk);

static int g_on = -1;
static rq4_fn g_rq4;
static rq8_fn g_rq8;
static dist_fn g_d4, g_d8;
static long long g_n[4];
static unsigned long long g_c[4];
static long long g_n_inter4, g_n_islice4;   /* 4x4 calls with intra == 0; calls made in I slices */
static unsigned long long g_c_inter4;
static unsigned long long g_tsc0;
static struct timespec g_ts0;

static int on(void)
{
  if (g_on < 0) {
    const char *e = getenv("JMME_F3_PROFILE");
    g_on = e && e[0] == '1';
    if (g_on) {
      clock_gettime(CLOCK_MONOTONIC, &g_ts0);
      g_tsc0 = __rdtsc();
    }
  }
  return g_on;
}

static int t_rq4(Macroblock *m, ColorPlane pl, int bx, int by, int *cc, int intra)
{
  unsigned long long t = __rdtsc();
  int r = g_rq4(m, pl, bx, by, cc, intra);
  unsigned long long dt = __rdtsc() - t;
  g_c[0] += dt;
  ++g_n[0];
  if (!intra) {   /* an inter residual: the prediction is a motion-compensated block */
    ++g_n_inter4;
    g_c_inter4 += dt;
  }
  if (m->p_Slice->slice_type == I_SLICE) ++g_n_islice4;
  return r;
}

static int t_rq8(Macroblock *m, ColorPlane pl, int b8, int *cc, int intra)
{
  unsigned long long t = __rdtsc();
  int r = g_rq8(m, pl, b8, cc, intra);
  g_c[1] += __rdtsc() - t;
  ++g_n[1];
  return r;
}

static distblk t_d4(short *d, distblk m)
{
  unsigned long long t = __rdtsc();
  distblk r = g_d4(d, m);
  g_c[2] += __rdtsc() - t;
  ++g_n[2];
  return r;
}

static distblk t_d8(short *d, distblk m)
{
  unsigned long long t = __rdtsc();
  distblk r = g_d8(d, m);
  g_c[3] += __rdtsc() - t;
  ++g_n[3];
  return r;
}

extern void __real_select_transform(Macroblock *currMB);
/* (weak: the CPU-only profiling build, lencod_f3prof, links no GPU server) */
extern int jm_f3_gpu_on(void) __attribute__((weak));
extern int jm_f3_gpu_rq4(Macroblock *m, ColorPlane pl, int bx, int by, int *cc, int intra) __attribute__((weak));
extern int residual_transform_quant_luma_4x4(Macroblock *, ColorPlane, int, int, int *, int);
void __wrap_select_transform(Macroblock *currMB)
{
  __real_select_transform(currMB);
  /* JMME_F3=1: the plain 4x4 residual coding goes through the GPU server (jm_f3_gpu.c) */
  if (jm_f3_gpu_on && jm_f3_gpu_on() && currMB->residual_transform_quant_luma_4x4 == residual_transform_quant_luma_4x4)
    currMB->residual_transform_quant_luma_4x4 = jm_f3_gpu_rq4;
  if (!on()) return;
  if (currMB->residual_transform_quant_luma_4x4 != t_rq4) {
    g_rq4 = currMB->residual_transform_quant_luma_4x4;
    currMB->residual_transform_quant_luma_4x4 = t_rq4;
  }
  if (currMB->residual_transform_quant_luma_8x8 != t_rq8) {
    g_rq8 = currMB->residual_transform_quant_luma_8x8;
    currMB->residual_transform_quant_luma_8x8 = t_rq8;
  }
}

extern void __real_select_distortion(VideoParameters *p_Vid, InputParameters *p_Inp);
void __wrap_select_distortion(VideoParameters *p_Vid, InputParameters *p_Inp)
{
  __real_select_distortion(p_Vid, p_Inp);
  if (!on()) return;
  g_d4 = p_Vid->distortion4x4;
  g_d8 = p_Vid->distortion8x8;
  p_Vid->distortion4x4 = t_d4;
  p_Vid->distortion8x8 = t_d8;
}

static void report(void) __attribute__((destructor));
static void report(void)
{
  static const char *name[4] = {"residual_transform_quant_luma_4x4", "residual_transform_quant_luma_8x8",
                                "distortion4x4", "distortion8x8"};
  struct timespec ts;
  double s, ghz;
  int i;
  if (g_on != 1) return;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  s = (double)(ts.tv_sec - g_ts0.tv_sec) + 1e-9 * (double)(ts.tv_nsec - g_ts0.tv_nsec);
  ghz = s > 0 ? (double)(__rdtsc() - g_tsc0) / s * 1e-9 : 1.0;
  fprintf(stderr, "jm_f3_profile: %.3f s profiled (TSC %.2f GHz)\n", s, ghz);
  for (i = 0; i < 4; i++)
    fprintf(stderr, "jm_f3_profile: %s: %lld calls, %.1f ms, %.1f ns per call\n", name[i], g_n[i],
            (double)g_c[i] / ghz * 1e-6, g_n[i] ? (double)g_c[i] / ghz / (double)g_n[i] : 0.0);
  fprintf(stderr, "jm_f3_profile: residual_transform_quant_luma_4x4 inter (intra == 0): %lld calls, %.1f ms; "
          "in I slices: %lld calls\n", g_n_inter4, (double)g_c_inter4 / ghz * 1e-6, g_n_islice4);
}
