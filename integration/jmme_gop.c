/*
 * jmme_gop.c -- closed-GOP multi-GPU launcher for the drop-in encoder
 * (JM's motion estimation is sequential inside a GOP --
 * frame t searches the reconstruction of t-1, store_picture_in_dpb,
 * JM/lencod/src/mbuffer.c:1905 -- so N GPUs encode N closed GOPs at once).
 *
 * The sequence [0, frames) is cut into GOPs of `gop` frames.  GOP k is encoded
 * by a fresh encoder process (lencod_jmme, or the stock lencod for a CPU
 * rehearsal) started with JM's own keys
 *     -p StartFrame=k*gop -p FramesToBeEncoded=<gop or the rest>
 *     -p OutputFile=<prefix>_gopK.264 -p ReconFile=<prefix>_gopK_rec.yuv
 * (StartFrame / FramesToBeEncoded: JM/lencod/inc/configfile.h:39,47), so each
 * GOP starts with an IDR picture and references nothing outside itself.  Its
 * GPU is chosen in the child's environment (HIP_VISIBLE_DEVICES) between fork
 * and exec -- this process never touches the GPU.  Up to `per_gpu` children
 * run on each GPU; a GPU whose child exits takes the next GOP.
 *
 * The GOP reconstructions, concatenated in order, equal the reconstruction of
 * one encoder run over the whole sequence with IntraPeriod = IDRPeriod = gop
 * (tests/test_gop_launch.py checks this on the CPU with the stock encoder and
 * on the GPU with lencod_jmme); the bitstreams differ only in their headers
 * (each GOP carries its own parameter sets and idr_pic_id).
 *
 * Host placement: the encoders are host-bound (JM's mode decision, entropy
 * coding and the adapter stay on the CPU), so each child is pinned to host cores
 * with sched_setaffinity between fork and exec when a core list is given
 * (--cpus; without it the scheduler places them).  The list is cut into one
 * contiguous share per GPU slot -- a rank-per-GPU caller passes its GPU's
 * NUMA-local cores -- and each running child of a slot takes a core of its
 * share to itself while there are enough (the whole share otherwise).
 *
 * GPU queues: the HIP runtime gives each process up to GPU_MAX_HW_QUEUES (4)
 * hardware queues, one per stream it uses.  With 8 encoders on one GPU that is
 * more user queues than the GPU's scheduler keeps mapped at once, and it then
 * time-slices them: measured on MI355X with 8 concurrent 4K EPZS encodes (whose
 * searches alone are round trips), JM's ME time per GOP went from 1.3 s to 5.4 s
 * (tools/exp_gop_queues.py).  So each child gets GPU_MAX_HW_QUEUES =
 * 16 / per_gpu, clamped to [1, 4] (--hw-queues N overrides, 0 leaves the
 * environment alone).
 *
 * Usage:
 *   jmme_gop --encoder PATH --gpus N [--per-gpu K] [--devices D0,D1,..] [--cpus LIST] [--hw-queues N]
 *            --gop G --frames F --prefix OUTPREFIX [--concat] -- <encoder arguments>
 * (--devices: the HIP device index each of the N GPU slots stands for; default
 * 0 .. N-1.  A rank-per-GPU caller passes its own device alone.  --cpus: a
 * Linux cpulist, e.g. "0-15,64-79".)
 * Prints one JSON line: GOPs, their GPU, wall time and JM's "Total ME time".
 */
#define _GNU_SOURCE
#include <errno.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

typedef struct gop_run {
  int gop, gpu, first, count;
  int core;        /* the core the child has to itself (index into g_cpus), -1: its slot's whole share */
  pid_t pid;
  double t0, t1, me_s;
  int status;
} gop_run;

static double now_s(void)
{
  struct timeval tv;
  gettimeofday(&tv, NULL);
  return tv.tv_sec + tv.tv_usec * 1e-6;
}

static void die(const char *msg)
{
  fprintf(stderr, "jmme_gop: %s\n", msg);
  exit(2);
}

static const char *g_encoder, *g_prefix;
static int g_dev_map[64];
static char **g_enc_args;
static int g_n_enc_args;
static int g_pin;
static int *g_cpus, g_n_cpus;      /* host cores the children run on */
static unsigned char *g_core_busy;  /* per entry of g_cpus: held by a running child */
static int g_gpus;
static int g_hw_queues;            /* GPU_MAX_HW_QUEUES for the children (0: inherited) */

/* "0-3,8,10-11" -> cores; returns the count (-1: malformed) */
static int parse_cpulist(const char *q, int **out)
{
  int n = 0, cap = 64;
  int *v = (int *)malloc(sizeof(int) * (size_t)cap);
  if (!v) die("out of memory");
  while (*q) {
    char *end;
    long a = strtol(q, &end, 10), b;
    if (end == q || a < 0) { free(v); return -1; }
    b = a;
    if (*end == '-') {
      q = end + 1;
      b = strtol(q, &end, 10);
      if (end == q || b < a) { free(v); return -1; }
    }
    for (; a <= b; a++) {
      if (n == cap) {
        cap *= 2;
        v = (int *)realloc(v, sizeof(int) * (size_t)cap);
        if (!v) die("out of memory");
      }
      v[n++] = (int)a;
    }
    if (*end && *end != ',') { free(v); return -1; }
    q = *end == ',' ? end + 1 : end;
  }
  *out = v;
  return n;
}

/* slot g's share of g_cpus: [lo, hi) */
static void slot_share(int g, int *lo, int *hi)
{
  *lo = (int)((long)g * g_n_cpus / g_gpus);
  *hi = (int)((long)(g + 1) * g_n_cpus / g_gpus);
  if (*hi <= *lo) {   /* fewer cores than slots: slots share cores round-robin */
    *lo = g % g_n_cpus;
    *hi = *lo + 1;
  }
}

/* a free core of slot g's share for a new child (-1: none free, the child takes the share) */
static int take_core(int g)
{
  int lo, hi, c;
  slot_share(g, &lo, &hi);
  for (c = lo; c < hi; c++)
    if (!g_core_busy[c]) { g_core_busy[c] = 1; return c; }
  return -1;
}

/* the child's cpulist as text (for the report) */
static void placement_text(const gop_run *r, char *buf, size_t n)
{
  int lo, hi;
  if (!g_pin) { snprintf(buf, n, "unpinned"); return; }
  if (r->core >= 0) { snprintf(buf, n, "%d", g_cpus[r->core]); return; }
  slot_share(r->gpu, &lo, &hi);
  snprintf(buf, n, hi - lo == 1 ? "%d" : "%d-%d", g_cpus[lo], g_cpus[hi - 1]);  /* (shares are listed in order) */
}

static void gop_path(char *buf, size_t n, int gop, const char *suffix)
{
  snprintf(buf, n, "%s_gop%03d%s", g_prefix, gop, suffix);
}

/* fork + exec one GOP's encoder on `gpu`; the child's stdout goes to its log */
static pid_t start_gop(gop_run *r)
{
  char start[64], count[64], out[4096], rec[4096], log[4096], errp[4096], dev[32];
  char outp[4200], recp[4200];
  pid_t pid;
  int i, k = 0;
  char **argv = (char **)calloc((size_t)g_n_enc_args + 16, sizeof(char *));
  if (!argv) die("out of memory");
  snprintf(start, sizeof start, "StartFrame=%d", r->first);
  snprintf(count, sizeof count, "FramesToBeEncoded=%d", r->count);
  gop_path(out, sizeof out, r->gop, ".264");
  gop_path(rec, sizeof rec, r->gop, "_rec.yuv");
  gop_path(log, sizeof log, r->gop, ".log");
  gop_path(errp, sizeof errp, r->gop, ".err");
  snprintf(outp, sizeof outp, "OutputFile=%s", out);
  snprintf(recp, sizeof recp, "ReconFile=%s", rec);
  snprintf(dev, sizeof dev, "%d", r->gpu < 64 ? g_dev_map[r->gpu] : r->gpu);
  argv[k++] = (char *)g_encoder;
  for (i = 0; i < g_n_enc_args; i++) argv[k++] = g_enc_args[i];
  argv[k++] = "-p"; argv[k++] = start;
  argv[k++] = "-p"; argv[k++] = count;
  argv[k++] = "-p"; argv[k++] = outp;
  argv[k++] = "-p"; argv[k++] = recp;
  argv[k] = NULL;
  pid = fork();
  if (pid < 0) die("fork failed");
  if (pid == 0) {
    FILE *f = freopen(log, "w", stdout);
    if (!f) _exit(127);
    if (!freopen(errp, "w", stderr)) _exit(127);   /* the encoder's (and libjmme's) reports, per GOP */
    if (g_pin) {   /* the host cores are fixed before the encoder starts, like the device */
      cpu_set_t set;
      int lo, hi, c;
      CPU_ZERO(&set);
      if (r->core >= 0) {
        CPU_SET(g_cpus[r->core], &set);
      } else {
        slot_share(r->gpu, &lo, &hi);
        for (c = lo; c < hi; c++) CPU_SET(g_cpus[c], &set);
      }
      if (sched_setaffinity(0, sizeof set, &set)) {
        fprintf(stderr, "jmme_gop: sched_setaffinity: %s\n", strerror(errno));
        _exit(127);
      }
    }
    /* the device is fixed before the encoder (and the HIP runtime in it) starts */
    setenv("HIP_VISIBLE_DEVICES", dev, 1);
    if (g_hw_queues > 0) {
      char hq[16];
      snprintf(hq, sizeof hq, "%d", g_hw_queues);
      setenv("GPU_MAX_HW_QUEUES", hq, 1);
    }
    execv(g_encoder, argv);
    fprintf(stderr, "jmme_gop: exec %s: %s\n", g_encoder, strerror(errno));
    _exit(127);
  }
  free(argv);
  r->pid = pid;
  r->t0 = now_s();
  return pid;
}

/* JM's own "Total ME time for sequence : x sec" (report.c:803) from the GOP's log */
static double me_time(int gop)
{
  char path[4096], line[512];
  double v = -1;
  FILE *f;
  gop_path(path, sizeof path, gop, ".log");
  f = fopen(path, "r");
  if (!f) return -1;
  while (fgets(line, sizeof line, f)) {
    const char *p = strstr(line, "Total ME time for sequence");
    if (p && (p = strchr(p, ':'))) v = atof(p + 1);
  }
  fclose(f);
  return v;
}

static int append_file(FILE *dst, const char *src)
{
  char buf[1 << 16];
  size_t n;
  FILE *f = fopen(src, "rb");
  if (!f) return -1;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0)
    if (fwrite(buf, 1, n, dst) != n) { fclose(f); return -1; }
  fclose(f);
  return 0;
}

int main(int argc, char **argv)
{
  int gpus = 1, per_gpu = 1, gop = 0, frames = 0, concat = 0, i, n_gops, next = 0, done = 0, failed = 0;
  int *busy;
  gop_run *runs;
  double t_start;
  const char *devices = NULL, *cpus = NULL;
  int hw_queues = -1;
  for (i = 0; i < 64; i++) g_dev_map[i] = i;
  for (i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "--")) { i++; break; }
    if (!strcmp(argv[i], "--concat")) { concat = 1; continue; }
    if (i + 1 >= argc) die("missing value");
    if (!strcmp(argv[i], "--encoder")) g_encoder = argv[++i];
    else if (!strcmp(argv[i], "--gpus")) gpus = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--per-gpu")) per_gpu = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--gop")) gop = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--frames")) frames = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--prefix")) g_prefix = argv[++i];
    else if (!strcmp(argv[i], "--devices")) devices = argv[++i];
    else if (!strcmp(argv[i], "--cpus")) cpus = argv[++i];
    else if (!strcmp(argv[i], "--hw-queues")) hw_queues = atoi(argv[++i]);
    else die("unknown option (see the usage in jmme_gop.c)");
  }
  if (!g_encoder || !g_prefix || gpus < 1 || per_gpu < 1 || gop < 1 || frames < 1)
    die("need --encoder, --prefix, --gpus >= 1, --gop >= 1, --frames >= 1");
  if (devices) {   /* "3" or "0,2,5": slot g runs on device devices[g] */
    const char *q = devices;
    int g = 0;
    while (*q && g < 64) {
      char *end;
      long v = strtol(q, &end, 10);
      if (end == q || v < 0 || (*end && *end != ',')) die("bad --devices list");
      g_dev_map[g++] = (int)v;
      q = *end == ',' ? end + 1 : end;
    }
    if (g < gpus) die("--devices names fewer devices than --gpus");
  }
  g_gpus = gpus;
  if (hw_queues < 0) hw_queues = per_gpu > 4 ? (16 / per_gpu < 1 ? 1 : 16 / per_gpu) : 4;
  if (hw_queues > 4) hw_queues = 4;
  g_hw_queues = hw_queues;
  g_pin = cpus != NULL;
  if (cpus) {
    g_n_cpus = parse_cpulist(cpus, &g_cpus);
    if (g_n_cpus <= 0) die("bad --cpus list");
  } else {   /* the launcher's own affinity */
    cpu_set_t set;
    int c;
    if (sched_getaffinity(0, sizeof set, &set)) die("sched_getaffinity failed");
    g_cpus = (int *)malloc(sizeof(int) * CPU_SETSIZE);
    if (!g_cpus) die("out of memory");
    for (c = 0; c < CPU_SETSIZE; c++)
      if (CPU_ISSET(c, &set)) g_cpus[g_n_cpus++] = c;
    if (!g_n_cpus) die("empty affinity");
  }
  g_core_busy = (unsigned char *)calloc((size_t)g_n_cpus, 1);
  if (!g_core_busy) die("out of memory");
  g_enc_args = argv + i;
  g_n_enc_args = argc - i;
  n_gops = (frames + gop - 1) / gop;
  runs = (gop_run *)calloc((size_t)n_gops, sizeof(gop_run));
  busy = (int *)calloc((size_t)gpus, sizeof(int));
  if (!runs || !busy) die("out of memory");
  for (i = 0; i < n_gops; i++) {
    runs[i].gop = i;
    runs[i].first = i * gop;
    runs[i].count = frames - i * gop < gop ? frames - i * gop : gop;
    runs[i].gpu = -1;
  }
  t_start = now_s();
  while (done < n_gops) {
    /* fill every free slot, GPU by GPU */
    int g;
    for (g = 0; g < gpus && next < n_gops; g++)
      while (busy[g] < per_gpu && next < n_gops) {
        runs[next].gpu = g;
        runs[next].core = g_pin ? take_core(g) : -1;
        start_gop(&runs[next]);
        busy[g]++;
        next++;
      }
    {
      int st = 0;
      pid_t pid = wait(&st);
      if (pid < 0) die("wait failed");
      for (i = 0; i < n_gops; i++)
        if (runs[i].pid == pid && runs[i].t1 == 0) {
          runs[i].t1 = now_s();
          runs[i].status = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
          runs[i].me_s = me_time(i);
          busy[runs[i].gpu]--;
          if (runs[i].core >= 0) g_core_busy[runs[i].core] = 0;
          if (runs[i].status) failed++;
          done++;
          break;
        }
    }
  }
  if (concat && !failed) {
    char path[4096], src[4096];
    FILE *fo, *fr;
    snprintf(path, sizeof path, "%s.264", g_prefix);
    fo = fopen(path, "wb");
    snprintf(path, sizeof path, "%s_rec.yuv", g_prefix);
    fr = fopen(path, "wb");
    if (!fo || !fr) die("cannot write the concatenated outputs");
    for (i = 0; i < n_gops; i++) {
      gop_path(src, sizeof src, i, ".264");
      if (append_file(fo, src)) die("cannot read a GOP bitstream");
      gop_path(src, sizeof src, i, "_rec.yuv");
      if (append_file(fr, src)) die("cannot read a GOP reconstruction");
    }
    fclose(fo);
    fclose(fr);
  }
  printf("{\"gops\": %d, \"gop\": %d, \"frames\": %d, \"gpus\": %d, \"per_gpu\": %d, \"wall_s\": %.3f, \"failed\": %d, "
         "\"host_cores\": %d, \"pinned\": %d, \"hw_queues\": %d, \"runs\": [", n_gops, gop, frames, gpus, per_gpu,
         now_s() - t_start, failed, g_n_cpus, g_pin, g_hw_queues);
  for (i = 0; i < n_gops; i++) {
    char place[64];
    placement_text(&runs[i], place, sizeof place);
    printf("%s{\"gop\": %d, \"gpu\": %d, \"device\": %d, \"cpus\": \"%s\", \"first\": %d, \"frames\": %d, "
           "\"wall_s\": %.3f, \"me_s\": %.3f, \"status\": %d}", i ? ", " : "", i, runs[i].gpu,
           runs[i].gpu < 64 ? g_dev_map[runs[i].gpu] : runs[i].gpu, place, runs[i].first, runs[i].count,
           runs[i].t1 - runs[i].t0, runs[i].me_s, runs[i].status);
  }
  printf("]}\n");
  free(runs);
  free(busy);
  free(g_cpus);
  free(g_core_busy);
  return failed ? 1 : 0;
}
