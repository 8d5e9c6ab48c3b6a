/* Measurement aid for the drop-in (JMME_SAMPLE=<file>): a wall-clock sampling
 * profile of JM's motion-estimation region -- the time JM's "Total ME time"
 * counts (PartitionMotionSearch / SubPartitionMotionSearch, JM/lencod/src/
 * mv_search.c:1564,1686, each timed by JM itself).  A POSIX timer on the
 * encoding thread fires every 20 us of wall time; while the thread is inside
 * one of those two functions the handler records the interrupted instruction
 * pointer.  At exit the samples and /proc/self/maps go to the file, and
 * tools/sample_report.py attributes them to functions (nm) and libraries.
 * Without JMME_SAMPLE the two wrappers only call JM's functions. */
#define _GNU_SOURCE
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include "global.h"

void __real_PartitionMotionSearch(Macroblock *currMB, int blocktype, int block8x8, int *lambda_factor);
void __real_SubPartitionMotionSearch(Macroblock *currMB, int blocktype, int block8x8, int *lambda_factor);

#define MAX_SAMPLES (1 << 22)
static uintptr_t *g_pcs = NULL;
static volatile sig_atomic_t g_in_me = 0;
static volatile long g_n = 0;
static long g_ticks = 0;
static int g_state = -1;   /* -1 not decided, 0 off, 1 on */
static const char *g_path = NULL;

static void on_tick(int sig, siginfo_t *si, void *uc_)
{
  (void)sig;
  (void)si;
  ++g_ticks;
  if (!g_in_me || g_n >= MAX_SAMPLES) return;
  g_pcs[g_n++] = (uintptr_t)((ucontext_t *)uc_)->uc_mcontext.gregs[REG_RIP];
}

static void dump(void)
{
  FILE *f = fopen(g_path, "w"), *m;
  char line[1024];
  long i;
  if (!f) return;
  fprintf(f, "# samples %ld ticks %ld period_us 20\n", (long)g_n, g_ticks);
  for (i = 0; i < g_n; i++) fprintf(f, "%lx\n", (unsigned long)g_pcs[i]);
  fprintf(f, "# maps\n");
  if ((m = fopen("/proc/self/maps", "r"))) {
    while (fgets(line, sizeof line, m)) fputs(line, f);
    fclose(m);
  }
  fclose(f);
}

static void start(void)
{
  struct sigaction sa;
  struct sigevent ev;
  struct itimerspec it;
  timer_t t;
  g_path = getenv("JMME_SAMPLE");
  g_state = g_path && *g_path;
  if (!g_state) return;
  g_pcs = (uintptr_t *)malloc(MAX_SAMPLES * sizeof(uintptr_t));
  if (!g_pcs) { g_state = 0; return; }
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_tick;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigaction(SIGRTMIN + 3, &sa, NULL);
  memset(&ev, 0, sizeof ev);
  ev.sigev_notify = SIGEV_THREAD_ID;
  ev.sigev_signo = SIGRTMIN + 3;
  ev._sigev_un._tid = (pid_t)syscall(SYS_gettid);   /* this (the encoding) thread only */
  if (timer_create(CLOCK_MONOTONIC, &ev, &t)) { g_state = 0; return; }
  memset(&it, 0, sizeof it);
  it.it_interval.tv_nsec = it.it_value.tv_nsec = 20000;
  timer_settime(t, 0, &it, NULL);
  atexit(dump);
}

void __wrap_PartitionMotionSearch(Macroblock *currMB, int blocktype, int block8x8, int *lambda_factor)
{
  if (g_state < 0) start();
  g_in_me = 1;
  __real_PartitionMotionSearch(currMB, blocktype, block8x8, lambda_factor);
  g_in_me = 0;
}

void __wrap_SubPartitionMotionSearch(Macroblock *currMB, int blocktype, int block8x8, int *lambda_factor)
{
  if (g_state < 0) start();
  g_in_me = 1;
  __real_SubPartitionMotionSearch(currMB, blocktype, block8x8, lambda_factor);
  g_in_me = 0;
}
