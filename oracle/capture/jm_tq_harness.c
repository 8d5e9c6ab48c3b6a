/*
 * jm_tq_harness.c -- TEST INFRASTRUCTURE (golden-vector generator).
 *
 * Linked against the JM 18.5 objects compiled by oracle/Makefile from the
 * reference sources (nothing is copied), it feeds seeded random blocks to
 * JM's own forward4x4 / inverse4x4 / hadamard4x4 / ihadamard4x4 /
 * hadamard4x2 / ihadamard4x2 / hadamard2x2 / ihadamard2x2 / forward8x8 /
 * inverse8x8 (lcommon/src/transform.c), HadamardSAD4x4 / HadamardSAD8x8
 * (lencod/src/me_distortion.c) and quant_4x4_normal
 * (lencod/src/quant4x4_normal.c), and writes inputs and JM's outputs as a
 * flat little-endian int32 stream that tests/golden/make_golden_tq.py turns
 * into tests/golden/tq_jm.npz.
 *
 * Usage: jm_tq_harness SEED N OUT.bin
 */
#include "global.h"
#include "mbuffer.h"
#include "transform.h"
#include "me_distortion.h"
#include "quant4x4.h"

#include <stdio.h>
#include <stdlib.h>

static unsigned long long g_state;
static int rnd(int lo, int hi)   /* inclusive, splitmix64 */
{
  unsigned long long z = (g_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return lo + (int)(z % (unsigned long long)(hi - lo + 1));
}

static FILE *g_out;
static void put(int v) { fwrite(&v, 4, 1, g_out); }
static void tag(const char *name, int n, int in_len, int out_len)
{
  char t[16] = {0};
  snprintf(t, sizeof t, "%s", name);
  fwrite(t, 1, 16, g_out);
  put(n); put(in_len); put(out_len);
}

/* a 16x16 int plane with row pointers, the shape JM's transforms index */
static int **plane16(void)
{
  int **p = (int **)malloc(16 * sizeof(int *));
  int *d = (int *)calloc(16 * 16, sizeof(int));
  int r;
  for (r = 0; r < 16; r++) p[r] = d + 16 * r;
  return p;
}

typedef void (*tf_pos)(int **, int **, int, int);

/* fixed_py: inverse8x8 takes no pos_y (it reads and writes rows 0..7) */
static void run_pos_transform(const char *name, tf_pos fn, int n, int sz, int lo, int hi, int fixed_py)
{
  int **a = plane16(), **b = plane16();
  int k, r, c;
  tag(name, n, sz * sz, sz * sz);
  for (k = 0; k < n; k++) {
    const int py = fixed_py ? 0 : sz * rnd(0, 16 / sz - 1), px = sz * rnd(0, 16 / sz - 1);
    for (r = 0; r < sz; r++)
      for (c = 0; c < sz; c++) { a[py + r][px + c] = rnd(lo, hi); put(a[py + r][px + c]); }
    fn(a, b, py, px);
    for (r = 0; r < sz; r++)
      for (c = 0; c < sz; c++) put(b[py + r][px + c]);
  }
}

static void inv8_wrap(int **t, int **b, int py, int px) { (void)py; inverse8x8(t, b, px); }

static void run_had(const char *name, void (*fn)(int **, int **), int n, int rows, int cols, int orows,
                    int ocols, int lo, int hi)
{
  int **a = plane16(), **b = plane16();
  int k, r, c;
  tag(name, n, rows * cols, orows * ocols);
  for (k = 0; k < n; k++) {
    for (r = 0; r < rows; r++)
      for (c = 0; c < cols; c++) { a[r][c] = rnd(lo, hi); put(a[r][c]); }
    fn(a, b);
    for (r = 0; r < orows; r++)
      for (c = 0; c < ocols; c++) put(b[r][c]);
  }
}

static void run_had2x2(int n)
{
  int **a = plane16();
  int k, t[4], u[4], v[4];
  tag("hadamard2x2", n, 4, 4);
  for (k = 0; k < n; k++) {
    a[0][0] = rnd(-65536, 65535); a[0][4] = rnd(-65536, 65535);
    a[4][0] = rnd(-65536, 65535); a[4][4] = rnd(-65536, 65535);
    put(a[0][0]); put(a[0][4]); put(a[4][0]); put(a[4][4]);
    hadamard2x2(a, t);
    put(t[0]); put(t[1]); put(t[2]); put(t[3]);
  }
  tag("ihadamard2x2", n, 4, 4);
  for (k = 0; k < n; k++) {
    int i;
    for (i = 0; i < 4; i++) { u[i] = rnd(-262144, 262143); put(u[i]); }
    ihadamard2x2(u, v);
    for (i = 0; i < 4; i++) put(v[i]);
  }
}

static void run_satd(int n)
{
  short d[64];
  int k, i;
  tag("satd4x4", n, 16, 1);
  for (k = 0; k < n; k++) {
    const int amp = (k % 4 == 0) ? 255 : rnd(1, 255);
    for (i = 0; i < 16; i++) { d[i] = (short)rnd(-amp, amp); put(d[i]); }
    put(HadamardSAD4x4(d));
  }
  tag("satd8x8", n, 64, 1);
  for (k = 0; k < n; k++) {
    const int amp = (k % 4 == 0) ? 255 : rnd(1, 255);
    for (i = 0; i < 64; i++) { d[i] = (short)rnd(-amp, amp); put(d[i]); }
    put(HadamardSAD8x8(d));
  }
}

/* H.264 4x4 scans (frame zig-zag, field), as (horizontal, vertical) pairs */
static const byte kFrameScan[16][2] = {{0,0},{1,0},{0,1},{0,2},{1,1},{2,0},{3,0},{2,1},
                                       {1,2},{0,3},{1,3},{2,2},{3,1},{3,2},{2,3},{3,3}};
static const byte kFieldScan[16][2] = {{0,0},{0,1},{1,0},{0,2},{0,3},{1,1},{1,2},{1,3},
                                       {2,0},{2,1},{2,2},{2,3},{3,0},{3,1},{3,2},{3,3}};
static const byte kCost[2][16] = {{3,2,2,1,1,1,0,0,0,0,0,0,0,0,0,0},
                                  {9,9,9,9,9,9,9,9,9,9,9,9,9,9,9,9}};
/* H.264 quantisation / dequantisation multipliers (spec tables, flat matrix) */
static const int kQuant[6][3] = {{13107,5243,8066},{11916,4660,7490},{10082,4194,6554},
                                 {9362,3647,5825},{8192,3355,5243},{7282,2893,4559}};
static const int kDequant[6][3] = {{10,16,13},{11,18,14},{13,20,16},{14,23,18},{16,25,20},{18,29,23}};

static void run_quant(int n)
{
  VideoParameters *vid = (VideoParameters *)calloc(1, sizeof(VideoParameters));
  QuantParameters *qpar = (QuantParameters *)calloc(1, sizeof(QuantParameters));
  Slice *sl = (Slice *)calloc(1, sizeof(Slice));
  Macroblock mb;
  int qp_per_matrix[52];
  LevelQuantParams qrow[4][4], *qrows[4];
  int **tb = plane16();
  int acl[18], acr[18];
  int k, i, j, q;
  for (q = 0; q < 52; q++) qp_per_matrix[q] = q / 6;
  qpar->qp_per_matrix = qp_per_matrix;
  vid->p_Quant = qpar;
  memset(&mb, 0, sizeof mb);
  mb.p_Vid = vid;
  mb.p_Slice = sl;
  for (j = 0; j < 4; j++) qrows[j] = qrow[j];

  /* record: [coef 16][scale 16][offset 16][inv 16][qp, cavlc, scan_sel, cost_sel, coeff_cost_in]
   *   -> [coef out 16][levels 17][runs 16][coeff_cost][nonzero] */
  tag("quant4x4", n, 16 * 4 + 5, 16 + 17 + 16 + 2);
  for (k = 0; k < n; k++) {
    QuantMethods qm;
    const int qp = rnd(0, 51), qp_rem = qp % 6, per = qp / 6;
    const int realistic = (k % 3) != 0;
    const int cavlc = rnd(0, 1), scan_sel = rnd(0, 1), cost_sel = rnd(0, 1);
    const int block_x = 4 * rnd(0, 3);
    const int qbits = 15 + per;
    int coeff_cost = rnd(0, 5), nz;
    const int amp = rnd(0, 3) == 0 ? 30000 : rnd(1, 4000);
    for (j = 0; j < 4; j++)
      for (i = 0; i < 4; i++) {
        const int cls = ((i & 1) == 0 && (j & 1) == 0) ? 0 : (((i & 1) && (j & 1)) ? 1 : 2);
        LevelQuantParams *p = &qrow[j][i];
        if (realistic) {
          p->ScaleComp = kQuant[qp_rem][cls];
          p->InvScaleComp = kDequant[qp_rem][cls] << 4;
          p->OffsetComp = rnd(0, (1 << 11) - 1) << (qbits - 11);
        } else {
          p->ScaleComp = rnd(0, 16384);
          p->InvScaleComp = rnd(0, 512);
          p->OffsetComp = rnd(0, (1 << qbits) - 1);
        }
        tb[j][block_x + i] = (rnd(0, 2) == 0) ? 0 : rnd(-amp, amp);
      }
    for (j = 0; j < 4; j++) for (i = 0; i < 4; i++) put(tb[j][block_x + i]);
    for (j = 0; j < 4; j++) for (i = 0; i < 4; i++) put(qrow[j][i].ScaleComp);
    for (j = 0; j < 4; j++) for (i = 0; i < 4; i++) put(qrow[j][i].OffsetComp);
    for (j = 0; j < 4; j++) for (i = 0; i < 4; i++) put(qrow[j][i].InvScaleComp);
    put(qp); put(cavlc); put(scan_sel); put(cost_sel); put(coeff_cost);
    sl->symbol_mode = (char)(cavlc ? CAVLC : CABAC);
    memset(&qm, 0, sizeof qm);
    memset(acl, 0x55, sizeof acl);
    memset(acr, 0, sizeof acr);
    qm.block_x = block_x;
    qm.qp = qp;
    qm.ACLevel = acl;
    qm.ACRun = acr;
    qm.q_params = qrows;
    qm.coeff_cost = &coeff_cost;
    qm.pos_scan = scan_sel ? kFieldScan : kFrameScan;
    qm.c_cost = kCost[cost_sel];
    nz = quant_4x4_normal(&mb, tb, &qm);
    for (j = 0; j < 4; j++) for (i = 0; i < 4; i++) put(tb[j][block_x + i]);
    for (i = 0; i < 17; i++) put(acl[i] == 0x55555555 ? 0 : acl[i]);
    for (i = 0; i < 16; i++) put(acr[i]);
    put(coeff_cost);
    put(nz);
  }
}

int main(int argc, char **argv)
{
  int n;
  if (argc != 4) { fprintf(stderr, "usage: %s SEED N OUT.bin\n", argv[0]); return 2; }
  g_state = strtoull(argv[1], NULL, 10);
  n = atoi(argv[2]);
  g_out = fopen(argv[3], "wb");
  if (!g_out) { perror(argv[3]); return 1; }
  run_pos_transform("forward4x4", forward4x4, n, 4, -255, 255, 0);
  run_pos_transform("inverse4x4", inverse4x4, n, 4, -8192, 8191, 0);
  run_had("hadamard4x4", hadamard4x4, n, 4, 4, 4, 4, -65536, 65535);
  run_had("ihadamard4x4", ihadamard4x4, n, 4, 4, 4, 4, -65536, 65535);
  run_had("hadamard4x2", hadamard4x2, n, 2, 4, 2, 4, -65536, 65535);
  run_had("ihadamard4x2", ihadamard4x2, n, 2, 4, 4, 2, -65536, 65535);
  run_had2x2(n);
  run_pos_transform("forward8x8", forward8x8, n, 8, -255, 255, 0);
  run_pos_transform("inverse8x8", inv8_wrap, n, 8, -16384, 16383, 1);
  run_satd(n);
  run_quant(n);
  fclose(g_out);
  return 0;
}
