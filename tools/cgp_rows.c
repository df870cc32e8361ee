// cgp_rows.c -- stochastic search for Life-rule v_bitop3 networks with
// vertical sharing, on the row-split layouts.
//
// A cell's 3x3 neighbourhood is three rows (u = above, c, d = below) of three
// raw cells (L, a, R); L and R are the exchanged neighbour columns.  Gates
// come in three kinds, each costing one v_bitop3 per 32-bit word:
//   row gates    f(signals of ONE row): computed once per row, read by the
//                three output rows that see it (offsets u, c, d).  The
//                horizontal sums h0 = xor3(L,a,R), h1 = maj(L,a,R) of
//                gen_split are two row gates.
//   pair gates   f(signals of rows r, r+1): computed once per row, read at
//                offsets (u, c) and (c, d).
//   output gates f(anything): per output row.
// Cost per word = R + P + O.  The network must give
//   next = (n == 3) | (a & n == 4),  n = inclusive 3x3 count,
// on all 512 neighbourhoods (LifeAPI.hpp:1196-1216 Step()).
//
// usage: cgp_rows R P O seconds seed [fix_h]
//   fix_h = 1 pins the first two row gates to xor3 / maj (the current h-layer).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define W 8  // 512 minterms
#define MAXR 4
#define MAXP 4
#define MAXO 8
typedef struct { uint64_t w[W]; } tt;

static int NR, NP, NO, FIXH;
static tt raw[3][3];  // [row u/c/d][L/a/R]
static tt target;

typedef struct {
  uint8_t rsrc[MAXR][3], rfn[MAXR];
  uint8_t psrc[MAXP][3], pfn[MAXP];
  uint8_t osrc[MAXO][3], ofn[MAXO];
} genome;

static inline uint64_t lut64(uint8_t f, uint64_t x, uint64_t y, uint64_t z) {
  uint64_t r = 0;
  for (int k = 0; k < 8; k++)
    if (f >> k & 1) r |= ((k & 4) ? x : ~x) & ((k & 2) ? y : ~y) & ((k & 1) ? z : ~z);
  return r;
}
static inline void lut(tt *o, uint8_t f, const tt *x, const tt *y, const tt *z) {
  for (int h = 0; h < W; h++) o->w[h] = lut64(f, x->w[h], y->w[h], z->w[h]);
}

// signal numbering
//   row signals of row t: t*RS + k, k < RS = 3 + NR
//   pair signals: 3*RS + q*NP + k (q = 0: pair (u,c), q = 1: pair (c,d))
//   output gates: 3*RS + 2*NP + k
#define RS (3 + NR)
static int eval(const genome *g, tt *sig) {
  for (int t = 0; t < 3; t++) {
    for (int k = 0; k < 3; k++) sig[t * RS + k] = raw[t][k];
    for (int i = 0; i < NR; i++)
      lut(&sig[t * RS + 3 + i], g->rfn[i], &sig[t * RS + g->rsrc[i][0]], &sig[t * RS + g->rsrc[i][1]],
          &sig[t * RS + g->rsrc[i][2]]);
  }
  // pair gate inputs: index < 2*RS selects a row signal of (first, second)
  // row; index >= 2*RS an earlier pair gate of the same pair
  for (int q = 0; q < 2; q++)
    for (int i = 0; i < NP; i++) {
      const tt *in[3];
      for (int j = 0; j < 3; j++) {
        int s = g->psrc[i][j];
        in[j] = s < 2 * RS ? &sig[(q + s / RS) * RS + s % RS] : &sig[3 * RS + q * NP + (s - 2 * RS)];
      }
      lut(&sig[3 * RS + q * NP + i], g->pfn[i], in[0], in[1], in[2]);
    }
  const int base = 3 * RS + 2 * NP;
  for (int i = 0; i < NO; i++)
    lut(&sig[base + i], g->ofn[i], &sig[g->osrc[i][0]], &sig[g->osrc[i][1]], &sig[g->osrc[i][2]]);
  int bad = 0;
  for (int h = 0; h < W; h++) bad += __builtin_popcountll(sig[base + NO - 1].w[h] ^ target.w[h]);
  return bad;
}

static uint64_t rs;
static inline uint32_t rnd(void) {
  rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
  return (uint32_t)(rs >> 11);
}
static void rsrc(genome *g, int i, int j) { g->rsrc[i][j] = rnd() % (3 + i); }
static void psrc(genome *g, int i, int j) { g->psrc[i][j] = rnd() % (2 * RS + i); }
static void osrc(genome *g, int i, int j) { g->osrc[i][j] = rnd() % (3 * RS + 2 * NP + i); }
static void fix(genome *g) {
  if (FIXH && NR >= 2) {
    for (int i = 0; i < 2; i++) g->rsrc[i][0] = 0, g->rsrc[i][1] = 1, g->rsrc[i][2] = 2;
    g->rfn[0] = 0x96, g->rfn[1] = 0xE8;
  }
}
static void randomise(genome *g) {
  for (int i = 0; i < NR; i++) { for (int j = 0; j < 3; j++) rsrc(g, i, j); g->rfn[i] = rnd(); }
  for (int i = 0; i < NP; i++) { for (int j = 0; j < 3; j++) psrc(g, i, j); g->pfn[i] = rnd(); }
  for (int i = 0; i < NO; i++) { for (int j = 0; j < 3; j++) osrc(g, i, j); g->ofn[i] = rnd(); }
  fix(g);
}
static void mutate(genome *g) {
  int n = 1 + rnd() % 3, tot = NR + NP + NO;
  while (n--) {
    int i = rnd() % tot, j = rnd() % 3, fb = rnd() & 1, bit = rnd() % 8;
    if (i < NR) { if (fb) g->rfn[i] ^= 1u << bit; else rsrc(g, i, j); }
    else if ((i -= NR) < NP) { if (fb) g->pfn[i] ^= 1u << bit; else psrc(g, i, j); }
    else { i -= NP; if (fb) g->ofn[i] ^= 1u << bit; else osrc(g, i, j); }
  }
  fix(g);
}

int main(int argc, char **argv) {
  if (argc < 6) { fprintf(stderr, "usage: cgp_rows R P O seconds seed [fix_h]\n"); return 2; }
  NR = atoi(argv[1]), NP = atoi(argv[2]), NO = atoi(argv[3]);
  double secs = atof(argv[4]);
  rs = strtoull(argv[5], 0, 0) * 0x9E3779B97F4A7C15ull + 1;
  FIXH = argc > 6 ? atoi(argv[6]) : 0;
  if (NR > MAXR || NP > MAXP || NO > MAXO || NO < 1) return 2;
  for (int m = 0; m < 512; m++) {
    int n = __builtin_popcount(m);
    for (int t = 0; t < 3; t++)
      for (int k = 0; k < 3; k++)
        if (m >> (3 * t + k) & 1) raw[t][k].w[m >> 6] |= 1ull << (m & 63);
    int a = m >> 4 & 1;  // centre: row c, cell a
    if (n == 3 || (a && n == 4)) target.w[m >> 6] |= 1ull << (m & 63);
  }
  tt sig[3 * (3 + MAXR) + 2 * MAXP + MAXO];
  clock_t t0 = clock();
  long restarts = 0, found = 0;
  while ((double)(clock() - t0) / CLOCKS_PER_SEC < secs) {
    genome par, ch;
    randomise(&par);
    int pf = eval(&par, sig);
    for (long it = 0; it < 300000 && pf; it++)
      for (int k = 0; k < 4; k++) {
        ch = par;
        mutate(&ch);
        int f = eval(&ch, sig);
        if (f <= pf) par = ch, pf = f;
      }
    restarts++;
    if (pf == 0) {
      found++;
      printf("FOUND R=%d P=%d O=%d:", NR, NP, NO);
      for (int i = 0; i < NR; i++) printf(" r%d=%02x(%d,%d,%d)", i, par.rfn[i], par.rsrc[i][0], par.rsrc[i][1], par.rsrc[i][2]);
      for (int i = 0; i < NP; i++) printf(" p%d=%02x(%d,%d,%d)", i, par.pfn[i], par.psrc[i][0], par.psrc[i][1], par.psrc[i][2]);
      for (int i = 0; i < NO; i++) printf(" o%d=%02x(%d,%d,%d)", i, par.ofn[i], par.osrc[i][0], par.osrc[i][1], par.osrc[i][2]);
      printf("\n");
      fflush(stdout);
    }
  }
  fprintf(stderr, "R=%d P=%d O=%d restarts %ld found %ld\n", NR, NP, NO, restarts, found);
  return 0;
}
