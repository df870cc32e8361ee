// cgp_weld.c -- cgp_search.c for LifeWeld::Step (LifeWeld.hpp:169-186): the
// same 7 inputs plus the frozen count planes f2, f1, f0 (10 inputs), target
// = the Life rule on (inclusive count mod 8) + frozen count, mod 8, exactly
// as the reference's HalfAdd / FullAdd / FullAdd chain computes it.
//
// Inputs per cell (7): the 2-bit horizontal 3-sums of the rows above, at and
// below the cell, in a chosen 2-bit encoding E of 0..3 (the h-layer: two
// LUTs per word, shared by the three output rows that read the word), and
// the centre cell a.  Target: next = (n == 3) | (a & n == 4) with n the
// inclusive 3x3 count (LifeAPI.hpp:1251-1252 / NeighbourCount.hpp:104-118
// rule).  Don't-cares: the centre row's sum includes a, so (a = 1, sum 0) and
// (a = 0, sum 3) never occur.  tools/exact_tail.c searched symmetric
// 2 + 2 first layers with a free `a`; this searches arbitrary DAGs of G LUTs.
//
// usage: cgp_search G seconds seed [encoding 0..23 | -1 = all]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define NIN 10
#define MAXG 16
#define TW 16
typedef struct { uint64_t w[TW]; } tt;

static tt in_tt[NIN], target, care;
static int G;

typedef struct { uint8_t src[MAXG][3]; uint8_t fn[MAXG]; uint8_t out; } genome;

static inline uint64_t lut64(uint8_t f, uint64_t x, uint64_t y, uint64_t z) {
  uint64_t r = 0;
  for (int k = 0; k < 8; k++)
    if (f >> k & 1) r |= ((k & 4) ? x : ~x) & ((k & 2) ? y : ~y) & ((k & 1) ? z : ~z);
  return r;
}

static int eval(const genome *g) {
  tt sig[NIN + MAXG];
  memcpy(sig, in_tt, sizeof(in_tt));
  for (int i = 0; i < G; i++)
    for (int h = 0; h < TW; h++)
      sig[NIN + i].w[h] = lut64(g->fn[i], sig[g->src[i][0]].w[h], sig[g->src[i][1]].w[h], sig[g->src[i][2]].w[h]);
  int bad = 0;
  for (int h = 0; h < TW; h++)
    bad += __builtin_popcountll((sig[g->out].w[h] ^ target.w[h]) & care.w[h]);
  return bad;
}

static uint64_t rs;
static inline uint32_t rnd(void) {
  rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
  return (uint32_t)(rs >> 11);
}

static void randomise(genome *g) {
  for (int i = 0; i < G; i++) {
    for (int j = 0; j < 3; j++) g->src[i][j] = rnd() % (NIN + i);
    g->fn[i] = rnd() & 255;
  }
  g->out = NIN + G - 1;
}

static void mutate(genome *g) {
  int n = 1 + rnd() % 3;
  while (n--) {
    int i = rnd() % G;
    if (rnd() & 1) g->src[i][rnd() % 3] = rnd() % (NIN + i);
    else g->fn[i] ^= 1u << (rnd() % 8);
  }
}

static void setup(int enc) {
  // the 24 bijections {0..3} -> 2-bit codes
  int perms[24][4], np = 0;
  for (int a = 0; a < 4; a++) for (int b = 0; b < 4; b++) for (int c = 0; c < 4; c++) for (int d = 0; d < 4; d++)
    if (a != b && a != c && a != d && b != c && b != d && c != d) { perms[np][0] = a, perms[np][1] = b, perms[np][2] = c, perms[np][3] = d; np++; }
  memset(in_tt, 0, sizeof in_tt); memset(&target, 0, sizeof target); memset(&care, 0, sizeof care);
  for (int m = 0; m < 1024; m++) {
    int code[3] = {m & 3, (m >> 2) & 3, (m >> 4) & 3}, a = (m >> 6) & 1, sum[3];
    const int fz = (m >> 7) & 7;  // bits 7, 8, 9 = f0, f1, f2
    for (int r = 0; r < 3; r++)
      for (int s = 0; s < 4; s++) if (perms[enc][s] == code[r]) sum[r] = s;
    for (int b = 0; b < NIN; b++) if (m >> b & 1) in_tt[b].w[m >> 6] |= 1ull << (m & 63);
    const int n = (sum[0] + sum[1] + sum[2]) & 7, t = (n + fz) & 7;
    int ok = !(a == 1 && sum[1] == 0) && !(a == 0 && sum[1] == 3);
    if (ok) care.w[m >> 6] |= 1ull << (m & 63);
    if (t == 3 || (a && t == 4)) target.w[m >> 6] |= 1ull << (m & 63);
  }
}

int main(int argc, char **argv) {
  G = argc > 1 ? atoi(argv[1]) : 10;
  double secs = argc > 2 ? atof(argv[2]) : 10;
  rs = argc > 3 ? strtoull(argv[3], 0, 0) * 0x9E3779B97F4A7C15ull + 1 : 88172645463325252ull;
  int enc_only = argc > 4 ? atoi(argv[4]) : -1;
  clock_t t0 = clock();
  long restarts = 0;
  while ((double)(clock() - t0) / CLOCKS_PER_SEC < secs) {
    int enc = enc_only >= 0 ? enc_only : (int)(rnd() % 24);
    setup(enc);
    genome par, ch;
    randomise(&par);
    int pf = eval(&par);
    for (long it = 0; it < 200000 && pf; it++) {
      for (int k = 0; k < 4; k++) {
        ch = par;
        mutate(&ch);
        int f = eval(&ch);
        if (f <= pf) { par = ch; pf = f; }
      }
    }
    restarts++;
    if (pf == 0) {
      printf("FOUND G=%d enc=%d:", G, enc);
      for (int i = 0; i < G; i++) printf(" n%d=f%02x(%d,%d,%d)", NIN + i, par.fn[i], par.src[i][0], par.src[i][1], par.src[i][2]);
      printf(" out=%d\n", par.out);
      fflush(stdout);
    }
  }
  fprintf(stderr, "restarts %ld\n", restarts);
  return 0;
}
