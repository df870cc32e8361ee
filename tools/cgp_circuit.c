// cgp_circuit.c -- shrink a multi-output v_bitop3 network by Cartesian
// genetic programming ((1+4) evolution with neutral drift), keeping it
// exact on a care set of input rows (tools/cgp_stable.py builds the problem:
// the rows the kernel's inputs can take).
//
// Problem file (binary, little-endian): int32 nin, nout, words; then nin
// input bit-vectors and nout target bit-vectors of `words` uint64 each (bit
// r of input i = input i on care row r; rows past the care count are padded
// with copies of row 0).  Seed / result file (text): "G NOUT", then G lines
// "fn a b c" (sources: 0..nin-1 inputs, nin + k gate k, k < own index), then
// NOUT lines "node inv".  Gates' truth tables follow v_bitop3:
// bit (a<<2 | b<<1 | c) of fn.  Output inversion is free (the consumers fold
// it into their own v_bitop3).
//
// usage: cgp_circuit problem.bin seed.txt out.txt seconds rngseed spare
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define MAXG 256
#define MAXIN 32
#define MAXOUT 16

static int NIN, NOUT, WORDS, G;
static uint64_t *in_tt, *target;  // [NIN][WORDS], [NOUT][WORDS]

typedef struct {
  uint16_t src[MAXG][3];
  uint8_t fn[MAXG];
  uint16_t out[MAXOUT];
  uint8_t inv[MAXOUT];
} genome;

static inline uint64_t lut3(uint8_t f, uint64_t x, uint64_t y, uint64_t z) {
  const uint64_t b0 = -(uint64_t)(f & 1), b1 = -(uint64_t)(f >> 1 & 1), b2 = -(uint64_t)(f >> 2 & 1),
                 b3 = -(uint64_t)(f >> 3 & 1), b4 = -(uint64_t)(f >> 4 & 1), b5 = -(uint64_t)(f >> 5 & 1),
                 b6 = -(uint64_t)(f >> 6 & 1), b7 = -(uint64_t)(f >> 7 & 1);
  const uint64_t q0 = ~y & ~z, q1 = ~y & z, q2 = y & ~z, q3 = y & z;
  const uint64_t g0 = (q0 & b0) | (q1 & b1) | (q2 & b2) | (q3 & b3);
  const uint64_t g1 = (q0 & b4) | (q1 & b5) | (q2 & b6) | (q3 & b7);
  return (~x & g0) | (x & g1);
}

static uint64_t rng_s;
static inline uint64_t rnd(void) {
  uint64_t z = (rng_s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// active gates: reachable from the outputs
static int active(const genome *g, uint8_t *act) {
  memset(act, 0, MAXG);
  for (int o = 0; o < NOUT; o++)
    if (g->out[o] >= NIN) act[g->out[o] - NIN] = 1;
  int n = 0;
  for (int i = G - 1; i >= 0; i--) {
    if (!act[i]) continue;
    n++;
    for (int k = 0; k < 3; k++)
      if (g->src[i][k] >= NIN) act[g->src[i][k] - NIN] = 1;
  }
  return n;
}

// exact on every care row?  vals: scratch [G][WORDS]
static int correct(const genome *g, const uint8_t *act, uint64_t *vals) {
  for (int w0 = 0; w0 < WORDS; w0 += 64) {  // blocks of 64 words: most wrong genomes fail early
    const int w1 = w0 + 64 < WORDS ? w0 + 64 : WORDS;
    for (int i = 0; i < G; i++) {
      if (!act[i]) continue;
      const uint64_t *a = g->src[i][0] < NIN ? in_tt + (size_t)g->src[i][0] * WORDS : vals + (size_t)(g->src[i][0] - NIN) * WORDS;
      const uint64_t *b = g->src[i][1] < NIN ? in_tt + (size_t)g->src[i][1] * WORDS : vals + (size_t)(g->src[i][1] - NIN) * WORDS;
      const uint64_t *c = g->src[i][2] < NIN ? in_tt + (size_t)g->src[i][2] * WORDS : vals + (size_t)(g->src[i][2] - NIN) * WORDS;
      uint64_t *d = vals + (size_t)i * WORDS;
      for (int w = w0; w < w1; w++) d[w] = lut3(g->fn[i], a[w], b[w], c[w]);
    }
    for (int o = 0; o < NOUT; o++) {
      const uint64_t *v = g->out[o] < NIN ? in_tt + (size_t)g->out[o] * WORDS : vals + (size_t)(g->out[o] - NIN) * WORDS;
      const uint64_t inv = g->inv[o] ? ~0ull : 0ull;
      const uint64_t *t = target + (size_t)o * WORDS;
      for (int w = w0; w < w1; w++)
        if ((v[w] ^ inv) != t[w]) return 0;
    }
  }
  return 1;
}

static void mutate(genome *g) {
  const int kinds = 3;
  int n = 1 + (int)(rnd() % 3);
  while (n--) {
    const int k = (int)(rnd() % kinds);
    if (k == 0) {  // a gate's source
      const int i = (int)(rnd() % G), s = (int)(rnd() % 3);
      g->src[i][s] = (uint16_t)(rnd() % (NIN + i));
    } else if (k == 1) {  // a gate's function
      const int i = (int)(rnd() % G);
      if (rnd() & 1) g->fn[i] ^= (uint8_t)(1u << (rnd() % 8));
      else g->fn[i] = (uint8_t)rnd();
    } else {  // an output
      const int o = (int)(rnd() % NOUT);
      if (rnd() & 3) g->out[o] = (uint16_t)(NIN + rnd() % G);
      else g->inv[o] ^= 1;
    }
  }
}

static int load_genome(const char *path, genome *g, int spare) {
  FILE *f = fopen(path, "r");
  if (!f) return -1;
  int gn, no;
  if (fscanf(f, "%d %d", &gn, &no) != 2 || no != NOUT || gn + spare > MAXG) return -2;
  memset(g, 0, sizeof *g);
  // spare gates first (inactive, inputs only), then the seed shifted by spare
  for (int i = 0; i < spare; i++) {
    g->fn[i] = (uint8_t)rnd();
    for (int k = 0; k < 3; k++) g->src[i][k] = (uint16_t)(rnd() % (NIN + i));
  }
  for (int i = 0; i < gn; i++) {
    int fn, s[3];
    if (fscanf(f, "%d %d %d %d", &fn, &s[0], &s[1], &s[2]) != 4) return -3;
    g->fn[spare + i] = (uint8_t)fn;
    for (int k = 0; k < 3; k++) g->src[spare + i][k] = (uint16_t)(s[k] < NIN ? s[k] : s[k] + spare);
  }
  for (int o = 0; o < NOUT; o++) {
    int node, inv;
    if (fscanf(f, "%d %d", &node, &inv) != 2) return -4;
    g->out[o] = (uint16_t)(node < NIN ? node : node + spare);
    g->inv[o] = (uint8_t)inv;
  }
  fclose(f);
  G = gn + spare;
  return 0;
}

static void save_genome(const char *path, const genome *g) {
  uint8_t act[MAXG];
  const int n = active(g, act);
  int map[MAXG], k = 0;
  for (int i = 0; i < G; i++) map[i] = act[i] ? k++ : -1;
  FILE *f = fopen(path, "w");
  fprintf(f, "%d %d\n", n, NOUT);
  for (int i = 0; i < G; i++) {
    if (!act[i]) continue;
    fprintf(f, "%d", g->fn[i]);
    for (int s = 0; s < 3; s++) {
      const int v = g->src[i][s];
      fprintf(f, " %d", v < NIN ? v : NIN + map[v - NIN]);
    }
    fprintf(f, "\n");
  }
  for (int o = 0; o < NOUT; o++) {
    const int v = g->out[o];
    fprintf(f, "%d %d\n", v < NIN ? v : NIN + map[v - NIN], g->inv[o]);
  }
  fclose(f);
}

int main(int argc, char **argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: cgp_circuit problem.bin seed.txt out.txt seconds rngseed spare\n");
    return 2;
  }
  FILE *f = fopen(argv[1], "rb");
  int32_t hdr[3];
  if (!f || fread(hdr, 4, 3, f) != 3) return 3;
  NIN = hdr[0], NOUT = hdr[1], WORDS = hdr[2];
  if (NIN > MAXIN || NOUT > MAXOUT) return 4;
  in_tt = malloc((size_t)NIN * WORDS * 8);
  target = malloc((size_t)NOUT * WORDS * 8);
  if (fread(in_tt, 8, (size_t)NIN * WORDS, f) != (size_t)NIN * WORDS) return 5;
  if (fread(target, 8, (size_t)NOUT * WORDS, f) != (size_t)NOUT * WORDS) return 6;
  fclose(f);
  const double secs = atof(argv[4]);
  rng_s = strtoull(argv[5], 0, 10) * 0x2545F4914F6CDD1DULL + 1;
  const int spare = atoi(argv[6]);
  genome parent, child;
  if (load_genome(argv[2], &parent, spare)) {
    fprintf(stderr, "bad seed genome\n");
    return 7;
  }
  uint64_t *vals = malloc((size_t)MAXG * WORDS * 8);
  uint8_t act[MAXG];
  int best = active(&parent, act);
  if (!correct(&parent, act, vals)) {
    fprintf(stderr, "seed genome is not exact on the care set\n");
    return 8;
  }
  fprintf(stderr, "seed: %d active gates\n", best);
  const clock_t t0 = clock();
  long evals = 0;
  while ((double)(clock() - t0) / CLOCKS_PER_SEC < secs) {
    for (int lam = 0; lam < 4; lam++) {
      child = parent;
      mutate(&child);
      const int n = active(&child, act);
      evals++;
      if (n > best) continue;
      if (!correct(&child, act, vals)) continue;
      if (n < best) {
        fprintf(stderr, "%.1fs %ld evals: %d active gates\n", (double)(clock() - t0) / CLOCKS_PER_SEC, evals, n);
        save_genome(argv[3], &child);
      }
      best = n;
      parent = child;  // neutral drift on ties
    }
  }
  save_genome(argv[3], &parent);
  fprintf(stderr, "done: %d active gates, %ld evals\n", best, evals);
  printf("%d\n", best);
  return 0;
}
