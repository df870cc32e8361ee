/*
 * lifeapi_oracle.c -- CPU restatement of the reference's Step() path.
 *
 * TEST INFRASTRUCTURE ONLY (see lifeapi_oracle.h).  Never linked into the
 * product library; the product fails loudly if its HIP code object is absent.
 *
 * Every function names the reference lines it restates.  Paths are relative
 * to the reference snapshot (scorbiclife/LifeAPI, 2025-02-22).
 */
#include "lifeapi_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t rotl64(uint64_t v, unsigned k) { return (v << k) | (v >> ((64 - k) & 63)); }
static inline uint64_t rotr64(uint64_t v, unsigned k) { return (v >> k) | (v << ((64 - k) & 63)); }

/* Vertical (in-column) 3-cell sum as two bit planes.
 * LifeAPI.hpp:897-907 (LifeState::CountRows). */
void oracle_count_rows(const uint64_t s[64], uint64_t col0[64], uint64_t col1[64]) {
  for (int x = 0; x < ORACLE_N; ++x) {
    const uint64_t a = s[x];
    const uint64_t up = rotl64(a, 1), dn = rotr64(a, 1);
    col0[x] = up ^ dn ^ a;
    col1[x] = ((up ^ dn) & a) | (up & dn);
  }
}

/* B3/S23 from the centre column and the neighbour columns' 2-bit sums.
 * LifeAPI.hpp:837-848 (LifeState::Rokicki). */
uint64_t oracle_rokicki(uint64_t a, uint64_t bU0, uint64_t bU1, uint64_t bB0, uint64_t bB1) {
  const uint64_t aw = rotl64(a, 1), ae = rotr64(a, 1);
  const uint64_t s0 = aw ^ ae, s1 = aw & ae;
  const uint64_t ts0 = bB0 ^ bU0;
  const uint64_t ts1 = (bB0 & bU0) | (ts0 & s0);
  return (bB1 ^ bU1 ^ ts1 ^ s1) & ((bB1 | bU1) ^ (ts1 | s1)) & ((ts0 ^ s0) | a);
}

/* One generation in place, torus wrap on the column index.
 * LifeAPI.hpp:1196-1216 (LifeState::Step). */
void oracle_step(uint64_t s[64]) {
  uint64_t c0[64], c1[64];
  oracle_count_rows(s, c0, c1);
  for (int x = 0; x < ORACLE_N; ++x) {
    const int xl = (x + ORACLE_N - 1) & (ORACLE_N - 1); /* idxU */
    const int xr = (x + 1) & (ORACLE_N - 1);            /* idxB */
    s[x] = oracle_rokicki(s[x], c0[xl], c1[xl], c0[xr], c1[xr]);
  }
}

/* Same generation via two full adders on the bit planes.
 * LifeAPI.hpp:1218-1254 (LifeState::StepAlt), adders from :822-833. */
void oracle_step_alt(uint64_t s[64]) {
  uint64_t c0[64], c1[64];
  oracle_count_rows(s, c0, c1);
  for (int x = 0; x < ORACLE_N; ++x) {
    const int xl = (x + ORACLE_N - 1) & (ORACLE_N - 1);
    const int xr = (x + 1) & (ORACLE_N - 1);
    const uint64_t a = s[x];
    /* FullAdd(final_sum, final_carry, u_on0, c_on0, l_on0) */
    uint64_t h = c0[xl] ^ c0[x];
    const uint64_t fs = h ^ c0[xr];
    const uint64_t fc = (c0[xl] & c0[x]) | (c0[xr] & h);
    /* FullAdd(carry_sum, carry_carry, u_on1, c_on1, l_on1) */
    h = c1[xl] ^ c1[x];
    const uint64_t cs = h ^ c1[xr];
    uint64_t cc = (c1[xl] & c1[x]) | (c1[xr] & h);
    cc ^= fc & cs;
    s[x] = (fs ^ cc) & (fc ^ cs ^ cc) & (a | fs);
  }
}

/* Inclusive 3x3 count 0..9 as four planes.
 * NeighbourCount.hpp:25-38 (halo CountRows) and :40-70 (adder chain). */
void oracle_neighbour_count(const uint64_t s[64], uint64_t bit3[64], uint64_t bit2[64],
                            uint64_t bit1[64], uint64_t bit0[64]) {
  uint64_t c0[66], c1[66];
  oracle_count_rows(s, c0 + 1, c1 + 1);
  c0[0] = c0[64]; c0[65] = c0[1];
  c1[0] = c1[64]; c1[65] = c1[1];
  for (int x = 0; x < ORACLE_N; ++x) {
    const uint64_t u0 = c0[x], m0 = c0[x + 1], l0 = c0[x + 2];
    const uint64_t u1 = c1[x], m1 = c1[x + 1], l1 = c1[x + 2];
    /* HalfAdd(uc0, uc_carry0, u_on0, c_on0) */
    const uint64_t uc0 = u0 ^ m0, ucc0 = u0 & m0;
    /* FullAdd(uc1, uc2, u_on1, c_on1, uc_carry0) */
    const uint64_t hh = u1 ^ m1;
    const uint64_t uc1 = hh ^ ucc0, uc2 = (u1 & m1) | (ucc0 & hh);
    /* HalfAdd(on0, on_carry0, uc0, l_on0) */
    const uint64_t on0 = uc0 ^ l0, occ0 = uc0 & l0;
    /* FullAdd(on1, on_carry1, uc1, l_on1, on_carry0) */
    const uint64_t h2 = uc1 ^ l1;
    const uint64_t on1 = h2 ^ occ0, occ1 = (uc1 & l1) | (occ0 & h2);
    /* HalfAdd(on2, on3, uc2, on_carry1) */
    bit0[x] = on0;
    bit1[x] = on1;
    bit2[x] = uc2 ^ occ1;
    bit3[x] = uc2 & occ1;
  }
}

/* Life via WithExactly(3) | (s & WithExactly(4)) on the inclusive count.
 * NeighbourCount.hpp:93-102 (WithExactly). */
void oracle_step_nc(uint64_t s[64]) {
  uint64_t b3[64], b2[64], b1[64], b0[64];
  oracle_neighbour_count(s, b3, b2, b1, b0);
  for (int x = 0; x < ORACLE_N; ++x) {
    const uint64_t exactly3 = ~b3[x] & ~b2[x] & b1[x] & b0[x];
    const uint64_t exactly4 = ~b3[x] & b2[x] & ~b1[x] & ~b0[x];
    s[x] = exactly3 | (s[x] & exactly4);
  }
}

/* OFF cells with exactly 1, exactly 2, and more neighbours, plus (optionally)
 * the next generation.  LifeAPI.hpp:956-993 (InteractionCounts) and
 * :997-1040 (InteractionCountsAndNext). */
void oracle_interaction_counts(const uint64_t s[64], uint64_t out1[64], uint64_t out2[64],
                               uint64_t out_more[64], uint64_t next[64]) {
  uint64_t c0[64], c1[64];
  oracle_count_rows(s, c0, c1);
  for (int x = 0; x < ORACLE_N; ++x) {
    const int xl = (x + ORACLE_N - 1) & (ORACLE_N - 1), xr = (x + 1) & (ORACLE_N - 1);
    uint64_t h = c0[xl] ^ c0[x];
    const uint64_t fsum = h ^ c0[xr], fcar = (c0[xl] & c0[x]) | (c0[xr] & h);
    h = c1[xl] ^ c1[x];
    const uint64_t csum = h ^ c1[xr];
    uint64_t ccar = (c1[xl] & c1[x]) | (c1[xr] & h);
    const uint64_t dead = ~s[x];
    out1[x] = dead & ~ccar & fsum & ~csum & ~fcar;
    out2[x] = dead & ~ccar & ~fsum & (csum ^ fcar);
    out_more[x] = dead & ~out2[x] & (fcar | csum | ccar);
    if (next) {
      ccar ^= csum & fcar;
      next[x] = (fsum ^ ccar) & (fcar ^ csum ^ ccar) & (s[x] | fsum);
    }
  }
}

/* LifeWeld::Step (LifeWeld.hpp:169-186), `gens` times, in place on the
 * LifeWeld layout {state, frozen2, frozen1, frozen0} (4 x 64 words): the
 * inclusive count's low three bits (CountNeighbourhood, bit3 dropped) plus
 * the frozen 3-bit count, then the Life rule on the sum. */
void oracle_weld_step(uint64_t w[256], unsigned gens) {
  uint64_t *s = w;
  const uint64_t *f2 = w + 64, *f1 = w + 128, *f0 = w + 192;
  for (unsigned g = 0; g < gens; ++g) {
    uint64_t b3[64], b2[64], b1[64], b0[64];
    oracle_neighbour_count(s, b3, b2, b1, b0);
    for (int x = 0; x < ORACLE_N; ++x) {
      const uint64_t s0 = b0[x] ^ f0[x], k0 = b0[x] & f0[x];
      const uint64_t h1 = b1[x] ^ f1[x];
      const uint64_t s1 = h1 ^ k0, k1 = (b1[x] & f1[x]) | (k0 & h1);
      const uint64_t s2 = b2[x] ^ f2[x] ^ k1;
      s[x] = (s0 ^ s2) & (s1 ^ s2) & (s[x] | s0);
    }
  }
}

/* LifeAPI.hpp:877-881 (LifeState::Step(unsigned)). */
void oracle_step_n(uint64_t s[64], unsigned gens) {
  for (unsigned g = 0; g < gens; ++g) oracle_step(s);
}

typedef struct {
  const uint64_t *in;
  uint64_t *out;
  size_t lo, hi;
  unsigned gens;
  int formulation;
} batch_job;

static void *batch_worker(void *p) {
  const batch_job *j = (const batch_job *)p;
  uint64_t s[64] __attribute__((aligned(64)));
  for (size_t u = j->lo; u < j->hi; ++u) {
    memcpy(s, j->in + u * 64, sizeof s);
    for (unsigned g = 0; g < j->gens; ++g) {
      if (j->formulation == ORACLE_FULLADD) oracle_step_alt(s);
      else if (j->formulation == ORACLE_NCOUNT) oracle_step_nc(s);
      else oracle_step(s);
    }
    memcpy(j->out + u * 64, s, sizeof s);
  }
  return NULL;
}

/* Batched form of LifeAPI.hpp:882-886 (Stepped(unsigned)) over independent
 * universes; each thread owns a contiguous slice. */
void oracle_step_batch(const uint64_t *in, uint64_t *out, size_t n, unsigned gens,
                       int formulation, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
  batch_job jobs[256];
  pthread_t tid[256];
  if (nthreads > 256) nthreads = 256;
  for (int t = 0; t < nthreads; ++t) {
    jobs[t].in = in; jobs[t].out = out;
    jobs[t].lo = n * (size_t)t / (size_t)nthreads;
    jobs[t].hi = n * (size_t)(t + 1) / (size_t)nthreads;
    jobs[t].gens = gens; jobs[t].formulation = formulation;
  }
  if (nthreads == 1) { batch_worker(&jobs[0]); return; }
  for (int t = 0; t < nthreads; ++t) pthread_create(&tid[t], NULL, batch_worker, &jobs[t]);
  for (int t = 0; t < nthreads; ++t) pthread_join(tid[t], NULL);
}

/* LifeAPI.hpp:290-298 (LifeState::GetPop). */
unsigned oracle_pop(const uint64_t s[64]) {
  unsigned p = 0;
  for (int x = 0; x < ORACLE_N; ++x) p += (unsigned)__builtin_popcountll(s[x]);
  return p;
}

void oracle_pop_batch(const uint64_t *s, uint32_t *pop, size_t n) {
  for (size_t u = 0; u < n; ++u) pop[u] = oracle_pop(s + u * 64);
}

/* LifeTarget.hpp:44-51 (LifeState::Contains(const LifeTarget&)). */
int oracle_contains_target(const uint64_t s[64], const uint64_t wanted[64],
                           const uint64_t unwanted[64]) {
  uint64_t diff = 0;
  for (int x = 0; x < ORACLE_N; ++x) diff |= (s[x] ^ wanted[x]) & (wanted[x] | unwanted[x]);
  return diff == 0;
}

/* Parsing.hpp:143-198 (GenericParse + LifeState::Parse): header lines that
 * start with 'x' are dropped, '$' with no count means 1, a count of 129 on
 * '$' stops parsing, any non-'o' cell char is dead.  Coordinates are NOT
 * wrapped by the reference (Set at LifeAPI.hpp:131); out-of-board cells are
 * reported as an error here instead of writing out of bounds. */
int oracle_parse_rle(const char *rle, uint64_t out[64]) {
  memset(out, 0, 64 * sizeof(uint64_t));
  int cnt = 0, x = 0, y = 0, bad = 0;
  const char *p = rle;
  while (*p) {
    const char *eol = strchr(p, '\n');
    const size_t len = eol ? (size_t)(eol - p) : strlen(p);
    if (len == 0 || p[0] != 'x') {
      for (size_t i = 0; i < len; ++i) {
        const char ch = p[i];
        if (ch >= '0' && ch <= '9') {
          cnt = cnt * 10 + (ch - '0');
        } else if (ch == '$') {
          if (cnt == 0) cnt = 1;
          if (cnt == 129) return bad ? -1 : 0;
          y += cnt; x = 0; cnt = 0;
        } else if (ch == '!') {
          return bad ? -1 : 0;
        } else if (ch == '\r' || ch == ' ') {
          continue;
        } else {
          if (cnt == 0) cnt = 1;
          for (int j = 0; j < cnt; ++j, ++x) {
            if (ch != 'o') continue;
            if (x < 0 || x >= 64 || y < 0 || y >= 64) { bad = 1; continue; }
            out[x] |= 1ULL << y;
          }
          cnt = 0;
        }
      }
    }
    if (!eol) break;
    p = eol + 1;
  }
  return bad ? -1 : 0;
}

/* LifeState::RLE() = GenericRLE with cellchar 'o'/'b' (Parsing.hpp:8-63,
 * 200-204): rows printed from y = 32 (torus_wrap(j + 32)), cells from
 * x = 32 (torus_wrap(i + N/2)); per row, runs "<n>o" / "<n>b" (n omitted
 * when 1) with a dead run at the end of a row dropped; a row's first live
 * cell is preceded by the rows passed since the last flush as "<k>$"; no
 * trailing "$" (flushtrailing = false); then "!".  Writes at most `cap`
 * bytes (no NUL) and returns the full length. */
static size_t rle_put_count(char *out, size_t n, size_t cap, unsigned count) {
  char digits[12];
  int k = 0;
  if (count <= 1) return n;
  while (count) { digits[k++] = (char)('0' + count % 10); count /= 10; }
  while (k) { if (n < cap) out[n] = digits[--k]; else --k; ++n; }
  return n;
}

size_t oracle_rle(const uint64_t s[64], char *out, size_t cap) {
  size_t n = 0;
  unsigned rows_pending = 0;
  for (unsigned j = 0; j < 64; ++j) {
    const unsigned y = (j + 32) & 63;
    int last = (int)((s[32] >> y) & 1);
    unsigned run = 0;
    for (unsigned i = 0; i < 64; ++i) {
      const int cell = (int)((s[(i + 32) & 63] >> y) & 1);
      if (cell && rows_pending) {
        n = rle_put_count(out, n, cap, rows_pending);
        if (n < cap) out[n] = '$';
        ++n;
        rows_pending = 0;
      }
      if (cell != last) {
        n = rle_put_count(out, n, cap, run);
        if (n < cap) out[n] = last ? 'o' : 'b';
        ++n;
        run = 0;
      }
      ++run;
      last = cell;
    }
    if (last) {
      n = rle_put_count(out, n, cap, run);
      if (n < cap) out[n] = 'o';
      ++n;
    }
    ++rows_pending;
  }
  if (n < cap) out[n] = '!';
  return n + 1;
}

/* ---- build-defined synthetic input and digests (no reference analogue) ---- */

#define GOLDEN 0x9E3779B97F4A7C15ULL

uint64_t oracle_splitmix64_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

/* Word w (global index u*64+x) = splitmix64 output number w+1 of `seed`.
 * mode 0: uniform density-0.5 columns.
 * mode 1: RandomState()-shaped columns, uniform on [2^61, 2^62) like
 *         LifeAPI.hpp:18-23,63-69 (row 61 on, rows 62-63 off). */
void oracle_fill(uint64_t *out, size_t n, uint64_t seed, uint64_t first_universe, int mode) {
  for (size_t i = 0; i < n * 64; ++i) {
    const uint64_t w = first_universe * 64 + i;
    uint64_t v = oracle_splitmix64_mix(seed + (w + 1) * GOLDEN);
    if (mode == 1) v = (v & ((1ULL << 61) - 1)) | (1ULL << 61);
    out[i] = v;
  }
}

/* Per-universe hash: mix(sum_x mix(s[x] + (x+1)*GOLDEN)), order sensitive in x. */
uint64_t oracle_universe_hash(const uint64_t s[64]) {
  uint64_t acc = 0;
  for (int x = 0; x < ORACLE_N; ++x) acc += oracle_splitmix64_mix(s[x] + (uint64_t)(x + 1) * GOLDEN);
  return oracle_splitmix64_mix(acc);
}

void oracle_hash_batch(const uint64_t *s, uint64_t *h, size_t n) {
  for (size_t u = 0; u < n; ++u) h[u] = oracle_universe_hash(s + u * 64);
}

/* Batch digest: sum_u mix(h_u + (u_global+1)*GOLDEN) -- additive, so shard
 * digests combine by 64-bit addition. */
uint64_t oracle_batch_digest(const uint64_t *hashes, size_t n, uint64_t first_universe) {
  uint64_t acc = 0;
  for (size_t u = 0; u < n; ++u)
    acc += oracle_splitmix64_mix(hashes[u] + (first_universe + u + 1) * GOLDEN);
  return acc;
}

/* ---- LifeStable passes (LifeStable.hpp:526-729) ----
 * planes: {state, unknown, live2, live3, dead0, dead1, dead2, dead4, dead5,
 * dead6} x 64 words (class member order, LifeStable.hpp:41-53; options are
 * "1 = ruled out").  The espresso fragments stable_count.hpp / stable_signal.hpp
 * are evaluated by TABLE LOOKUP in their complete truth tables (tests/golden/
 * stable_{count,signal}_tt.npz, extracted from the reference build):
 * tt_count = 9 x 512 bytes, tt_signal = 4 x 131072 bytes.  Returns
 * consistent | changed << 1, like LifeStable::PropagateResult. */
enum { ST, UN, L2, L3, D0, D1, D2, D4, D5, D6 };
#define PL(p, k) ((p) + (k) * 64)

/* LifeStable.hpp:526-556 */
static int stable_sync(uint64_t *p) {
  uint64_t changes = 0, abort_ = 0, ml[64], md[64];
  for (int x = 0; x < 64; ++x) {
    const uint64_t known_on = ~PL(p, UN)[x] & PL(p, ST)[x];
    md[x] = ~(PL(p, D0)[x] & PL(p, D1)[x] & PL(p, D2)[x] & PL(p, D4)[x] & PL(p, D5)[x] & PL(p, D6)[x]);
    changes |= md[x] & known_on;
    for (int k = D0; k <= D6; ++k) PL(p, k)[x] |= known_on;
    const uint64_t known_off = ~PL(p, UN)[x] & ~PL(p, ST)[x];
    ml[x] = ~(PL(p, L2)[x] & PL(p, L3)[x]);
    changes |= ml[x] & known_off;
    PL(p, L2)[x] |= known_off;
    PL(p, L3)[x] |= known_off;
    abort_ |= ~ml[x] & ~md[x];
  }
  if (abort_) return 0;
  for (int x = 0; x < 64; ++x) {
    changes |= ~PL(p, ST)[x] & (ml[x] & ~md[x]);
    PL(p, ST)[x] |= ml[x] & ~md[x];
    changes |= ~PL(p, UN)[x] & (ml[x] & md[x]);
    PL(p, UN)[x] &= ml[x] & md[x];
  }
  return 1 | (changes ? 2 : 0);
}

static unsigned cell_index(const uint64_t *w, int nin, int y) {
  unsigned idx = 0;
  for (int i = 0; i < nin; ++i) idx |= (unsigned)((w[i] >> y) & 1u) << i;
  return idx;
}

/* LifeStable.hpp:558-615 */
static int stable_options(uint64_t *p, const uint8_t *tt) {
  uint64_t off[64], s3[64], s2[64], s1[64], s0[64], o3[64], o2[64], o1[64], o0[64];
  for (int x = 0; x < 64; ++x) off[x] = ~PL(p, UN)[x] & ~PL(p, ST)[x];
  oracle_neighbour_count(PL(p, ST), s3, s2, s1, s0);
  oracle_neighbour_count(off, o3, o2, o1, o0);
  uint64_t has_abort = 0, changes = 0;
  for (int x = 0; x < 64; ++x) {
    const uint64_t in[9] = {s2[x], s1[x], s0[x], o3[x], o2[x], o1[x], o0[x], PL(p, ST)[x], off[x]};
    uint64_t r[9] = {0};
    for (int y = 0; y < 64; ++y) {
      const unsigned idx = cell_index(in, 9, y);
      for (int k = 0; k < 9; ++k) r[k] |= (uint64_t)(tt[k * 512 + idx] & 1u) << y;
    }
    for (int k = 0; k < 8; ++k) {  /* l2 l3 d0 d1 d2 d4 d5 d6 -> planes L2.. D6 */
      changes |= r[k] & ~PL(p, L2 + k)[x];
      PL(p, L2 + k)[x] |= r[k];
    }
    has_abort |= r[8];
  }
  return (has_abort == 0) | (changes ? 2 : 0);
}

/* LifeAPI.hpp:541-562 (ZOIHollow) */
static void zoi_hollow(const uint64_t *s, uint64_t *out) {
  uint64_t t[64], m[64];
  for (int x = 0; x < 64; ++x) {
    m[x] = rotl64(s[x], 1) | rotr64(s[x], 1);
    t[x] = s[x] | m[x];
  }
  for (int x = 0; x < 64; ++x) out[x] = t[(x + 63) & 63] | m[x] | t[(x + 1) & 63];
}

/* LifeStable.hpp:617-675 */
static int stable_signal(uint64_t *p, const uint8_t *tt) {
  uint64_t mx[64], s3[64], s2[64], s1[64], s0[64], m3[64], m2[64], m1[64], m0[64];
  uint64_t soff[64], son[64], coff[64], con[64], offz[64], onz[64];
  for (int x = 0; x < 64; ++x) mx[x] = PL(p, ST)[x] | PL(p, UN)[x];
  oracle_neighbour_count(PL(p, ST), s3, s2, s1, s0);
  oracle_neighbour_count(mx, m3, m2, m1, m0);
  for (int x = 0; x < 64; ++x) {
    const uint64_t in[17] = {PL(p, L2)[x], PL(p, L3)[x], PL(p, D0)[x], PL(p, D1)[x], PL(p, D2)[x],
                             PL(p, D4)[x], PL(p, D5)[x], PL(p, D6)[x], s2[x], s1[x], s0[x],
                             m3[x], m2[x], m1[x], m0[x], PL(p, ST)[x], PL(p, UN)[x]};
    uint64_t r[4] = {0};
    for (int y = 0; y < 64; ++y) {
      const unsigned idx = cell_index(in, 17, y);
      for (int k = 0; k < 4; ++k) r[k] |= (uint64_t)(tt[k * 131072 + idx] & 1u) << y;
    }
    soff[x] = r[0]; son[x] = r[1]; coff[x] = r[2]; con[x] = r[3];
  }
  zoi_hollow(soff, offz);
  zoi_hollow(son, onz);
  uint64_t clash = 0, changes = 0;
  for (int x = 0; x < 64; ++x) {
    offz[x] |= coff[x];
    onz[x] |= con[x];
    clash |= offz[x] & onz[x] & PL(p, UN)[x];
  }
  if (clash) return 0;
  for (int x = 0; x < 64; ++x) {
    changes |= (offz[x] & PL(p, UN)[x]) | (onz[x] & PL(p, UN)[x]);
    const uint64_t w_off = offz[x] & PL(p, UN)[x];   /* SetOff, LifeStable.hpp:330-335 */
    PL(p, ST)[x] &= ~w_off;
    PL(p, UN)[x] &= ~w_off;
    PL(p, L2)[x] |= w_off;
    PL(p, L3)[x] |= w_off;
    const uint64_t w_on = onz[x] & PL(p, UN)[x];     /* SetOn, LifeStable.hpp:320-329 */
    PL(p, ST)[x] |= w_on;
    PL(p, UN)[x] &= ~w_on;
    for (int k = D0; k <= D6; ++k) PL(p, k)[x] |= w_on;
  }
  return 1 | (changes ? 2 : 0);
}

/* LifeStable.hpp:695-716 */
static int stable_step(uint64_t *p, const uint8_t *ttc, const uint8_t *tts) {
  const int k = stable_sync(p);
  if (!(k & 1)) return 0;
  const int o = stable_options(p, ttc);
  if (!(o & 1)) return 0;
  const int s = stable_signal(p, tts);
  if (!(s & 1)) return 0;
  return 1 | ((k | o | s) & 2);
}

/* LifeStable::Vulnerable() (LifeStable.hpp:366-412): the cells whose
 * neighbourhood admits both an ON and an OFF stable completion.  The
 * stable_vulnerable.hpp fragment (15 inputs: options, NeighbourCount bits
 * 2..0 of state, bits 3..0 of unknown) is evaluated by table lookup in tt
 * (4 x 2^15, extracted from the reference build); then
 * on = ZOIHollow(vulnerable_on) | vulnerable_center_on, likewise off, and
 * the result is on & off. */
void oracle_stable_vulnerable(const uint64_t *p, uint64_t out[64], const uint8_t *tt) {
  uint64_t s3[64], s2[64], s1[64], s0[64], u3[64], u2[64], u1[64], u0[64];
  uint64_t von[64], voff[64], vcon[64], vcoff[64], onz[64], offz[64];
  oracle_neighbour_count(PL(p, ST), s3, s2, s1, s0);
  oracle_neighbour_count(PL(p, UN), u3, u2, u1, u0);
  for (int x = 0; x < 64; ++x) {
    const uint64_t in[15] = {PL(p, L2)[x], PL(p, L3)[x], PL(p, D0)[x], PL(p, D1)[x], PL(p, D2)[x],
                             PL(p, D4)[x], PL(p, D5)[x], PL(p, D6)[x], s2[x], s1[x], s0[x],
                             u3[x], u2[x], u1[x], u0[x]};
    uint64_t r[4] = {0};
    for (int y = 0; y < 64; ++y) {
      const unsigned idx = cell_index(in, 15, y);
      for (int k = 0; k < 4; ++k) r[k] |= (uint64_t)(tt[k * 32768 + idx] & 1u) << y;
    }
    von[x] = r[0]; voff[x] = r[1]; vcon[x] = r[2]; vcoff[x] = r[3];
  }
  zoi_hollow(von, onz);
  zoi_hollow(voff, offz);
  for (int x = 0; x < 64; ++x) out[x] = (onz[x] | vcon[x]) & (offz[x] | vcoff[x]);
}

int oracle_stable_pass(uint64_t *planes, int which, const uint8_t *tt_count,
                       const uint8_t *tt_signal) {
  switch (which) {
    case 0: return stable_sync(planes);
    case 1: return stable_options(planes, tt_count);
    case 2: return stable_signal(planes, tt_signal);
    case 3: return stable_step(planes, tt_count, tt_signal);
    case 5: { /* StabiliseOptions, LifeStable.hpp:677-693 */
      int ever = 0;
      for (;;) {
        const int k = stable_sync(planes);
        if (!(k & 1)) return 0;
        const int o = stable_options(planes, tt_count);
        if (!(o & 1)) return 0;
        if (!((k | o) & 2)) return 1 | ever;
        ever = 2;
      }
    }
    default: { /* LifeStable.hpp:718-729 */
      int ever = 0;
      for (;;) {
        const int r = stable_step(planes, tt_count, tt_signal);
        if (!(r & 1)) return 0;
        if (!(r & 2)) return 1 | ever;
        ever = 2;
      }
    }
  }
}

/* ---- config 5: the unknown_step_refined harness ----
 * bitslicing/unknown_step_refined.hpp:1-85 is an espresso sum-of-products
 * over 16 per-cell inputs.  The oracle evaluates that function by TABLE
 * LOOKUP: tt holds the fragment's complete truth table (3 x 65536 bytes of
 * 0/1, index bit i = input i in the order l2 l3 d0 d1 d2 d4 d5 d6
 * current_unknown current_on s2 s1 s0 on2 on1 on0), extracted from the
 * reference build by tests/golden/make_golden.py.  Inputs per universe: 11
 * planes (stable.state, current.state, current.unknown, live2, live3, dead0,
 * dead1, dead2, dead4, dead5, dead6); s* / on* = bits 2..0 of the inclusive
 * NeighbourCount (NeighbourCount.hpp:40-70) of stable.state / current.state.
 * Output: next_on, next_unknown, next_unknown_stable planes. */
void oracle_refined_step_batch(const uint64_t *in, uint64_t *out, size_t n, const uint8_t *tt) {
  for (size_t u = 0; u < n; ++u) {
    const uint64_t *p = in + u * 11 * 64;
    uint64_t *o = out + u * 3 * 64;
    uint64_t s3[64], s2[64], s1[64], s0[64], c3[64], c2[64], c1[64], c0[64];
    oracle_neighbour_count(p, s3, s2, s1, s0);
    oracle_neighbour_count(p + 64, c3, c2, c1, c0);
    for (int x = 0; x < 64; ++x) {
      const uint64_t planes[16] = {p[3 * 64 + x], p[4 * 64 + x], p[5 * 64 + x], p[6 * 64 + x],
                                   p[7 * 64 + x], p[8 * 64 + x], p[9 * 64 + x], p[10 * 64 + x],
                                   p[2 * 64 + x], p[1 * 64 + x], s2[x], s1[x], s0[x],
                                   c2[x], c1[x], c0[x]};
      uint64_t r0 = 0, r1 = 0, r2 = 0;
      for (int y = 0; y < 64; ++y) {
        unsigned idx = 0;
        for (int i = 0; i < 16; ++i) idx |= (unsigned)((planes[i] >> y) & 1u) << i;
        r0 |= (uint64_t)(tt[idx] & 1u) << y;
        r1 |= (uint64_t)(tt[65536 + idx] & 1u) << y;
        r2 |= (uint64_t)(tt[2 * 65536 + idx] & 1u) << y;
      }
      o[x] = r0;
      o[64 + x] = r1;
      o[128 + x] = r2;
    }
  }
}
