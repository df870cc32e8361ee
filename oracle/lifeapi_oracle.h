/*
 * lifeapi_oracle.h -- CPU restatement of LifeAPI's Step() path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the timed CPU baseline.  The product path
 * (lifeapi_amd/, include/lifeapi/) never calls into it.
 *
 * Parity status: PINNED.  The restatement is checked bit-for-bit against the
 * reference's own Step()/StepAlt()/NeighbourCount built from
 * /root/reference by oracle/Makefile (target `ref`, outputs in oracle/_ref/)
 * and against the golden vectors under tests/golden/ that the reference
 * build generated (tests/golden/make_golden.py).
 *
 * Layout (LifeAPI.hpp:39-40,131): a universe is uint64_t state[64]; word x
 * is column x, bit y of that word is cell (x, y).  Batches are contiguous
 * arrays of universes (64 words = 512 bytes each).
 */
#ifndef LIFEAPI_ORACLE_H
#define LIFEAPI_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_N 64

/* formulation selector for oracle_step_batch */
enum {
  ORACLE_ROKICKI = 0, /* LifeState::Step()       LifeAPI.hpp:1196-1216 */
  ORACLE_FULLADD = 1, /* LifeState::StepAlt()    LifeAPI.hpp:1218-1254 */
  ORACLE_NCOUNT = 2   /* NeighbourCount rule     NeighbourCount.hpp:40-102 */
};

void oracle_count_rows(const uint64_t s[64], uint64_t col0[64], uint64_t col1[64]);
uint64_t oracle_rokicki(uint64_t a, uint64_t bU0, uint64_t bU1, uint64_t bB0, uint64_t bB1);
void oracle_step(uint64_t s[64]);
void oracle_step_alt(uint64_t s[64]);
void oracle_neighbour_count(const uint64_t s[64], uint64_t bit3[64], uint64_t bit2[64],
                            uint64_t bit1[64], uint64_t bit0[64]);
void oracle_step_nc(uint64_t s[64]);
void oracle_step_n(uint64_t s[64], unsigned gens);

/* in -> out (in == out allowed), n universes, `gens` generations each. */
void oracle_step_batch(const uint64_t *in, uint64_t *out, size_t n, unsigned gens,
                       int formulation, int nthreads);

unsigned oracle_pop(const uint64_t s[64]);
void oracle_pop_batch(const uint64_t *s, uint32_t *pop, size_t n);
int oracle_contains_target(const uint64_t s[64], const uint64_t wanted[64],
                           const uint64_t unwanted[64]);
/* returns 0 on success, -1 on a cell outside the 64x64 board */
int oracle_parse_rle(const char *rle, uint64_t out[64]);
size_t oracle_rle(const uint64_t s[64], char *out, size_t cap);

/* build-defined synthetic input: splitmix64 stream indexed by global word */
uint64_t oracle_splitmix64_mix(uint64_t z);
void oracle_fill(uint64_t *out, size_t n, uint64_t seed, uint64_t first_universe, int mode);

/* build-defined digests (checksum of checksums, additive over shards) */
uint64_t oracle_universe_hash(const uint64_t s[64]);
void oracle_hash_batch(const uint64_t *s, uint64_t *h, size_t n);
uint64_t oracle_batch_digest(const uint64_t *hashes, size_t n, uint64_t first_universe);

/* LifeAPI.hpp:956-1040 (InteractionCounts / InteractionCountsAndNext);
 * next may be NULL */
void oracle_interaction_counts(const uint64_t s[64], uint64_t out1[64], uint64_t out2[64],
                               uint64_t out_more[64], uint64_t next[64]);

/* LifeWeld.hpp:169-186: in place on {state, frozen2, frozen1, frozen0} */
void oracle_weld_step(uint64_t w[256], unsigned gens);

/* LifeStable passes, in place on 10 planes (see lifeapi_oracle.c):
 * which = 0 SynchroniseStateKnown, 1 UpdateOptions, 2 SignalNeighbours,
 * 3 PropagateStep, 4 Propagate, 5 StabiliseOptions (LifeStable.hpp:677-693).
 * Returns consistent | changed << 1. */
void oracle_stable_vulnerable(const uint64_t *planes, uint64_t out[64], const uint8_t *tt);
int oracle_stable_pass(uint64_t *planes, int which, const uint8_t *tt_count,
                       const uint8_t *tt_signal);

/* config 5 harness (see lifeapi_oracle.c): 11 planes in, 3 planes out per
 * universe; tt = the reference fragment's truth table, 3 x 65536 bytes */
void oracle_refined_step_batch(const uint64_t *in, uint64_t *out, size_t n, const uint8_t *tt);

#ifdef __cplusplus
}
#endif
#endif
