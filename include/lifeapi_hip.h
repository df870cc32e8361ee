/*
 * lifeapi_hip.h -- C ABI of the MI355X (gfx950) batched LifeState::Step().
 *
 * The reference (scorbiclife/LifeAPI) is a header-only C++ library with no
 * FFI; its "operator API" is the inline member functions of LifeState.  Each
 * entry point below is the batched, device-resident replacement for one of
 * them, cited as file:line into the reference snapshot:
 *
 *   lifeapi_step_batch[_dev]     LifeState::Step()          LifeAPI.hpp:1196-1216
 *                                LifeState::Step(unsigned)  LifeAPI.hpp:877-881
 *                                LifeState::Stepped(unsigned) LifeAPI.hpp:882-886
 *   lifeapi_pop_batch_dev        LifeState::GetPop()        LifeAPI.hpp:290-298
 *   lifeapi_contains_batch_dev   LifeState::Contains(const LifeTarget&)
 *                                                           LifeTarget.hpp:44-51
 *   lifeapi_fill_random_dev      LifeState::RandomState()   LifeAPI.hpp:63-69
 *                                (seeded splitmix64; mode 1 = RandomState's
 *                                 [2^61, 2^62) column distribution)
 *   lifeapi_parse_rle_batch[_dev] LifeState::Parse          Parsing.hpp:143-198
 *   lifeapi_rle_*batch[_dev]     LifeState::RLE()           Parsing.hpp:8-63,200-204
 *   lifeapi_hash_batch_dev       (build-defined digest; stands in for
 *                                 LifeState::GetHash, LifeAPI.hpp:373, which
 *                                 needs the un-vendored xxHash)
 *
 * Data layout: a universe is the reference's LifeState, i.e. uint64_t[64]
 * (word x = column x, bit y = row y; LifeAPI.hpp:39-40,131), 512 bytes.  A
 * batch is a contiguous array of n universes = n*64 words.  Pointers must be
 * 8-byte aligned (LifeState is 64-byte aligned, so a LifeState[] always is).
 * in == out is allowed (in-place, like Step()); any other overlap is rejected.
 *
 * Conventions: every function returns 0 on success; a negative LIFEAPI_E_*
 * for a caller error; a positive hipError_t from the HIP runtime otherwise.
 * lifeapi_last_error() gives this thread's message for the last failure.
 * Nothing throws across this ABI.  The library owns only internal staging
 * buffers and streams (one per device, created lazily); the caller owns all
 * arguments.  *_dev functions take device pointers and enqueue on `stream`
 * (a hipStream_t; NULL = the null stream) without synchronising.  The host
 * functions are synchronous and thread-safe (one lock per device).
 */
#ifndef LIFEAPI_HIP_H
#define LIFEAPI_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LIFEAPI_ABI_VERSION 2

#define LIFEAPI_OK 0
#define LIFEAPI_E_INVALID (-1)   /* null/misaligned pointer, overlap, bad argument */
#define LIFEAPI_E_NODEVICE (-2)  /* no gfx950 device / bad device index */
#define LIFEAPI_E_NOKERNEL (-3)  /* code object for this GPU missing */

int lifeapi_abi_version(void);
const char *lifeapi_last_error(void);
int lifeapi_device_count(void);
/* which shipped kernel configuration lifeapi_step_batch[_dev] runs for this
 * many generations on a batch of n universes (the launch shape changes with
 * the batch size above 4M universes; a static string, for logs and benchmark
 * records); lifeapi_step_kernel_name(g) is the name for batches of at most 4M */
const char *lifeapi_step_kernel_name_n(uint32_t generations, size_t n);
const char *lifeapi_step_kernel_name(uint32_t generations);

/* ---- device-resident, stream-ordered (the hot path) -------------------- */

/* out[u] = in[u] stepped `generations` times (0 = copy), for u < n.  For
 * 1-2 generations and 192K <= n <= 4M a call whose input is a batch an
 * earlier call wrote walks it in the opposite order to that call (a per-device
 * book of the last batches written; a cache-locality choice for back-to-back
 * calls on the batch just written); above 4M each XCD takes a contiguous
 * eighth of the batch.  Results never depend on either, and
 * calls from several threads are safe.                                    */
int lifeapi_step_batch_dev(const uint64_t *d_in, uint64_t *d_out, size_t n,
                           uint32_t generations, void *stream);
/* d_pop[u] = population of universe u                                     */
int lifeapi_pop_batch_dev(const uint64_t *d_states, uint32_t *d_pop, size_t n, void *stream);
/* d_hash[u] = build-defined 64-bit hash of universe u     */
int lifeapi_hash_batch_dev(const uint64_t *d_states, uint64_t *d_hash, size_t n, void *stream);
/* d_out[u] = Contains(target) for target = (wanted, unwanted), both device
 * pointers to 64 words (LifeTarget.hpp:44-51).  Only the columns holding the
 * target's care cells (wanted | unwanted) are read from each universe.  With
 * unwanted = 0 this is Contains(pat), with wanted = 0 AreDisjoint(pat)
 * (LifeAPI.hpp:377-397); the (dx, dy) forms are these on the pattern moved by
 * (dx, dy) (LifeAPI.hpp:399-421).                                           */
int lifeapi_contains_batch_dev(const uint64_t *d_states, const uint64_t *d_wanted,
                               const uint64_t *d_unwanted, uint8_t *d_out, size_t n,
                               void *stream);
/* fused Step^gens + Contains: d_out[u] = first generation g in 1..gens at
 * which Stepped(g) contains the target, or 0 if none (all 0 for gens = 0);
 * d_final (may be NULL) receives Stepped(gens).  With d_final NULL (the
 * search filter) only the target's light cone is read and stepped: at 1-2
 * generations the columns within gens of its care columns, from 3 the
 * columns of a cone of at most 32 columns and the rows of a cone that fits
 * 32 rows; a target with neither is stepped whole.  Nothing is remembered
 * between calls: the target buffers may be rewritten between them.         */
int lifeapi_step_contains_batch_dev(const uint64_t *d_in, uint64_t *d_final,
                                    const uint64_t *d_wanted, const uint64_t *d_unwanted,
                                    uint32_t *d_first_gen, size_t n, uint32_t generations,
                                    void *stream);
/* Inclusive 3x3 neighbourhood count of each universe as 4 planes:
 * d_out = n x {bit3, bit2, bit1, bit0} x 64 words.
 * Replaces NeighbourCount(const LifeState&) (NeighbourCount.hpp:40-70) and
 * LifeState::CountNeighbourhood (LifeAPI.hpp:909-952).                    */
int lifeapi_neighbour_count_batch_dev(const uint64_t *d_in, uint64_t *d_out, size_t n, void *stream);
/* LifeState::InteractionCounts (LifeAPI.hpp:956-993): d_out = n x {out1,
 * out2, outMore} x 64 words; with_next != 0: InteractionCountsAndNext
 * (LifeAPI.hpp:997-1040), d_out = n x {out1, out2, outMore, next} x 64.     */
int lifeapi_interaction_counts_batch_dev(const uint64_t *d_in, uint64_t *d_out, size_t n,
                                         int with_next, void *stream);
/* LifeStable propagation passes, in place on LifeStable[n] = {state,
 * unknown, live2, live3, dead0, dead1, dead2, dead4, dead5, dead6} x 64
 * words (member order, LifeStable.hpp:41-53; option planes 1 = ruled out).
 * pass: 0 SynchroniseStateKnown (LifeStable.hpp:526-556), 1 UpdateOptions
 * (:558-615), 2 SignalNeighbours (:617-675), 3 PropagateStep (:695-716),
 * 4 Propagate (:718-729, at most max_iters steps; 0 = 2^20),
 * 5 StabiliseOptions (:677-693, the same bound).
 * d_flags[u] = consistent | changed << 1 (| 4 if max_iters stopped 4 / 5),
 * i.e. the PropagateResult; planes are left exactly as the reference leaves
 * them, including on an inconsistent early return.  Only the 128-byte lines
 * holding a changed column are written back (the rest is already there).  */
int lifeapi_stable_pass_batch_dev(uint64_t *d_planes, uint8_t *d_flags, size_t n, int pass,
                                  uint32_t max_iters, void *stream);
/* LifeStable::Vulnerable() (LifeStable.hpp:366-412) of every LifeStable[n]
 * (layout as above): d_out = n LifeStates.                                */
int lifeapi_stable_vulnerable_batch_dev(const uint64_t *d_planes, uint64_t *d_out, size_t n, void *stream);
/* LifeWeld::Step() (LifeWeld.hpp:169-186) `generations` times, in place on
 * LifeWeld[n] = {state, frozen2, frozen1, frozen0} x 64 words (the struct's
 * member order, LifeWeld.hpp:18-20); only the state planes change.        */
int lifeapi_weld_step_batch_dev(uint64_t *d_welds, size_t n, uint32_t generations, void *stream);
/* Config-5 ternary step: bitslicing/unknown_step_refined.hpp:1-85 applied
 * per column with s2..s0 / on2..on0 = bits 2..0 of NeighbourCount
 * (NeighbourCount.hpp:40-70) of stable.state / current.state.
 * d_in: n x 11 planes x 64 words (stable.state, current.state,
 * current.unknown, live2, live3, dead0, dead1, dead2, dead4, dead5, dead6;
 * option planes 1 = ruled out, LifeStable.hpp:41-53).  d_out: n x 3 planes
 * (next_on, next_unknown, next_unknown_stable).  No overlap allowed.      */
int lifeapi_refined_step_batch_dev(const uint64_t *d_in, uint64_t *d_out, size_t n, void *stream);
/* synthetic universes: word w = u*64+x (u counted from first_universe) is
 * splitmix64(seed + (w+1)*0x9E3779B97F4A7C15); mode 1 maps each column to
 * [2^61, 2^62) like RandomState()                                         */
int lifeapi_fill_random_dev(uint64_t *d_out, size_t n, uint64_t seed,
                            uint64_t first_universe, int mode, void *stream);
/* RLE batch I/O.  Text is a byte blob; pattern u is bytes
 * [offsets[u], offsets[u+1]) (n+1 offsets, no terminators).
 * LifeState::RLE() (Parsing.hpp:8-63,200-204; rows and columns printed
 * from 32, as the reference does): lengths first, the caller scans them
 * into offsets, then the write.                                           */
int lifeapi_rle_lengths_batch_dev(const uint64_t *d_states, uint32_t *d_len, size_t n, void *stream);
int lifeapi_rle_write_batch_dev(const uint64_t *d_states, const uint64_t *d_offsets, char *d_text,
                                size_t n, void *stream);
/* LifeState::Parse (GenericParse, Parsing.hpp:143-198) of every pattern.
 * d_status[u] bit 0: a live cell off the 64x64 board was dropped (the
 * reference writes out of bounds there); bit 1: parsing stopped at a "$"
 * count of 129 (the reference's early return, Parsing.hpp:171-173).       */
int lifeapi_parse_rle_batch_dev(const char *d_text, const uint64_t *d_offsets, size_t n,
                                uint64_t *d_out, uint8_t *d_status, void *stream);

/* ---- host pointers, synchronous ----------------------------------------- */

/* Stages through device memory of `device` (or of every visible device,
 * contiguous shards, one host thread each, when device == -1; the
 * environment variable LIFEAPI_HOST_SHARDS=k overrides that shard count,
 * shard s running on device s mod count -- a rehearsal knob for machines
 * with fewer GPUs).                                                        */
int lifeapi_step_batch(const uint64_t *in, uint64_t *out, size_t n, uint32_t generations,
                       int device);
int lifeapi_pop_batch(const uint64_t *states, uint32_t *pop, size_t n, int device);
/* host-pointer forms of the *_dev entry points above (same layouts); each
 * stages through `device` in chunks of <= 64 MiB per array, two chunks in
 * flight (one per direction of the link); device -1 shards over every
 * visible device as above                                                 */
int lifeapi_weld_step_batch(uint64_t *welds, size_t n, uint32_t generations, int device);
int lifeapi_stable_pass_batch(uint64_t *planes, uint8_t *flags, size_t n, int pass,
                              uint32_t max_iters, int device);
int lifeapi_stable_vulnerable_batch(const uint64_t *planes, uint64_t *out, size_t n, int device);
int lifeapi_neighbour_count_batch(const uint64_t *in, uint64_t *out, size_t n, int device);
int lifeapi_interaction_counts_batch(const uint64_t *in, uint64_t *out, size_t n, int with_next,
                                     int device);
int lifeapi_refined_step_batch(const uint64_t *in, uint64_t *out, size_t n, int device);
int lifeapi_contains_batch(const uint64_t *states, const uint64_t *wanted, const uint64_t *unwanted,
                           uint8_t *out, size_t n, int device);
/* host form of lifeapi_step_contains_batch_dev: the search-loop idiom
 * "for g in 1..gens: s.Step(); if (s.Contains(target)) ..." (LifeAPI.hpp:
 * 1196-1216, LifeTarget.hpp:44-51) over n host universes; final (may be NULL,
 * may equal in) receives Stepped(gens); device -1 shards the batch over all
 * visible GPUs as lifeapi_step_batch does                                  */
int lifeapi_step_contains_batch(const uint64_t *in, uint64_t *final_states, const uint64_t *wanted,
                                const uint64_t *unwanted, uint32_t *first_gen, size_t n,
                                uint32_t generations, int device);
/* RLE of every state: fills offsets[0..n] (offsets[n] = total bytes); with
 * text == NULL only the offsets (size query), else writes the patterns to
 * text (LIFEAPI_E_INVALID if text_cap < offsets[n])                       */
int lifeapi_rle_batch(const uint64_t *states, size_t n, char *text, size_t text_cap, uint64_t *offsets,
                      int device);
int lifeapi_parse_rle_batch(const char *text, const uint64_t *offsets, size_t n, uint64_t *out,
                            uint8_t *status, int device);

/* Page-lock a host array the caller reuses across calls (hipHostRegister,
 * portable to every device).  The host-pointer entry points move page-locked
 * memory by DMA in both directions at once (about 97 GB/s combined against
 * 56 GB/s for pageable memory, profiles/r01/host_bench.jsonl).  A call moving
 * at least 8 MiB pins pageable arrays itself for its duration, so this is
 * optional: it holds the pin across calls, and covers smaller calls.
 * Unregister before freeing the memory, and do not register or unregister
 * an array while another thread's call on it is in flight (the per-call
 * pins are counted across threads; the runtime does not count
 * registrations).  New in this build: the reference has no host/device
 * split at all.                                                            */
int lifeapi_host_register(void *p, size_t bytes);
int lifeapi_host_unregister(void *p);

#ifdef __cplusplus
}
#endif
#endif /* LIFEAPI_HIP_H */
