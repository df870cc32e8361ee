// step.hip -- batched LifeState::Step() (LifeAPI.hpp:1196-1216, Stepped(n)
// :877-886) and the fused Step + Contains (LifeTarget.hpp:44-51): the
// shipped kernel configurations and their C ABI (include/lifeapi_hip.h).
// The kernels are in step_kernels.hpp; the measured alternatives (other
// networks, exchanges, layouts and schedules) live in the tuning build,
// tools/tune/tune_step.hip, and are not part of this library.
#include <algorithm>

#include "cone_kernels.hpp"

using namespace lifeapi_impl;

namespace {

using StepFn = void (*)(const uint64_t *, uint64_t *, uint64_t, uint32_t, uint64_t);

// The shipped configurations (profiles/r01/tune_*.jsonl):
// * gens <= 2 -- HBM-streaming: natural layout, DPP exchange, the 7-LUT
//   network, 4 universes in flight per wave, nontemporal loads (no layout
//   change to pay for);
// * gens > 2 -- VALU-bound: 8-way row split with 4 universes interleaved bit
//   by bit, LDS exchange, the 6-LUT tail, state resident in VGPRs for all
//   generations, as the hand-allocated loop of split_asm.inc; nontemporal
//   below 32 generations.  One-shot grids: every capped grid-stride grid
//   measured slower.
// Batches above kCachedUniverses run with at most 7 blocks (28 waves)
// resident per CU instead of the 8 its registers allow, set by unused dynamic
// LDS: fewer concurrent streams per CU, better served by HBM.  Round 3,
// exact caps (host.hip occupancy_lds), same process, ping-pong with the
// batch-keyed order (tools/ab/order_interleave_ab.py --caps,
// profiles/r03/order_caps.jsonl): 8M universes 6.25 TB/s with 7 and 6.22
// with 6 against 6.09 uncapped and 5.76 with 5; 16M 6.13 with 6 or 7 against
// 5.95 uncapped and 5.71 with 5; at 4M 7 and uncapped equal (6.44 / 6.39),
// at 1M-3M uncapped best (7 is 3-4 % slower, 6 up to 7 %).  The fixed-order
// sweep agrees (tools/ab/step_occupancy_ab.py, profiles/r03/step_occupancy.jsonl:
// 16M 6.09 / 6.07 TB/s with 6 / 7 against 5.78 uncapped and 5.67 with 5).
// Round 2 shipped "6", but its LDS arithmetic rounded the share up and gave
// one block fewer whenever the cap did not divide 160 KiB (6 -> 5, 7 -> 6):
// it ran 5; occupancy_lds now checks the count on the occupancy API.
// Launch order and store policy (tools/ab/order_ab.py, profiles/r02/order_*.jsonl,
// same process, ping-pong as the bench): a launch whose input batch an
// earlier launch wrote takes the groups in the reverse of that launch's order
// (host.hpp launch_reverse, keyed on the batch), so it starts on what was
// written last; the groups that store the last min(256 MiB, half
// the batch) of a launch use plain stores, which leave that part in the 256 MB
// memory-side Infinity Cache, and the rest nontemporal ones, which do not
// evict it.  Batches of up to kCachedUniverses use every block slot, larger
// ones the cap.  Against round 2's launch (nontemporal, one order, capped at
// what turned out to be 5 blocks per CU): +12 % at 1M universes, +10 % at 2M,
// +3-5 % at 512K and 4M, equal at 8M-16M -- most of it from dropping the cap:
// against one fixed order with every store nontemporal and no cap the order
// policy gains +1-4 % at 1M (round 3's same-process A/B +4 %, round 4's
// footprint sweeps +1-2 %, profiles/r04/r04e/footprint.jsonl).
constexpr uint64_t kCachedUniverses = 1ull << 22;
constexpr int kStreamResidentBlocks = 7;
// Below this batch size the order stays fixed: at 64K universes (64 MiB per
// launch) the fixed order was 4 % faster, single batch and two interleaved,
// and at 128K the two boxes disagreed (-4 / +1 %); from 192K on the
// batch-keyed order is as fast or faster (+1-3 % at 192K-384K, +7-8 % for two
// interleaved 512K batches, +16 % for one 1M batch; tools/ab/order_interleave_ab.py,
// profiles/r03/order_interleave*.jsonl)
constexpr uint64_t kOrderMinUniverses = 3ull << 16;
constexpr uint64_t kPlainBytes = 256ull << 20;
constexpr uint64_t kFilterOrderUniverses = 1ull << 21;  // the same for the 1-2 generation search filter
constexpr const char *kStreamName =
    "k_step<dpp, 4 universes/wave, nt loads, 7-LUT network; alternating order, the last min(256 MiB, half) of "
    "each launch stored plain, the rest nt>";
// Above kCachedUniverses there is no Infinity Cache reuse to arrange: one
// order, every store nontemporal, and each XCD streams a contiguous eighth
// of the batch (kXcdChunk, device.hpp xcd_chunk_block).  Same process,
// ping-pong, 7 blocks per CU (tools/ab/step_xcd_ab.py,
// profiles/r03/step_xcd_ab.jsonl): 16M universes 2.736 ms against 2.836 for
// the order/plain-tail launch and 2.845 with the plain block mapping; 8M
// 1.396 against 1.410 / 1.427; at 4M the chunked mapping was 1 % slower, at
// 1M equal.
// Round 4: 8 universes per wave for these batches (4 KiB in flight per
// wave): same process, interleaved, 7 rounds (tools/ab/big_upw_ab.py,
// profiles/r04/r04d/big_upw_ab.jsonl): 8M 6.12 against 5.83 TB/s back to
// back (6.40 / 6.17 after a read-only scrub), 16M and 4M equal (6.38 / 6.38,
// 6.40 / 6.36).
constexpr const char *kStreamBigName =
    "k_step<dpp, 8 universes/wave, nt, 7-LUT network; each XCD a contiguous eighth, one order>";
struct StepLaunch {
  StepFn fn;
  uint64_t universes_per_wave;
  int resident_blocks;   // per CU, 0 = as many as fit
  bool alternate;        // alternate the group order between launches
  uint64_t plain_bytes;  // the last bytes of a launch stored plain
  const char *name;
  uint32_t flags;        // kXcdChunk or 0
};
StepLaunch shipped_step(uint32_t gens, uint64_t n) {
  if (gens <= 2 && n > kCachedUniverses)
    return {k_step<XDPP, 8, true, 3, true>, 8, kStreamResidentBlocks, false, 0, kStreamBigName, kXcdChunk};
  if (gens <= 2)
    return {k_step<XDPP, 4, true, 3, true>, 4, 0, true, std::min<uint64_t>(kPlainBytes, n * 512 / 2), kStreamName,
            0u};
  if (gens < 32)
    return {k_step_split<8, 1, true, 6, kAsmLoop>, 4, 0, false, 0,
            "k_step_split<8-way split, 4 universes/wave, nt, 6-LUT tail, assembly loop>", 0u};
  return {k_step_split<8, 1, false, 6, kAsmLoop>, 4, 0, false, 0,
          "k_step_split<8-way split, 4 universes/wave, 6-LUT tail, assembly loop>", 0u};
}

}  // namespace

extern "C" {

const char *lifeapi_step_kernel_name_n(uint32_t generations, size_t n) {
  return shipped_step(generations, n).name;
}
const char *lifeapi_step_kernel_name(uint32_t generations) { return shipped_step(generations, 1).name; }

int lifeapi_step_batch_dev(const uint64_t *d_in, uint64_t *d_out, size_t n, uint32_t generations,
                           void *stream) {
  int rc = check_batch(d_in, d_out, n);
  if (rc != LIFEAPI_OK || n == 0) return rc;
  int cus = 0;
  rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const StepLaunch l = shipped_step(generations, n);
  const uint64_t waves = (n + l.universes_per_wave - 1) / l.universes_per_wave;
  unsigned lds = 0;
  if (l.resident_blocks) {
    rc = occupancy_lds(reinterpret_cast<const void *>(l.fn), l.resident_blocks, lds);
    if (rc != LIFEAPI_OK) return rc;
  }
  const uint64_t plain = (l.plain_bytes + l.universes_per_wave * 512 - 1) / (l.universes_per_wave * 512);
  uint32_t order = 0;
  if (l.alternate && n >= kOrderMinUniverses) order = launch_reverse(d_in, d_out, (uint64_t)n * 512) ? kReverse : 0u;
  else note_forward_write(d_out, (uint64_t)n * 512);
  hipLaunchKernelGGL(l.fn, dim3(grid_for(waves, cus, 0)), dim3(kBlock), lds, (hipStream_t)stream, d_in,
                     d_out, (uint64_t)n, generations | order | l.flags, plain < waves ? waves - plain : (uint64_t)0);
  return launched("k_step launch");
}

int lifeapi_step_contains_batch_dev(const uint64_t *d_in, uint64_t *d_final,
                                    const uint64_t *d_wanted, const uint64_t *d_unwanted,
                                    uint32_t *d_first_gen, size_t n, uint32_t generations,
                                    void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_in || !d_wanted || !d_unwanted || !d_first_gen || !aligned8(d_in) ||
      !aligned8(d_wanted) || !aligned8(d_unwanted) || ((uintptr_t)d_first_gen & 3u))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_step_contains_batch_dev%s");
  if (d_final) {
    int rc = check_batch(d_in, d_final, n);
    if (rc != LIFEAPI_OK) return rc;
  }
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  if (!d_final && generations <= 2) {
    // the search filter proper (first hits only) at 1-2 generations: the
    // target's light cone, or the whole board, in the natural layout
    // (cone_kernels.hpp k_cone_adapt, DMA form): a whole-board target takes
    // the universes through LDS (cone_wave_full_dma / cone_wave_rows_dma, 8
    // per pass by global_load_lds, the next pass fetched while this one
    // steps), every other window its cone (cone_wave); every wave decides,
    // on a grid of at most kConeAdaptBlocksPerCU blocks per CU looping over
    // the batch.  Round 6: no launch report -- round 5 chose the grid per
    // target pointers from the last call's report, which a loop that rewrites
    // its target buffers read stale (+13 % per call, tools/report_loop_probe.py,
    // profiles/r06/).  1M universes, median of 5 x 10 back to back
    // (tools/filter_iter_probe.py, profiles/r06/): the one-row whole board
    // 0.083 / 0.086 ms at 1 / 2 generations against 0.082 / 0.081 on the
    // reported uncapped grid, the full-height and random whole boards 5-9 %
    // faster, the block + ring unchanged (0.023 / 0.026).
    return launch_cone_adapt<kConeSets, true, uint32_t, true>(d_in, d_wanted, d_unwanted, d_first_gen, n,
                                                              generations, cus, (hipStream_t)stream,
                                                              kConeAdaptBlocksPerCU, kWave, kConeAdaptBlocksPerCU);
  }
  if (!d_final) {
    // 3+ generations, first hits only (round 6): one launch of the merged
    // split kernel (step_kernels.hpp k_step_contains_split, kContainsAll),
    // whose waves take the pass their target calls for -- no report, so a
    // loop that rewrites its target buffers loses nothing:
    // * care rows that fit 32 with the light cone (cone_rows): on a whole
    //   board below kConeWholeWinGens generations the packed LDS-DMA pass
    //   (cone_wave_rows_dma), else the window split layout (cone_split.hpp)
    //   on the column window, on half the lanes once the cone's columns fit
    //   (a whole board's chunks fetched by LDS-DMA);
    // * else a cone of <= 32 columns: the natural layout on the cone
    //   (cone_wave);
    // * else the 8-way row split with the test fused (the loop its row
    //   window picks), the next group of universes fetched into LDS while
    //   this one steps.
    // 1M universes, median of 5 x 10 back to back (tools/filter_iter_probe.py,
    // profiles/r06/): block + ring at 3 / 5 / 8 / 13 generations 0.042 / 0.058
    // / 0.096 / 0.137 ms (round 5: 0.047 / 0.057 / 0.154 / 0.222;
    // profiles/r06/shrink_ab/), a full-height target 0.179 / 0.235 / 0.309 /
    // 0.435 (0.18 / 0.24 / 0.32 / 0.47 on the split pair).
    using Fn = void (*)(const uint64_t *, uint64_t *, const uint64_t *, const uint64_t *, uint32_t *, uint64_t,
                        uint32_t, uint32_t);
    const Fn fn = aligned16(d_in) ? k_step_contains_split<8, kContainsNet, kContainsAll, true, true>
                                  : k_step_contains_split<8, kContainsNet, kContainsAll, false, true>;
    hipLaunchKernelGGL(fn, dim3(grid_for((n + 3) / 4, cus, kFilterIterBlocksPerCU)), dim3(kBlock), 0,
                       (hipStream_t)stream, d_in, (uint64_t *)nullptr, d_wanted, d_unwanted, d_first_gen, (uint64_t)n,
                       generations, kConeIterColumns);
    return launched("k_step_contains_split launch");
  }
  if (generations > 2) {  // the layout of the shipped step for gens > 2
    // Without final states, a target whose light cone over `generations`
    // spans at most kConeIterColumns columns is answered on that cone:
    // kContainsLo's waves step only those columns in the natural layout
    // (cone_wave) and kContainsHi's return.  Both grids are capped (blocks
    // per CU, looping over the batch), so that the idle kernel's waves cost a
    // few microseconds instead of a wave launch per 4 universes
    // (tools/ab/search_iter_caps_ab.py).  With final states
    // the capped grids help too: 1M universes x 8 / 64
    // generations 0.467 -> 0.394-0.398 / 1.78-1.80 -> 1.70 ms, 256K 0.112 ->
    // 0.101 ms; at config 3's 64K the cap does not bind (tools/ab/final_caps_ab.py,
    // profiles/r04/r04ar).
    const int split_cap = kSplitIterBlocksPerCU;
    const uint32_t cone_max = 0;  // (final states: every universe steps the whole board)
    // two kernels, one per register layout (a target window of <= 4 rows in
    // 62 VGPRs, 8 waves per SIMD; the rest in 70, 7 waves): each wave finds
    // the window and only the matching kernel works (step_kernels.hpp
    // kContainsLo / kContainsHi)
    using Fn = void (*)(const uint64_t *, uint64_t *, const uint64_t *, const uint64_t *, uint32_t *, uint64_t,
                        uint32_t, uint32_t);
    const Fn fns[2] = {k_step_contains_split<8, kContainsNet, kContainsLo>,
                       k_step_contains_split<8, kContainsNet, kContainsHi>};
    const dim3 grid(grid_for((n + 3) / 4, cus, split_cap));
    if (d_final) note_forward_write(d_final, (uint64_t)n * 512);
    for (const Fn fn : fns) {
      hipLaunchKernelGGL(fn, grid, dim3(kBlock), 0, (hipStream_t)stream, d_in, d_final, d_wanted, d_unwanted,
                         d_first_gen, (uint64_t)n, generations, cone_max);
      rc = launched("k_step_contains_split launch");
      if (rc != LIFEAPI_OK) return rc;
    }
    return LIFEAPI_OK;
  } else {
    // 8 universes per wave, every block slot (tools/ab/filter_ab.py,
    // profiles/r02/filter_ab.jsonl, 1M universes x 1 generation, same
    // process): 0.087 ms = 6.25 TB/s on the 516 B per universe of the bare
    // filter, 0.181 ms with final states (5.96 TB/s on 1028 B); 4 per wave
    // 0.107 / 0.179, with fewer blocks resident slower; one per wave 0.229.
    // With final states, the launch order and plain-stored tail of the step
    // (above): a loop that filters the states the last call left gets them
    // partly from the Infinity Cache (tools/ab/filter_order_ab.py).
    const uint64_t groups = (n + 7) / 8;
    // Up to 2M universes: +3.4 % at 512K and 1M, +2 % at 2M, none at 4M
    // (profiles/r02/filter_order_ab.jsonl).
    const bool order = d_final && n <= kFilterOrderUniverses && n >= kOrderMinUniverses;
    const uint64_t plain = order ? (std::min<uint64_t>(kPlainBytes, n * 512 / 2) + 8 * 512 - 1) / (8 * 512) : 0;
    uint32_t rev = 0;
    if (order) rev = launch_reverse(d_in, d_final, (uint64_t)n * 512) ? kReverse : 0u;
    else if (d_final) note_forward_write(d_final, (uint64_t)n * 512);
    hipLaunchKernelGGL(k_step_contains<8>, dim3(grid_for(groups, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream,
                       d_in, d_final, d_wanted, d_unwanted, d_first_gen, (uint64_t)n, generations | rev,
                       plain < groups ? groups - plain : (uint64_t)0);
  }
  return launched("k_step_contains launch");
}

}  // extern "C"
