// stencils.hip -- the other per-generation stencils of SURVEY 8(f):
// NeighbourCount / InteractionCounts (LifeAPI.hpp:909-1040), LifeWeld::Step
// (LifeWeld.hpp:169-186), the LifeStable propagation passes
// (LifeStable.hpp:526-729) and the config-5 unknown_step_refined step.
#include "device.hpp"
#include "host.hpp"
#include "split_layout.hpp"
#include "stable_kernels.hpp"
#include "stencil_kernels.hpp"

using namespace lifeapi_impl;

extern "C" {

// LifeStable kernels: one wave per LifeStable, at most this many blocks (of
// kWavesPerBlock waves) resident per CU (see lifeapi_stable_pass_batch_dev)
constexpr int kStableResidentBlocks = 4;
constexpr int kWeldResidentBlocks = 7;  // k_weld (below 12 generations)
// per pass (sync, options, signal, step, propagate, stabilise): 0 = every
// slot.  Round 3, exact caps, 1M LifeStables of three families, same process
// (tools/ab/stable_grid_ab.py, profiles/r03/stable_caps_1m.jsonl): the single
// passes 2-5 % faster with 3 resident blocks than with 4 (sync 1.79-1.81
// against 1.86 ms, signal 1.80-1.82 against 1.83-1.87); Propagate keeps
// every slot (3 blocks: +25 % on still lifes; 4-6 within 3 % of it) and
// StabiliseOptions 4 (3 and 4 within 1 %).  Round 2's "3" had been 2 (its
// LDS share was rounded up).
constexpr int kStablePassResident[6] = {3, 3, 3, 3, 0, kStableResidentBlocks};
// the LDS-DMA passes (below): at most 5 blocks resident per CU
constexpr int kStableDmaResident = 5;

static int counts_launch(const uint64_t *d_in, uint64_t *d_out, size_t n, int mode, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_in || !d_out || !aligned8(d_in) || !aligned8(d_out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to a neighbourhood-count entry point%s");
  const size_t planes = mode == 1 ? 3 : 4;
  const uintptr_t a = (uintptr_t)d_in, b = (uintptr_t)d_out;
  if (a < b + n * planes * 512 && b < a + n * 512)
    return fail(LIFEAPI_E_INVALID, "count input and output overlap%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  using Fn = void (*)(const uint64_t *, uint64_t *, uint64_t);
  Fn fn = mode == 0 ? (Fn)k_counts<0> : mode == 1 ? (Fn)k_counts<1> : (Fn)k_counts<2>;
  note_forward_write(d_out, (uint64_t)n * planes * 512);
  hipLaunchKernelGGL(fn, dim3(grid_for(n, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream, d_in,
                     d_out, (uint64_t)n);
  return launched("k_counts launch");
}

int lifeapi_stable_pass_batch_dev(uint64_t *d_planes, uint8_t *d_flags, size_t n, int pass,
                                  uint32_t max_iters, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_planes || !d_flags || !aligned8(d_planes) || pass < 0 || pass > 5)
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_stable_pass_batch_dev%s");
  const uintptr_t a = (uintptr_t)d_planes, b = (uintptr_t)d_flags;
  if (b < a + n * 10 * 512 && a < b + n) return fail(LIFEAPI_E_INVALID, "flags overlap planes%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  using Fn = void (*)(uint64_t *, uint8_t *, uint64_t, uint32_t, uint32_t);
  const Fn fns[6] = {k_stable<0>, k_stable<1>, k_stable<2>, k_stable<3>, k_stable<4>, k_stable<5>};
  // Launch shape (same-process A/Bs, tools/ab/stable_grid_ab.py, on still lifes
  // around an unknown window with fresh options -- the state a search
  // propagates from --, sparse soups and random planes, 64K and 1M
  // LifeStables; profiles/r02/stable_occupancy_*.jsonl): one wave per
  // LifeStable with at most kStablePassResident[pass] blocks resident per
  // CU (round 3's exact caps, above), set by unused dynamic LDS; round 2's
  // measurements below were of 4 (and its "3" of 2).  Every pass reads and writes its 5 KiB in place; fewer concurrent
  // streams per CU serve that better (the in-place copy of the same shape,
  // build/membw inplace: 5.73 TB/s uncapped, 5.87 at 2 blocks per CU).  At
  // 1M: 5-10 % faster than one wave per LifeStable unlimited or a
  // 32-blocks-per-CU grid that loops over the batch on soups and random
  // planes, within 1-4 % of the looping grid on still lifes, where that one
  // had been best; at 64K the best or within 2 % everywhere.
  // Propagate (pass 4) loops PropagateStep to its fixpoint, a data-dependent
  // amount of VALU work per LifeStable: it keeps every wave slot (4 blocks
  // resident: +1.4 % on still lifes at 1M, and 8 % slower on tools/rows_bench.py's
  // random planes, whose fixpoints take more steps).
  unsigned lds = 0;
  if (kStablePassResident[pass]) {
    rc = occupancy_lds(reinterpret_cast<const void *>(fns[pass]), kStablePassResident[pass], lds);
    if (rc != LIFEAPI_OK) return rc;
  }
  // One order: alternating it, as k_weld does, was 1-2 % slower on repeated
  // passes in place (tools/ab/stable_order_ab.py, profiles/r02/stable_order_ab.jsonl).
  // Each XCD takes a contiguous eighth of the batch (the last argument's bit
  // 1, device.hpp xcd_chunk_block): on 1M LifeStables, same process, fresh
  // copies (tools/ab/stable_xcd_ab.py, profiles/r03/stable_xcd_ab.jsonl)
  // Propagate 1.96 -> 1.77 ms, sync 1.77 -> 1.63, options 1.62 -> 1.54,
  // signal 1.83 -> 1.72, PropagateStep 1.95 -> 1.86, StabiliseOptions
  // 1.79 -> 1.66.
  note_forward_write(d_planes, (uint64_t)n * 10 * 512);
  if ((pass == 0 || pass == 1 || pass == 2 || pass == 3 || pass == 5) && aligned16(d_planes)) {
    // Round 5: SynchroniseStateKnown, UpdateOptions, SignalNeighbours and
    // PropagateStep move their LifeStable through LDS (k_stable_dma, U = 1, WIDE): five
    // 16-byte-per-lane global_load_lds in, ds_read_b64 out to lane =
    // column; the changed lines back through the image, 16 bytes per lane;
    // at most 5 blocks resident per CU.  Same process, 1M LifeStables of
    // three families, ms (tools/stable_dma_ab.py, profiles/r05/
    // stable_dma_ab_r05m.jsonl; fresh options / a search's next node /
    // random planes): signal 0.791 / 0.786 / 0.790 against 0.802 / 0.798 /
    // 0.802 for k_stable (round 4: 1.10-1.15); PropagateStep 1.654 / 1.074
    // / 1.645 against 1.697 / 1.368 / 1.631; sync 1.649 / 1.058 / 1.649
    // against 1.625 / 1.142 / 1.632; UpdateOptions, which stores only the
    // option planes, 1.491 / 1.042 / 1.491 against 1.551 / 1.210 / 1.560
    // (profiles/r05/stall/options_dma_ab.jsonl; storing state and unknown
    // too, as the image holds them, it lost 6 % where every column
    // changes).  SynchroniseStateKnown, UpdateOptions and StabiliseOptions
    // store only the planes that changed: sync 1.499 / 0.929 / 1.494,
    // UpdateOptions 1.496 / 0.940 / 1.495, StabiliseOptions (uncapped grid:
    // at most 5 blocks per CU it loses on the next node, 1.22) 1.553 /
    // 1.068 / 1.555 against 1.711 / 1.103 / 1.708 (profiles/r05/stall/
    // skip_planes_ab*.jsonl).  Propagate gains nothing: it keeps k_stable
    // (DESIGN.md 3.5).  The loads and stores are 16 bytes wide: an 8-byte
    // aligned batch keeps k_stable.
    using DFn = void (*)(uint64_t *, uint8_t *, uint64_t, uint32_t, uint32_t);
    const DFn dma = pass == 0   ? (DFn)k_stable_dma<0, 2, true, true>
                    : pass == 1 ? (DFn)k_stable_dma<1, 2, true, true>
                    : pass == 2 ? (DFn)k_stable_dma<2, 2, true, true>
                    : pass == 3 ? (DFn)k_stable_dma<3, 2, true, true>
                                : (DFn)k_stable_dma<5, 2, true, true>;
    unsigned dlds = 0;
    if (pass != 5) {  // (StabiliseOptions: every block the LDS holds)
      rc = occupancy_lds(reinterpret_cast<const void *>(dma), kStableDmaResident, dlds);
      if (rc != LIFEAPI_OK) return rc;
    }
    hipLaunchKernelGGL(dma, dim3(grid_for(n, cus, 0)), dim3(kBlock), dlds, (hipStream_t)stream, d_planes, d_flags,
                       (uint64_t)n, max_iters ? max_iters : 1u << 20, 1u << 8);
    return launched("k_stable_dma launch");
  }
  hipLaunchKernelGGL(fns[pass], dim3(grid_for(n, cus, 0)), dim3(kBlock), lds, (hipStream_t)stream,
                     d_planes, d_flags, (uint64_t)n, max_iters ? max_iters : 1u << 20, 2u);
  return launched("k_stable launch");
}

int lifeapi_stable_vulnerable_batch_dev(const uint64_t *d_planes, uint64_t *d_out, size_t n, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_planes || !d_out || !aligned8(d_planes) || !aligned8(d_out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_stable_vulnerable_batch_dev%s");
  const uintptr_t a = (uintptr_t)d_planes, b = (uintptr_t)d_out;
  if (b < a + n * 10 * 512 && a < b + n * 512) return fail(LIFEAPI_E_INVALID, "out overlaps planes%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  // as the passes: one wave per LifeStable, at most 4 blocks resident per
  // CU (0.96-0.97 ms at 1M against 0.97-1.00 unlimited and 1.02-1.04 on a
  // looping grid; profiles/r02/stable_occupancy_*.jsonl), each XCD a
  // contiguous eighth of the batch (0.998 -> 0.905 ms at 1M, same process;
  // tools/ab/stencil_xcd_ab.py, profiles/r03/stencil_xcd_ab.jsonl; the counts,
  // k_weld and k_refined at config 5's 256K measured within noise or slower
  // with it and keep the plain mapping)
  unsigned lds = 0;
  rc = occupancy_lds(reinterpret_cast<const void *>(k_stable_vulnerable<true>), kStableResidentBlocks, lds);
  if (rc != LIFEAPI_OK) return rc;
  note_forward_write(d_out, (uint64_t)n * 512);
  hipLaunchKernelGGL(k_stable_vulnerable<true>, dim3(grid_for(n, cus, 0)), dim3(kBlock), lds, (hipStream_t)stream,
                     d_planes, d_out, (uint64_t)n);
  return launched("k_stable_vulnerable launch");
}

int lifeapi_weld_step_batch_dev(uint64_t *d_welds, size_t n, uint32_t generations, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_welds || !aligned8(d_welds))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_weld_step_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  if (generations >= 12) {  // state resident in VGPRs on the split layout (k_weld_split)
    note_forward_write(d_welds, (uint64_t)n * 2048);
    hipLaunchKernelGGL(generations < 32 ? k_weld_split<true> : k_weld_split<false>,
                       dim3(grid_for((n + 3) / 4, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream,
                       d_welds, (uint64_t)n, generations);
  } else {
    // the order keyed on the batch (host.hpp launch_reverse: in place, so
    // it alternates between calls on the same welds), nontemporal
    // throughout: in a loop stepping the batch in place, +15 % at 256K
    // welds, +7 % at 512K, +3.5 % at 1M, +1.5 % at 2M; a plain-stored tail
    // adds nothing here (tools/ab/weld_order_ab.py, profiles/r02/weld_order_ab.jsonl)
    // At most 7 blocks resident per CU: 0.459 against 0.484 ms for 1M welds
    // with every slot (6: 0.458; 5: 0.472), same process, exact caps
    // (tools/ab/stencil_occupancy_ab.py, profiles/r03/stencil_caps.jsonl).
    // Round 4: two welds per wave (their 8 loads issued together) and each XCD
    // a contiguous eighth of the batch.  The A/B (profiles/r04/r04b/
    // weld_u_ab.jsonl) ran the new shape in one fixed order: 0.4218 ms for 1M
    // welds against 0.4680 with one weld per wave and 0.4505 for round 3's
    // launch (0.796 / 0.717 / 0.745 of 8 TB/s).  What ships keeps the
    // batch-keyed alternating order above; that exact launch, in place, back
    // to back, measured 0.799-0.801 of 8 TB/s (0.791-0.795 after a read-only
    // scrub) in tools/rows_bench.py (profiles/r04/r04u, r04e).
    constexpr int kWeldU = 2;
    unsigned lds = 0;
    rc = occupancy_lds(reinterpret_cast<const void *>(k_weld<true, kWeldU>), kWeldResidentBlocks, lds);
    if (rc != LIFEAPI_OK) return rc;
    const uint32_t rev = launch_reverse(d_welds, d_welds, (uint64_t)n * 2048) ? kWeldReverse : 0u;
    const uint64_t groups = (n + kWeldU - 1) / kWeldU;
    hipLaunchKernelGGL((k_weld<true, kWeldU>), dim3(grid_for(groups, cus, 0)), dim3(kBlock), lds,
                       (hipStream_t)stream, d_welds, (uint64_t)n, generations | rev, groups);
  }
  return launched("k_weld launch");
}

int lifeapi_neighbour_count_batch_dev(const uint64_t *d_in, uint64_t *d_out, size_t n, void *stream) {
  return counts_launch(d_in, d_out, n, 0, stream);
}

int lifeapi_interaction_counts_batch_dev(const uint64_t *d_in, uint64_t *d_out, size_t n,
                                         int with_next, void *stream) {
  return counts_launch(d_in, d_out, n, with_next ? 2 : 1, stream);
}

int lifeapi_refined_step_batch_dev(const uint64_t *d_in, uint64_t *d_out, size_t n, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_in || !d_out || !aligned8(d_in) || !aligned8(d_out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_refined_step_batch_dev%s");
  const uintptr_t a = (uintptr_t)d_in, b = (uintptr_t)d_out;
  if (a < b + n * 3 * 512 && b < a + n * 11 * 512)
    return fail(LIFEAPI_E_INVALID, "refined step input and output overlap%s");
  // the measured best with the 192-op SOP network (profiles/r01/tune_c5.jsonl):
  // prefetch the next universe, one-shot grid, no occupancy bound -> 6.3 TB/s
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  note_forward_write(d_out, (uint64_t)n * 3 * 512);
  hipLaunchKernelGGL((k_refined<1, 0>), dim3(grid_for(n, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream, d_in,
                     d_out, (uint64_t)n);
  return launched("k_refined launch");
}

}  // extern "C"
