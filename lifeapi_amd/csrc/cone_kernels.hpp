// cone_kernels.hpp -- Contains(LifeTarget) (LifeTarget.hpp:44-51) and the
// 1-2 generation search filter (Step(), LifeAPI.hpp:1196-1216, then
// Contains) reading only the target's light cone.
//
// Whether generation g of a universe contains a target depends only on the
// input columns within distance g of the target's care columns (wanted |
// unwanted): a cell's next state reads its 3x3 neighbourhood.  Every wave
// finds the smallest cyclic window [x0, x0 + w) of columns holding the care
// cells (care_window, the same search as the row window of the iterated
// kernel) and loads only columns [x0 - g, x0 + w + g) mod 64 -- K = w + 2g
// columns, K * 8 bytes of each 512-byte universe, so that the 128-byte lines
// outside never leave HBM.
//
// Lane layout: P = the next power of two >= K lanes per universe, 64 / P
// universes per wave register ("set"); lane j of group q holds column
// (x0 - g + j) mod 64 of its universe.  The generation is the streaming
// step's network (life_gen<XDPP, 3>) unchanged: its 64-lane DPP rotate hands
// a group's edge lanes their neighbour group's columns, which is wrong data
// -- but only for the g margin columns on either side, which the test never
// reads (after g generations the error has moved g columns in).  The care
// columns are exact.  A window with K >= 64 loads the whole board from
// column 0, where the rotate is the true torus.
//
// The pass over a wave's universes (cone_wave) and the window tests
// (cone_window, cone_whole, cone_fits) live in step_kernels.hpp, shared with
// the iterated search loop's kContainsLo.  This file holds the kernels that
// launch them: k_cone_adapt (shipped: the chunk of universes per wave chosen
// from the window), k_cone (fixed shapes, the tuning build's A/Bs) and the
// whole-board Contains pass with 16-byte loads.
#pragma once

#include <type_traits>

#include "step_kernels.hpp"

namespace lifeapi_impl {
namespace {

// Contains over the whole board (K = 64) on a 16-byte aligned batch: lane l
// reads words 2(l mod 32), 2(l mod 32) + 1 of universe 2k + l / 32 (one
// dwordx4 moves two universes per wave-instruction, as k_contains16), RMAX
// loads in flight per pass.
template <int UPW, int RMAX>
__device__ __forceinline__ void cone_wave_full16(const uint64_t *in, const uint64_t *__restrict__ wanted,
                                                 const uint64_t *__restrict__ unwanted, uint8_t *__restrict__ out,
                                                 uint64_t n, uint64_t u_first, uint64_t u_step, int lane) {
  constexpr int RB = UPW / 2 < RMAX ? UPW / 2 : RMAX;
  static_assert(UPW % (2 * RB) == 0, "passes of 2 RB universes");
  const int half = lane >> 5, col = (lane & 31) * 2;
  const uint64_t w0 = wanted[col], w1 = wanted[col + 1];
  const uint64_t m0 = w0 | unwanted[col], m1 = w1 | unwanted[col + 1];
  for (uint64_t u0 = u_first; u0 < n; u0 += u_step) {
    uint32_t mine = 0;  // lane L: the answer for universe u0 + L
#pragma unroll 1
    for (int pass = 0; pass < UPW / (2 * RB); ++pass) {
      const uint64_t ub = u0 + (uint64_t)pass * 2 * RB;
      u64x2 v[RB];
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const uint64_t u = ub + 2 * k + half;
        v[k] = u < n ? __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(in + u * kWave + col))
                     : u64x2{w0, w1};
      }
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const uint64_t d = ((v[k][0] ^ w0) & m0) | ((v[k][1] ^ w1) & m1);
        const uint64_t bad = __ballot(d != 0ull);  // lanes 0-31: universe 2k, 32-63: 2k+1
        const uint32_t rel = (uint32_t)lane - (uint32_t)(pass * 2 * RB + 2 * k);
        if (rel < 2u) mine = (uint32_t)(bad >> (32 * rel)) == 0u ? 1u : 0u;
      }
    }
    if (lane < UPW && u0 + lane < n) out[u0 + lane] = (uint8_t)mine;
  }
}

// (dma_fetch_pass: cone_split.hpp)

// The whole-board pass (K = 64) through LDS: each register set is one
// universe, RB sets per pass; the RB universes of a pass (RB * 512
// contiguous bytes) arrive by RB / 2 sixteen-byte-per-lane global_load_lds
// (LDS-DMA, no VGPR destination: lanes 0-31 fill one universe, 32-63 the
// next) and leave by ds_read_b64 with lane = column, and the next pass's are
// fetched as soon as this pass has been read out, so that they stream in
// while this pass steps.  Chunks of 2 RB universes per wave, u_step apart;
// one coalesced store of answers per chunk.  `img`: this wave's RB * 512
// bytes of LDS.  The batch must be 16-byte aligned.
template <int RB, bool FIRST, typename OutT>
__device__ __forceinline__ void cone_wave_full_dma(const uint64_t *in, uint64_t w64, uint64_t m64,
                                                   OutT *__restrict__ out, uint64_t n, uint64_t u_first,
                                                   uint64_t u_step, uint32_t gens, int lane, uint64_t *img,
                                                   bool prefetched) {
  static_assert(RB % 2 == 0 && 2 * RB <= kWave, "passes of pairs of universes, one answer per lane");
  const W tw = split(w64), tm = split(m64);
  auto clean = [&](W s) __attribute__((always_inline)) {
    const uint32_t d = ((s.lo ^ tw.lo) & tm.lo) | ((s.hi ^ tw.hi) & tm.hi);
    return __ballot(d != 0u) == 0ull;
  };
  // pass t: universes [base(t), base(t) + RB); chunk t / 2
  auto base = [&](uint64_t t) { return u_first + (t >> 1) * u_step + (t & 1) * RB; };
  auto fetch = [&](uint64_t ub) __attribute__((always_inline)) { dma_fetch_pass<RB>(in, n, ub, lane, img); };
  if (u_first >= n) return;
  if (!prefetched) fetch(u_first);  // (else the caller issued it)
  uint32_t mine = 0;  // lane L: the answer for universe (chunk start) + L
  int after = 0;      // vector-memory ops issued after the pending fetch (the chunk's answer store)
  for (uint64_t t = 0;; ++t) {
    const uint64_t ub = base(t);
    if (ub >= n) break;
    if (after) __builtin_amdgcn_s_waitcnt(kWaitVm1);
    else __builtin_amdgcn_s_waitcnt(kWaitVm0);
    W a[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) a[k] = split(img[k * kWave + lane]);
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);  // read out before the next fetch lands
    const uint64_t nb = base(t + 1);
    if (nb < n) fetch(nb);
    uint32_t res[RB];
    if constexpr (FIRST) {
#pragma unroll
      for (int k = 0; k < RB; ++k) res[k] = 0;
      for (uint32_t g = 1; g <= gens; ++g) {
#pragma unroll
        for (int k = 0; k < RB; ++k) {
          a[k] = life_gen<XDPP, 3>(a[k], nullptr, lane);
          if (res[k] == 0 && clean(a[k])) res[k] = g;
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < RB; ++k) res[k] = clean(a[k]) ? 1u : 0u;
    }
#pragma unroll
    for (int k = 0; k < RB; ++k)
      if ((uint32_t)lane == (uint32_t)((t & 1) * RB + k)) mine = res[k];
    after = 0;
    if ((t & 1) || ub + RB >= n) {  // the chunk's last pass: store its answers
      const uint64_t u0 = base(t & ~1ull);
      if (lane < 2 * RB && u0 + lane < n) out[u0 + lane] = (OutT)mine;
      mine = 0;
      after = 1;
    }
  }
}

// (cone_wave_rows_dma: cone_split.hpp)

// (cone_rows and kConeRowsWindowGens: step_kernels.hpp)

// UPW universes per wave (one-shot grid of ceil(n / UPW) waves), every wave
// choosing its lane layout from the window (wave-uniform: the target is the
// same for all).  Each choice runs its own copy of the pass.  A16: the batch
// is 16-byte aligned (Contains over the whole board then takes 16-byte loads).
// kmax: a wave whose window K exceeds it returns at once (the iterated
// search loop's split-layout kernels answer those, step.hip).
template <int UPW, int RMAX, bool FIRST, typename OutT, bool A16 = false, bool PIPE = false>
__global__ __launch_bounds__(kBlock) void k_cone(const uint64_t *in, const uint64_t *__restrict__ wanted,
                                                 const uint64_t *__restrict__ unwanted, OutT *__restrict__ out,
                                                 uint64_t n, uint32_t gens, uint32_t kmax) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t u0 = wave * UPW, step = (uint64_t)gridDim.x * kWavesPerBlock * UPW;  // grid-stride (capped grids)
  if (u0 >= n) return;
  const uint32_t g = FIRST ? gens : 0u;
  const uint64_t care_col = wanted[lane] | unwanted[lane];
  uint32_t xs = 0, K = kWave;
  if (!cone_whole(care_col, g)) cone_window(care_col, g, xs, K);  // (a whole-board target skips the search)
  if (K > kmax) return;
  if constexpr (!FIRST && A16) {
    if (K == (uint32_t)kWave) return cone_wave_full16<UPW, RMAX>(in, wanted, unwanted, out, n, u0, step, lane);
  }
  // (a wave of UPW universes takes whole register sets: P >= 64 / UPW)
  auto pass = [&](auto p) __attribute__((always_inline)) {
    cone_wave<decltype(p)::value, UPW, RMAX, FIRST, OutT, PIPE>(in, wanted, unwanted, out, n, u0, step, gens, xs, K,
                                                                lane);
  };
  if (K <= 4 && UPW >= 16) pass(std::integral_constant<int, (UPW >= 16 ? 4 : 8)>{});
  else if (K <= 8) pass(std::integral_constant<int, 8>{});
  else if (K <= 16) pass(std::integral_constant<int, 16>{});
  else if (K <= 32) pass(std::integral_constant<int, 32>{});
  else pass(std::integral_constant<int, 64>{});
}

// k_cone with the chunk size chosen by the window: 64 universes per wave
// chunk while P <= 8 lanes per universe (one pass), 16 for wider cones (one
// pass of 16 / 4 / 1 universes per register set), on a grid of ceil(n / 16)
// waves capped at the caller's blocks per CU, every wave looping over the
// batch with its own chunk size.
// DMA (a 16-byte aligned batch): the whole board (K = 64) through LDS
// (cone_wave_full_dma, RMAX sets per pass, chunks of 2 RMAX universes), on
// the uncapped grid; every other window keeps the capped shape, the first
// cap_waves waves looping over the batch and the rest returning after the
// whole-board test (0: no cap).
// WIN: from kConeRowsWindowGens generations on, a target whose rows fit
// 32 (16) takes the window split layout (cone_split.hpp cone_wave_split) on
// the capped grid instead of the packed row-window passes.
// EARLY (DMA): a whole board's first pass is fetched as soon as the
// whole-board test passes, so the row-window search runs under it.  1M
// universes, back to back, against the tuning build's EARLY = false
// (profiles/r06/ab/early_fetch.jsonl): full-height and random whole boards at
// 2 generations 0.133 / 0.132 ms against 0.138 / 0.139, the one-row target
// and 1 generation within +-3 %, small targets unchanged.
template <int RMAX, bool FIRST, typename OutT, bool A16 = false, bool DMA = false, bool ROWS = true, bool WIN = false,
          bool EARLY = true>
__global__ __launch_bounds__(kBlock) void k_cone_adapt(const uint64_t *in, const uint64_t *__restrict__ wanted,
                                                       const uint64_t *__restrict__ unwanted, OutT *__restrict__ out,
                                                       uint64_t n, uint32_t gens, uint32_t kmax, uint32_t cap_waves) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  uint64_t nw = (uint64_t)gridDim.x * kWavesPerBlock;
  // (the smallest chunk any path takes: a wave starting past n has no work)
  // (WIN: the window split layout's sets are as small as 8 universes, 64
  // lanes x 32 rows)
  constexpr uint64_t kMinChunk = WIN ? 8 : DMA && 2 * RMAX < 16 ? 2 * RMAX : 16;
  if (wave * kMinChunk >= n) return;
  const uint32_t g = FIRST ? gens : 0u;
  const uint64_t w64 = wanted[lane], m64 = w64 | unwanted[lane], care_col = m64;
  uint32_t xs = 0, K = kWave;
  // the window split layout (WIN, cone_split.hpp)
  auto split_pass = [&](int pk_, uint32_t y0_, uint64_t nw_) __attribute__((always_inline)) {
    cone_split_pass(in, wanted, unwanted, out, n, wave, nw_, gens, xs, K, pk_, y0_, lane);
  };
  if constexpr (DMA) {
    __shared__ uint64_t img_all[kWavesPerBlock][RMAX * kWave];
    uint64_t *img = img_all[__builtin_amdgcn_readfirstlane(threadIdx.x / kWave)];
    const uint64_t c = 2 * RMAX;
    // (round 5 fetched a whole board's first pass before the whole-board test
    // when the last launch on the same target pointers had reported one;
    // round 6 reads no report and fetches it right after that test, DESIGN.md
    // 3.2)
    int pk = 0;
    uint32_t y0 = 0;
    if (cone_whole(care_col, g)) {
      // (not before a pass that loads by itself: the window split layout)
      const bool early = EARLY && kmax >= (uint32_t)kWave && wave * c < n &&
                         !(WIN && FIRST && gens >= kConeWholeWinGens);
      if (early) dma_fetch_pass<RMAX>(in, n, wave * c, lane, img);
      if constexpr (FIRST) pk = cone_rows(care_col, gens, y0);
      if (kmax < (uint32_t)kWave) return;
      if constexpr (FIRST && WIN) {
        if (pk > 0 && gens >= kConeWholeWinGens) {  // (its sets may be 8 universes: before the chunk test)
          if (cap_waves) {
            if (wave >= cap_waves) return;
            nw = nw < cap_waves ? nw : cap_waves;
          }
          return split_pass(pk, y0, nw);
        }
      }
      if (wave * c >= n) return;
      if constexpr (FIRST && ROWS) {
        auto rows = [&](auto pk_c, auto wrap_c) __attribute__((always_inline)) {
          cone_wave_rows_dma<RMAX, decltype(pk_c)::value, decltype(wrap_c)::value>(
              in, w64, m64, out, n, wave * c, nw * c, gens, y0, lane, img, early);
        };
        using T = std::true_type;
        using F = std::false_type;
        using P1 = std::integral_constant<int, 1>;
        using P2 = std::integral_constant<int, 2>;
        using P4 = std::integral_constant<int, 4>;
        if (pk == 4) return y0 >= 32u ? rows(P4{}, T{}) : rows(P4{}, F{});
        if (pk == 2) return y0 >= 32u ? rows(P2{}, T{}) : rows(P2{}, F{});
        if (pk == 1) return y0 >= 32u ? rows(P1{}, T{}) : rows(P1{}, F{});
      }
      return cone_wave_full_dma<RMAX, FIRST>(in, w64, m64, out, n, wave * c, nw * c, gens, lane, img, early);
    }
    if (cap_waves) {
      if (wave >= cap_waves) return;
      nw = nw < cap_waves ? nw : cap_waves;
    }
    cone_window(care_col, g, xs, K);
    if (K > kmax) return;
    if (K == (uint32_t)kWave) {
      if (wave * c >= n) return;
      return cone_wave_full_dma<RMAX, FIRST>(in, w64, m64, out, n, wave * c, nw * c, gens, lane, img, false);
    }
  } else {
    int pk = 0;
    uint32_t y0 = 0;
    if (!cone_whole(care_col, g)) {
      cone_window(care_col, g, xs, K);
      // (the row window of a column window: cone_wave_rows, below)
      if constexpr (FIRST && ROWS) {
        if (gens >= kConeRowsWindowGens) pk = cone_rows(care_col, gens, y0);
      }
    } else if constexpr (FIRST && ROWS) {
      if (gens >= kConeRowsWindowGens) pk = cone_rows(care_col, gens, y0);
    }
    if (K > kmax) return;
    if constexpr (FIRST && ROWS) {
      // a column window of more than 4 columns (the whole board too, in this
      // capped form) whose rows, widened by the cone, fit 32 (16) rows: 1 (2)
      // universes per register and lane, rows cut to the window
      // (cone_wave_rows)
      if constexpr (WIN) {
        if (pk > 0 && K > 4u && gens >= kConeRowsWindowGens) return split_pass(pk, y0, nw);
      }
      if (pk > 0 && K > 4u && gens >= kConeRowsWindowGens) {
        auto rw = [&](auto p_c, auto upw_c, auto pk_c, auto wrap_c) __attribute__((always_inline)) {
          constexpr int UPWc = decltype(upw_c)::value;
          if (wave * UPWc >= n) return;
          cone_wave_rows<decltype(p_c)::value, UPWc, RMAX, decltype(pk_c)::value, decltype(wrap_c)::value>(
              in, wanted, unwanted, out, n, wave * UPWc, nw * UPWc, gens, xs, K, y0, lane);
        };
        using I8 = std::integral_constant<int, 8>;
        using I16 = std::integral_constant<int, 16>;
        using I32 = std::integral_constant<int, 32>;
        using I64 = std::integral_constant<int, 64>;
        using K1 = std::integral_constant<int, 1>;
        using K2 = std::integral_constant<int, 2>;
        using T = std::true_type;
        using F = std::false_type;
        const bool wrap = y0 >= 32u, two = pk >= 2;
        if (K <= 8u) {
          if (two) return wrap ? rw(I8{}, I64{}, K2{}, T{}) : rw(I8{}, I64{}, K2{}, F{});
          return wrap ? rw(I8{}, I64{}, K1{}, T{}) : rw(I8{}, I64{}, K1{}, F{});
        }
        if (K <= 16u) {
          if (two) return wrap ? rw(I16{}, I16{}, K2{}, T{}) : rw(I16{}, I16{}, K2{}, F{});
          return wrap ? rw(I16{}, I16{}, K1{}, T{}) : rw(I16{}, I16{}, K1{}, F{});
        }
        if (K <= 32u) {
          if (two) return wrap ? rw(I32{}, I16{}, K2{}, T{}) : rw(I32{}, I16{}, K2{}, F{});
          return wrap ? rw(I32{}, I16{}, K1{}, T{}) : rw(I32{}, I16{}, K1{}, F{});
        }
        if (two) return wrap ? rw(I64{}, I16{}, K2{}, T{}) : rw(I64{}, I16{}, K2{}, F{});
        return wrap ? rw(I64{}, I16{}, K1{}, T{}) : rw(I64{}, I16{}, K1{}, F{});
      }
    }
  }
  if constexpr (!FIRST && A16 && !DMA) {
    if (K == (uint32_t)kWave) return cone_wave_full16<16, RMAX>(in, wanted, unwanted, out, n, wave * 16, nw * 16, lane);
  }
  if (K <= 8) {
    if (wave * 64 >= n) return;
    if (K <= 4) cone_wave<4, 64, RMAX, FIRST>(in, wanted, unwanted, out, n, wave * 64, nw * 64, gens, xs, K, lane);
    else cone_wave<8, 64, RMAX, FIRST>(in, wanted, unwanted, out, n, wave * 64, nw * 64, gens, xs, K, lane);
  } else if (K <= 16) {
    cone_wave<16, 16, RMAX, FIRST>(in, wanted, unwanted, out, n, wave * 16, nw * 16, gens, xs, K, lane);
  } else if (K <= 32) {
    cone_wave<32, 16, RMAX, FIRST>(in, wanted, unwanted, out, n, wave * 16, nw * 16, gens, xs, K, lane);
  } else {
    cone_wave<64, 16, RMAX, FIRST>(in, wanted, unwanted, out, n, wave * 16, nw * 16, gens, xs, K, lane);
  }
}

// The shipped shape (round 4's last): k_cone_adapt, register sets 8 at a
// time, at most 16 blocks per CU, for Contains and the 1-2 generation filter.
// Same process, 1M universes, back to back (tools/cone_ab.py,
// profiles/r04/r04x/cone_ab.jsonl), against k_cone with 64 universes per wave
// on a one-shot grid (shipped before): filter 0.0223 / 0.0226 ms on the
// 4-column target, 0.0436 / 0.0471 on 14 columns, 0.0658 / 0.0696 on 30, the
// whole board 0.0884 / 0.0898; Contains 0.0199 / 0.0213, 0.0409 / 0.0411,
// 0.0616 / 0.0626, 0.0790 / 0.0803.  Caps of 4 / 8 / 32 and no cap: slower
// on some target each (32: +7 % on the 4-column filter; none: +40 %).
// k_cone's fixed shapes, before: 64 per wave best for P <= 8 (0.0270 against
// 0.0288 ms with 32 per wave, each launch after a scrub,
// profiles/r04/r04g/cone_grid_ab.jsonl), 16 per wave best for 14-30 columns.
constexpr int kConeSets = 8;
constexpr int kConeAdaptBlocksPerCU = 16;
// (Round 5 routed the filter without final states by the generation count,
// the batch size and the last launch report: k_cone_adapt alone up to 4
// generations (6 for batches of at most 256K), the row-window passes up to
// 15, the split pair beyond; its constants and measurements are in the git
// history and DESIGN.md 3.2.)
// Round 6: the merged split kernel (step.hip, 3+ generations without final
// states) on a grid of at most this many blocks per CU looping over the
// batch (1M universes: 16 and 32 within 1-3 % of each other on every
// target, 8 up to 9 % slower on the one-row whole board; profiles/r06/ab/)
constexpr int kFilterIterBlocksPerCU = 16;
// (kConeWholeWinGens: step_kernels.hpp)
// The iterated search loop (gens > 2, no final states) steps the light cone
// while it spans at most this many columns (P <= 32 lanes per universe: at
// most half the natural layout's work per universe-generation, against the
// split layout's 18 issue slots plus its layout change) -- inside
// kContainsLo (step_kernels.hpp, kConeLoUniverses = 8 universes per wave
// chunk: that work is VALU-bound, and 64 per wave would leave 64K universes
// one wave per SIMD).
constexpr uint32_t kConeIterColumns = 32;
static_assert(kConeIterColumns <= 32, "kContainsLo's cone passes take P <= 32");
// The split kernels (step.hip, with or without final states) run on grids of
// at most 32 blocks per CU looping over the batch: one of the two always
// idles, and the working one is faster capped from 256K universes on.
constexpr int kSplitIterBlocksPerCU = 32;
// The tuning build's separate-launch form of the same (k_cone before the
// pair): 8 universes per wave.
constexpr int kConeIterUniverses = 8;

// Launches k_cone on a one-shot grid.
template <int UPW, int RMAX, bool FIRST, typename OutT, bool PIPE = false>
int launch_cone(const uint64_t *d_in, const uint64_t *d_wanted, const uint64_t *d_unwanted, OutT *d_out, size_t n,
                uint32_t gens, int cus, hipStream_t stream, int blocks_per_cu = 0, uint32_t kmax = kWave) {
  const dim3 grid(grid_for((n + UPW - 1) / UPW, cus, blocks_per_cu));
  bool a16 = false;
  if constexpr (!FIRST) a16 = aligned16(d_in);
  if constexpr (!FIRST) {
    if (a16) {
      hipLaunchKernelGGL((k_cone<UPW, RMAX, FIRST, OutT, true, PIPE>), grid, dim3(kBlock), 0, stream, d_in, d_wanted,
                         d_unwanted, d_out, (uint64_t)n, gens, kmax);
      return launched("k_cone launch");
    }
  }
  hipLaunchKernelGGL((k_cone<UPW, RMAX, FIRST, OutT, false, PIPE>), grid, dim3(kBlock), 0, stream, d_in, d_wanted,
                     d_unwanted, d_out, (uint64_t)n, gens, kmax);
  return launched("k_cone launch");
}

// Launches k_cone_adapt on ceil(n / 16) waves, at most blocks_per_cu blocks
// per CU (0: no cap).  DMA: a whole-board window takes cone_wave_full_dma
// when the batch is 16-byte aligned, on a grid of at most dma_blocks_per_cu
// blocks per CU (0: uncapped; blocks_per_cu then caps the waves of a
// windowed target).
template <int RMAX, bool FIRST, typename OutT, bool DMA = false, bool ROWS = true, bool WIN = false, bool EARLY = true>
int launch_cone_adapt(const uint64_t *d_in, const uint64_t *d_wanted, const uint64_t *d_unwanted, OutT *d_out,
                      size_t n, uint32_t gens, int cus, hipStream_t stream, int blocks_per_cu,
                      uint32_t kmax = kWave, int dma_blocks_per_cu = 0) {
  const dim3 grid(grid_for((n + 15) / 16, cus, blocks_per_cu));
  if constexpr (DMA) {
    if (aligned16(d_in)) {
      const uint32_t cap_waves = blocks_per_cu > 0 ? (uint32_t)(cus * blocks_per_cu * kWavesPerBlock) : 0u;
      hipLaunchKernelGGL((k_cone_adapt<RMAX, FIRST, OutT, true, true, ROWS, WIN, EARLY>),
                         dim3(grid_for((n + 15) / 16, cus, dma_blocks_per_cu)), dim3(kBlock), 0, stream, d_in,
                         d_wanted, d_unwanted, d_out, (uint64_t)n, gens, kmax, cap_waves);
      return launched("k_cone_adapt launch");
    }
  }
  bool a16 = false;
  if constexpr (!FIRST) a16 = aligned16(d_in);
  if (a16) {
    if constexpr (!FIRST) {
      hipLaunchKernelGGL((k_cone_adapt<RMAX, FIRST, OutT, true, false, ROWS, WIN>), grid, dim3(kBlock), 0, stream, d_in,
                         d_wanted, d_unwanted, d_out, (uint64_t)n, gens, kmax, 0u);
      return launched("k_cone_adapt launch");
    }
  }
  hipLaunchKernelGGL((k_cone_adapt<RMAX, FIRST, OutT, false, false, ROWS, WIN>), grid, dim3(kBlock), 0, stream, d_in,
                     d_wanted, d_unwanted, d_out, (uint64_t)n, gens, kmax, 0u);
  return launched("k_cone_adapt launch");
}

}  // namespace
}  // namespace lifeapi_impl
