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
#pragma once

#include "step_kernels.hpp"

namespace lifeapi_impl {
namespace {

// One wave's chunks of UPW universes u0 .. u0 + UPW - 1, u0 = u_first,
// u_first + u_step, ... (< n), under the window (xs = first loaded column,
// K <= P loaded columns).  FIRST: out[u] = the first
// generation in 1..gens whose state contains the target (0 = never), else
// out[u] = Contains(target) of the state as loaded (gens unused).  Register
// sets go RMAX at a time: all their loads are issued before the first test.
template <int P, int UPW, int RMAX, bool FIRST, typename OutT>
__device__ __forceinline__ void cone_wave(const uint64_t *in, const uint64_t *__restrict__ wanted,
                                          const uint64_t *__restrict__ unwanted, OutT *__restrict__ out,
                                          uint64_t n, uint64_t u_first, uint64_t u_step, uint32_t gens,
                                          uint32_t xs, uint32_t K, int lane) {
  constexpr int GPS = kWave / P;  // universes per register set
  static_assert(UPW % GPS == 0, "a wave takes whole register sets");
  constexpr int R = UPW / GPS;
  constexpr int RB = R < RMAX ? R : RMAX;
  static_assert(R % RB == 0, "passes of RB sets");
  const uint32_t j = (uint32_t)lane & (P - 1), q = (uint32_t)lane / P;
  const uint32_t col = (xs + j) & (kWave - 1);
  const bool live = j < K;
  // the target's column under this lane (zero outside the window: the care
  // columns all lie in [x0, x0 + w), and no lane j >= K or margin lane maps
  // onto one while K <= 64)
  const uint64_t w64 = live ? wanted[col] : 0ull, m64 = live ? (w64 | unwanted[col]) : 0ull;
  const W tw = split(w64), tm = split(m64);
  const uint32_t sh = q * P;
  auto clean = [&](W s) __attribute__((always_inline)) {
    const uint32_t d = ((s.lo ^ tw.lo) & tm.lo) | ((s.hi ^ tw.hi) & tm.hi);
    const uint64_t bad = __ballot(d != 0u);  // wave-uniform
    if constexpr (P == kWave) return bad == 0ull;
    else return ((bad >> sh) & ((1ull << P) - 1)) == 0ull;
  };
  static_assert(UPW <= kWave, "one result per lane");
  for (uint64_t u0 = u_first; u0 < n; u0 += u_step) {
    uint32_t mine = 0;  // lane L: the result of universe u0 + L (one coalesced store per chunk)
#pragma unroll 1
    for (int pass = 0; pass < R / RB; ++pass) {
      const uint64_t ub = u0 + (uint64_t)pass * RB * GPS + q;
      W a[RB];
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const uint64_t u = ub + (uint64_t)k * GPS;
        a[k] = (live && u < n) ? ld<true>(in + u * kWave + col) : W{0u, 0u};
      }
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
      // set k's group q is universe u0 + pass * RB * GPS + k * GPS + q: its
      // result (uniform over the group) moves to that lane
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const uint32_t first = (uint32_t)(pass * RB + k) * GPS, rel = (uint32_t)lane - first;
        uint32_t v = res[k];
        if constexpr (GPS > 1) v = (uint32_t)__shfl((int)v, (int)((rel & (GPS - 1)) * P));
        if (rel < (uint32_t)GPS) mine = v;
      }
    }
    if (lane < UPW && u0 + lane < n) out[u0 + lane] = (OutT)mine;
  }
}

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

// UPW universes per wave (one-shot grid of ceil(n / UPW) waves), every wave
// choosing its lane layout from the window (wave-uniform: the target is the
// same for all).  Each choice runs its own copy of the pass.  A16: the batch
// is 16-byte aligned (Contains over the whole board then takes 16-byte loads).
// kmax: a wave whose window K exceeds it returns at once (the iterated
// search loop's split-layout kernels answer those, step.hip).
template <int UPW, int RMAX, bool FIRST, typename OutT, bool A16 = false>
__global__ __launch_bounds__(kBlock) void k_cone(const uint64_t *in, const uint64_t *__restrict__ wanted,
                                                 const uint64_t *__restrict__ unwanted, OutT *__restrict__ out,
                                                 uint64_t n, uint32_t gens, uint32_t kmax) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t u0 = wave * UPW, step = (uint64_t)gridDim.x * kWavesPerBlock * UPW;  // grid-stride (capped grids)
  if (u0 >= n) return;
  uint32_t xs, K;
  cone_window(wanted, unwanted, FIRST ? gens : 0u, lane, xs, K);
  if (K > kmax) return;
  if constexpr (!FIRST && A16) {
    if (K == (uint32_t)kWave) return cone_wave_full16<UPW, RMAX>(in, wanted, unwanted, out, n, u0, step, lane);
  }
  // (a wave of UPW universes takes whole register sets: P >= 64 / UPW)
  if (K <= 4 && UPW >= 16) cone_wave<UPW >= 16 ? 4 : 8, UPW, RMAX, FIRST>(in, wanted, unwanted, out, n, u0, step, gens,
                                                                         xs, K, lane);
  else if (K <= 8) cone_wave<8, UPW, RMAX, FIRST>(in, wanted, unwanted, out, n, u0, step, gens, xs, K, lane);
  else if (K <= 16) cone_wave<16, UPW, RMAX, FIRST>(in, wanted, unwanted, out, n, u0, step, gens, xs, K, lane);
  else if (K <= 32) cone_wave<32, UPW, RMAX, FIRST>(in, wanted, unwanted, out, n, u0, step, gens, xs, K, lane);
  else cone_wave<64, UPW, RMAX, FIRST>(in, wanted, unwanted, out, n, u0, step, gens, xs, K, lane);
}

// The shipped shape: 64 universes per wave, register sets 8 at a time, one-
// shot grid.  Same process, 1M universes, each launch after a read-only scrub
// (tools/ab/cone_grid_ab.py, profiles/r04/r04g/cone_grid_ab.jsonl): the
// 4-column target's filter 0.0270 against 0.0288 ms with 32 per wave (back to
// back 0.0221 / 0.0240), Contains 0.0246 / 0.0256, a loaf box alike; the
// whole-board filter 0.0933 / 0.0892 (back to back 0.0928 / 0.0940).  Capped
// grids whose waves find the window once and loop over the batch: within
// +-3 % of the one-shot grid for small targets, slower for the whole board.
constexpr int kConeUniverses = 64, kConeSets = 8;
// The iterated search loop (gens > 2, no final states) takes the light-cone
// kernel while the cone spans at most this many columns (P <= 32 lanes per
// universe: at most half the natural layout's work per universe-generation,
// against the split layout's 18 issue slots plus its layout change).
constexpr uint32_t kConeIterColumns = 32;
// ... with 8 universes per wave (1-4 register sets): that work is VALU-bound,
// and 64 universes per wave would leave 64K universes one wave per SIMD.
constexpr int kConeIterUniverses = 8;
// ... on a grid of at most 16 blocks (64 waves) per CU looping over the
// batch: when the split kernels answer (wider cones), the cone launch's waves
// all return after the window search, and a one-shot grid of n / 8 waves
// would cost that many wave launches.
constexpr int kConeIterBlocksPerCU = 16;
// ... and the split pair after it on grids of at most 32 blocks per CU
// (step.hip): one of the two always idles.
constexpr int kSplitIterBlocksPerCU = 32;

// Launches k_cone on a one-shot grid.
template <int UPW, int RMAX, bool FIRST, typename OutT>
int launch_cone(const uint64_t *d_in, const uint64_t *d_wanted, const uint64_t *d_unwanted, OutT *d_out, size_t n,
                uint32_t gens, int cus, hipStream_t stream, int blocks_per_cu = 0, uint32_t kmax = kWave) {
  const dim3 grid(grid_for((n + UPW - 1) / UPW, cus, blocks_per_cu));
  bool a16 = false;
  if constexpr (!FIRST) a16 = aligned16(d_in);
  if constexpr (!FIRST) {
    if (a16) {
      hipLaunchKernelGGL((k_cone<UPW, RMAX, FIRST, OutT, true>), grid, dim3(kBlock), 0, stream, d_in, d_wanted,
                         d_unwanted, d_out, (uint64_t)n, gens, kmax);
      return launched("k_cone launch");
    }
  }
  hipLaunchKernelGGL((k_cone<UPW, RMAX, FIRST, OutT, false>), grid, dim3(kBlock), 0, stream, d_in, d_wanted,
                     d_unwanted, d_out, (uint64_t)n, gens, kmax);
  return launched("k_cone launch");
}

}  // namespace
}  // namespace lifeapi_impl
