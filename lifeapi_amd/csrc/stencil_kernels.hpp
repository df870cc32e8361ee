// stencil_kernels.hpp -- the streaming stencils of SURVEY 8(f) other than
// Step and LifeStable: NeighbourCount / InteractionCounts (k_counts),
// LifeWeld::Step (k_weld, k_weld_split) and the config-5 unknown_step_refined
// step (k_refined).  stencils.hip launches them (the product ABI); the tuning
// build (tools/tune/tune_stencils.hip) launches the same kernels with other
// occupancy settings for A/Bs.
#pragma once

#include <type_traits>

#include "device.hpp"
#include "split_layout.hpp"

namespace lifeapi_impl {
namespace {

// ---- neighbourhood counters --------------------------

// Bits 2..0 of the inclusive 3x3 count of this lane's column: the
// NeighbourCount adder chain (NeighbourCount.hpp:40-70) in the row-first
// order of life_gen<RULE 2> (4 DPP moves): count = fs + 2(fc+cs) + 4cc.
__device__ __forceinline__ void ncount3(W a, W &b2, W &b1, W &b0) {
  W L, R;
  neighbour_cols<XDPP>(a, L, R, nullptr, 0);
  const W h0 = lut3<kXor3>(L, a, R), h1 = lut3<kMaj>(L, a, R);
  const W h0u = rot_up(h0), h0d = rot_dn(h0), h1u = rot_up(h1), h1d = rot_dn(h1);
  const W fs = lut3<kXor3>(h0u, h0, h0d), fc = lut3<kMaj>(h0u, h0, h0d);
  const W cs = lut3<kXor3>(h1u, h1, h1d), cc = lut3<kMaj>(h1u, h1, h1d);
  b0 = fs;
  b1 = W{fc.lo ^ cs.lo, fc.hi ^ cs.hi};
  b2 = lut3<kCarry2>(cc, fc, cs);
}
// Same stencil as Step(), different output planes.  The two FullAdds of the
// vertical planes give the inclusive 3x3 count = fs + 2(fc + cs) + 4cc.
// MODE 0: NeighbourCount / CountNeighbourhood (NeighbourCount.hpp:40-70,
//         LifeAPI.hpp:909-952): planes bit3, bit2, bit1, bit0.
// MODE 1: InteractionCounts (LifeAPI.hpp:956-993): out1, out2, outMore.
// MODE 2: InteractionCountsAndNext (LifeAPI.hpp:997-1040): out1, out2,
//         outMore, next.
template <int MODE, bool CHUNK = false>
__global__ __launch_bounds__(kBlock) void k_counts(const uint64_t *__restrict__ in,
                                                   uint64_t *__restrict__ out, uint64_t n) {
  constexpr int P = MODE == 1 ? 3 : 4;
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t u = block_index<CHUNK>() * kWavesPerBlock + wib; u < n; u += stride) {
    const W a = ld<true>(in + u * kWave + lane);
    const W up = rot_up(a), dn = rot_dn(a);
    const W c0 = lut3<kXor3>(up, dn, a), c1 = lut3<kMaj>(up, dn, a);
    W L0, R0, L1, R1;
    neighbours<XDPP>(c0, c1, L0, R0, L1, R1, nullptr, lane);
    const W fs = lut3<kXor3>(L0, c0, R0), fc = lut3<kMaj>(L0, c0, R0);
    const W cs = lut3<kXor3>(L1, c1, R1), cc = lut3<kMaj>(L1, c1, R1);
    uint64_t *q = out + u * P * kWave + lane;
    const uint64_t s = join(a), vfs = join(fs), vfc = join(fc), vcs = join(cs), vcc = join(cc);
    if constexpr (MODE == 0) {
      const uint64_t carry = vfc & vcs;
      st<true>(q + 0 * kWave, split(vcc & carry));          // bit3
      st<true>(q + 1 * kWave, split(vcc ^ carry));          // bit2
      st<true>(q + 2 * kWave, split(vfc ^ vcs));            // bit1
      st<true>(q + 3 * kWave, fs);                          // bit0
    } else {
      const uint64_t o1 = ~s & ~vcc & vfs & ~vcs & ~vfc;
      const uint64_t o2 = ~s & ~vcc & ~vfs & (vcs ^ vfc);
      const uint64_t om = ~s & ~o2 & (vfc | vcs | vcc);
      st<true>(q + 0 * kWave, split(o1));
      st<true>(q + 1 * kWave, split(o2));
      st<true>(q + 2 * kWave, split(om));
      if constexpr (MODE == 2) {
        const uint64_t c2 = vcc ^ (vcs & vfc);
        st<true>(q + 3 * kWave, split((vfs ^ c2) & (vfc ^ vcs ^ c2) & (s | vfs)));
      }
    }
  }
}

// ---- LifeWeld::Step ----------------------------------
// LifeWeld.hpp:169-186: inclusive count bits 2..0 (CountNeighbourhood, bit3
// dropped) + the frozen 3-bit count (HalfAdd, FullAdd, FullAdd), then the
// Life rule on the sum.  The frozen planes are loop-invariant, so `gens`
// generations run in registers.  In place on LifeWeld[] = {state, frozen2,
// frozen1, frozen0} x 64 words; only the state plane is written back.
__device__ __forceinline__ W weld_gen(W s, W f2, W f1, W f0) {
  W b2, b1, b0;
  ncount3(s, b2, b1, b0);
  const W s0 = W{b0.lo ^ f0.lo, b0.hi ^ f0.hi}, k0 = W{b0.lo & f0.lo, b0.hi & f0.hi};
  const W s1 = lut3<kXor3>(b1, f1, k0), k1 = lut3<kMaj>(b1, f1, k0);
  const W s2 = lut3<kXor3>(b2, f2, k1);
  const W p = lut3<kLive>(s0, s2, s);  // (s0 ^ s2) & (s | s0)
  return W{p.lo & (s1.lo ^ s2.lo), p.hi & (s1.hi ^ s2.hi)};
}

// In place, one wave per LifeWeld.  Bit 31 of `gens` (kWeldReverse)
// reverses the order in which waves take the welds, and the welds taken
// from position `plain_from` on load and store with plain (not
// nontemporal) accesses: alternated between launches, a launch on the batch
// the last one stepped starts on the welds that launch touched last, part of
// which the memory-side Infinity Cache still holds (as k_step).
constexpr uint32_t kWeldReverse = 1u << 31;
// U welds per wave (their 4 U loads issued before the first generation); the
// tuning build measures U = 2, 4 (tools/ab/weld_u_ab.py)
template <bool CHUNK = false, int U = 1>
__global__ __launch_bounds__(kBlock) void k_weld(uint64_t *__restrict__ welds, uint64_t n,
                                                 uint32_t gens, uint64_t plain_from) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const bool rev = (gens & kWeldReverse) != 0;
  gens &= ~kWeldReverse;
  const uint64_t groups = (n + U - 1) / U;
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t k = block_index<CHUNK>() * kWavesPerBlock + wib; k < groups; k += stride) {
    const uint64_t g0 = (rev ? groups - 1 - k : k) * U;
    auto run = [&](auto nt) __attribute__((always_inline)) {
      constexpr bool NT = decltype(nt)::value;
      W s[U], f2[U], f1[U], f0[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const uint64_t *p = welds + (g0 + j) * 4 * kWave + lane;
        const bool ok = U == 1 || g0 + j < n;
        s[j] = ok ? ld<NT>(p) : W{0u, 0u};
        f2[j] = ok ? ld<NT>(p + kWave) : W{0u, 0u};
        f1[j] = ok ? ld<NT>(p + 2 * kWave) : W{0u, 0u};
        f0[j] = ok ? ld<NT>(p + 3 * kWave) : W{0u, 0u};
      }
      for (uint32_t g = 0; g < gens; ++g) {
#pragma unroll
        for (int j = 0; j < U; ++j) s[j] = weld_gen(s[j], f2[j], f1[j], f0[j]);
      }
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (U == 1 || g0 + j < n) st<NT>(welds + (g0 + j) * 4 * kWave + lane, s[j]);
    };
    if (k < plain_from) run(std::true_type{});
    else run(std::false_type{});
  }
}

// LifeWeld::Step iterated on the 8-way row split (split_layout.hpp): a wave
// holds 4 welds, state and the three frozen planes each in 8 VGPRs per lane,
// the state exchanged through LDS as in gen_split.
//
// The tail: the reference adds the inclusive count's bits 2..0 to the frozen
// count (HalfAdd, FullAdd, FullAdd, mod 8) and applies the Life rule to the
// sum (LifeWeld.hpp:169-186): 13 v_bitop3 after the h-layer when written as
// that adder chain.  tools/cgp_weld.c (the network search of
// tools/cgp_search.c with f2, f1, f0 as three more inputs) found this 10-gate
// network for the same function on all 4096 combinations of neighbourhood
// and frozen count, using the centre-row don't-cares; checked by
// tests/test_oracle.py::test_weld_tail_truth, and every GPU result is
// compared with the reference's own LifeWeld::Step.  Per 32-bit word and
// generation: 12 v_bitop3 with the h-layer, against about 25 slots on the
// natural layout (k_weld).  Its layout change of four planes costs more than
// the plain step's, so it pays from about 12 generations up: 256K welds x 16
// gens 0.24 vs 0.29 ms, x 256 gens 2.30 vs 3.31 ms, x 3 gens 0.14 vs 0.11 ms
// (profiles/r01/weld_ab.jsonl).
constexpr uint32_t kW0 = 0x69, kW2 = 0x52, kW5 = 0x95, kW6 = 0xA5, kW8 = 0x31, kW9 = 0x28;
__device__ __forceinline__ uint32_t weld_tail(uint32_t h0u, uint32_t h0, uint32_t h0d, uint32_t h1u,
                                              uint32_t h1, uint32_t h1d, uint32_t a, uint32_t f2,
                                              uint32_t f1, uint32_t f0) {
  const uint32_t w0 = lut3<kW0>(h0u, h0d, f0);
  const uint32_t w1 = lut3<kXor3>(f1, h1u, h1d);
  const uint32_t w2 = lut3<kW2>(w0, a, h0);
  const uint32_t w3 = lut3<kMaj>(h0d, f0, w0);
  const uint32_t w4 = lut3<kMaj>(h1d, f1, h1u);
  const uint32_t w5 = lut3<kW5>(w1, w3, f2);
  const uint32_t w6 = lut3<kW6>(w5, h1d, w4);
  const uint32_t w7 = lut3<kXor3>(w1, w2, w3);
  const uint32_t w8 = lut3<kW8>(a, w6, w2);
  return lut3<kW9>(h1, w7, w8);
}

__device__ __forceinline__ void gen_weld_split(uint32_t (&r)[8], const uint32_t (&f2)[8],
                                               const uint32_t (&f1)[8], const uint32_t (&f0)[8],
                                               uint32_t *slot, int lane) {
  constexpr int S = 8, P = 4;
  uint32_t lv[S], rv[S];
  lds_exchange<S>(r, lv, rv, slot, lane);
  uint32_t h0[S], h1[S];
#pragma unroll
  for (int j = 0; j < S; ++j) {
    h0[j] = lut3<kXor3>(lv[j], r[j], rv[j]);
    h1[j] = lut3<kMaj>(lv[j], r[j], rv[j]);
  }
  const uint32_t h0u = __builtin_amdgcn_alignbit(h0[S - 1], h0[S - 1], 32 - P);  // rotl P
  const uint32_t h1u = __builtin_amdgcn_alignbit(h1[S - 1], h1[S - 1], 32 - P);
  const uint32_t h0d = __builtin_amdgcn_alignbit(h0[0], h0[0], P);  // rotr P
  const uint32_t h1d = __builtin_amdgcn_alignbit(h1[0], h1[0], P);
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const uint32_t a0 = j == 0 ? h0u : h0[j - 1], c0 = j == S - 1 ? h0d : h0[j + 1];
    const uint32_t a1 = j == 0 ? h1u : h1[j - 1], c1 = j == S - 1 ? h1d : h1[j + 1];
    r[j] = weld_tail(a0, h0[j], c0, a1, h1[j], c1, r[j], f2[j], f1[j], f0[j]);
  }
}

template <bool NT>
__global__ __launch_bounds__(kBlock) void k_weld_split(uint64_t *__restrict__ welds, uint64_t n,
                                                       uint32_t gens) {
  constexpr int S = 8, P = 4;
  __shared__ uint32_t lds[kWavesPerBlock * S * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * P;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wib) * P; u0 < n; u0 += stride) {
    uint32_t r[S], f2[S], f1[S], f0[S];
    {
      W c[4][P];  // [plane][weld]: state, frozen2, frozen1, frozen0 (LifeWeld.hpp:18-20)
#pragma unroll
      for (int u = 0; u < P; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          c[q][u] = u0 + u < n ? ld<NT>(welds + ((u0 + u) * 4 + q) * kWave + lane) : W{0u, 0u};
      Split<S>::load(c[0], r);
      Split<S>::load(c[1], f2);
      Split<S>::load(c[2], f1);
      Split<S>::load(c[3], f0);
    }
    for (uint32_t g = 0; g < gens; ++g) gen_weld_split(r, f2, f1, f0, lds + wib * S * kWave, lane);
    W c[P];
    Split<S>::store(r, c);
#pragma unroll
    for (int u = 0; u < P; ++u)
      if (u0 + u < n) st<NT>(welds + (u0 + u) * 4 * kWave + lane, c[u]);
  }
}

// ---- config 5: the unknown_step_refined ternary step --------------------

// bitslicing/unknown_step_refined.hpp:1-85 as a v_bitop3 network.  The
// network is generated (tools/synth_sop.py) from the fragment's complete
// truth table, which tests/golden/make_golden.py extracts from the reference
// build, and is verified against all 2^16 input combinations when generated.
template <class T>
__device__ __forceinline__ void refined_circuit(const T (&x)[16], T &next_on, T &next_unknown,
                                                T &next_unknown_stable) {
#include "refined_circuit.inc"
}

__device__ __forceinline__ void refined_load(W (&pl)[11], const uint64_t *in, uint64_t u, int lane) {
  const uint64_t *p = in + u * 11 * kWave + lane;
#pragma unroll
  for (int k = 0; k < 11; ++k) pl[k] = ld<true>(p + k * kWave);
}

__device__ __forceinline__ void refined_one(const W (&pl)[11], uint64_t *out, uint64_t u, int lane) {
  W x[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = pl[3 + k];  // l2 l3 d0 d1 d2 d4 d5 d6
  x[8] = pl[2];                                  // current_unknown
  x[9] = pl[1];                                  // current_on
  ncount3(pl[0], x[10], x[11], x[12]);           // s2 s1 s0
  ncount3(pl[1], x[13], x[14], x[15]);           // on2 on1 on0
  // Evaluate the ~500-node network on the low and then the high 32 bits of
  // the column: the scheduling barrier keeps the two halves from being
  // interleaved, which halves the live temporaries (VGPR pressure).
  uint32_t xl[16], xh[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    xl[k] = x[k].lo;
    xh[k] = x[k].hi;
  }
  W o0, o1, o2;
  refined_circuit(xl, o0.lo, o1.lo, o2.lo);
  __builtin_amdgcn_sched_barrier(0);
  refined_circuit(xh, o0.hi, o1.hi, o2.hi);
  uint64_t *q = out + u * 3 * kWave + lane;
  st<true>(q, o0);
  st<true>(q + kWave, o1);
  st<true>(q + 2 * kWave, o2);
}

// One wave per universe at a time, grid-strided.  In: 11 planes x 64 words
// (stable.state, current.state, current.unknown, live2, live3, dead0, dead1,
// dead2, dead4, dead5, dead6 -- LifeStable.hpp:41-53 with options stored as
// "1 = ruled out").  Out: 3 planes (next_on, next_unknown,
// next_unknown_stable).  PF = 1: the next universe's 11 loads are issued
// before this one's ~1000-instruction network runs (register double buffer),
// so HBM traffic overlaps the VALU work of the same wave.  OCC = minimum
// waves per SIMD requested from the register allocator (0 = no bound).
template <int PF, int OCC, bool CHUNK = false>
__global__ __launch_bounds__(kBlock, OCC > 0 ? OCC : 1) void k_refined(
    const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t n) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  uint64_t u = block_index<CHUNK>() * kWavesPerBlock + wib;
  if (u >= n) return;
  if constexpr (PF == 0) {
    for (; u < n; u += stride) {
      W pl[11];
      refined_load(pl, in, u, lane);
      refined_one(pl, out, u, lane);
    }
  } else {
    W cur[11];
    refined_load(cur, in, u, lane);
    for (; u < n; u += stride) {
      const uint64_t un = u + stride;
      W nxt[11];
      if (un < n) refined_load(nxt, in, un, lane);
      refined_one(cur, out, u, lane);
      if (un < n) {
#pragma unroll
        for (int k = 0; k < 11; ++k) cur[k] = nxt[k];
      }
    }
  }
}

}  // namespace
}  // namespace lifeapi_impl
