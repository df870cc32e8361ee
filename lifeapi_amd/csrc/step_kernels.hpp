// step_kernels.hpp -- the generation networks and the two step kernels of
// batched LifeState::Step() (LifeAPI.hpp:1196-1216, Stepped(n) :877-886):
// k_step (natural layout, one column per lane) and k_step_split (8-way row
// split, state resident in VGPRs across generations).  step.hip instantiates
// the shipped configurations; the tuning build (tools/tune/tune_step.hip)
// instantiates the measured alternatives.
#pragma once

#include "host.hpp"
#include "split_layout.hpp"
#include "split_asm.inc"
#include "cone_split.hpp"

namespace lifeapi_impl {
// internal linkage: every library that includes this header gets its own
// kernels (the product and the tuning build never share instantiations)
namespace {

template <int X, int RULE>
__device__ __forceinline__ W life_gen(W a, uint64_t *slot, int lane) {
  if constexpr (RULE == 4) {
    // the RULE 3 network on the (E, O) layout: 18 v_bitop3 + 4 v_alignbit
    // per generation plus the exchange
    W L, R;
    neighbour_cols<X>(a, L, R, slot, lane);
    const W h0 = lut3<kXor3>(L, a, R), h1 = lut3<kMaj>(L, a, R);
    const uint32_t h0u = rotl1(h0.hi), h0d = rotr1(h0.lo);  // rows 2k-1 (for E), 2k+2 (for O)
    const uint32_t h1u = rotl1(h1.hi), h1d = rotr1(h1.lo);
    const W s0{lut3<kLe1>(h0u, h0.lo, h0.hi), lut3<kLe1>(h0.lo, h0.hi, h0d)};
    const W s1{lut3<kNae>(h0u, h0.lo, h0.hi), lut3<kNae>(h0.lo, h0.hi, h0d)};
    const W s2{lut3<kLe1>(h1u, h1.lo, h1.hi), lut3<kLe1>(h1.lo, h1.hi, h1d)};
    const W s3{lut3<kEven>(h1u, h1.lo, h1.hi), lut3<kEven>(h1.lo, h1.hi, h1d)};
    const W t1 = lut3<kT1>(s0, s1, a);
    const W t2 = lut3<kT2>(s2, a, t1);
    return lut3<kT3>(s1, s3, t2);
  }
  if constexpr (RULE == 3) {
    // row-first exchange and rotations as RULE 2, then the 7-LUT network:
    // 26 VALU per generation plus the exchange
    W L, R;
    neighbour_cols<X>(a, L, R, slot, lane);
    const W h0 = lut3<kXor3>(L, a, R), h1 = lut3<kMaj>(L, a, R);
    const W h0u = rot_up(h0), h0d = rot_dn(h0), h1u = rot_up(h1), h1d = rot_dn(h1);
    const W s0 = lut3<kLe1>(h0u, h0, h0d), s1 = lut3<kNae>(h0u, h0, h0d);
    const W s2 = lut3<kLe1>(h1u, h1, h1d), s3 = lut3<kEven>(h1u, h1, h1d);
    const W t1 = lut3<kT1>(s0, s1, a);
    const W t2 = lut3<kT2>(s2, a, t1);
    return lut3<kT3>(s1, s3, t2);
  }
  if constexpr (RULE == 14) {
    // RULE 3's exchange, h-layer and rotates with the 6-LUT tail
    // (life_tail6) per 32-bit half: 24 VALU per generation plus the exchange
    W L, R;
    neighbour_cols<X>(a, L, R, slot, lane);
    const W h0 = lut3<kXor3>(L, a, R), h1 = lut3<kMaj>(L, a, R);
    const W h0u = rot_up(h0), h0d = rot_dn(h0), h1u = rot_up(h1), h1d = rot_dn(h1);
    return W{life_tail6(h0u.lo, h0.lo, h0d.lo, h1u.lo, h1.lo, h1d.lo, a.lo),
             life_tail6(h0u.hi, h0.hi, h0d.hi, h1u.hi, h1.hi, h1d.hi, a.hi)};
  }
  if constexpr (RULE == 2) {
    // Row-first form of the same adder network.  A DPP move issues at half
    // the VALU rate on gfx950 (tools/ab/valu_probe.hip: 8 DPP of 32 instructions
    // cost 25 % of the loop), so exchange the raw column (4 DPP) instead of
    // its two vertical-sum planes (8 DPP):
    //   horizontal 3-sums  H0 = xor3(L,a,R), H1 = maj(L,a,R)   (2-bit, 0..3)
    //   vertical    FullAdd(H0 up, H0, H0 down) -> fs, fc
    //               FullAdd(H1 up, H1, H1 down) -> cs, cc
    // and the 3x3 count is again fs + 2(fc + cs) + 4cc, so the rule tail is
    // StepAlt's (LifeAPI.hpp:1251-1252).  Addition is commutative, so this is
    // bit-identical to CountRows-then-columns (LifeAPI.hpp:897-907,1218-1254).
    W L, R;
    neighbour_cols<X>(a, L, R, slot, lane);
    const W h0 = lut3<kXor3>(L, a, R), h1 = lut3<kMaj>(L, a, R);
    const W h0u = rot_up(h0), h0d = rot_dn(h0), h1u = rot_up(h1), h1d = rot_dn(h1);
    const W fs = lut3<kXor3>(h0u, h0, h0d), fc = lut3<kMaj>(h0u, h0, h0d);
    const W cs = lut3<kXor3>(h1u, h1, h1d), cc = lut3<kMaj>(h1u, h1, h1d);
    const W b2 = lut3<kCarry2>(cc, fc, cs);
    const W p = lut3<kLive>(fs, b2, a);
    const W q = lut3<kXor3>(fc, cs, b2);
    return W{p.lo & q.lo, p.hi & q.hi};
  }
  const W up = rot_up(a), dn = rot_dn(a);
  if constexpr (RULE == 0) {
    // CountRows (LifeAPI.hpp:897-907): vertical 3-sum as two planes
    const W c0 = lut3<kXor3>(up, dn, a);
    const W c1 = lut3<kMaj>(up, dn, a);
    W L0, R0, L1, R1;
    neighbours<X>(c0, c1, L0, R0, L1, R1, slot, lane);
    // FullAdd x2 (LifeAPI.hpp:826-833, StepAlt :1246-1249): 3x3 inclusive
    // count = fs + 2(fc + cs) + 4cc
    const W fs = lut3<kXor3>(L0, c0, R0), fc = lut3<kMaj>(L0, c0, R0);
    const W cs = lut3<kXor3>(L1, c1, R1), cc = lut3<kMaj>(L1, c1, R1);
    // StepAlt :1251-1252: cc ^= fc & cs;  next = (fs^cc) & (fc^cs^cc) & (a|fs)
    const W b2 = lut3<kCarry2>(cc, fc, cs);
    const W p = lut3<kLive>(fs, b2, a);
    const W q = lut3<kXor3>(fc, cs, b2);
    return W{p.lo & q.lo, p.hi & q.hi};
  } else {
    // the same network in plain and/or/xor (the compiler folds the DPP moves
    // into v_*_dpp consumers); kept as an ablation of the bitop3 form
    const uint64_t av = join(a), u = join(up), d = join(dn);
    const uint64_t c0v = u ^ d ^ av, c1v = (u & d) | ((u ^ d) & av);
    W L0, R0, L1, R1;
    neighbours<X>(split(c0v), split(c1v), L0, R0, L1, R1, slot, lane);
    const uint64_t l0 = join(L0), r0 = join(R0), l1 = join(L1), r1 = join(R1);
    const uint64_t h0 = l0 ^ c0v, h1 = l1 ^ c1v;
    const uint64_t fs = h0 ^ r0, fc = (l0 & c0v) | (r0 & h0);
    const uint64_t cs = h1 ^ r1;
    uint64_t cc = (l1 & c1v) | (r1 & h1);
    cc ^= fc & cs;
    return split((fs ^ cc) & (fc ^ cs ^ cc) & (av | fs));
  }
}

// out[u] = in[u] stepped `gens` times.  Wave w of the grid takes groups of U
// consecutive universes, grid-strided.  All branches are wave-uniform.
// in == out is allowed (Step() in place), so neither pointer is
// __restrict__: each wave loads its universes before it stores them and no
// wave touches another's (the same holds for k_step_split).
// Bit 31 of `gens` (kReverse) reverses the order in which waves take the
// groups: alternated between launches, each launch first reads what the one
// before it wrote last.  The groups taken from position `plain_from` on (in
// the launch's order) store with plain stores, the rest as NTS says: the
// last-written part then stays in the memory-side Infinity Cache for the next
// launch to read first, and the nontemporal rest does not evict it
// (DESIGN.md 3.1).  The launcher sets both only for gens <= 2.
constexpr uint32_t kReverse = 1u << 31;
// Bit 30 of `gens` (kXcdChunk): each XCD takes a contiguous eighth of the
// groups (xcd_chunk_block); the launcher sets it for large batches.
constexpr uint32_t kXcdChunk = 1u << 30;
// NTS: nontemporal stores (default: as the loads) before `plain_from`.
template <int X, int U, bool NT, int RULE, bool NTS>
__device__ __forceinline__ void step_body(const uint64_t *in, uint64_t *out, uint64_t n, uint32_t gens,
                                          uint64_t plain_from) {
  __shared__ uint64_t lds[uses_lds(X) ? kWavesPerBlock * U * 2 * kWave : 1];
  const int lane = threadIdx.x & (kWave - 1);
  // wave index in the block, made provably wave-uniform so that the tail
  // tests below are scalar branches
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const bool rev = (gens & kReverse) != 0;
  const uint64_t blk = (gens & kXcdChunk) ? xcd_chunk_block() : (uint64_t)blockIdx.x;
  gens &= ~(kReverse | kXcdChunk);
  const uint64_t groups = (n + U - 1) / U, wstride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t grp = blk * kWavesPerBlock + wib; grp < groups; grp += wstride) {
    const uint64_t u0 = (rev ? groups - 1 - grp : grp) * U;
    W a[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      a[k] = (u0 + k < n) ? ld<NT>(in + (u0 + k) * kWave + lane) : W{0u, 0u};
    if constexpr (RULE == 4) {
#pragma unroll
      for (int k = 0; k < U; ++k) a[k] = to_eo(a[k]);
    }
    for (uint32_t g = 0; g < gens; ++g) {
#pragma unroll
      for (int k = 0; k < U; ++k)
        a[k] = life_gen<X, RULE>(a[k], lds + (wib * U + k) * 2 * kWave, lane);
    }
    if constexpr (RULE == 4) {
#pragma unroll
      for (int k = 0; k < U; ++k) a[k] = from_eo(a[k]);
    }
    if (grp < plain_from) {
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (u0 + k < n) st<NTS>(out + (u0 + k) * kWave + lane, a[k]);
    } else {
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (u0 + k < n) st<false>(out + (u0 + k) * kWave + lane, a[k]);
    }
  }
}

template <int X, int U, bool NT, int RULE, bool NTS = NT>
__global__ __launch_bounds__(kBlock) void k_step(const uint64_t *in, uint64_t *out, uint64_t n,
                                                 uint32_t gens, uint64_t plain_from) {
  step_body<X, U, NT, RULE, NTS>(in, out, n, gens, plain_from);
}
// The same kernel under another name, for the tuning build's side launches
// (bench.py's cache-neutral and copy figures, the order A/Bs), so that a
// rocprofv3 trace of the bench tells them from the product's launches.
template <int X, int U, bool NT, int RULE, bool NTS = NT>
__global__ __launch_bounds__(kBlock) void k_step_ab(const uint64_t *in, uint64_t *out, uint64_t n,
                                                    uint32_t gens, uint64_t plain_from) {
  step_body<X, U, NT, RULE, NTS>(in, out, n, gens, plain_from);
}

// step_body with the wave's U universes moved through LDS (the LifeStable
// passes' LDS-DMA form, stable_kernels.hpp k_stable_dma): U / 2
// sixteen-byte-per-lane global_load_lds in (lanes 0-31 one universe, 32-63 the
// next), ds_read_b64 out to lane = column; WIDE: the results back through the
// image, 16 bytes per lane (ds_write_b64, ds_read_b128, global_store_dwordx4),
// else 8-byte stores from the lanes.  Order, plain-stored tail and XCD
// chunking as step_body.  The batch must be 16-byte aligned.
template <int U, int RULE, bool NTS, bool WIDE>
__device__ __forceinline__ void step_body_dma(const uint64_t *in, uint64_t *out, uint64_t n, uint32_t gens,
                                              uint64_t plain_from) {
  static_assert(U % 2 == 0, "pairs of universes per 16-byte load");
  __shared__ uint64_t img_all[kWavesPerBlock][U * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  uint64_t *img = img_all[wib];
  const bool rev = (gens & kReverse) != 0;
  const uint64_t blk = (gens & kXcdChunk) ? xcd_chunk_block() : (uint64_t)blockIdx.x;
  gens &= ~(kReverse | kXcdChunk);
  const uint64_t groups = (n + U - 1) / U, wstride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t grp = blk * kWavesPerBlock + wib; grp < groups; grp += wstride) {
    const uint64_t u0 = (rev ? groups - 1 - grp : grp) * U;
#pragma unroll
    for (int i = 0; i < U / 2; ++i) {
      uint64_t u = u0 + 2 * i + (lane >> 5);
      if (u >= n) u = n - 1;  // (a valid address; the result is not stored)
      const char *src = reinterpret_cast<const char *>(in + u * kWave) + (lane & 31) * 16;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                       (__attribute__((address_space(3))) void *)(img + i * 2 * kWave), 16, 0, 2);
    }
    __builtin_amdgcn_s_waitcnt(kWaitVm0);
    W a[U];
#pragma unroll
    for (int k = 0; k < U; ++k) a[k] = split(img[k * kWave + lane]);
    for (uint32_t g = 0; g < gens; ++g) {
#pragma unroll
      for (int k = 0; k < U; ++k) a[k] = life_gen<XDPP, RULE>(a[k], nullptr, lane);
    }
    const bool nt = NTS && grp < plain_from;
    if constexpr (WIDE) {
#pragma unroll
      for (int k = 0; k < U; ++k) img[k * kWave + lane] = join(a[k]);
      const u64x2 *src = reinterpret_cast<const u64x2 *>(img) + lane;
#pragma unroll
      for (int i = 0; i < U / 2; ++i) {
        const uint64_t u = u0 + 2 * i + (lane >> 5);
        const u64x2 v = src[i * kWave];
        u64x2 *dst = reinterpret_cast<u64x2 *>(out + u * kWave) + (lane & 31);
        if (u < n) {
          if (nt) __builtin_nontemporal_store(v, dst);
          else *dst = v;
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (u0 + k < n) {
          if (nt) st<true>(out + (u0 + k) * kWave + lane, a[k]);
          else st<false>(out + (u0 + k) * kWave + lane, a[k]);
        }
    }
  }
}

template <int U, int RULE, bool NTS, bool WIDE>
__global__ __launch_bounds__(kBlock) void k_step_dma(const uint64_t *in, uint64_t *out, uint64_t n, uint32_t gens,
                                                     uint64_t plain_from) {
  step_body_dma<U, RULE, NTS, WIDE>(in, out, n, gens, plain_from);
}

// k_step for the split layouts: wave w takes G groups of P = S/2
// consecutive universes, grid-strided; all branches wave-uniform.  NET: the
// tail network (7 = RULE 3's, 6 = life_tail6); D: registers exchanged by DPP
// instead of LDS (gen_split), or kPipe: the software-pipelined LDS loop
// (gens_split_pipe).
constexpr int kPipe = -1;
constexpr int kAsmLoop = -3;  // the hand-allocated rule-11 loop (split_asm.inc)
// WPB: waves per block (the tuning build's A/B of finer blocks; the product
// launches kWavesPerBlock).
template <int S, int G, bool NT, int NET, int D = 0, int V = 0, int WPB = kWavesPerBlock>
__global__ __launch_bounds__(WPB * kWave) void k_step_split(const uint64_t *in, uint64_t *out, uint64_t n,
                                                            uint32_t gens, uint64_t /* plain_from: k_step's */) {
  constexpr int P = S / 2;
  __shared__ uint32_t lds[WPB * G * S * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t per_wave = (uint64_t)G * P;
  const uint64_t stride = (uint64_t)gridDim.x * WPB * per_wave;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * WPB + wib) * per_wave; u0 < n; u0 += stride) {
    uint32_t r[G][S];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      W c[P];
#pragma unroll
      for (int u = 0; u < P; ++u) {
        const uint64_t x = u0 + g * P + u;
        c[u] = x < n ? ld<NT>(in + x * kWave + lane) : W{0u, 0u};
      }
      Split<S>::load(c, r[g]);
    }
    if constexpr (D == kPipe) {
#pragma unroll
      for (int g = 0; g < G; ++g) gens_split_pipe<S, NET>(r[g], lds + (wib * G + g) * S * kWave, lane, gens);
    } else if constexpr (D == kAsmLoop) {
      static_assert(S == 8 && NET == 6 && G <= 2, "split_asm.inc is rule 11, one or two groups");
      const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)(
          lds + wib * G * S * kWave);  // group g's planes at base + 2 KiB * g
      const uint32_t self = base + lane * 16u, prev = base + ((lane + kWave - 1) & (kWave - 1)) * 16u,
                     next = base + ((lane + 1) & (kWave - 1)) * 16u;
      if constexpr (G == 2) split_gens_asm2(r[0], r[1], gens, self, prev, next);
      else if constexpr (V == 1) split_gens_asm_v1(r[0], gens, self, prev, next);
      else if constexpr (V == 2) split_gens_asm_v2(r[0], gens, self, prev, next);
      else if constexpr (V == 3) split_gens_asm_v3(r[0], gens, self, prev, next);
      else split_gens_asm_v0(r[0], gens, self, prev, next);
    } else {
      for (uint32_t it = 0; it < gens; ++it) {
#pragma unroll
        for (int g = 0; g < G; ++g) gen_split<S, NET, D>(r[g], lds + (wib * G + g) * S * kWave, lane);
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      W c[P];
      Split<S>::store(r[g], c);
#pragma unroll
      for (int u = 0; u < P; ++u) {
        const uint64_t x = u0 + g * P + u;
        if (x < n) st<NT>(out + x * kWave + lane, c[u]);
      }
    }
  }
}

// Step + Contains fused for gens <= 2 (k_step_contains_split takes more):
// first generation in 1..gens whose state contains the target (0 = never);
// the state keeps stepping to `gens` for d_final.  The streaming step's
// shape -- U universes per wave, loads issued first, nontemporal -- so the
// search filter of SURVEY 8(f) row 1 reads 512 B and writes 4 B per
// universe.  `in` and `fin` may be the same array (the host form stages
// through one buffer), so neither is __restrict__: each wave loads its
// universes before it stores them, and no wave touches another's universes.
// Group order (kReverse in `gens`) and the plain-stored tail of the final
// states (`plain_from`) as k_step's.
// X / RULE: the exchange and network of the generation (life_gen).  PF: each
// wave loads the next group's states before it works on the current one (a
// grid of at most the resident waves, looping over the batch).
template <int U, bool WIDE = false, int X = XDPP, int RULE = 3, bool PF = false>
__global__ __launch_bounds__(kBlock) void k_step_contains(const uint64_t *in, uint64_t *fin,
                                                          const uint64_t *__restrict__ wanted,
                                                          const uint64_t *__restrict__ unwanted,
                                                          uint32_t *__restrict__ first,
                                                          uint64_t n, uint32_t gens, uint64_t plain_from) {
  // WIDE: the states move as 16-byte accesses (two adjacent columns per
  // lane, two universes per wave-instruction) staged through the wave's own
  // U x 512 B of LDS, which turns them into lane = column (and back for the
  // final states); the batch must be 16-byte aligned
  __shared__ uint64_t stage[WIDE || uses_lds(X) ? kWavesPerBlock * U * kWave : 1];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const W w = split(wanted[lane]), uw = split(unwanted[lane]);
  const bool rev = (gens & kReverse) != 0;
  const uint64_t blk = (gens & kXcdChunk) ? xcd_chunk_block() : (uint64_t)blockIdx.x;
  gens &= ~(kReverse | kXcdChunk);
  const uint64_t groups = (n + U - 1) / U, wstride = (uint64_t)gridDim.x * kWavesPerBlock;
  uint64_t *st_w = stage + (WIDE || uses_lds(X) ? wib * U * kWave : 0);
  const int half = lane >> 5, col = (lane & 31) * 2;
  static_assert(!(PF && WIDE), "the prefetching loop is the 8-byte form's");
  W an[U];
  auto load_group = [&](uint64_t g, W (&dst)[U]) __attribute__((always_inline)) {
    const uint64_t v0 = (rev ? groups - 1 - g : g) * U;
#pragma unroll
    for (int k = 0; k < U; ++k) dst[k] = (v0 + k < n) ? ld<true>(in + (v0 + k) * kWave + lane) : W{0u, 0u};
  };
  if constexpr (PF) {
    const uint64_t g0 = blk * kWavesPerBlock + wib;
    if (g0 < groups) load_group(g0, an);
  }
  for (uint64_t grp = blk * kWavesPerBlock + wib; grp < groups; grp += wstride) {
    const uint64_t u0 = (rev ? groups - 1 - grp : grp) * U;
    W a[U];
    if constexpr (PF) {
#pragma unroll
      for (int k = 0; k < U; ++k) a[k] = an[k];
      if (grp + wstride < groups) load_group(grp + wstride, an);
    } else if constexpr (WIDE) {
      static_assert(U % 2 == 0, "universes come in pairs");
      u64x2 v[U / 2];
#pragma unroll
      for (int k = 0; k < U / 2; ++k) {
        const uint64_t u = u0 + 2 * k + half;
        v[k] = u < n ? __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(in + u * kWave + col))
                     : u64x2{0ull, 0ull};
      }
#pragma unroll
      for (int k = 0; k < U / 2; ++k)
        *reinterpret_cast<u64x2 *>(st_w + (2 * k + half) * kWave + col) = v[k];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < U; ++k) a[k] = split(st_w[k * kWave + lane]);
      __builtin_amdgcn_wave_barrier();  // (the final states reuse the stage below)
    } else {
#pragma unroll
      for (int k = 0; k < U; ++k) a[k] = (u0 + k < n) ? ld<true>(in + (u0 + k) * kWave + lane) : W{0u, 0u};
    }
    uint32_t hit[U];
#pragma unroll
    for (int k = 0; k < U; ++k) hit[k] = 0;
    for (uint32_t g = 1; g <= gens; ++g) {
#pragma unroll
      for (int k = 0; k < U; ++k) {
        a[k] = life_gen<X, RULE>(a[k], uses_lds(X) ? st_w + k * kWave : nullptr, lane);
        if (hit[k] == 0 && wave_contains(a[k], w, uw)) hit[k] = g;
      }
    }
    if constexpr (WIDE) {
      if (fin) {
#pragma unroll
        for (int k = 0; k < U; ++k) st_w[k * kWave + lane] = join(a[k]);
        __builtin_amdgcn_wave_barrier();
        const bool nt = grp < plain_from;
#pragma unroll
        for (int k = 0; k < U / 2; ++k) {
          const uint64_t u = u0 + 2 * k + half;
          const u64x2 v = *reinterpret_cast<const u64x2 *>(st_w + (2 * k + half) * kWave + col);
          u64x2 *dst = reinterpret_cast<u64x2 *>(fin + u * kWave + col);
          if (u < n) {
            if (nt) __builtin_nontemporal_store(v, dst);
            else *dst = v;
          }
        }
        __builtin_amdgcn_wave_barrier();  // (the next group's loads reuse the stage)
      }
    } else if (fin && grp < plain_from) {
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (u0 + k < n) st<true>(fin + (u0 + k) * kWave + lane, a[k]);
    } else if (fin) {
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (u0 + k < n) st<false>(fin + (u0 + k) * kWave + lane, a[k]);
    }
    // lanes 0..U-1 write the U first-hit generations with one store
    uint32_t h = hit[0];
#pragma unroll
    for (int k = 1; k < U; ++k) h = lane == k ? hit[k] : h;
    if (lane < U && u0 + lane < n) first[u0 + lane] = h;
  }
}

// The same on the 8-way split layout (k_step_split): 4 universes per wave.
// The target is put into the same register layout once, replicated for the
// 4 universes; after every generation (r ^ w) & (w | u) is OR-ed over the
// registers and tested per universe (its bits are every P-th).
// Without d_final, a wave of the compiled loop stops once all its universes
// have hit.
constexpr uint32_t kDiff = ((TA ^ TB) & (TB | TC)) & 0xFF;  // (s ^ wanted) & (wanted | unwanted)
constexpr int kContainsNet = 6;  // tail network of the fused kernel (as k_step's default, rule 11)
// ASM selects the loop (times: config 3, 64K universes x 1024 generations,
// a block + ring target, against the plain step's 1.27-1.30 ms;
// profiles/r02/contains_ab*.jsonl):
//   0  the compiled loop below (a ballot per universe and generation)
//   1  the assembly loop of split_asm.inc with the test after every
//      generation: 8 differences, 3 OR3, per universe a masked OR + compare
//      and 8 SALU (1.760 ms)
//   2  1 with lean bookkeeping: two SALU per universe and generation, hits
//      on a slow path (1.668)
//   3  2 on the target's row window: every wave finds the smallest cyclic
//      window [y0, y0 + h) of rows that holds all of the target's care cells
//      (wanted | unwanted) and, when h <= 8, rotates the universes and the
//      target up by y0 rows (Life on the torus commutes with translation,
//      and so does Contains), so that the care rows are the split layout's
//      residues 0..h-1 and the test differences only h of the 8 registers;
//      d_final is rotated back (1.558-1.621; 78-87 VGPRs, 5-6 waves/SIMD)
//   4  3 with the scalar part after the plane-1 exchange (no gain)
//   5  3 with the test batched over eight generations for h <= 7: each
//      generation's OR of differences occupies bits 0..3 only, so it packs
//      into a nibble of one word, whose lane OR (DPP) and scalar test run
//      once per block (1.456; 92 VGPRs, 4 waves)
//   6  3 in the low register layout: a window of at most 4 rows, the target
//      in v52..v59 (1.563: the occupancy alone gains nothing)
//   7  5 in the low layout (1.397, +9.8 %: 64 VGPRs, 8 waves)
//   8  the rest of 5: windows of more than 4 rows (batched up to 7, the
//      per-generation test on 8 and on targets with no window)
// 6 and 7 do nothing for a window wider than 4 rows, 8 nothing for the
// others.  step.hip ships kContainsLo then kContainsHi: every wave of both
// finds the same window, so exactly one of them works and the other's waves
// return at once.  Each wave-uniform choice of loop runs its own copy of the
// pass over the universes (`universes` below), so the register allocator
// sees one assembly loop's pins at a time: 8 takes 70 VGPRs (7 waves per
// SIMD), where one shared pass took 84 (5), and 7 takes 62 (8 waves).
constexpr int kContainsLo = 7, kContainsHi = 8;
// 9: both in one kernel (each wave takes the loop its window calls for), so
// that one launch answers any target; the kernel takes kContainsHi's 72
// VGPRs (7 waves per SIMD), which costs the low layout nothing measurable
// (6 above: the low layout's occupancy alone gained nothing)
constexpr int kContainsAll = 9;
// (Measured, commit 5278498: targets with no row window of at most 7 rows
// batched over eight generations, each generation's differences folded onto
// a nibble, instead of the lean per-generation test -- no gain, 1M x 3-13
// generations within -2 .. +3 %, profiles/r06/batch_h8_ab/; the lean test
// stays.  tools/tune/split_asm_tune.inc keeps split_contains_asm_batch_h8.)
// the light-cone path of kContainsLo (cone_max below): universes per wave chunk
// (Measured in the compiler's allocation, not shipped: the whole board in the
// natural layout for wider cones at <= 4 generations -- 10-35 % faster there
// -- costs kContainsLo 7 VGPRs (62 -> 69, any register-set count) or
// kContainsHi 7 (70 -> 77), a wave per SIMD for every other target.)
// (16-universe chunks for cones of 9-32 columns: 6-8 % slower at 64K x 8-13
// generations, +4 % at 1M x 3, equal at 1M x 8-13; profiles/r04/r04ag)
constexpr int kConeLoUniverses = 8;
constexpr uint32_t kLowRows = 4;  // tools/gen_split_asm.py LOW_H

// (rotr64, care_window: device.hpp)
// The column window of a target's care cells, widened by the light cone of
// `gens` generations: xs = first column, K = columns (64: the whole board
// from column 0; also for gens >= 32, whatever the window).  The light-cone
// kernels (cone_kernels.hpp) load exactly these columns.
// care_col: this lane's column of care cells (wanted | unwanted).
__device__ __forceinline__ void cone_window(uint64_t care_col, uint32_t gens, uint32_t &xs, uint32_t &K) {
  const uint64_t cols = __ballot(care_col != 0ull);  // bit x: column x has care cells
  uint32_t x0, w;
  care_window(cols, x0, w);
  K = gens >= (uint32_t)kWave / 2 ? (uint32_t)kWave : w + 2 * gens;
  xs = (x0 - gens) & (kWave - 1);
  if (K >= (uint32_t)kWave) K = kWave, xs = 0;
}
// Whether the cyclic mask e holds a run of at least L (1 .. 64) set bits:
// runs of 2^k by doubling, then the binary digits of L (about 40 scalar
// instructions, no data-dependent selects).
__device__ __forceinline__ bool has_run(uint64_t e, uint32_t L) {
  if (L >= 64u) return e == ~0ull;
  uint64_t run[6];
  run[0] = e;
#pragma unroll
  for (int k = 1; k < 6; ++k) run[k] = run[k - 1] & rotr64(run[k - 1], 1u << (k - 1));
  uint64_t cur = ~0ull;
  uint32_t len = 0;
#pragma unroll
  for (int k = 5; k >= 0; --k)
    if ((L >> k) & 1u) cur &= rotr64(run[k], len), len += 1u << k;
  return cur != 0ull;
}
// Whether cone_window's K is 64 (the whole board from column 0): the care
// columns leave no cyclic run of 2 gens + 1 empty columns, or gens >= 32.
// The light-cone kernels ask this before the full window search, which a
// whole-board target then skips.
__device__ __forceinline__ bool cone_whole(uint64_t care_col, uint32_t gens) {
  return gens >= (uint32_t)kWave / 2 || !has_run(~__ballot(care_col != 0ull), 2u * gens + 1u);
}
// Whether cone_window's K is at most kmax, for 2 gens < kmax <= 64: the care
// columns then leave a cyclic run of at least L = 64 - kmax + 2 gens > 32
// empty columns -- tested directly (runs of 32 by doubling, then one shifted
// AND for the rest, about 25 scalar instructions against care_window's ~100;
// the split kernels' waves ask this on every launch of the iterated loop).
__device__ __forceinline__ bool cone_fits(uint64_t care_col, uint32_t gens, uint32_t kmax) {
  uint64_t run = ~__ballot(care_col != 0ull);  // bit p: column p empty
#pragma unroll
  for (int k = 0; k < 5; ++k) run &= rotr64(run, 1u << k);  // bit p: columns p .. p + 2^(k+1) - 1 empty
  return (run & rotr64(run, 64u - kmax + 2u * gens - 32u)) != 0ull;
}
__device__ __forceinline__ void cone_window(const uint64_t *__restrict__ wanted,
                                            const uint64_t *__restrict__ unwanted, uint32_t gens, int lane,
                                            uint32_t &xs, uint32_t &K) {
  cone_window(wanted[lane] | unwanted[lane], gens, xs, K);
}

// The row window of a filter's whole-board pass (cone_kernels.hpp
// cone_wave_rows_dma) and of the window split layout (cone_split.hpp): the
// smallest cyclic window of the target's care rows, widened by `gens` rows on
// either side, and the most universes per 32-bit word whose field holds it
// (PK = 4, 2, 1: fields of 8, 16, 32 rows); 0 when it needs more than 32 rows.
__device__ __forceinline__ int cone_rows(uint64_t care_col, uint32_t gens, uint32_t &y0) {
  const uint32_t lo = wave_or_u32_dpp((uint32_t)care_col), hi = wave_or_u32_dpp((uint32_t)(care_col >> 32));
  uint32_t cy0, h;
  care_window((uint64_t)lo | (uint64_t)hi << 32, cy0, h);
  if (gens >= 16u) return 0;
  const uint32_t need = h + 2u * gens;
  y0 = (cy0 - gens) & 63u;
  return need <= 8u ? 4 : need <= 16u ? 2 : need <= 32u ? 1 : 0;
}

// A column window (5-32 columns) takes the row window too from this many
// generations on (cone_wave_rows; below it the pass is not VALU-bound).
constexpr uint32_t kConeRowsWindowGens = 3;
// A whole board whose care rows fit a row window takes the LDS-DMA packed
// form (cone_wave_rows_dma) below this many generations, the
// window split layout (cone_split.hpp) from it on (one-row target, 1M
// universes: 3 / 5 generations 0.080 / 0.116 ms against 0.102 / 0.113 for
// the split window; 8 / 13: 0.203 / 0.289 against 0.199 / 0.279;
// profiles/r06/ab/)
constexpr uint32_t kConeWholeWinGens = 8;

// The light-cone pass (cone_kernels.hpp; here for the iterated search
// loop's low-layout kernel, below).  One wave's chunks of UPW universes u0 .. u0 + UPW - 1, u0 = u_first,
// u_first + u_step, ... (< n), under the window (xs = first loaded column,
// K <= P loaded columns).  FIRST: out[u] = the first
// generation in 1..gens whose state contains the target (0 = never), else
// out[u] = Contains(target) of the state as loaded (gens unused).  Register
// sets go RMAX at a time: all their loads are issued before the first test.
// PIPE: a pass issues the next pass's loads before it steps its own sets
// (twice the registers for the data; an A/B, tools/cone_ab.py).
template <int P, int UPW, int RMAX, bool FIRST, typename OutT, bool PIPE = false>
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
    auto load = [&](int pass, W (&a)[RB]) __attribute__((always_inline)) {
      const uint64_t ub = u0 + (uint64_t)pass * RB * GPS + q;
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const uint64_t u = ub + (uint64_t)k * GPS;
        a[k] = (live && u < n) ? ld<true>(in + u * kWave + col) : W{0u, 0u};
      }
    };
    W nx[RB];
    if constexpr (PIPE) load(0, nx);
#pragma unroll 1
    for (int pass = 0; pass < R / RB; ++pass) {
      W a[RB];
      if constexpr (PIPE) {
#pragma unroll
        for (int k = 0; k < RB; ++k) a[k] = nx[k];
        if (pass + 1 < R / RB) load(pass + 1, nx);
      } else {
        load(pass, a);
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

// cone_wave with the rows cut to the light cone too (the column window's
// counterpart of cone_kernels.hpp cone_wave_rows_dma): each lane's column is
// cut to rows y0 .. y0 + FW - 1 (FW = 32 / PK) by one v_alignbit (WRAP: the
// window crosses row 63), PK universes share one 32-bit register (universe
// field f in bits f FW ..), and the generation runs with 1-bit shifts for the
// vertical neighbours: the bits shifted in at a field's edges are wrong and
// move one row inwards per generation, never onto a care row, which lies at
// least `gens` rows inside its field (FIRST only; gens < 16).  Lanes as
// cone_wave: P per universe, GPS = 64 / P universes per register set, so one
// register holds PK GPS universes: register k, field f, group q is universe
// u0 + k PK GPS + f GPS + q.
template <int P, int UPW, int RMAX, int PK, bool WRAP, typename OutT>
__device__ __forceinline__ void cone_wave_rows(const uint64_t *in, const uint64_t *__restrict__ wanted,
                                               const uint64_t *__restrict__ unwanted, OutT *__restrict__ out,
                                               uint64_t n, uint64_t u_first, uint64_t u_step, uint32_t gens,
                                               uint32_t xs, uint32_t K, uint32_t y0, int lane) {
  constexpr int GPS = kWave / P, FW = 32 / PK, UPR = GPS * PK;
  static_assert(PK == 1 || PK == 2 || PK == 4, "fields of 32, 16 or 8 rows");
  static_assert(UPW % UPR == 0 && UPW <= kWave, "a wave takes whole registers, one result per lane");
  constexpr int R = UPW / UPR;
  constexpr int RB = R < RMAX ? R : RMAX;
  static_assert(R % RB == 0, "passes of RB registers");
  constexpr uint32_t fmask = FW == 32 ? ~0u : (1u << FW) - 1u;
  constexpr uint32_t rep = PK == 1 ? 1u : PK == 2 ? 0x00010001u : 0x01010101u;
  constexpr uint32_t kDiff = ((TA ^ TB) & TC) & 0xFF;  // (s ^ wanted) & care
  const uint32_t j = (uint32_t)lane & (P - 1), q = (uint32_t)lane / P;
  const uint32_t col = (xs + j) & (kWave - 1);
  const bool live = j < K;
  const uint32_t sh = y0 & 31u, gsh = q * P;
  auto cut = [&](uint64_t v) __attribute__((always_inline)) {
    const W w = split(v);
    return WRAP ? __builtin_amdgcn_alignbit(w.lo, w.hi, sh) : __builtin_amdgcn_alignbit(w.hi, w.lo, sh);
  };
  const uint64_t w64 = live ? wanted[col] : 0ull, m64 = live ? (w64 | unwanted[col]) : 0ull;
  const uint32_t tw = (cut(w64) & fmask) * rep, tm = (cut(m64) & fmask) * rep;
  for (uint64_t u0 = u_first; u0 < n; u0 += u_step) {
    uint32_t mine = 0;  // lane L: the result of universe u0 + L
#pragma unroll 1
    for (int pass = 0; pass < R / RB; ++pass) {
      const uint64_t ub = u0 + (uint64_t)pass * RB * UPR + q;
      uint32_t a[RB];
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        uint32_t e[PK];
#pragma unroll
        for (int f = 0; f < PK; ++f) {
          const uint64_t u = ub + (uint64_t)(k * UPR + f * GPS);
          e[f] = (live && u < n) ? cut(__builtin_nontemporal_load(in + u * kWave + col)) : 0u;
        }
        if constexpr (PK == 1) {
          a[k] = e[0];
        } else if constexpr (PK == 2) {
          a[k] = __builtin_amdgcn_perm(e[1], e[0], 0x05040100u);
        } else {
          const uint32_t p01 = __builtin_amdgcn_perm(e[1], e[0], 0x0C0C0400u);
          const uint32_t p23 = __builtin_amdgcn_perm(e[3], e[2], 0x0C0C0400u);
          a[k] = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
        }
      }
      uint32_t res[RB][PK];
#pragma unroll
      for (int k = 0; k < RB; ++k)
#pragma unroll
        for (int f = 0; f < PK; ++f) res[k][f] = 0;
      for (uint32_t g = 1; g <= gens; ++g) {
#pragma unroll
        for (int k = 0; k < RB; ++k) {
          const uint32_t L = dpp_prev(a[k]), Rt = dpp_next(a[k]);
          const uint32_t h0 = lut3<kXor3>(L, a[k], Rt), h1 = lut3<kMaj>(L, a[k], Rt);
          a[k] = life_tail6(h0 << 1, h0, h0 >> 1, h1 << 1, h1, h1 >> 1, a[k]);
          const uint32_t d = lut3<kDiff>(a[k], tw, tm);
#pragma unroll
          for (int f = 0; f < PK; ++f) {
            const uint64_t bad = __ballot((d & (fmask << (f * FW))) != 0u);
            bool clean;
            if constexpr (P == kWave) clean = bad == 0ull;
            else clean = ((bad >> gsh) & ((1ull << P) - 1)) == 0ull;
            if (res[k][f] == 0 && clean) res[k][f] = g;
          }
        }
      }
      // register k, field f, group q is universe u0 + (pass RB + k) UPR + f GPS + q:
      // its result (uniform over the group) moves to that lane
#pragma unroll
      for (int k = 0; k < RB; ++k)
#pragma unroll
        for (int f = 0; f < PK; ++f) {
          const uint32_t first = (uint32_t)((pass * RB + k) * UPR + f * GPS), rel = (uint32_t)lane - first;
          uint32_t v = res[k][f];
          if constexpr (GPS > 1) v = (uint32_t)__shfl((int)v, (int)((rel & (GPS - 1)) * P));
          if (rel < (uint32_t)GPS) mine = v;
        }
    }
    if (lane < UPW && u0 + lane < n) out[u0 + lane] = (OutT)mine;
  }
}

// cone_max: with no final states, a target whose light cone spans at most
// cone_max columns (0 = never) is answered on that cone: kContainsLo's waves
// step only those columns in the natural layout (cone_wave, 8 universes per
// wave chunk, looping over the batch), every other ASM's waves return at once.
// PF (16-byte aligned batch, no final states): the wave's next group of P
// universes is fetched into LDS by P / 2 sixteen-byte-per-lane
// global_load_lds (LDS-DMA: no VGPR destination, so the assembly loops keep
// their registers) as soon as the current group has been read out, and
// streams in while the current group steps; the generation loops' own LDS
// traffic is the exchange area, a different 2 KiB.
// WIN (no final states, 3 <= gens < 16): a target whose care rows, widened
// by the light cone, fit 32 rows (cone_rows) takes the window split layout
// (cone_split.hpp) on its column window -- or, on a whole board below
// kConeWholeWinGens generations, the packed LDS-DMA row pass.
template <int S, int NET, int ASM = 0, bool PF = false, bool WIN = false>
// (amdgpu_waves_per_eu(7): the shrinking window pass (cone_split.hpp) lifts
// the kernel's allocation 72 -> 76 VGPRs on its own, a wave per SIMD for
// every target; held at 72 it spills 12 bytes, reloaded once per chunk)
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(7))) void k_step_contains_split(const uint64_t *in, uint64_t *fin,
                                                                const uint64_t *__restrict__ wanted,
                                                                const uint64_t *__restrict__ unwanted,
                                                                uint32_t *__restrict__ first, uint64_t n,
                                                                uint32_t gens, uint32_t cone_max) {
  constexpr int P = S / 2;
  constexpr uint32_t every = P == 1 ? ~0u : P == 2 ? 0x55555555u : P == 4 ? 0x11111111u : 0x01010101u;
  // 4 KiB of LDS per wave: the exchange area of the generation loops
  // (S words per lane), then PF's fetch stage (P universes); the whole-board
  // row-window pass (WIN) takes all of it as its image (8 universes)
  static_assert(S * kWave * 4 + P * kWave * 8 <= 4096, "4 KiB per wave");
  __shared__ uint64_t wave_lds[kWavesPerBlock][512];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  uint32_t *const lds = reinterpret_cast<uint32_t *>(wave_lds[0]);  // (wave w's area: lds + w * 1024)
  // the target's care cells in this lane's column (both windows read it;
  // the cone test first: after the row window's, it costs kContainsHi 6
  // VGPRs, 70 -> 76)
  const uint64_t care_col = wanted[lane] | unwanted[lane];
  if constexpr (WIN) {
    if (!fin && gens >= kConeRowsWindowGens && gens < 16u) {
      uint32_t y0w = 0;
      const int pk = cone_rows(care_col, gens, y0w);
      if (pk > 0) {
        const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + wib, nw = (uint64_t)gridDim.x * kWavesPerBlock;
        uint32_t xs = 0, K = kWave;
        const bool whole = cone_whole(care_col, gens);
        if (!whole) cone_window(care_col, gens, xs, K);
        if constexpr (PF) {  // (a 16-byte aligned batch)
          if (whole && gens < kConeWholeWinGens) {
            // the whole board's row window below kConeWholeWinGens: the
            // packed LDS-DMA pass (cone_split.hpp cone_wave_rows_dma, chunks
            // of 16 universes, 8 per pass fetched while the last steps)
            const uint64_t w64 = wanted[lane], m64 = w64 | unwanted[lane];
            uint64_t *img = wave_lds[wib];
            auto rows = [&](auto pk_c, auto wrap_c) __attribute__((always_inline)) {
              cone_wave_rows_dma<8, decltype(pk_c)::value, decltype(wrap_c)::value>(
                  in, w64, m64, first, n, wave * 16, nw * 16, gens, y0w, lane, img, false);
            };
            using T = std::true_type;
            using F = std::false_type;
            using P1 = std::integral_constant<int, 1>;
            using P2 = std::integral_constant<int, 2>;
            using P4 = std::integral_constant<int, 4>;
            if (pk == 4) return y0w >= 32u ? rows(P4{}, T{}) : rows(P4{}, F{});
            if (pk == 2) return y0w >= 32u ? rows(P2{}, T{}) : rows(P2{}, F{});
            return y0w >= 32u ? rows(P1{}, T{}) : rows(P1{}, F{});
          }
        }
        return cone_split_pass(in, wanted, unwanted, first, n, wave, nw, gens, xs, K, pk, y0w, lane,
                               reinterpret_cast<uint32_t *>(wave_lds[wib]), PF);
      }
    }
  }
  // (2 gens in 64 bits: in 32 it wraps for gens >= 2^31)
  if (cone_max && cone_max <= 32u && !fin && 2ull * gens < cone_max && cone_fits(care_col, gens, cone_max)) {
    if constexpr (ASM == kContainsLo || ASM == kContainsAll) {
      uint32_t cxs, cK;
      cone_window(care_col, gens, cxs, cK);  // cK <= cone_max (cone_fits)
      {
        constexpr int U = kConeLoUniverses;
        const uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wib) * U,
                       step = (uint64_t)gridDim.x * kWavesPerBlock * U;
        if (cK <= 8) cone_wave<8, U, 8, true>(in, wanted, unwanted, first, n, u0, step, gens, cxs, cK, lane);
        else if (cK <= 16) cone_wave<16, U, 8, true>(in, wanted, unwanted, first, n, u0, step, gens, cxs, cK, lane);
        else cone_wave<32, U, 8, true>(in, wanted, unwanted, first, n, u0, step, gens, cxs, cK, lane);
      }
    }
    return;
  }
  uint32_t y0 = 0, h = S;  // the row window of ASM 3 (else: no rotation, all registers)
  if constexpr (ASM >= 3) {
    const uint32_t lo = wave_or_u32_dpp((uint32_t)care_col), hi = wave_or_u32_dpp((uint32_t)(care_col >> 32));
    care_window((uint64_t)lo | (uint64_t)hi << 32, y0, h);
    if (h > S) y0 = 0, h = S;
    if (ASM == 8 && h <= kLowRows) return;  // the low layout's target
  }
  if constexpr (ASM == 6 || ASM == 7) {
    if (h > kLowRows) return;  // the low layout: windows of <= 4 rows only (8 the rest)
  }
  uint32_t tw[S], tu[S];
  {
    W c[P];
#pragma unroll
    for (int u = 0; u < P; ++u) c[u] = split(rotr64(wanted[lane], y0));
    Split<S>::load(c, tw);
#pragma unroll
    for (int u = 0; u < P; ++u) c[u] = split(rotr64(unwanted[lane], y0));
    Split<S>::load(c, tu);
  }
  uint32_t tm[S];  // wanted | unwanted (the assembly loop's second target plane)
#pragma unroll
  for (int j = 0; j < S; ++j) tm[j] = tw[j] | tu[j];

  // one pass over this wave's groups of P universes with `gens_loop(r, hit)`
  // as the generation loop; every wave-uniform choice of loop (below) gets
  // its own copy of this pass, so that each assembly loop's pinned registers
  // are all the register allocator sees around it
  auto universes_pf = [&](auto &&gens_loop) __attribute__((always_inline)) {
    static_assert(P % 2 == 0, "pairs of universes per 16-byte load");
    uint64_t *img = wave_lds[wib] + S * kWave / 2;  // (after the exchange area)
    const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * P;
    auto fetch = [&](uint64_t ub) __attribute__((always_inline)) {
      const uint32_t ln = lane_id_fresh();
#pragma unroll
      for (int i = 0; i < P / 2; ++i) {
        uint64_t u = ub + 2 * i + (ln >> 5);
        if (u >= n) u = n - 1;  // (a valid address; its answer is not stored)
        const char *src = reinterpret_cast<const char *>(in + u * kWave) + (ln & 31) * 16;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                         (__attribute__((address_space(3))) void *)(img + i * 2 * kWave), 16, 0, 2);
      }
    };
    uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wib) * P;
    if (u0 >= n) return;
    fetch(u0);
    bool stored = false;  // an answer store was issued after the pending fetch
    for (; u0 < n; u0 += stride) {
      const uint64_t left = n - u0;
      const uint32_t avail = (left >> 2) ? (uint32_t)P : (uint32_t)left;
      // the fetch is the only older vector-memory op but the answer store
      // (in issue order: MI355X_MICROARCH.md, s_waitcnt vmcnt)
      if (stored) __builtin_amdgcn_s_waitcnt(kWaitVm1);
      else __builtin_amdgcn_s_waitcnt(kWaitVm0);
      uint32_t r[S];
      {
        // the P columns of this lane, read in one assembly block: a compiled
        // LDS read after an LDS-DMA makes the compiler wait for every
        // outstanding vector-memory op (vmcnt(0)), the last answer store
        // included; the counted wait above is the one this read needs
        static_assert(P == 4, "four universes per group");
        const uint32_t at = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)img +
                            lane_id_fresh() * 8u;
        uint64_t v0, v1, v2, v3;
        asm volatile(
            "ds_read_b64 %0, %4\n"
            "ds_read_b64 %1, %4 offset:512\n"
            "ds_read_b64 %2, %4 offset:1024\n"
            "ds_read_b64 %3, %4 offset:1536\n"
            "s_waitcnt lgkmcnt(0)\n"
            : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
            : "v"(at)
            : "memory");
        W c[P] = {split(v0), split(v1), split(v2), split(v3)};
        if (y0) {  // (wave-uniform)
#pragma unroll
          for (int u = 0; u < P; ++u) c[u] = split(rotr64(join(c[u]), y0));
        }
        if (u0 + stride < n) fetch(u0 + stride);  // (the stage is read out: the next group may land)
        Split<S>::load(c, r);
      }
      uint32_t hit[P];
#pragma unroll
      for (int u = 0; u < P; ++u) hit[u] = 0;
      gens_loop(r, hit);
      const uint32_t ln2 = lane_id_fresh();
      uint32_t h = hit[0];
#pragma unroll
      for (int u = 1; u < P; ++u) h = ln2 == (uint32_t)u ? hit[u] : h;
      if (ln2 < avail) first[u0 + ln2] = h;  // one store instruction
      stored = true;
    }
  };
  auto universes = [&](auto &&gens_loop) __attribute__((always_inline)) {
    if constexpr (PF) {
      if (!fin) return universes_pf(gens_loop);
    }
    const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * P;
    for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wib) * P; u0 < n; u0 += stride) {
      // the wave's universes u0 .. u0 + avail - 1 from scalar bases: a 64-bit
      // lane address or a vector copy of n kept across the loop would cost
      // VGPRs, and the low layout's occupancy hangs on the last four
      const uint64_t left = n - u0;
      const uint32_t avail = (left >> 2) ? (uint32_t)P : (uint32_t)left;
      const uint64_t *src = in + u0 * kWave;
      const uint32_t ln = lane_id_fresh();
      uint32_t r[S];
      W c[P];
#pragma unroll
      for (int u = 0; u < P; ++u) c[u] = (uint32_t)u < avail ? split(src[u * kWave + ln]) : W{0u, 0u};
      if (y0) {  // (wave-uniform: the row window's rotation, none for a window of 8 rows from row 0)
#pragma unroll
        for (int u = 0; u < P; ++u) c[u] = split(rotr64(join(c[u]), y0));
      }
      Split<S>::load(c, r);
      uint32_t hit[P];
#pragma unroll
      for (int u = 0; u < P; ++u) hit[u] = 0;
      gens_loop(r, hit);
      const uint32_t ln2 = lane_id_fresh();  // not kept live across the loop
      if (fin) {
        Split<S>::store(r, c);
        uint64_t *dst = fin + u0 * kWave;
#pragma unroll
        for (int u = 0; u < P; ++u)
          if ((uint32_t)u < avail) dst[u * kWave + ln2] = y0 ? rotr64(join(c[u]), 64 - y0) : join(c[u]);
      }
      if (ln2 == 0) {
#pragma unroll
        for (int u = 0; u < P; ++u)
          if ((uint32_t)u < avail) first[u0 + u] = hit[u];
      }
    }
  };
  if constexpr (ASM) {  // split_asm.inc: the default generation loop with the test fused in
    static_assert(S == 8 && NET == 6 && P == 4, "split_contains_asm is rule 11");
    const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)(lds + wib * 1024);
    const uint32_t self = base + lane * 16u, prev = base + ((lane + kWave - 1) & (kWave - 1)) * 16u,
                   next = base + ((lane + 1) & (kWave - 1)) * 16u;
#define LIFEAPI_RUN(fn)                                                                          \
  universes([&](uint32_t(&r)[S], uint32_t(&hit)[P]) __attribute__((always_inline)) {            \
    fn(r, tw, tm, gens, self, prev, next, hit);                                                  \
  })
#define LIFEAPI_BY_H(pre, wide)                                                                  \
  switch (h) { /* wave-uniform */                                                                \
    case 1: LIFEAPI_RUN(pre##1); break;                                                          \
    case 2: LIFEAPI_RUN(pre##2); break;                                                          \
    case 3: LIFEAPI_RUN(pre##3); break;                                                          \
    case 4: LIFEAPI_RUN(pre##4); break;                                                          \
    case 5: LIFEAPI_RUN(pre##5); break;                                                          \
    case 6: LIFEAPI_RUN(pre##6); break;                                                          \
    case 7: LIFEAPI_RUN(pre##7); break;                                                          \
    default: LIFEAPI_RUN(wide); break;                                                           \
  }
    if constexpr (ASM == 2) {
      LIFEAPI_RUN(split_contains_asm_lean);
    } else if constexpr (ASM == 8) {
      if (h == 5) LIFEAPI_RUN(split_contains_asm_batch_h5);
      else if (h == 6) LIFEAPI_RUN(split_contains_asm_batch_h6);
      else if (h == 7) LIFEAPI_RUN(split_contains_asm_batch_h7);
      else LIFEAPI_RUN(split_contains_asm_lean);
    } else if constexpr (ASM == kContainsAll) {
      if (h <= kLowRows) LIFEAPI_RUN(split_contains_asm_batch_lo);
      else if (h == 5) LIFEAPI_RUN(split_contains_asm_batch_h5);
      else if (h == 6) LIFEAPI_RUN(split_contains_asm_batch_h6);
      else if (h == 7) LIFEAPI_RUN(split_contains_asm_batch_h7);
      else LIFEAPI_RUN(split_contains_asm_lean);
    } else if constexpr (ASM == 7) {
      LIFEAPI_RUN(split_contains_asm_batch_lo);
    } else if constexpr (ASM == 6) {
      LIFEAPI_RUN(split_contains_asm_lean_lo);
    } else if constexpr (ASM == 5) {
      LIFEAPI_BY_H(split_contains_asm_batch_h, split_contains_asm_lean)
    } else if constexpr (ASM == 4) {
      LIFEAPI_BY_H(split_contains_asm_lean_late_h, split_contains_asm_lean_late)
    } else if constexpr (ASM == 3) {
      LIFEAPI_BY_H(split_contains_asm_lean_h, split_contains_asm_lean)
    } else {
      LIFEAPI_RUN(split_contains_asm);
    }
#undef LIFEAPI_BY_H
#undef LIFEAPI_RUN
  } else {
    universes([&](uint32_t(&r)[S], uint32_t(&hit)[P]) __attribute__((always_inline)) {
      uint32_t found = 0;
      for (uint32_t g = 1; g <= gens; ++g) {
        gen_split<S, NET>(r, lds + wib * 1024, lane);
        uint32_t d = 0;
#pragma unroll
        for (int j = 0; j < S; ++j) d |= lut3<kDiff>(r[j], tw[j], tu[j]);
        // straight-line: a ballot per universe, the bookkeeping in scalar registers
        uint32_t clean = 0;
#pragma unroll
        for (int u = 0; u < P; ++u) clean |= (__ballot((d & (every << u)) != 0) == 0 ? 1u : 0u) << u;
        const uint32_t fresh = clean & ~found;
#pragma unroll
        for (int u = 0; u < P; ++u) hit[u] = (fresh >> u) & 1 ? g : hit[u];
        found |= fresh;
        if (!fin && found == (1u << P) - 1) break;
      }
    });
  }
}


}  // namespace
}  // namespace lifeapi_impl
