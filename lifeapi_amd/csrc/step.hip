// step.hip -- batched LifeState::Step() (LifeAPI.hpp:1196-1216, Stepped(n)
// :877-886) and the fused Step + Contains (LifeTarget.hpp:44-51): the
// generation networks, k_step / k_step_split and their launch configuration.
#include <algorithm>

#include "host.hpp"
#include "split_layout.hpp"
#include "tile_asm.inc"
#include "split_asm.inc"

using namespace lifeapi_impl;

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
  if constexpr (RULE == 2) {
    // Row-first form of the same adder network.  A DPP move issues at half
    // the VALU rate on gfx950 (tools/valu_probe.hip: 8 DPP of 32 instructions
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

// `gens` generations of one universe in the (E, O) layout (RULE 4), as one
// hand-allocated loop.  The compiler's allocation puts two or three sources
// of about half of the v_bitop3 in one VGPR bank (tools/vbank.py), and such an
// instruction issues at half rate (tools/bank_probe.hip).  Here every VALU
// instruction reads its sources from distinct banks (bank = vN mod 4):
//   A = (E, O) v0:v1 (banks 0,1)   R = right column v2:v3 (2,3)
//   L = left column v5 (E, bank 1), v4 (O, bank 0)
// The exchange goes through this wave's 512-B LDS slot (ds_write_b64 of A,
// ds_read_b64 of the right neighbour's word, two ds_read_b32 of the left
// one); a wave's LDS operations complete in order and each generation waits
// for its reads before the next write.  Network: life_gen<_, 4>.
__device__ __forceinline__ void gens_asm(W &a, uint32_t gens, uint32_t lds_self, uint32_t lds_prev,
                                         uint32_t lds_next) {
  asm volatile(
      "v_mov_b32 v0, %[e]\n"
      "v_mov_b32 v1, %[o]\n"
      "s_cmp_eq_u32 %[g], 0\n"
      "s_cbranch_scc1 2f\n"
      "1:\n"
      "ds_write_b64 %[as], v[0:1]\n"
      "ds_read_b64 v[2:3], %[an]\n"
      "ds_read_b32 v5, %[ap]\n"
      "ds_read_b32 v4, %[ap] offset:4\n"
      "s_sub_u32 %[g], %[g], 1\n"
      "s_waitcnt lgkmcnt(0)\n"
      "v_bitop3_b32 v8, v5, v0, v2 bitop3:0x96\n"      // h0 E = xor3(L, A, R)
      "v_bitop3_b32 v9, v4, v1, v3 bitop3:0x96\n"      // h0 O
      "v_bitop3_b32 v10, v5, v0, v2 bitop3:0xe8\n"     // h1 E = maj(L, A, R)
      "v_bitop3_b32 v11, v4, v1, v3 bitop3:0xe8\n"     // h1 O
      "v_alignbit_b32 v6, v9, v9, 31\n"                // u0 = rotl1(h0 O): row 2k-1
      "v_alignbit_b32 v14, v8, v8, 1\n"                // d0 = rotr1(h0 E): row 2k+2
      "v_alignbit_b32 v12, v11, v11, 31\n"             // u1
      "v_alignbit_b32 v16, v10, v10, 1\n"              // d1
      "v_bitop3_b32 v13, v6, v8, v9 bitop3:0x17\n"     // s0 E = SA <= 1
      "v_bitop3_b32 v18, v6, v8, v9 bitop3:0x7e\n"     // s1 E = SA in {1,2}
      "v_bitop3_b32 v20, v8, v9, v14 bitop3:0x17\n"    // s0 O
      "v_bitop3_b32 v22, v8, v9, v14 bitop3:0x7e\n"    // s1 O
      "v_bitop3_b32 v17, v12, v10, v11 bitop3:0x17\n"  // s2 E = SB <= 1
      "v_bitop3_b32 v24, v12, v10, v11 bitop3:0x69\n"  // s3 E = SB in {0,2}
      "v_bitop3_b32 v28, v10, v11, v16 bitop3:0x17\n"  // s2 O
      "v_bitop3_b32 v21, v10, v11, v16 bitop3:0x69\n"  // s3 O
      "v_bitop3_b32 v15, v13, v18, v0 bitop3:0x34\n"   // t1 E = T1(s0, s1, a)
      "v_bitop3_b32 v19, v20, v22, v1 bitop3:0x34\n"   // t1 O
      "v_bitop3_b32 v25, v17, v0, v15 bitop3:0x58\n"   // t2 E = T2(s2, a, t1)
      "v_bitop3_b32 v23, v28, v1, v19 bitop3:0x58\n"   // t2 O
      "v_bitop3_b32 v0, v18, v24, v25 bitop3:0x28\n"   // a E = T3(s1, s3, t2)
      "v_bitop3_b32 v1, v22, v21, v23 bitop3:0x28\n"   // a O
      "s_cmp_lg_u32 %[g], 0\n"
      "s_cbranch_scc1 1b\n"
      "2:\n"
      "v_mov_b32 %[e], v0\n"
      "v_mov_b32 %[o], v1\n"
      : [e] "+v"(a.lo), [o] "+v"(a.hi), [g] "+s"(gens)
      : [as] "v"(lds_self), [ap] "v"(lds_prev), [an] "v"(lds_next)
      : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v8", "v9", "v10", "v11", "v12", "v13", "v14",
        "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v28", "scc",
        "memory");
  static_assert(kT1 == 0x34 && kT2 == 0x58 && kT3 == 0x28 && kLe1 == 0x17 && kNae == 0x7E &&
                    kEven == 0x69 && kXor3 == 0x96 && kMaj == 0xE8,
                "gens_asm spells out the RULE 4 tables");
}

// out[u] = in[u] stepped `gens` times.  Wave w of the grid takes groups of U
// consecutive universes, grid-strided.  All branches are wave-uniform.
template <int X, int U, bool NT, int RULE>
__global__ __launch_bounds__(kBlock) void k_step(const uint64_t *__restrict__ in,
                                                 uint64_t *__restrict__ out, uint64_t n,
                                                 uint32_t gens) {
  __shared__ uint64_t lds[uses_lds(X) ? kWavesPerBlock * U * 2 * kWave : 1];
  const int lane = threadIdx.x & (kWave - 1);
  // wave index in the block, made provably wave-uniform so that the tail
  // tests below are scalar branches
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * U;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wib) * U; u0 < n; u0 += stride) {
    W a[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      a[k] = (u0 + k < n) ? ld<NT>(in + (u0 + k) * kWave + lane) : W{0u, 0u};
    if constexpr (RULE == 4) {
#pragma unroll
      for (int k = 0; k < U; ++k) a[k] = to_eo(a[k]);
    }
    if constexpr (X == XASM) {
      static_assert(RULE == 4, "the hand-allocated loop is the RULE 4 network");
#pragma unroll
      for (int k = 0; k < U; ++k) {
        // LDS byte addresses of this wave's slot: own word, left and right neighbours
        const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)(
            lds + (wib * U + k) * 2 * kWave);
        gens_asm(a[k], gens, base + lane * 8u, base + ((lane + kWave - 1) & (kWave - 1)) * 8u,
                 base + ((lane + 1) & (kWave - 1)) * 8u);
      }
    } else {
      for (uint32_t g = 0; g < gens; ++g) {
#pragma unroll
        for (int k = 0; k < U; ++k)
          a[k] = life_gen<X, RULE>(a[k], lds + (wib * U + k) * 2 * kWave, lane);
      }
    }
    if constexpr (RULE == 4) {
#pragma unroll
      for (int k = 0; k < U; ++k) a[k] = from_eo(a[k]);
    }
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (u0 + k < n) st<NT>(out + (u0 + k) * kWave + lane, a[k]);
  }
}

// k_step for the split layouts: wave w takes G groups of P = S/2
// consecutive universes, grid-strided; all branches wave-uniform.  NET: the
// tail network (7 = RULE 3's, 6 = life_tail6); D: registers exchanged by DPP
// instead of LDS (gen_split), or kPipe: the software-pipelined LDS loop
// (gens_split_pipe).
constexpr int kPipe = -1;
constexpr int kAsmLoop = -3;  // the hand-allocated rule-11 loop (split_asm.inc)
template <int S, int G, bool NT, int NET, int D = 0, int V = 0>
__global__ __launch_bounds__(kBlock) void k_step_split(const uint64_t *__restrict__ in,
                                                       uint64_t *__restrict__ out, uint64_t n,
                                                       uint32_t gens) {
  constexpr int P = S / 2;
  __shared__ uint32_t lds[kWavesPerBlock * G * S * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t per_wave = (uint64_t)G * P;
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * per_wave;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wib) * per_wave; u0 < n; u0 += stride) {
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

// k_step for the tile layouts (gen_tile): a wave holds C groups of P = S/2
// universes, lane i of group g columns C*i .. C*i+C-1 of each (C*8
// contiguous bytes per universe: two dwordx4 loads for C = 4).
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ u64x2 ld2(const uint64_t *p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(p));
  else return *reinterpret_cast<const u64x2 *>(p);
}
template <bool NT>
__device__ __forceinline__ void st2(uint64_t *p, u64x2 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u64x2 *>(p));
  else *reinterpret_cast<u64x2 *>(p) = v;
}

template <int S, int C, int X, bool NT, int NET>
__global__ __launch_bounds__(kBlock) void k_step_tile(const uint64_t *__restrict__ in,
                                                      uint64_t *__restrict__ out, uint64_t n,
                                                      uint32_t gens) {
  constexpr int P = S / 2, LPG = kWave / C;
  static_assert(C % 2 == 0, "columns are moved in pairs");
  __shared__ uint32_t lds[X == XDPP ? 1 : kWavesPerBlock * 2 * S * kWave];  // 4 planes of 1 KiB per wave (S = 8)
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int grp = lane / LPG, col0 = (lane & (LPG - 1)) * C;
  const uint64_t per_wave = (uint64_t)C * P;
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * per_wave;
  uint32_t *slot = lds + (X == XDPP ? 0 : wib * 2 * S * kWave);
  // per-lane offsets stay 32-bit and the tile's base pointer wave-uniform, so
  // little beyond the state is live across the generation loop
  const uint32_t lane_off = (uint32_t)(grp * P * kWave + col0);
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wib) * per_wave; u0 < n; u0 += stride) {
    const uint64_t left = n - u0;  // universes from u0 on (wave-uniform)
    const uint64_t *src = in + u0 * kWave;
    uint32_t off = lane_off, first = (uint32_t)(grp * P);
    // opaque to the optimiser: keeps it from hoisting 64-bit copies of the
    // lane offsets out of the loop (they would stay live across the generations)
    asm volatile("" : "+v"(off), "+v"(first));
    const uint32_t room = left < per_wave ? (uint32_t)left : (uint32_t)per_wave;
    uint32_t r[C][S];
    {
      uint64_t w[P][C];
#pragma unroll
      for (int u = 0; u < P; ++u) {
        const bool ok = first + u < room;
#pragma unroll
        for (int c = 0; c < C; c += 2) {
          const u64x2 v = ok ? ld2<NT>(src + off + u * kWave + c) : u64x2{0, 0};
          w[u][c] = v[0], w[u][c + 1] = v[1];
        }
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        W cc[P];
#pragma unroll
        for (int u = 0; u < P; ++u) cc[u] = split(w[u][c]);
        Split<S>::load(cc, r[c]);
      }
    }
    if constexpr (X == XASM) {
      static_assert(S == 8 && C == 4, "tile_asm.inc is the 8-way split, 4 columns per lane");
      const uint32_t base =
          (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)slot;
      const int g0 = lane & ~(LPG - 1);
      tile_gens_asm(r, gens, base + lane * 16u, base + (g0 | ((lane + LPG - 1) & (LPG - 1))) * 16u,
                    base + (g0 | ((lane + 1) & (LPG - 1))) * 16u);
    } else {
      for (uint32_t it = 0; it < gens; ++it) gen_tile<S, C, X, NET>(r, slot, lane);
    }
    asm volatile("" : "+v"(off), "+v"(first));  // (store addresses: recomputed here)
    uint64_t w[P][C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      W cc[P];
      Split<S>::store(r[c], cc);
#pragma unroll
      for (int u = 0; u < P; ++u) w[u][c] = join(cc[u]);
    }
    uint64_t *dst = out + u0 * kWave;
#pragma unroll
    for (int u = 0; u < P; ++u) {
      if (first + u < room) {
#pragma unroll
        for (int c = 0; c < C; c += 2) st2<NT>(dst + off + u * kWave + c, u64x2{w[u][c], w[u][c + 1]});
      }
    }
  }
}

// Step + Contains fused: first generation in 1..gens whose state contains the
// target (0 = never); the state keeps stepping to `gens` for d_final.
__global__ __launch_bounds__(kBlock) void k_step_contains(const uint64_t *__restrict__ in,
                                                          uint64_t *__restrict__ fin,
                                                          const uint64_t *__restrict__ wanted,
                                                          const uint64_t *__restrict__ unwanted,
                                                          uint32_t *__restrict__ first,
                                                          uint64_t n, uint32_t gens) {
  const int lane = threadIdx.x & (kWave - 1);
  const W w = split(wanted[lane]), uw = split(unwanted[lane]);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t u = (uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave; u < n; u += stride) {
    W a = split(in[u * kWave + lane]);
    uint32_t hit = 0;
    for (uint32_t g = 1; g <= gens; ++g) {
      a = life_gen<XDPP, 3>(a, nullptr, lane);
      if (hit == 0 && wave_contains(a, w, uw)) hit = g;
    }
    if (fin) fin[u * kWave + lane] = join(a);
    if (lane == 0) first[u] = hit;
  }
}

// The same on the 8-way split layout (k_step_split): 4 universes per wave.
// The target is put into the same register layout once, replicated for the
// 4 universes; after every generation (r ^ w) & (w | u) is OR-ed over the
// registers and one ballot per universe (its bits are every P-th) tests it,
// with no branch per universe.  The check costs about 5 VALU per
// universe-generation on top of the 18 of the step (+20-25 % measured,
// profiles/r01/contains_bench.jsonl); branching around the bookkeeping
// when no universe is clean measured slower still.
// Without d_final, a wave stops once all its universes have hit.
constexpr uint32_t kDiff = ((TA ^ TB) & (TB | TC)) & 0xFF;  // (s ^ wanted) & (wanted | unwanted)
constexpr int kContainsNet = 6;  // tail network of the fused kernel (as k_step's default, rule 11)
// the fused kernel runs the assembly loop of split_asm.inc (split_contains_asm)
// for gens > 2; the compiled loop above stays for comparison
constexpr bool kContainsAsm = true;
template <int S, int NET, bool ASM = false>
__global__ __launch_bounds__(kBlock) void k_step_contains_split(const uint64_t *__restrict__ in,
                                                                uint64_t *__restrict__ fin,
                                                                const uint64_t *__restrict__ wanted,
                                                                const uint64_t *__restrict__ unwanted,
                                                                uint32_t *__restrict__ first, uint64_t n,
                                                                uint32_t gens) {
  constexpr int P = S / 2;
  constexpr uint32_t every = P == 1 ? ~0u : P == 2 ? 0x55555555u : P == 4 ? 0x11111111u : 0x01010101u;
  __shared__ uint32_t lds[kWavesPerBlock * S * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  uint32_t tw[S], tu[S];
  {
    W c[P];
#pragma unroll
    for (int u = 0; u < P; ++u) c[u] = split(wanted[lane]);
    Split<S>::load(c, tw);
#pragma unroll
    for (int u = 0; u < P; ++u) c[u] = split(unwanted[lane]);
    Split<S>::load(c, tu);
  }
  uint32_t tm[S];  // wanted | unwanted (the assembly loop's second target plane)
#pragma unroll
  for (int j = 0; j < S; ++j) tm[j] = tw[j] | tu[j];

  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * P;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wib) * P; u0 < n; u0 += stride) {
    uint32_t r[S];
    W c[P];
#pragma unroll
    for (int u = 0; u < P; ++u) c[u] = u0 + u < n ? split(in[(u0 + u) * kWave + lane]) : W{0u, 0u};
    Split<S>::load(c, r);
    uint32_t hit[P];
#pragma unroll
    for (int u = 0; u < P; ++u) hit[u] = 0;
    uint32_t found = 0;
    if constexpr (ASM) {  // split_asm.inc: the default generation loop with the test fused in
      static_assert(S == 8 && NET == 6, "split_contains_asm is rule 11");
      const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)(
          lds + wib * S * kWave);
      split_contains_asm(r, tw, tm, gens, base + lane * 16u, base + ((lane + kWave - 1) & (kWave - 1)) * 16u,
                         base + ((lane + 1) & (kWave - 1)) * 16u, hit);
    } else for (uint32_t g = 1; g <= gens; ++g) {
      gen_split<S, NET>(r, lds + wib * S * kWave, lane);
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
    if (fin) {
      Split<S>::store(r, c);
#pragma unroll
      for (int u = 0; u < P; ++u)
        if (u0 + u < n) fin[(u0 + u) * kWave + lane] = join(c[u]);
    }
    if (lane == 0) {
#pragma unroll
      for (int u = 0; u < P; ++u)
        if (u0 + u < n) first[u0 + u] = hit[u];
    }
  }
}

using StepFn = void (*)(const uint64_t *, uint64_t *, uint64_t, uint32_t);

template <int X, int U, bool NT, int RULE>
constexpr StepFn step_ptr() { return k_step<X, U, NT, RULE>; }

template <int X, bool NT, int RULE>
StepFn pick_u(int u) {
  switch (u) {
    case 1: return step_ptr<X, 1, NT, RULE>();
    case 2: return step_ptr<X, 2, NT, RULE>();
    case 4: return step_ptr<X, 4, NT, RULE>();
    case 8: return step_ptr<X, 8, NT, RULE>();
    default: return nullptr;
  }
}
template <int X, int RULE>
StepFn pick_nt(int u, bool nt) { return nt ? pick_u<X, true, RULE>(u) : pick_u<X, false, RULE>(u); }
template <int X>
StepFn pick_rule(int u, bool nt, int rule) {
  if constexpr (X == XASM) {
    return rule == 4 ? pick_nt<X, 4>(u, nt) : nullptr;
  } else {
    switch (rule) {
      case 0: return pick_nt<X, 0>(u, nt);
      case 1: return pick_nt<X, 1>(u, nt);
      case 2: return pick_nt<X, 2>(u, nt);
      case 3: return pick_nt<X, 3>(u, nt);
      case 4: return pick_nt<X, 4>(u, nt);
      default: return nullptr;
    }
  }
}
template <int S, int NET, int D = 0, int V = 0>
StepFn pick_split(int groups, bool nt) {
  switch (groups) {
    case 1: return nt ? k_step_split<S, 1, true, NET, D, V> : k_step_split<S, 1, false, NET, D, V>;
    case 2: return nt ? k_step_split<S, 2, true, NET, D, V> : k_step_split<S, 2, false, NET, D, V>;
    default: return nullptr;
  }
}
// universes one wave holds per universes_per_wave unit (rules 5-7, 10-12:
// groups; rules 8, 9, 13: one tile of C groups)
int group_size(int rule) {
  switch (rule) {
    case 5: case 10: return 2;
    case 6: case 11: return 4;
    case 7: case 12: return 8;
    case 8: case 13: return 16;
    case 9: return 8;
    default: return 1;
  }
}

template <int NET>
StepFn pick_tile4(int xchg, bool nt) {
  if (xchg == LIFEAPI_XCHG_LDS) return nt ? k_step_tile<8, 4, XLDS, true, NET> : k_step_tile<8, 4, XLDS, false, NET>;
  if (xchg == LIFEAPI_XCHG_DPP) return nt ? k_step_tile<8, 4, XDPP, true, NET> : k_step_tile<8, 4, XDPP, false, NET>;
  return nullptr;
}

StepFn pick_step(const lifeapi_launch_cfg &c) {
  if (c.rule == 8 || c.rule == 9 || c.rule == 13) {  // tile layouts: one tile per wave
    if (c.universes_per_wave != 1) return nullptr;
    const bool nt = c.nontemporal != 0;
    if (c.rule == 9)
      return c.xchg == LIFEAPI_XCHG_LDS ? (nt ? k_step_tile<8, 2, XLDS, true, 7> : k_step_tile<8, 2, XLDS, false, 7>)
                                        : nullptr;
    if (c.rule == 13) return pick_tile4<6>(c.xchg, nt);
    if (c.xchg == LIFEAPI_XCHG_ASM) return nt ? k_step_tile<8, 4, XASM, true, 7> : k_step_tile<8, 4, XASM, false, 7>;
    return pick_tile4<7>(c.xchg, nt);
  }
  if ((c.rule >= 5 && c.rule <= 7) || (c.rule >= 10 && c.rule <= 12)) {  // split layouts
    const bool nt = c.nontemporal != 0;
    if (c.xchg == LIFEAPI_XCHG_ASM) {
      return c.rule == 11 ? pick_split<8, 6, kAsmLoop>(c.universes_per_wave, nt) : nullptr;
    }
    if (c.xchg > LIFEAPI_XCHG_ASM_V(0) && c.xchg <= LIFEAPI_XCHG_ASM_V(3) && c.rule == 11 &&
        c.universes_per_wave == 1) {  // the other schedules of the assembly loop
      switch (c.xchg - LIFEAPI_XCHG_ASM_V(0)) {
        case 1: return pick_split<8, 6, kAsmLoop, 1>(1, nt);
        case 2: return pick_split<8, 6, kAsmLoop, 2>(1, nt);
        default: return pick_split<8, 6, kAsmLoop, 3>(1, nt);
      }
    }
    if (c.xchg == LIFEAPI_XCHG_LDS_PIPE) {
      switch (c.rule) {
        case 6: return pick_split<8, 7, kPipe>(c.universes_per_wave, nt);
        case 11: return pick_split<8, 6, kPipe>(c.universes_per_wave, nt);
        case 12: return pick_split<16, 6, kPipe>(c.universes_per_wave, nt);
        default: return nullptr;
      }
    }
    if (c.xchg > LIFEAPI_XCHG_LDS_DPP(0) && (c.rule == 11 || c.rule == 12)) {
      // LDS for most registers, DPP for D of them
      const int d = c.xchg - LIFEAPI_XCHG_LDS_DPP(0);
      if (c.rule == 11) {
        switch (d) {
          case 1: return pick_split<8, 6, 1>(c.universes_per_wave, nt);
          case 2: return pick_split<8, 6, 2>(c.universes_per_wave, nt);
          case 3: return pick_split<8, 6, 3>(c.universes_per_wave, nt);
          case 4: return pick_split<8, 6, 4>(c.universes_per_wave, nt);
          default: return nullptr;
        }
      }
      switch (d) {
        case 2: return pick_split<16, 6, 2>(c.universes_per_wave, nt);
        case 4: return pick_split<16, 6, 4>(c.universes_per_wave, nt);
        default: return nullptr;
      }
    }
    if (c.xchg != LIFEAPI_XCHG_LDS) return nullptr;
    switch (c.rule) {
      case 5: return pick_split<4, 7>(c.universes_per_wave, nt);
      case 6: return pick_split<8, 7>(c.universes_per_wave, nt);
      case 7: return pick_split<16, 7>(c.universes_per_wave, nt);
      case 10: return pick_split<4, 6>(c.universes_per_wave, nt);
      case 11: return pick_split<8, 6>(c.universes_per_wave, nt);
      default: return pick_split<16, 6>(c.universes_per_wave, nt);
    }
  }
  switch (c.xchg) {
    case LIFEAPI_XCHG_DPP: return pick_rule<XDPP>(c.universes_per_wave, c.nontemporal != 0, c.rule);
    case LIFEAPI_XCHG_LDS: return pick_rule<XLDS>(c.universes_per_wave, c.nontemporal != 0, c.rule);
    case LIFEAPI_XCHG_BPERM: return pick_rule<XBPERM>(c.universes_per_wave, c.nontemporal != 0, c.rule);
    case LIFEAPI_XCHG_MIX: return pick_rule<XMIX>(c.universes_per_wave, c.nontemporal != 0, c.rule);
    case LIFEAPI_XCHG_MIX1: return pick_rule<XMIX1>(c.universes_per_wave, c.nontemporal != 0, c.rule);
    case LIFEAPI_XCHG_MIX3: return pick_rule<XMIX3>(c.universes_per_wave, c.nontemporal != 0, c.rule);
    case LIFEAPI_XCHG_LDSR: return pick_rule<XLDSR>(c.universes_per_wave, c.nontemporal != 0, c.rule);
    case LIFEAPI_XCHG_LDSR3: return pick_rule<XLDSR3>(c.universes_per_wave, c.nontemporal != 0, c.rule);
    case LIFEAPI_XCHG_ASM: return pick_rule<XASM>(c.universes_per_wave, c.nontemporal != 0, c.rule);
    default: return nullptr;
  }
}

}  // namespace

extern "C" {

void lifeapi_default_cfg(lifeapi_launch_cfg *cfg, uint32_t generations) {
  if (!cfg) return;
  // Measured on MI355X (profiles/r01/tune_c3x.jsonl, tune_gsweep.jsonl): a
  // one-shot grid (no grid-stride cap) beats every capped grid.
  cfg->blocks_per_cu = 0;
  if (generations <= 2) {
    // HBM-streaming regime: 4 x 512 B loads in flight per wave, DPP exchange,
    // the 7-LUT network on the natural layout (no layout change to pay for)
    cfg->xchg = LIFEAPI_XCHG_DPP;
    cfg->rule = 3;
    cfg->universes_per_wave = 4;
    cfg->nontemporal = 1;
  } else {
    // VALU regime: 8-way row split, 4 universes per wave interleaved bit by
    // bit, LDS exchange, the 6-LUT tail; state resident in VGPRs for all
    // generations (rule 11 over rule 6: 1.47 vs 1.61 ms on config 3,
    // profiles/r01/tune_c3net.jsonl), as the hand-allocated loop of
    // split_asm.inc (2-2.5 % over the compiled one, tune_c3asm.jsonl)
    cfg->xchg = LIFEAPI_XCHG_ASM;
    cfg->rule = 11;
    cfg->universes_per_wave = 1;
    cfg->nontemporal = generations < 32 ? 1 : 0;
  }
}

int lifeapi_step_batch_dev_cfg(const uint64_t *d_in, uint64_t *d_out, size_t n,
                               uint32_t generations, void *stream,
                               const lifeapi_launch_cfg *cfg) {
  int rc = check_batch(d_in, d_out, n);
  if (rc != LIFEAPI_OK || n == 0) return rc;
  lifeapi_launch_cfg c;
  if (cfg) c = *cfg;
  else lifeapi_default_cfg(&c, generations);
  StepFn fn = pick_step(c);
  if (!fn) return fail(LIFEAPI_E_INVALID, "unsupported launch cfg%s");
  int cus = 0;
  rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const uint64_t per_wave = (uint64_t)c.universes_per_wave * group_size(c.rule);
  const uint64_t waves = (n + per_wave - 1) / per_wave;
  const unsigned grid = grid_for(waves, cus, c.blocks_per_cu);
  hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, d_in, d_out,
                     (uint64_t)n, generations);
  return launched("k_step launch");
}

int lifeapi_step_batch_dev(const uint64_t *d_in, uint64_t *d_out, size_t n,
                           uint32_t generations, void *stream) {
  return lifeapi_step_batch_dev_cfg(d_in, d_out, n, generations, stream, nullptr);
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
  if (generations > 2) {  // the default layout of k_step for gens > 2 (lifeapi_default_cfg)
    hipLaunchKernelGGL((k_step_contains_split<8, kContainsNet, kContainsAsm>), dim3(grid_for((n + 3) / 4, cus, 0)), dim3(kBlock), 0,
                       (hipStream_t)stream, d_in, d_final, d_wanted, d_unwanted, d_first_gen,
                       (uint64_t)n, generations);
  } else {
    hipLaunchKernelGGL(k_step_contains, dim3(grid_for(n, cus, 0)), dim3(kBlock), 0,
                       (hipStream_t)stream, d_in, d_final, d_wanted, d_unwanted, d_first_gen,
                       (uint64_t)n, generations);
  }
  return launched("k_step_contains launch");
}

}  // extern "C"
