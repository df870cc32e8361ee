// tune_step.hip -- the TUNING build of batched Step(): every measured
// alternative to the shipped kernels (other rule networks, exchanges,
// layouts, tiles and assembly-loop schedules), selectable per launch by
// lifeapi_launch_cfg (lifeapi_tune.h).  Built into tools/tune/
// liblifeapi_tune.so by __graft_entry__.build_tools(); used by
// tools/ab/tune.py and the ablation parity tests (tests/test_tune_parity.py).
// Not part of the product library or its header: the shipped
// configurations are fixed in lifeapi_amd/csrc/step.hip.
#include <algorithm>

#include "lifeapi_tune.h"
#include "step_kernels.hpp"
#include "split_asm_tune.inc"
#include "tile_asm.inc"
#include "pair_asm.inc"

using namespace lifeapi_impl;

static_assert(XDPP == LIFEAPI_XCHG_DPP && XLDS == LIFEAPI_XCHG_LDS && XBPERM == LIFEAPI_XCHG_BPERM &&
                  XMIX == LIFEAPI_XCHG_MIX && XMIX1 == LIFEAPI_XCHG_MIX1 && XMIX3 == LIFEAPI_XCHG_MIX3 &&
                  XLDSR == LIFEAPI_XCHG_LDSR && XLDSR3 == LIFEAPI_XCHG_LDSR3 && XASM == LIFEAPI_XCHG_ASM,
              "device.hpp's exchange numbering");

namespace {

// `gens` generations of one universe in the (E, O) layout (RULE 4), as one
// hand-allocated loop.  The compiler's allocation puts two or three sources
// of about half of the v_bitop3 in one VGPR bank (tools/vbank.py), and such an
// instruction issues at half rate (tools/ab/bank_probe.hip).  Here every VALU
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

// k_step with the hand-allocated RULE 4 loop (X == XASM)
template <int X, int U, bool NT, int RULE>
__global__ __launch_bounds__(kBlock) void k_step_asm4(const uint64_t *__restrict__ in,
                                                 uint64_t *__restrict__ out, uint64_t n,
                                                 uint32_t gens, uint64_t /* plain_from */) {
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

// k_step for the tile layouts (gen_tile): a wave holds C groups of P = S/2
// universes, lane i of group g columns C*i .. C*i+C-1 of each (C*8
// contiguous bytes per universe: two dwordx4 loads for C = 4).
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

// ---- the streaming step with two adjacent columns per lane (round 3 A/B) --
// Lane l of a wave holds columns 2i, 2i+1 (i = l & 31) of universe 2k + (l >> 5):
// one 16-byte access per lane moves two universes per wave-instruction.  Only
// a lane's outer columns cross lanes: column 2i's left neighbour is lane
// i-1's column 2i+1 and column 2i+1's right one lane i+1's column 2i (within
// the 32-lane half, wrapping), fetched by ds_bpermute on the LDS pipe (4 per
// two universes) instead of DPP moves on the VALU (8 per two universes).
__device__ __forceinline__ void pair_neighbours(W c0, W c1, W &l1, W &r0, int lane) {
  const int h = lane & 32, i = lane & 31;
  const int pa = (h | ((i + 31) & 31)) << 2, na = (h | ((i + 1) & 31)) << 2;
  l1 = W{(uint32_t)__builtin_amdgcn_ds_bpermute(pa, (int)c1.lo), (uint32_t)__builtin_amdgcn_ds_bpermute(pa, (int)c1.hi)};
  r0 = W{(uint32_t)__builtin_amdgcn_ds_bpermute(na, (int)c0.lo), (uint32_t)__builtin_amdgcn_ds_bpermute(na, (int)c0.hi)};
}

template <int U, bool NTS>
__global__ __launch_bounds__(kBlock) void k_step_pairnat(const uint64_t *in, uint64_t *out, uint64_t n,
                                                         uint32_t gens, uint64_t plain_from) {
  static_assert(U % 2 == 0, "universes come in pairs");
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int h = lane >> 5, col = (lane & 31) * 2;
  const bool rev = (gens & kReverse) != 0;
  const uint64_t blk = (gens & kXcdChunk) ? xcd_chunk_block() : (uint64_t)blockIdx.x;
  gens &= ~(kReverse | kXcdChunk);
  const uint64_t groups = (n + U - 1) / U, wstride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t grp = blk * kWavesPerBlock + wib; grp < groups; grp += wstride) {
    const uint64_t u0 = (rev ? groups - 1 - grp : grp) * U;
    W c0[U / 2], c1[U / 2];
#pragma unroll
    for (int k = 0; k < U / 2; ++k) {
      const uint64_t u = u0 + 2 * k + h;
      const u64x2 v = u < n ? ld2<true>(in + u * kWave + col) : u64x2{0, 0};
      c0[k] = split(v[0]);
      c1[k] = split(v[1]);
    }
    for (uint32_t g = 0; g < gens; ++g) {
#pragma unroll
      for (int k = 0; k < U / 2; ++k) {
        W l1, r0;
        pair_neighbours(c0[k], c1[k], l1, r0, lane);
        const W a0 = c0[k], a1 = c1[k];
        // column 2i: (L, a, R) = (l1, a0, a1); column 2i+1: (a0, a1, r0)
        const W h00 = lut3<kXor3>(l1, a0, a1), h10 = lut3<kMaj>(l1, a0, a1);
        const W h01 = lut3<kXor3>(a0, a1, r0), h11 = lut3<kMaj>(a0, a1, r0);
        auto tail = [](W a, W h0, W h1) __attribute__((always_inline)) {
          const W h0u = rot_up(h0), h0d = rot_dn(h0), h1u = rot_up(h1), h1d = rot_dn(h1);
          const W s0 = lut3<kLe1>(h0u, h0, h0d), s1 = lut3<kNae>(h0u, h0, h0d);
          const W s2 = lut3<kLe1>(h1u, h1, h1d), s3 = lut3<kEven>(h1u, h1, h1d);
          const W t1 = lut3<kT1>(s0, s1, a);
          const W t2 = lut3<kT2>(s2, a, t1);
          return lut3<kT3>(s1, s3, t2);
        };
        c0[k] = tail(a0, h00, h10);
        c1[k] = tail(a1, h01, h11);
      }
    }
    const bool nt = grp < plain_from;
#pragma unroll
    for (int k = 0; k < U / 2; ++k) {
      const uint64_t u = u0 + 2 * k + h;
      if (u < n) {
        const u64x2 v = {join(c0[k]), join(c1[k])};
        if (nt && NTS) st2<true>(out + u * kWave + col, v);
        else st2<false>(out + u * kWave + col, v);
      }
    }
  }
}

template <int S, int C, int X, bool NT, int NET>
__global__ __launch_bounds__(kBlock) void k_step_tile(const uint64_t *__restrict__ in,
                                                      uint64_t *__restrict__ out, uint64_t n,
                                                      uint32_t gens, uint64_t /* plain_from */) {
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

using StepFn = void (*)(const uint64_t *, uint64_t *, uint64_t, uint32_t, uint64_t);

template <int X, int U, bool NT, int RULE>
constexpr StepFn step_ptr() {
  if constexpr (X == XASM) return k_step_asm4<X, U, NT, RULE>;
  else return k_step<X, U, NT, RULE>;
}

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
      case 14: return pick_nt<X, 14>(u, nt);
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

// Diagnostic build of the shipped gens > 2 kernel (k_step_split<8, 1, NT,
// 6, kAsmLoop>): the same load / layout change / assembly loop / store, with
// the shader clock (s_memtime) and the 100 MHz real-time counter
// (s_memrealtime) stamped around the generation loop of every wave, lane 0
// writing {t0, q0, t1, q1} to a stamp buffer nothing else reads
// (MI355X_MICROARCH.md, DVFS item 6).  The held clock is
// (t1 - t0) / (q1 - q0) x 100 MHz.
template <bool NT>
__global__ __launch_bounds__(kBlock) void k_step_split_clock(const uint64_t *in, uint64_t *out, uint64_t n,
                                                             uint32_t gens, uint64_t *stamps) {
  constexpr int S = 8, P = 4;
  __shared__ uint32_t lds[kWavesPerBlock * S * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + wib;
  const uint64_t u0 = wave * P;
  if (u0 >= n) return;
  uint32_t r[S];
  W c[P];
#pragma unroll
  for (int u = 0; u < P; ++u) c[u] = u0 + u < n ? ld<NT>(in + (u0 + u) * kWave + lane) : W{0u, 0u};
  Split<S>::load(c, r);
  const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)(lds + wib * S * kWave);
  const uint32_t self = base + lane * 16u, prev = base + ((lane + kWave - 1) & (kWave - 1)) * 16u,
                 next = base + ((lane + 1) & (kWave - 1)) * 16u;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), q0 = __builtin_amdgcn_s_memrealtime();
  split_gens_asm_v0(r, gens, self, prev, next);
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), q1 = __builtin_amdgcn_s_memrealtime();
  Split<S>::store(r, c);
#pragma unroll
  for (int u = 0; u < P; ++u)
    if (u0 + u < n) st<NT>(out + (u0 + u) * kWave + lane, c[u]);
  if (lane == 0) {
    stamps[wave * 4 + 0] = t0;
    stamps[wave * 4 + 1] = q0;
    stamps[wave * 4 + 2] = t1;
    stamps[wave * 4 + 3] = q1;
  }
}

// The pair layout (tools/gen_pair_asm.py): two adjacent columns per lane, 32
// lanes and 4 interleaved universes per group, 2 groups (8 universes) per
// wave; the exchange moves only the outer columns.  V = schedule.  The
// assembly loop pins v0..v63, so nothing lane-varying may stay live across
// it: the lane index is re-derived afterwards (v_mbcnt, opaque to CSE) and
// every address is rebuilt from it and wave-uniform scalars.
template <bool NT, int V>
__global__ __launch_bounds__(kBlock) void k_step_pair(const uint64_t *in, uint64_t *out, uint64_t n, uint32_t gens) {
  constexpr int S = 8, P = 4;
  __shared__ uint32_t lds[kWavesPerBlock * 1024];  // 4 KiB per wave
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * 2 * P;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wib) * 2 * P; u0 < n; u0 += stride) {
    const uint32_t room = n - u0 < 2 * P ? (uint32_t)(n - u0) : 2 * P;  // wave-uniform
    uint32_t a[S], b[S];
    {
      const uint32_t lane = lane_id_fresh(), grp = lane >> 5, i = lane & 31;
      const uint64_t *src = in + u0 * kWave;
      W c0[P], c1[P];
#pragma unroll
      for (int u = 0; u < P; ++u) {
        u64x2 v = {0, 0};
        if (grp * P + u < room) v = ld2<NT>(src + ((grp * P + u) * kWave + 2 * i));
        c0[u] = split(v[0]);
        c1[u] = split(v[1]);
      }
      Split<S>::load(c0, a);
      Split<S>::load(c1, b);
    }
    {
      const uint32_t lane = lane_id_fresh();
      const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)(lds + wib * 1024);
      const uint32_t self = base + lane * 16u, prev = base + ((lane & 32) | ((lane + 31) & 31)) * 16u,
                     next = base + ((lane & 32) | ((lane + 1) & 31)) * 16u;
      if constexpr (V == 0) pair_gens_asm_v0(a, b, gens, self, prev, next);
      else if constexpr (V == 1) pair_gens_asm_v1(a, b, gens, self, prev, next);
      else if constexpr (V == 2) pair_gens_asm_v2(a, b, gens, self, prev, next);
      else if constexpr (V == 3) pair_gens_asm_v3(a, b, gens, self, prev, next);
      else if constexpr (V == 4) pair_gens_asm_v4(a, b, gens, self, prev, next);
      else pair_gens_asm_v5(a, b, gens, self, prev, next);
    }
    {
      const uint32_t lane = lane_id_fresh(), grp = lane >> 5, i = lane & 31;
      uint64_t *dst = out + u0 * kWave;
      W c0[P], c1[P];
      Split<S>::store(a, c0);
      Split<S>::store(b, c1);
#pragma unroll
      for (int u = 0; u < P; ++u)
        if (grp * P + u < room) st2<NT>(dst + ((grp * P + u) * kWave + 2 * i), u64x2{join(c0[u]), join(c1[u])});
    }
  }
}

}  // namespace

extern "C" {

/* fused Step + Contains on the split layout: variant = step_kernels.hpp's
 * ASM (0 compiled loop ... 7 / 8 the shipped pair's halves) */
int lifeapi_tune_step_contains(const uint64_t *d_in, uint64_t *d_final, const uint64_t *d_wanted,
                               const uint64_t *d_unwanted, uint32_t *d_first_gen, size_t n, uint32_t generations,
                               int variant, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_in || !d_wanted || !d_unwanted || !d_first_gen) return fail(LIFEAPI_E_INVALID, "null pointer%s");
  if (d_final) {
    int rc = check_batch(d_in, d_final, n);
    if (rc != LIFEAPI_OK) return rc;
  }
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  using Fn = void (*)(const uint64_t *, uint64_t *, const uint64_t *, const uint64_t *, uint32_t *, uint64_t, uint32_t,
                      uint32_t);
  const Fn fns[9] = {k_step_contains_split<8, kContainsNet, 0>, k_step_contains_split<8, kContainsNet, 1>,
                     k_step_contains_split<8, kContainsNet, 2>, k_step_contains_split<8, kContainsNet, 3>,
                     k_step_contains_split<8, kContainsNet, 4>, k_step_contains_split<8, kContainsNet, 5>,
                     k_step_contains_split<8, kContainsNet, 6>, k_step_contains_split<8, kContainsNet, 7>,
                     k_step_contains_split<8, kContainsNet, 8>};
  if (variant < 0 || variant > 8) return fail(LIFEAPI_E_INVALID, "unknown contains variant%s");
  hipLaunchKernelGGL(fns[variant], dim3(grid_for((n + 3) / 4, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream, d_in,
                     d_final, d_wanted, d_unwanted, d_first_gen, (uint64_t)n, generations, 0u);
  return launched("k_step_contains_split (tuning) launch");
}

/* the natural-layout fused kernel (gens <= 2) with `upw` universes per wave
 * and at most `resident` blocks per CU (0 = as many as fit)               */
int lifeapi_tune_step_contains_nat(const uint64_t *d_in, uint64_t *d_final, const uint64_t *d_wanted,
                                   const uint64_t *d_unwanted, uint32_t *d_first_gen, size_t n,
                                   uint32_t generations, int upw, int resident, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  // upw + 1024: each XCD a contiguous eighth of the batch (kXcdChunk)
  const uint32_t chunk = upw >= 1024 ? kXcdChunk : 0u;
  upw &= 1023;
  if (!d_in || !d_wanted || !d_unwanted || !d_first_gen) return fail(LIFEAPI_E_INVALID, "bad argument%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  unsigned lds = 0;
  const int cap = resident < 0 ? -resident : 0;  // resident < 0: a grid-stride grid of -resident blocks per CU
  using Fn = void (*)(const uint64_t *, uint64_t *, const uint64_t *, const uint64_t *, uint32_t *, uint64_t, uint32_t,
                      uint64_t);
  // upw 16 + U: the 16-byte staged form (k_step_contains<U, true>), U = 2, 4, 8
  Fn fn = upw == 1 ? (Fn)k_step_contains<1> : upw == 2 ? (Fn)k_step_contains<2> : upw == 4 ? (Fn)k_step_contains<4>
        : upw == 8 ? (Fn)k_step_contains<8> : upw == 18 ? (Fn)k_step_contains<2, true>
        : upw == 20 ? (Fn)k_step_contains<4, true> : upw == 24 ? (Fn)k_step_contains<8, true>
        // 32 + U: LDS exchange; 64 + U: the 6-LUT tail (RULE 14); 96 + U: both
        : upw == 36 ? (Fn)k_step_contains<4, false, XLDS, 3> : upw == 40 ? (Fn)k_step_contains<8, false, XLDS, 3>
        : upw == 68 ? (Fn)k_step_contains<4, false, XDPP, 14> : upw == 72 ? (Fn)k_step_contains<8, false, XDPP, 14>
        : upw == 100 ? (Fn)k_step_contains<4, false, XLDS, 14> : upw == 104 ? (Fn)k_step_contains<8, false, XLDS, 14>
        // 128 + U: the prefetching loop (give a capped grid, resident < 0); 192 + U: with RULE 14
        : upw == 132 ? (Fn)k_step_contains<4, false, XDPP, 3, true> : upw == 136 ? (Fn)k_step_contains<8, false, XDPP, 3, true>
        : upw == 200 ? (Fn)k_step_contains<8, false, XDPP, 14, true>
        : upw == 16 ? (Fn)k_step_contains<16> : upw == 12 ? (Fn)k_step_contains<12>
        : nullptr;
  if (!fn) return fail(LIFEAPI_E_INVALID, "universes per wave: 1, 2, 4 or 8 (16 + 2, 4, 8: 16-byte form)%s");
  if (upw > 16 && (((uintptr_t)d_in | (uintptr_t)d_final) & 15u))
    return fail(LIFEAPI_E_INVALID, "the 16-byte form needs 16-byte aligned batches%s");
  const int universes_per_wave = upw == 16 ? 16 : upw == 12 ? 12 : upw & 15;
  if (resident > 0) {
    rc = occupancy_lds((const void *)fn, resident, lds);
    if (rc != LIFEAPI_OK) return rc;
  }
  // one order, nontemporal stores (the launch before the product's order policy)
  hipLaunchKernelGGL(fn, dim3(grid_for((n + universes_per_wave - 1) / universes_per_wave, cus, cap)), dim3(kBlock), lds,
                     (hipStream_t)stream, d_in, d_final, d_wanted, d_unwanted, d_first_gen, (uint64_t)n,
                     generations | chunk, ~(uint64_t)0);
  return launched("k_step_contains (tuning) launch");
}

/* the two-kernel form (variants 7 then 8) with each kernel's grid capped at
 * cap_lo / cap_hi blocks per CU (0 = one block per 4 waves of work)      */
int lifeapi_tune_step_contains_pair(const uint64_t *d_in, uint64_t *d_final, const uint64_t *d_wanted,
                                    const uint64_t *d_unwanted, uint32_t *d_first_gen, size_t n,
                                    uint32_t generations, int cap_lo, int cap_hi, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_in || !d_wanted || !d_unwanted || !d_first_gen || generations <= 2 || cap_lo < 0 || cap_hi < 0)
    return fail(LIFEAPI_E_INVALID, "bad argument%s");
  if (d_final) {
    int rc = check_batch(d_in, d_final, n);
    if (rc != LIFEAPI_OK) return rc;
  }
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL((k_step_contains_split<8, kContainsNet, 7>), dim3(grid_for((n + 3) / 4, cus, cap_lo)),
                     dim3(kBlock), 0, (hipStream_t)stream, d_in, d_final, d_wanted, d_unwanted, d_first_gen,
                     (uint64_t)n, generations, 0u);
  rc = launched("k_step_contains_split (tuning) launch");
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL((k_step_contains_split<8, kContainsNet, 8>), dim3(grid_for((n + 3) / 4, cus, cap_hi)),
                     dim3(kBlock), 0, (hipStream_t)stream, d_in, d_final, d_wanted, d_unwanted, d_first_gen,
                     (uint64_t)n, generations, 0u);
  return launched("k_step_contains_split (tuning) launch");
}

/* the iterated search filter without final states on the split pair
 * (round 6 A/B, tools/filter_iter_probe.py): variant bits 0-7 = blocks per
 * CU of both grids (0: one-shot), bit 8 = the LDS-DMA prefetch form (PF),
 * bit 9 = kContainsHi alone (the Lo kernel not launched: answers only for
 * targets whose row window exceeds 4 rows), bit 10 = kContainsLo alone,
 * bit 11 = the merged kernel (kContainsAll) alone: one launch, any target */
int lifeapi_tune_filter_iter(const uint64_t *d_in, const uint64_t *d_wanted, const uint64_t *d_unwanted,
                             uint32_t *d_first_gen, size_t n, uint32_t generations, int variant, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_in || !d_wanted || !d_unwanted || !d_first_gen || generations <= 2 || variant < 0 ||
      ((variant & 0x100) && !aligned16(d_in)))
    return fail(LIFEAPI_E_INVALID, "bad argument%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const int cap = variant & 0xFF;
  const bool pf = (variant & 0x100) != 0, hi_only = (variant & 0x200) != 0, lo_only = (variant & 0x400) != 0;
  using Fn = void (*)(const uint64_t *, uint64_t *, const uint64_t *, const uint64_t *, uint32_t *, uint64_t, uint32_t,
                      uint32_t);
  const Fn lo = pf ? k_step_contains_split<8, kContainsNet, kContainsLo, true>
                   : k_step_contains_split<8, kContainsNet, kContainsLo>;
  const Fn hi = pf ? k_step_contains_split<8, kContainsNet, kContainsHi, true>
                   : k_step_contains_split<8, kContainsNet, kContainsHi>;
  const dim3 grid(grid_for((n + 3) / 4, cus, cap));
  if (variant & 0x800) {  // bit 12: with the window split layout (WIN)
    const bool win = (variant & 0x1000) != 0;
    const Fn all = win ? (pf ? k_step_contains_split<8, kContainsNet, kContainsAll, true, true>
                             : k_step_contains_split<8, kContainsNet, kContainsAll, false, true>)
                       : (pf ? k_step_contains_split<8, kContainsNet, kContainsAll, true>
                             : k_step_contains_split<8, kContainsNet, kContainsAll>);
    hipLaunchKernelGGL(all, grid, dim3(kBlock), 0, (hipStream_t)stream, d_in, nullptr, d_wanted, d_unwanted,
                       d_first_gen, (uint64_t)n, generations, 32u);
    return launched("k_step_contains_split (tuning) launch");
  }
  for (int k = 0; k < 2; ++k) {
    if ((k == 0 && hi_only) || (k == 1 && lo_only)) continue;
    hipLaunchKernelGGL(k == 0 ? lo : hi, grid, dim3(kBlock), 0, (hipStream_t)stream, d_in, nullptr, d_wanted,
                       d_unwanted, d_first_gen, (uint64_t)n, generations, 32u);  // (cone_max: cone_kernels.hpp kConeIterColumns)
    rc = launched("k_step_contains_split (tuning) launch");
    if (rc != LIFEAPI_OK) return rc;
  }
  return LIFEAPI_OK;
}

/* the pair layout (k_step_pair), schedule `variant` 0..5 */
int lifeapi_tune_step_pair(const uint64_t *d_in, uint64_t *d_out, size_t n, uint32_t generations, int variant,
                           void *stream) {
  int rc = check_batch(d_in, d_out, n);
  if (rc != LIFEAPI_OK || n == 0) return rc;
  int cus = 0;
  rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const bool nt = generations < 32;
  using Fn = void (*)(const uint64_t *, uint64_t *, uint64_t, uint32_t);
  const Fn fns[2][6] = {{k_step_pair<false, 0>, k_step_pair<false, 1>, k_step_pair<false, 2>, k_step_pair<false, 3>,
                         k_step_pair<false, 4>, k_step_pair<false, 5>},
                        {k_step_pair<true, 0>, k_step_pair<true, 1>, k_step_pair<true, 2>, k_step_pair<true, 3>,
                         k_step_pair<true, 4>, k_step_pair<true, 5>}};
  if (variant < 0 || variant > 5) return fail(LIFEAPI_E_INVALID, "unknown pair schedule%s");
  hipLaunchKernelGGL(fns[nt][variant], dim3(grid_for((n + 7) / 8, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_in, d_out, (uint64_t)n, generations);
  return launched("k_step_pair launch");
}

/* the shipped gens <= 2 kernel (k_step<dpp, U, nt loads, rule 3>) with
 * nontemporal (nts = 1) or plain stores (0), but plain for the groups that
 * store the last `plain_bytes` of the launch's order, at most `resident` blocks per CU
 * (0 = as many as fit), U = upw universes per wave (2, 4 or 8; shipped 4);
 * bit 31 of `generations` reverses the group order                         */
extern "C++" {
template <int U>
StepFn order_fn(int nts) { return nts ? k_step_ab<XDPP, U, true, 3, true> : k_step_ab<XDPP, U, true, 3, false>; }
}

int lifeapi_tune_step_order(const uint64_t *d_in, uint64_t *d_out, size_t n, uint32_t generations, void *stream,
                            int nts, int resident, int upw, uint64_t plain_bytes) {
  int rc = check_batch(d_in, d_out, n);
  if (rc != LIFEAPI_OK || n == 0) return rc;
  if ((generations & ~(kReverse | kXcdChunk)) > 2) return fail(LIFEAPI_E_INVALID, "streaming step: generations <= 2%s");
  // upw 32 + U: the column-pair form (k_step_pairnat<U>, 16-byte accesses; 16-byte-aligned batches)
  const StepFn fn = upw == 2 ? order_fn<2>(nts) : upw == 4 ? order_fn<4>(nts) : upw == 8 ? order_fn<8>(nts)
                  : upw == 36 ? (nts ? (StepFn)k_step_pairnat<4, true> : (StepFn)k_step_pairnat<4, false>)
                  : upw == 40 ? (nts ? (StepFn)k_step_pairnat<8, true> : (StepFn)k_step_pairnat<8, false>)
                  // upw 64 + U / 96 + U: through LDS (k_step_dma<U>, 8-byte / 16-byte stores; 16-byte-aligned batches)
                  : upw == 68 ? (nts ? (StepFn)k_step_dma<4, 3, true, false> : (StepFn)k_step_dma<4, 3, false, false>)
                  : upw == 72 ? (nts ? (StepFn)k_step_dma<8, 3, true, false> : (StepFn)k_step_dma<8, 3, false, false>)
                  : upw == 100 ? (nts ? (StepFn)k_step_dma<4, 3, true, true> : (StepFn)k_step_dma<4, 3, false, true>)
                  : upw == 104 ? (nts ? (StepFn)k_step_dma<8, 3, true, true> : (StepFn)k_step_dma<8, 3, false, true>)
                  : nullptr;
  if (!fn) return fail(LIFEAPI_E_INVALID, "universes per wave: 2, 4 or 8%s");
  upw &= 31;
  int cus = 0;
  rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  unsigned lds = 0;
  if (resident > 0) {
    rc = occupancy_lds((const void *)fn, resident, lds);
    if (rc != LIFEAPI_OK) return rc;
  }
  const uint64_t groups = (n + upw - 1) / upw, plain = (plain_bytes + upw * 512 - 1) / (upw * 512);
  hipLaunchKernelGGL(fn, dim3(grid_for(groups, cus, 0)), dim3(kBlock), lds, (hipStream_t)stream, d_in, d_out,
                     (uint64_t)n, generations, plain < groups ? groups - plain : (uint64_t)0);
  return launched("k_step (order) launch");
}

/* the shipped gens > 2 kernel (k_step_split<8, 1, NT, 6, asm loop>) with
 * `wpb` waves per block (1, 2 or 4 = shipped): finer blocks let the
 * dispatcher balance the last round of waves over the SIMDs              */
int lifeapi_tune_step_split_wpb(const uint64_t *d_in, uint64_t *d_out, size_t n, uint32_t generations, int wpb,
                                void *stream) {
  int rc = check_batch(d_in, d_out, n);
  if (rc != LIFEAPI_OK || n == 0) return rc;
  const bool nt = generations < 32;
  const uint64_t waves = (n + 3) / 4;
  const dim3 grid((unsigned)((waves + wpb - 1) / wpb)), block(64 * wpb);
  StepFn fn = nullptr;
  if (wpb == 1) fn = nt ? k_step_split<8, 1, true, 6, kAsmLoop, 0, 1> : k_step_split<8, 1, false, 6, kAsmLoop, 0, 1>;
  if (wpb == 2) fn = nt ? k_step_split<8, 1, true, 6, kAsmLoop, 0, 2> : k_step_split<8, 1, false, 6, kAsmLoop, 0, 2>;
  if (wpb == 4) fn = nt ? k_step_split<8, 1, true, 6, kAsmLoop, 0, 4> : k_step_split<8, 1, false, 6, kAsmLoop, 0, 4>;
  if (!fn) return fail(LIFEAPI_E_INVALID, "waves per block: 1, 2 or 4%s");
  hipLaunchKernelGGL(fn, grid, block, 0, (hipStream_t)stream, d_in, d_out, (uint64_t)n, generations, (uint64_t)0);
  return launched("k_step_split (wpb) launch");
}

/* the shipped gens > 2 kernel with clock stamps (see k_step_split_clock);
 * d_stamps: 4 words per wave, one wave per 4 universes, one-shot grid      */
int lifeapi_tune_step_clock(const uint64_t *d_in, uint64_t *d_out, size_t n, uint32_t generations,
                            void *stream, uint64_t *d_stamps) {
  int rc = check_batch(d_in, d_out, n);
  if (rc != LIFEAPI_OK || n == 0) return rc;
  if (!d_stamps) return fail(LIFEAPI_E_INVALID, "null stamp buffer%s");
  const uint64_t waves = (n + 3) / 4;
  hipLaunchKernelGGL(generations < 32 ? k_step_split_clock<true> : k_step_split_clock<false>,
                     dim3((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, d_in, d_out, (uint64_t)n, generations, d_stamps);
  return launched("k_step_split_clock launch");
}

void lifeapi_tune_default_cfg(lifeapi_launch_cfg *cfg, uint32_t generations) {
  if (!cfg) return;
  cfg->blocks_per_cu = 0;
  if (generations <= 2) {
    cfg->xchg = LIFEAPI_XCHG_DPP;
    cfg->rule = 3;
    cfg->universes_per_wave = 4;
    cfg->nontemporal = 1;
  } else {
    cfg->xchg = LIFEAPI_XCHG_ASM;
    cfg->rule = 11;
    cfg->universes_per_wave = 1;
    cfg->nontemporal = generations < 32 ? 1 : 0;
  }
}

int lifeapi_tune_step_batch_dev_cfg(const uint64_t *d_in, uint64_t *d_out, size_t n,
                                    uint32_t generations, void *stream,
                                    const lifeapi_launch_cfg *cfg) {
  int rc = check_batch(d_in, d_out, n);
  if (rc != LIFEAPI_OK || n == 0) return rc;
  lifeapi_launch_cfg c;
  if (cfg) c = *cfg;
  else lifeapi_tune_default_cfg(&c, generations);
  StepFn fn = pick_step(c);
  if (!fn) return fail(LIFEAPI_E_INVALID, "unsupported launch cfg%s");
  int cus = 0;
  rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const uint64_t per_wave = (uint64_t)c.universes_per_wave * group_size(c.rule);
  const uint64_t waves = (n + per_wave - 1) / per_wave;
  const unsigned grid = grid_for(waves, cus, c.blocks_per_cu);
  // blocks_per_cu < 0: no grid cap, at most -blocks_per_cu blocks resident
  // per CU (unused dynamic LDS on top of the kernel's own)
  unsigned lds = 0;
  if (c.blocks_per_cu < 0) {
    rc = occupancy_lds((const void *)fn, -c.blocks_per_cu, lds);
    if (rc != LIFEAPI_OK) return rc;
  }
  hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlock), lds, (hipStream_t)stream, d_in, d_out,
                     (uint64_t)n, generations, ~(uint64_t)0);
  return launched("k_step (tuning) launch");
}

}  // extern "C"
