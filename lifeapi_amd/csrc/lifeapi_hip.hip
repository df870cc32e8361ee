// lifeapi_hip.hip -- MI355X (gfx950) batched LifeState::Step() and friends.
//
// One 64-lane wavefront steps one 64x64 torus universe: lane x owns column x
// (the reference's state[x], LifeAPI.hpp:39-40) as two 32-bit VGPRs.  The
// vertical (in-column) neighbours are a 1-bit rotate of the lane's own word
// (v_alignbit_b32); the horizontal neighbours are the adjacent lanes' column
// sums, fetched with DPP wave_ror:1 / wave_rol:1 (64-lane rotates, so the torus
// wrap at columns 0/63 is free), or -- as ablations -- through LDS or
// ds_bpermute.  The B3/S23 rule is the reference's bitsliced adder network
// (CountRows LifeAPI.hpp:897-907 feeding the FullAdd form of StepAlt,
// LifeAPI.hpp:1218-1254, which the reference proves equal to Step()'s
// Rokicki form in tests/StepAltTest.cpp:5-13), evaluated with gfx950's
// 3-input v_bitop3_b32.  A wave keeps U universes in flight; the grid
// strides over the batch.  No MFMA: the work is pure integer/bitwise.
//
// All entry points are the C ABI in include/lifeapi_hip.h.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "lifeapi_hip.h"

namespace {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ULL;

// ------------------------------------------------------------------------
// lane-level primitives
// ------------------------------------------------------------------------

struct W {  // one column word, split in VGPR halves: bits 0-31 / 32-63
  uint32_t lo, hi;
};

__device__ __forceinline__ W split(uint64_t v) { return W{(uint32_t)v, (uint32_t)(v >> 32)}; }
__device__ __forceinline__ uint64_t join(W w) { return (uint64_t)w.lo | ((uint64_t)w.hi << 32); }

// 64-bit rotates by one row: rotl(a,1) (cell y <- y-1) and rotr(a,1).
__device__ __forceinline__ W rot_up(W a) {
  return W{__builtin_amdgcn_alignbit(a.lo, a.hi, 31), __builtin_amdgcn_alignbit(a.hi, a.lo, 31)};
}
__device__ __forceinline__ W rot_dn(W a) {
  return W{__builtin_amdgcn_alignbit(a.hi, a.lo, 1), __builtin_amdgcn_alignbit(a.lo, a.hi, 1)};
}

// v_bitop3_b32 truth tables: bit i of the table is f(bit i of 0xF0, 0xCC, 0xAA)
// for (src0, src1, src2).
constexpr uint32_t TA = 0xF0, TB = 0xCC, TC = 0xAA;
constexpr uint32_t kXor3 = (TA ^ TB ^ TC) & 0xFF;                     // 0x96
constexpr uint32_t kMaj = ((TA & TB) | (TA & TC) | (TB & TC)) & 0xFF;  // 0xE8
constexpr uint32_t kCarry2 = (TA ^ (TB & TC)) & 0xFF;                 // a ^ (b & c)
constexpr uint32_t kLive = ((TA ^ TB) & (TC | TA)) & 0xFF;            // (a ^ b) & (c | a)

template <uint32_t TT>
__device__ __forceinline__ uint32_t lut3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
}
template <uint32_t TT>
__device__ __forceinline__ W lut3(W a, W b, W c) {
  return W{lut3<TT>(a.lo, b.lo, c.lo), lut3<TT>(a.hi, b.hi, c.hi)};
}

// ------------------------------------------------------------------------
// neighbour-column exchange (lane x <- lanes x-1 and x+1, mod 64)
// ------------------------------------------------------------------------

enum Xchg {
  XDPP = LIFEAPI_XCHG_DPP,
  XLDS = LIFEAPI_XCHG_LDS,
  XBPERM = LIFEAPI_XCHG_BPERM,
  XMIX = LIFEAPI_XCHG_MIX,
  XMIX1 = LIFEAPI_XCHG_MIX1,
  XMIX3 = LIFEAPI_XCHG_MIX3,
  XLDSR = LIFEAPI_XCHG_LDSR,
  XLDSR3 = LIFEAPI_XCHG_LDSR3,
  XASM = LIFEAPI_XCHG_ASM
};
constexpr bool uses_lds(int x) { return x == XLDS || x == XLDSR || x == XLDSR3 || x == XASM; }

// A full-wave rotate has no out-of-range source lane, so bound_ctrl (read 0
// for invalid lanes) never fires; it lets the compiler skip the old-value init.
__device__ __forceinline__ uint32_t dpp_prev(uint32_t v) {  // wave_ror:1
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_next(uint32_t v) {  // wave_rol:1
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x134, 0xF, 0xF, true);
}
// the same rotates through the LDS crossbar (ds_bpermute: no LDS memory, but
// it issues on the LDS pipe instead of the VALU)
__device__ __forceinline__ uint32_t bperm_prev(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(((lane + kWave - 1) & (kWave - 1)) << 2, (int)v);
}
__device__ __forceinline__ uint32_t bperm_next(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(((lane + 1) & (kWave - 1)) << 2, (int)v);
}

template <int X>
__device__ __forceinline__ void neighbour_cols(W a, W &L, W &R, uint64_t *slot, int lane);

// slot: 128 words of this wave's LDS scratch (only used by XLDS)
template <int X>
__device__ __forceinline__ void neighbours(W c0, W c1, W &L0, W &R0, W &L1, W &R1,
                                           uint64_t *slot, int lane) {
  if constexpr (X != XLDS) {  // (the LDSR variants stage each plane in turn)
    neighbour_cols<X>(c0, L0, R0, slot, lane);
    neighbour_cols<X>(c1, L1, R1, slot, lane);
  } else {
    // Stage the two column-sum planes through LDS: [0,64) plane 0, [64,128)
    // plane 1, one 8-byte word per lane (ds_write_b64 / ds_read_b64, bank-
    // conflict free: consecutive lanes, consecutive 8-byte words).  DS ops of
    // one wave complete in order, so a wave only needs compiler ordering,
    // which the possible aliasing of the store and the loads already gives.
    uint64_t *s = slot;
    s[lane] = join(c0);
    s[kWave + lane] = join(c1);
    __builtin_amdgcn_wave_barrier();
    const int xp = (lane + kWave - 1) & (kWave - 1), xn = (lane + 1) & (kWave - 1);
    L0 = split(s[xp]);
    R0 = split(s[xn]);
    L1 = split(s[kWave + xp]);
    R1 = split(s[kWave + xn]);
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------------
// one generation of one universe (this lane's column)
// ------------------------------------------------------------------------

// one 64-bit neighbour word from lanes x-1 / x+1 (used by the row-first rule)
template <int X>
__device__ __forceinline__ void neighbour_cols(W a, W &L, W &R, uint64_t *slot, int lane) {
  if constexpr (X == XDPP) {
    L = W{dpp_prev(a.lo), dpp_prev(a.hi)};
    R = W{dpp_next(a.lo), dpp_next(a.hi)};
  } else if constexpr (X == XBPERM) {
    L = W{bperm_prev(a.lo, lane), bperm_prev(a.hi, lane)};
    R = W{bperm_next(a.lo, lane), bperm_next(a.hi, lane)};
  } else if constexpr (X == XMIX) {
    L = W{dpp_prev(a.lo), dpp_prev(a.hi)};
    R = W{bperm_next(a.lo, lane), bperm_next(a.hi, lane)};
  } else if constexpr (X == XMIX1) {
    L = W{dpp_prev(a.lo), dpp_prev(a.hi)};
    R = W{dpp_next(a.lo), bperm_next(a.hi, lane)};
  } else if constexpr (X == XMIX3) {
    L = W{dpp_prev(a.lo), bperm_prev(a.hi, lane)};
    R = W{bperm_next(a.lo, lane), bperm_next(a.hi, lane)};
  } else if constexpr (X == XLDSR || X == XLDSR3) {
    // one ds_write_b64 of the column, then the right neighbour by one
    // ds_read_b64 (and, for LDSR3, the left high word by one ds_read_b32).
    // A wave's LDS operations complete in order, so the only ordering needed
    // is the compiler's: the store and the loads may alias.
    uint64_t *s = slot;
    s[lane] = join(a);
    __builtin_amdgcn_wave_barrier();
    R = split(s[(lane + 1) & (kWave - 1)]);
    if constexpr (X == XLDSR) {
      L = W{dpp_prev(a.lo), dpp_prev(a.hi)};
    } else {
      const uint32_t *s32 = reinterpret_cast<const uint32_t *>(s);
      L = W{dpp_prev(a.lo), s32[2 * ((lane + kWave - 1) & (kWave - 1)) + 1]};
    }
    __builtin_amdgcn_wave_barrier();
  } else {
    uint64_t *s = slot;  // (ordering as in neighbours<XLDS>)
    s[lane] = join(a);
    __builtin_amdgcn_wave_barrier();
    L = split(s[(lane + kWave - 1) & (kWave - 1)]);
    R = split(s[(lane + 1) & (kWave - 1)]);
    __builtin_amdgcn_wave_barrier();
  }
}

// Tables of the 7-LUT network (RULE 3).  Over the vertical triples of the
// horizontal 3-sum planes h0 (A) and h1 (B), with SA, SB their 0..3 sums and
// count = SA + 2 SB (inclusive of the centre):
//   s0 = SA <= 1,  s1 = SA in {1,2},  s2 = SB <= 1,  s3 = SB in {0,2}
//   next = T3(s1, s3, T2(s2, a, T1(s0, s1, a)))
// T1..T3 were found by exhaustive search over all 3-gate tails on every pair
// of symmetric encodings (tools/exact_tail.c) and are checked on all 512
// 3x3 neighbourhoods by tests/test_oracle.py::test_rule3_network_truth.
// No 3-gate tail exists for the FullAdd encoding (fs, fc, cs, cc), so this
// saves one v_bitop3 per 32-bit half over StepAlt's tail.
constexpr uint32_t kLe1 = (~kMaj) & 0xFF;                        // 0x17: sum <= 1
constexpr uint32_t kNae = ((TA ^ TB) | (TB ^ TC)) & 0xFF;         // 0x7E: sum in {1,2}
constexpr uint32_t kEven = (~kXor3) & 0xFF;                       // 0x69: sum in {0,2}
constexpr uint32_t kT1 = 0x34, kT2 = 0x58, kT3 = 0x28;

// ---- even/odd row layout (RULE 4) ----
// A 64-bit column held as (E, O): E bit k = row 2k, O bit k = row 2k+1.  The
// vertical neighbours of row 2k are O bits k-1 and k; those of row 2k+1 are
// E bits k and k+1.  So a vertical triple costs one 32-bit rotate per plane
// and parity instead of two 64-bit rotates (four v_alignbit) per plane, and a
// v_alignbit issues at half rate on gfx950 (tools/bank_probe.hip).
__device__ __forceinline__ uint32_t delta_swap(uint32_t x, uint32_t m, int s) {
  const uint32_t t = ((x >> s) ^ x) & m;
  return x ^ t ^ (t << s);
}
// even bits -> low half, odd bits -> high half
__device__ __forceinline__ uint32_t unzip32(uint32_t x) {
  x = delta_swap(x, 0x22222222u, 1);
  x = delta_swap(x, 0x0C0C0C0Cu, 2);
  x = delta_swap(x, 0x00F000F0u, 4);
  return delta_swap(x, 0x0000FF00u, 8);
}
__device__ __forceinline__ uint32_t zip32(uint32_t x) {
  x = delta_swap(x, 0x0000FF00u, 8);
  x = delta_swap(x, 0x00F000F0u, 4);
  x = delta_swap(x, 0x0C0C0C0Cu, 2);
  return delta_swap(x, 0x22222222u, 1);
}
__device__ __forceinline__ W to_eo(W a) {  // (lo, hi) rows -> (E, O)
  const uint32_t l = unzip32(a.lo), h = unzip32(a.hi);
  return W{__builtin_amdgcn_perm(h, l, 0x05040100u), __builtin_amdgcn_perm(h, l, 0x07060302u)};
}
__device__ __forceinline__ W from_eo(W e) {
  return W{zip32(__builtin_amdgcn_perm(e.hi, e.lo, 0x05040100u)),
           zip32(__builtin_amdgcn_perm(e.hi, e.lo, 0x07060302u))};
}
__device__ __forceinline__ uint32_t rotl1(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 31); }
__device__ __forceinline__ uint32_t rotr1(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 1); }

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

template <bool NT>
__device__ __forceinline__ W ld(const uint64_t *p) {
  if constexpr (NT) return split(__builtin_nontemporal_load(p));
  else return split(*p);
}
template <bool NT>
__device__ __forceinline__ void st(uint64_t *p, W v) {
  if constexpr (NT) __builtin_nontemporal_store(join(v), p);
  else *p = join(v);
}

// ------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------

// out[u] = in[u] stepped `gens` times.  Wave w of the grid takes groups of U
// consecutive universes, grid-strided.  All branches are wave-uniform.
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

// ------------------------------------------------------------------------
// Row-split layouts (RULE 5: S = 4, RULE 6: S = 8, RULE 7: S = 16)
// ------------------------------------------------------------------------
//
// P = S/2 universes share a lane's S registers: bit P*k + u of R_j holds
// universe u, row S*k + j (k < 64/S).  The vertical neighbours of R_j are
// R_{j-1} and R_{j+1} at the same bit, except at the ends of the register
// ring: R_0's upper neighbour is R_{S-1} rotated left by P bits, R_{S-1}'s
// lower one is R_0 rotated right by P bits.  Because the P universes are
// interleaved bit by bit, one 32-bit rotate by P rotates all P of their
// 64/S-row rings at once.  Per register and generation that leaves the nine
// v_bitop3 of the RULE 3 network plus 4/S v_alignbit (two per plane per
// ring), against 9 + 2 for the even/odd split (S = 2, RULE 4).  The
// exchange goes through LDS (lane-major, S words per lane).

// Layout change by index-bit transpositions.  Number the 8*P source words
// X[2u + h] = universe u's column, h = high half (rows 32..63); a bit is then
// addressed by (register index bits | 5 position bits).  Exchanging register
// index bit a with position bit b (shift s = 2^b) is one delta swap per pair
// of registers:  t = ((A >> s) ^ B) & m_b;  B ^= t;  A ^= t << s.  Five such
// swaps route the row's upper bits k to the top of the word, the universe
// bits below them and the row's low bits j into the register index; the
// target register R_j is then a fixed renaming of X.  Each swap is its own
// inverse, so the store path runs them backwards.  About 30 VALU per
// universe each way (tools/split_layout.py checks the tables).
template <int S>
struct SplitNet;
template <>
struct SplitNet<2> {  // R_j: j = row bit 0;            (E, O) of RULE 4
  [[maybe_unused]] static constexpr int a[5] = {0, 0, 0, 0, 0};
  static constexpr __device__ int reg(int j) { return j; }
};
template <>
struct SplitNet<4> {  // R_j: j = row bits 1..0, 2 universes
  static constexpr int a[5] = {0, 0, 0, 0, 1};
  static constexpr __device__ int reg(int j) { return ((j & 1) << 1) | (j >> 1); }
};
template <>
struct SplitNet<8> {  // R_j: j = row bits 2..0, 4 universes
  static constexpr int a[5] = {0, 0, 0, 2, 1};
  static constexpr __device__ int reg(int j) { return ((j & 3) << 1) | (j >> 2); }
};

template <>
struct SplitNet<16> {  // R_j: j = row bits 3..0, 8 universes
  static constexpr int a[5] = {0, 0, 3, 2, 1};
  static constexpr __device__ int reg(int j) { return ((j & 7) << 1) | (j >> 3); }
};

template <int S>
__device__ __forceinline__ void split_swap(uint32_t (&x)[S], int stage) {
  constexpr uint32_t masks[5] = {0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
  const int a = SplitNet<S>::a[stage], sh = 16 >> stage;
  const uint32_t m = masks[stage];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    if ((i >> a) & 1) continue;
    const int k = i | (1 << a);
    const uint32_t t = ((x[i] >> sh) ^ x[k]) & m;
    x[k] ^= t;
    x[i] ^= t << sh;
  }
}

template <int S>
struct Split {
  static constexpr int P = S / 2;
  static __device__ __forceinline__ void load(const W (&c)[P], uint32_t (&r)[S]) {
    uint32_t x[S];
#pragma unroll
    for (int u = 0; u < P; ++u) x[2 * u] = c[u].lo, x[2 * u + 1] = c[u].hi;
#pragma unroll
    for (int st = 0; st < 5; ++st) split_swap<S>(x, st);
#pragma unroll
    for (int j = 0; j < S; ++j) r[j] = x[SplitNet<S>::reg(j)];
  }
  static __device__ __forceinline__ void store(const uint32_t (&r)[S], W (&c)[P]) {
    uint32_t x[S];
#pragma unroll
    for (int j = 0; j < S; ++j) x[SplitNet<S>::reg(j)] = r[j];
#pragma unroll
    for (int st = 4; st >= 0; --st) split_swap<S>(x, st);
#pragma unroll
    for (int u = 0; u < P; ++u) c[u] = W{x[2 * u], x[2 * u + 1]};
  }
};

// one generation of the P universes in r[] (RULE 3 network per register)
template <int S>
__device__ __forceinline__ void gen_split(uint32_t (&r)[S], uint32_t *slot, int lane) {
  constexpr int P = S / 2;
  // LDS planes of Q <= 4 words per lane: 16-B lane stride keeps ds_write_b128
  // / ds_read_b128 free of bank conflicts (a 32-B stride would be 2-way)
  constexpr int Q = S < 4 ? S : 4;
  typedef uint32_t vec __attribute__((ext_vector_type(Q)));
  vec *v = reinterpret_cast<vec *>(slot);
  const int xp = (lane + kWave - 1) & (kWave - 1), xn = (lane + 1) & (kWave - 1);
#pragma unroll
  for (int p = 0; p < S / Q; ++p) {
    vec mine;
#pragma unroll
    for (int q = 0; q < Q; ++q) mine[q] = r[p * Q + q];
    v[p * kWave + lane] = mine;  // a wave's LDS operations complete in order; the
  }                              // store and the loads may alias, so the compiler
  uint32_t lv[S], rv[S];         // keeps their order
#pragma unroll
  for (int p = 0; p < S / Q; ++p) {
    const vec l = v[p * kWave + xp], rr = v[p * kWave + xn];
#pragma unroll
    for (int q = 0; q < Q; ++q) lv[p * Q + q] = l[q], rv[p * Q + q] = rr[q];
  }
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
    const uint32_t s0 = lut3<kLe1>(a0, h0[j], c0), s1 = lut3<kNae>(a0, h0[j], c0);
    const uint32_t s2 = lut3<kLe1>(a1, h1[j], c1), s3 = lut3<kEven>(a1, h1[j], c1);
    const uint32_t t1 = lut3<kT1>(s0, s1, r[j]);
    const uint32_t t2 = lut3<kT2>(s2, r[j], t1);
    r[j] = lut3<kT3>(s1, s3, t2);
  }
}

// k_step for the split layouts: wave w takes G groups of P = S/2
// consecutive universes, grid-strided; all branches wave-uniform.
template <int S, int G, bool NT>
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
    for (uint32_t it = 0; it < gens; ++it) {
#pragma unroll
      for (int g = 0; g < G; ++g) gen_split<S>(r[g], lds + (wib * G + g) * S * kWave, lane);
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

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// ------------------------------------------------------------------------
// RLE batch I/O (Parsing.hpp:143-204), one wave per pattern
// ------------------------------------------------------------------------

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, int lane) {
  uint32_t inc = v;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const uint32_t t = __shfl_up(inc, off, kWave);
    if (lane >= off) inc += t;
  }
  return inc - v;
}
__device__ __forceinline__ uint64_t below_lane(int lane) { return (1ull << lane) - 1; }
__device__ __forceinline__ int last_set(uint64_t m) { return m ? 63 - __builtin_clzll(m) : -1; }

// LifeState::RLE() prints row y = (j + 32) & 63 as output row j, cells from
// x = 32 (GenericRLE, Parsing.hpp:13-16).  Lane j gets output row j with bit
// i = cell x = (i + 32) & 63: a 64x64 bit transpose by 64 ballots.
__device__ __forceinline__ uint64_t rle_row(uint64_t col, int lane) {
  uint64_t mine = 0;
  for (int j = 0; j < kWave; ++j) {
    const uint64_t m = __ballot((col >> ((j + 32) & 63)) & 1);
    if (lane == j) mine = (m >> 32) | (m << 32);
  }
  return mine;
}

// One output row's tokens (GenericRLE's loop body, Parsing.hpp:18-50): "<k>$"
// before the row's first live cell (k = rows since the last flush, omitted
// when 1), then "<n>o" / "<n>b" runs (n omitted when 1), a dead run that
// ends the row dropped.  Counts are at most 64, so at most two digits.
// Returns the byte count; writes them when WRITE.
template <bool WRITE>
__device__ uint32_t rle_row_tokens(uint64_t r, uint32_t eol, char *out) {
  uint32_t n = 0;
  auto count = [&](uint32_t c) {
    if (c <= 1) return;
    if (c >= 10) {
      if (WRITE) out[n] = (char)('0' + c / 10);
      ++n;
    }
    if (WRITE) out[n] = (char)('0' + c % 10);
    ++n;
  };
  if (r == 0) return 0;
  if (eol) {
    count(eol);
    if (WRITE) out[n] = '$';
    ++n;
  }
  uint32_t pos = 0, v = (uint32_t)(r & 1);
  while (pos < 64) {
    const uint64_t rest = r >> pos;
    const uint64_t ends = v ? ~rest : rest;  // first cell of the other value
    const uint32_t len = ends ? (uint32_t)__builtin_ctzll(ends) : 64u - pos;
    const uint32_t run = len < 64u - pos ? len : 64u - pos;
    if (!v && pos + run >= 64) break;  // dead run to the end of the row
    count(run);
    if (WRITE) out[n] = v ? 'o' : 'b';
    ++n;
    pos += run;
    v ^= 1u;
  }
  return n;
}

// longest RLE() of a 64x64 board: per row at most a 3-byte "<k>$" and 64
// bytes of runs (a run of n cells costs at most n bytes), then "!"
constexpr uint32_t kRleMaxBytes = 64 * (3 + 64) + 1 + 63;

// WRITE = false: len[u] = strlen(RLE()); WRITE = true: RLE() at text + offs[u]
template <bool WRITE>
__global__ __launch_bounds__(kBlock) void k_rle(const uint64_t *__restrict__ s, uint32_t *__restrict__ len,
                                                const uint64_t *__restrict__ offs, char *__restrict__ text,
                                                uint64_t n) {
  // the pattern is assembled in LDS and then copied out 64 consecutive bytes
  // per store (the rows' tokens land at scattered offsets)
  __shared__ char stage_all[WRITE ? kWavesPerBlock : 1][WRITE ? kRleMaxBytes : 1];
  char *stage = stage_all[WRITE ? threadIdx.x / kWave : 0];
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t u = (uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave; u < n; u += stride) {
    const uint64_t r = rle_row(s[u * kWave + lane], lane);
    // rows since the previous live row (or since the top): GenericRLE's eol_count
    const int prev = last_set(__ballot(r != 0) & below_lane(lane));
    const uint32_t eol = (uint32_t)(lane - (prev < 0 ? 0 : prev));
    const uint32_t mine = rle_row_tokens<false>(r, eol, nullptr);
    if constexpr (!WRITE) {
      const uint32_t total = wave_sum_u32(mine) + 1;  // + "!"
      if (lane == 0) len[u] = total;
    } else {
      const uint32_t at = wave_excl_scan(mine, lane);
      rle_row_tokens<true>(r, eol, stage + at);
      if (lane == kWave - 1) stage[at + mine] = '!';
      const uint32_t total = __shfl(at + mine, kWave - 1, kWave) + 1;
      char *base = text + offs[u];
      for (uint32_t i = lane; i < total; i += kWave) base[i] = stage[i];
    }
  }
}

// LifeState::Parse (GenericParse, Parsing.hpp:143-198) of text[offs[u],
// offs[u+1]), 64 bytes per step, one byte per lane:
//  * a line whose first byte is 'x' is dropped (:148-151); '\n' goes with it
//    (getline), '\r' and ' ' are skipped (:181-182);
//  * a decimal count accumulates across skipped bytes and lines (:164-166);
//  * '$' moves down count rows (0 -> 1), a count of 129 ends the parse
//    (:171-173); '!' ends it (:178-179);
//  * any other byte is a run of count cells (0 -> 1), live iff 'o' (:196).
// Per step: ballots give the line starts, kept bytes, digit and tag masks;
// each tag's count comes from the digit bit planes; wave scans give every
// tag's (x, y); every 'o' run ORs its cells into its row in LDS (one
// ds_or_b64 for all runs of the step), and the rows are turned into
// columns at the end.  status[u] bit 0: a live cell fell off the 64x64 board and was
// dropped (the reference writes out of bounds there); bit 1: stopped by a
// "$" count of 129.
__global__ __launch_bounds__(kBlock) void k_parse_rle(const char *__restrict__ text,
                                                      const uint64_t *__restrict__ offs,
                                                      uint64_t *__restrict__ out, uint8_t *__restrict__ status,
                                                      uint64_t n) {
  __shared__ uint64_t board[kWavesPerBlock][kWave];  // row y of this wave's pattern
  const int lane = threadIdx.x & (kWave - 1);
  uint64_t *rows = board[threadIdx.x / kWave];
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t u = (uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave; u < n; u += stride) {
    const uint64_t b = offs[u], e = offs[u + 1] > b ? offs[u + 1] : b;
    rows[lane] = 0;
    int64_t x = 0, y = 0;
    uint32_t cnt = 0, st = 0;
    bool line_start = true, header = false, done = false, off_board = false;
    for (uint64_t p0 = b; p0 < e && !done; p0 += kWave) {
      const uint64_t p = p0 + lane;
      const bool valid = p < e;
      const uint32_t c = valid ? (uint32_t)(uint8_t)text[p] : 0u;
      // header lines: first byte of my line
      const int nl_before = last_set(__ballot(valid && c == '\n') & below_lane(lane));
      const uint32_t first = __shfl(c, nl_before < 0 ? 0 : nl_before + 1, kWave);
      const bool hdr = nl_before >= 0 ? first == 'x' : (line_start ? first == 'x' : header);
      const bool kept = valid && c != '\n' && !hdr && c != '\r' && c != ' ';
      const bool dig = kept && c >= '0' && c <= '9';
      const bool tag = kept && !dig;
      const uint64_t D = __ballot(dig), T = __ballot(tag);
      const uint32_t dv = dig ? c - '0' : 0u;
      const uint64_t d0 = __ballot(dv & 1), d1 = __ballot(dv & 2), d2 = __ballot(dv & 4), d3 = __ballot(dv & 8);
      auto digits_value = [&](uint64_t m, uint32_t v) {  // digits in m, ascending, after v
        for (; m; m &= m - 1) {
          const int k = __builtin_ctzll(m);
          v = v * 10u + (uint32_t)(((d0 >> k) & 1) | ((d1 >> k) & 1) << 1 | ((d2 >> k) & 1) << 2 |
                                   ((d3 >> k) & 1) << 3);
        }
        return v;
      };
      auto after = [](int k) { return k < 0 ? ~0ull : ~((2ull << k) - 1); };
      // this tag's count: digits since the previous tag (or carried in)
      const int pt = last_set(T & below_lane(lane));
      uint32_t v = 0;
      if (tag) v = digits_value(D & below_lane(lane) & after(pt), pt < 0 ? cnt : 0u);
      const uint32_t cv = v == 0 ? 1u : v;
      const uint64_t S = __ballot(tag && (c == '!' || (c == '$' && cv == 129)));
      const uint64_t live_tags = S ? T & below_lane(__builtin_ctzll(S)) : T;
      const bool active = (live_tags >> lane) & 1;
      const bool dollar = active && c == '$';
      const bool cell = active && c != '$';
      const uint32_t dy = dollar ? cv : 0u, dx = cell ? cv : 0u;
      const uint32_t ey = wave_excl_scan(dy, lane), ex = wave_excl_scan(dx, lane);
      const uint64_t Dl = __ballot(dollar);
      const int ld = last_set(Dl & below_lane(lane));
      const uint32_t ex_ld = __shfl(ex, ld < 0 ? 0 : ld, kWave);
      const int64_t my_y = y + ey;
      const int64_t my_x = ld < 0 ? x + ex : (int64_t)(ex - ex_ld);
      if (cell && c == 'o') {  // each 'o' run ORs its cells into its row of the board
        if (my_y < 0 || my_y >= 64 || my_x < 0 || my_x + cv > 64) off_board = true;
        if (my_y >= 0 && my_y < 64 && my_x >= 0 && my_x < 64) {
          const uint64_t end = my_x + cv < 64 ? my_x + cv : 64;
          const uint64_t hi = end == 64 ? ~0ull : (1ull << end) - 1;
          __hip_atomic_fetch_or(&rows[my_y], hi & ~((1ull << my_x) - 1), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      // carry to the next 64 bytes
      const uint32_t ey_all = __shfl(ey + dy, kWave - 1, kWave), ex_all = __shfl(ex + dx, kWave - 1, kWave);
      const int lda = last_set(Dl);
      y += ey_all;
      x = lda < 0 ? x + ex_all : (int64_t)(ex_all - __shfl(ex, lda < 0 ? 0 : lda, kWave));
      if (S) {
        done = true;
        const int k = __builtin_ctzll(S);
        if (__shfl(c, k, kWave) == '$') st |= 2u;
      } else {
        const int lt = last_set(T);
        cnt = digits_value(D & after(lt), lt < 0 ? cnt : 0u);
      }
      line_start = __shfl(c, kWave - 1, kWave) == '\n';
      header = __shfl((uint32_t)hdr, kWave - 1, kWave) != 0;
    }
    // rows -> columns: lane x collects bit x of every row
    uint64_t word = 0;
#pragma unroll 8
    for (int r = 0; r < kWave; ++r) word |= ((rows[r] >> lane) & 1ull) << r;
    if (__ballot(off_board)) st |= 1u;
    out[u * kWave + lane] = word;
    if (lane == 0) status[u] = (uint8_t)st;
  }
}

// The per-universe reductions below take kRedU universes per wave, all loads
// issued before the first reduction (one wave per universe and a grid-stride
// loop left them latency-bound at 36-60 % of HBM, tools/rows_bench.py).
constexpr int kRedU = 4;

// GetPop (LifeAPI.hpp:290-298): two universes' popcounts per 32-bit reduction
__global__ __launch_bounds__(kBlock) void k_pop(const uint64_t *__restrict__ s,
                                                uint32_t *__restrict__ pop, uint64_t n) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * kRedU;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave) * kRedU; u0 < n;
       u0 += stride) {
    uint32_t c[kRedU];
#pragma unroll
    for (int k = 0; k < kRedU; ++k) c[k] = u0 + k < n ? (uint32_t)__popcll(s[(u0 + k) * kWave + lane]) : 0u;
#pragma unroll
    for (int k = 0; k < kRedU; k += 2) {
      const uint32_t t = wave_sum_u32(c[k] | c[k + 1] << 16);  // each sum <= 4096
      if (lane == 0) {
        if (u0 + k < n) pop[u0 + k] = t & 0xFFFF;
        if (u0 + k + 1 < n) pop[u0 + k + 1] = t >> 16;
      }
    }
  }
}

// build-defined universe hash: mix(sum_x mix(s[x] + (x+1)*G))
__global__ __launch_bounds__(kBlock) void k_hash(const uint64_t *__restrict__ s,
                                                 uint64_t *__restrict__ h, uint64_t n) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * kRedU;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave) * kRedU; u0 < n;
       u0 += stride) {
    uint64_t m[kRedU];
#pragma unroll
    for (int k = 0; k < kRedU; ++k) m[k] = u0 + k < n ? s[(u0 + k) * kWave + lane] : 0ull;
#pragma unroll
    for (int k = 0; k < kRedU; ++k) {
      const uint64_t t = wave_sum_u64(mix64(m[k] + (uint64_t)(lane + 1) * kGolden));
      if (lane == 0 && u0 + k < n) h[u0 + k] = mix64(t);
    }
  }
}

// Contains(LifeTarget) (LifeTarget.hpp:44-51): (s ^ w) & (w | u) == 0 on all columns
__device__ __forceinline__ bool wave_contains(W s, W w, W u) {
  const uint32_t dlo = (s.lo ^ w.lo) & (w.lo | u.lo), dhi = (s.hi ^ w.hi) & (w.hi | u.hi);
  return __ballot((dlo | dhi) != 0u) == 0ull;
}

__global__ __launch_bounds__(kBlock) void k_contains(const uint64_t *__restrict__ s,
                                                     const uint64_t *__restrict__ wanted,
                                                     const uint64_t *__restrict__ unwanted,
                                                     uint8_t *__restrict__ out, uint64_t n) {
  const int lane = threadIdx.x & (kWave - 1);
  const W w = split(wanted[lane]), uw = split(unwanted[lane]);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * kRedU;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave) * kRedU; u0 < n;
       u0 += stride) {
    W a[kRedU];
#pragma unroll
    for (int k = 0; k < kRedU; ++k) a[k] = u0 + k < n ? split(s[(u0 + k) * kWave + lane]) : W{0u, 0u};
#pragma unroll
    for (int k = 0; k < kRedU; ++k) {
      const bool c = wave_contains(a[k], w, uw);
      if (lane == 0 && u0 + k < n) out[u0 + k] = c ? 1 : 0;
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
// universe-generation on top of the 20 of the step (+25 % measured,
// profiles/r01/contains_bench.jsonl); branching around the bookkeeping
// when no universe is clean measured slower still.
// Without d_final, a wave stops once all its universes have hit.
constexpr uint32_t kDiff = ((TA ^ TB) & (TB | TC)) & 0xFF;  // (s ^ wanted) & (wanted | unwanted)
template <int S>
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
    for (uint32_t g = 1; g <= gens; ++g) {
      gen_split<S>(r, lds + wib * S * kWave, lane);
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
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_counts(const uint64_t *__restrict__ in,
                                                   uint64_t *__restrict__ out, uint64_t n) {
  constexpr int P = MODE == 1 ? 3 : 4;
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t u = (uint64_t)blockIdx.x * kWavesPerBlock + wib; u < n; u += stride) {
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

__global__ __launch_bounds__(kBlock) void k_weld(uint64_t *__restrict__ welds, uint64_t n,
                                                 uint32_t gens) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t u = (uint64_t)blockIdx.x * kWavesPerBlock + wib; u < n; u += stride) {
    uint64_t *p = welds + u * 4 * kWave + lane;
    W s = ld<false>(p);
    const W f2 = ld<false>(p + kWave), f1 = ld<false>(p + 2 * kWave), f0 = ld<false>(p + 3 * kWave);
    for (uint32_t g = 0; g < gens; ++g) s = weld_gen(s, f2, f1, f0);
    st<false>(p, s);
  }
}

// ---- LifeStable passes --------------------------------
// One wave per LifeStable: lane x holds column x of its 10 planes {state,
// unknown, live2, live3, dead0, dead1, dead2, dead4, dead5, dead6}
// (LifeStable.hpp:41-53; options "1 = ruled out").  The espresso fragments
// the passes #include (bitslicing/stable_count.hpp, stable_signal.hpp) are
// v_bitop3 networks generated by tools/synth_sop.py from their complete
// truth tables.  Whole-universe tests (abort, changed) are wave ballots.

__device__ __forceinline__ W operator&(W a, W b) { return W{a.lo & b.lo, a.hi & b.hi}; }
__device__ __forceinline__ W operator|(W a, W b) { return W{a.lo | b.lo, a.hi | b.hi}; }
__device__ __forceinline__ W operator~(W a) { return W{~a.lo, ~a.hi}; }
__device__ __forceinline__ bool wave_any(W a) { return __ballot((a.lo | a.hi) != 0u) != 0ull; }

// all four bits of the inclusive 3x3 count (NeighbourCount.hpp:40-70)
__device__ __forceinline__ void ncount4(W a, W &b3, W &b2, W &b1, W &b0) {
  W L, R;
  neighbour_cols<XDPP>(a, L, R, nullptr, 0);
  const W h0 = lut3<kXor3>(L, a, R), h1 = lut3<kMaj>(L, a, R);
  const W h0u = rot_up(h0), h0d = rot_dn(h0), h1u = rot_up(h1), h1d = rot_dn(h1);
  const W fs = lut3<kXor3>(h0u, h0, h0d), fc = lut3<kMaj>(h0u, h0, h0d);
  const W cs = lut3<kXor3>(h1u, h1, h1d), cc = lut3<kMaj>(h1u, h1, h1d);
  constexpr uint32_t kAnd3 = (TA & TB & TC) & 0xFF;
  b0 = fs;
  b1 = W{fc.lo ^ cs.lo, fc.hi ^ cs.hi};
  b2 = lut3<kCarry2>(cc, fc, cs);
  b3 = lut3<kAnd3>(cc, fc, cs);
}

// LifeState::ZOIHollow (LifeAPI.hpp:541-562): the 8 neighbours' OR
__device__ __forceinline__ W zoi_hollow(W s) {
  const W m = rot_up(s) | rot_dn(s);
  const W t = s | m;
  W L, R;
  neighbour_cols<XDPP>(t, L, R, nullptr, 0);
  return L | m | R;
}

template <class T>
__device__ __forceinline__ void stable_count_circuit(const T (&x)[9], T &l2, T &l3, T &d0, T &d1,
                                                     T &d2, T &d4, T &d5, T &d6, T &abort) {
#include "stable_count_circuit.inc"
}
template <class T>
__device__ __forceinline__ void stable_signal_circuit(const T (&x)[17], T &signaloff, T &signalon,
                                                      T &centeroff, T &centeron) {
#include "stable_signal_circuit.inc"
}

enum { PST, PUN, PL2, PL3, PD0, PD1, PD2, PD4, PD5, PD6 };

// SynchroniseStateKnown, LifeStable.hpp:526-556
__device__ __forceinline__ int stable_sync(W (&p)[10]) {
  const W known_on = ~p[PUN] & p[PST];
  const W maybe_dead = ~(p[PD0] & p[PD1] & p[PD2] & p[PD4] & p[PD5] & p[PD6]);
  W changes = maybe_dead & known_on;
#pragma unroll
  for (int k = PD0; k <= PD6; ++k) p[k] = p[k] | known_on;
  const W known_off = ~p[PUN] & ~p[PST];
  const W maybe_live = ~(p[PL2] & p[PL3]);
  changes = changes | (maybe_live & known_off);
  p[PL2] = p[PL2] | known_off;
  p[PL3] = p[PL3] | known_off;
  if (wave_any(~maybe_live & ~maybe_dead)) return 0;
  changes = changes | (~p[PST] & (maybe_live & ~maybe_dead));
  p[PST] = p[PST] | (maybe_live & ~maybe_dead);
  changes = changes | (~p[PUN] & (maybe_live & maybe_dead));
  p[PUN] = p[PUN] & (maybe_live & maybe_dead);
  return 1 | (wave_any(changes) ? 2 : 0);
}

// UpdateOptions, LifeStable.hpp:558-615 (stable_count.hpp at :591)
__device__ __forceinline__ int stable_options(W (&p)[10]) {
  const W off = ~p[PUN] & ~p[PST];
  W s3, s2, s1, s0, o3, o2, o1, o0;
  ncount4(p[PST], s3, s2, s1, s0);
  ncount4(off, o3, o2, o1, o0);
  const W x[9] = {s2, s1, s0, o3, o2, o1, o0, p[PST], off};
  W r[8], ab;
  stable_count_circuit(x, r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7], ab);
  W changes = W{0u, 0u};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    changes = changes | (r[k] & ~p[PL2 + k]);
    p[PL2 + k] = p[PL2 + k] | r[k];
  }
  return (wave_any(ab) ? 0 : 1) | (wave_any(changes) ? 2 : 0);
}

// SignalNeighbours, LifeStable.hpp:617-675 (stable_signal.hpp at :654),
// then SetOff / SetOn (:320-335)
__device__ __forceinline__ int stable_signal(W (&p)[10]) {
  W s3, s2, s1, s0, m3, m2, m1, m0;
  ncount4(p[PST], s3, s2, s1, s0);
  ncount4(p[PST] | p[PUN], m3, m2, m1, m0);
  const W x[17] = {p[PL2], p[PL3], p[PD0], p[PD1], p[PD2], p[PD4], p[PD5], p[PD6], s2, s1, s0,
                   m3, m2, m1, m0, p[PST], p[PUN]};
  W soff, son, coff, con;
  stable_signal_circuit(x, soff, son, coff, con);
  const W off_zoi = zoi_hollow(soff) | coff, on_zoi = zoi_hollow(son) | con;
  if (wave_any(off_zoi & on_zoi & p[PUN])) return 0;
  const W changes = (off_zoi & p[PUN]) | (on_zoi & p[PUN]);
  const W w_off = off_zoi & p[PUN];
  p[PST] = p[PST] & ~w_off;
  p[PUN] = p[PUN] & ~w_off;
  p[PL2] = p[PL2] | w_off;
  p[PL3] = p[PL3] | w_off;
  const W w_on = on_zoi & p[PUN];
  p[PST] = p[PST] | w_on;
  p[PUN] = p[PUN] & ~w_on;
#pragma unroll
  for (int k = PD0; k <= PD6; ++k) p[k] = p[k] | w_on;
  return 1 | (wave_any(changes) ? 2 : 0);
}

// PropagateStep, LifeStable.hpp:695-716
__device__ __forceinline__ int stable_step(W (&p)[10]) {
  const int k = stable_sync(p);
  if (!(k & 1)) return 0;
  const int o = stable_options(p);
  if (!(o & 1)) return 0;
  const int s = stable_signal(p);
  if (!(s & 1)) return 0;
  return 1 | ((k | o | s) & 2);
}

// PASS 0..3: one pass; 4: Propagate (LifeStable.hpp:718-729), at most
// max_iters PropagateSteps (flag bit 2 set if that bound stopped it).
template <int PASS>
__global__ __launch_bounds__(kBlock) void k_stable(uint64_t *__restrict__ planes,
                                                   uint8_t *__restrict__ flags, uint64_t n,
                                                   uint32_t max_iters) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t u = (uint64_t)blockIdx.x * kWavesPerBlock + wib; u < n; u += stride) {
    uint64_t *q = planes + u * 10 * kWave + lane;
    W p[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) p[k] = ld<false>(q + k * kWave);
    int r;
    if constexpr (PASS == 0) r = stable_sync(p);
    else if constexpr (PASS == 1) r = stable_options(p);
    else if constexpr (PASS == 2) r = stable_signal(p);
    else if constexpr (PASS == 3) r = stable_step(p);
    else {
      int ever = 0;
      r = -1;
      for (uint32_t it = 0; it < max_iters; ++it) {
        const int s = stable_step(p);
        if (!(s & 1)) { r = 0; break; }
        if (!(s & 2)) { r = 1 | ever; break; }
        ever = 2;
      }
      if (r < 0) r = 1 | ever | 4;
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) st<false>(q + k * kWave, p[k]);
    if (lane == 0) flags[u] = (uint8_t)r;
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
template <int PF, int OCC>
__global__ __launch_bounds__(kBlock, OCC > 0 ? OCC : 1) void k_refined(
    const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t n) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  uint64_t u = (uint64_t)blockIdx.x * kWavesPerBlock + wib;
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

__global__ __launch_bounds__(kBlock) void k_fill(uint64_t *__restrict__ out, uint64_t nwords,
                                                 uint64_t seed, uint64_t first_word, int mode) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nwords; i += stride) {
    uint64_t v = mix64(seed + (first_word + i + 1) * kGolden);
    if (mode == 1) v = (v & ((1ULL << 61) - 1)) | (1ULL << 61);
    __builtin_nontemporal_store(v, out + i);
  }
}

// ------------------------------------------------------------------------
// host side: errors, device info, dispatch
// ------------------------------------------------------------------------

thread_local std::string g_err;

int fail(int code, const char *fmt, const char *arg = nullptr) {
  char buf[512];
  std::snprintf(buf, sizeof buf, fmt, arg ? arg : "");
  g_err = buf;
  return code;
}
int fail_hip(hipError_t e, const char *what) {
  char buf[512];
  std::snprintf(buf, sizeof buf, "%s: %s (hipError %d)", what, hipGetErrorString(e), (int)e);
  g_err = buf;
  if (e == hipErrorNoBinaryForGpu || e == hipErrorInvalidDeviceFunction ||
      e == hipErrorInvalidImage || e == hipErrorSharedObjectInitFailed)
    return LIFEAPI_E_NOKERNEL;
  return (int)e;
}

struct DevInfo {
  int cus = 0;
  bool ok = false;
};
std::mutex g_info_mu;
std::vector<DevInfo> g_info;

int device_cus(int &cus) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return fail_hip(e, "hipGetDevice");
  std::lock_guard<std::mutex> lk(g_info_mu);
  if ((int)g_info.size() <= dev) g_info.resize(dev + 1);
  if (!g_info[dev].ok) {
    hipDeviceProp_t p;
    e = hipGetDeviceProperties(&p, dev);
    if (e != hipSuccess) return fail_hip(e, "hipGetDeviceProperties");
    if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
      return fail(LIFEAPI_E_NODEVICE, "device is %s, this library is built for gfx950 only",
                  p.gcnArchName);
    g_info[dev].cus = p.multiProcessorCount;
    g_info[dev].ok = true;
  }
  cus = g_info[dev].cus;
  return LIFEAPI_OK;
}

bool aligned8(const void *p) { return ((uintptr_t)p & 7u) == 0; }

int check_batch(const void *in, const void *out, size_t n) {
  if (n == 0) return LIFEAPI_OK;
  if (!in || !out) return fail(LIFEAPI_E_INVALID, "null universe pointer%s");
  if (!aligned8(in) || !aligned8(out)) return fail(LIFEAPI_E_INVALID, "universe pointers must be 8-byte aligned%s");
  if (n > (SIZE_MAX / 512)) return fail(LIFEAPI_E_INVALID, "n too large%s");
  const uintptr_t a = (uintptr_t)in, b = (uintptr_t)out, bytes = (uintptr_t)n * 512u;
  if (a != b && a < b + bytes && b < a + bytes)
    return fail(LIFEAPI_E_INVALID, "input and output batches overlap (only in == out is allowed)%s");
  return LIFEAPI_OK;
}

unsigned grid_for(uint64_t waves_needed, int cus, int blocks_per_cu) {
  uint64_t blocks = (waves_needed + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks_per_cu > 0) blocks = std::min<uint64_t>(blocks, (uint64_t)cus * blocks_per_cu);
  blocks = std::min<uint64_t>(blocks, 1u << 30);
  return (unsigned)std::max<uint64_t>(blocks, 1);
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
template <int S>
StepFn pick_split(int groups, bool nt) {
  switch (groups) {
    case 1: return nt ? k_step_split<S, 1, true> : k_step_split<S, 1, false>;
    case 2: return nt ? k_step_split<S, 2, true> : k_step_split<S, 2, false>;
    default: return nullptr;
  }
}
// universes one wave holds per universes_per_wave unit (rules 5, 6: groups)
int group_size(int rule) { return rule == 5 ? 2 : rule == 6 ? 4 : rule == 7 ? 8 : 1; }

StepFn pick_step(const lifeapi_launch_cfg &c) {
  if (c.rule >= 5 && c.rule <= 7) {  // split layouts: LDS exchange only
    if (c.xchg != LIFEAPI_XCHG_LDS) return nullptr;
    const bool nt = c.nontemporal != 0;
    return c.rule == 5 ? pick_split<4>(c.universes_per_wave, nt)
         : c.rule == 6 ? pick_split<8>(c.universes_per_wave, nt)
                       : pick_split<16>(c.universes_per_wave, nt);
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

int launched(const char *what) {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? LIFEAPI_OK : fail_hip(e, what);
}

// ---- host-pointer staging: one context per device ----
struct HostCtx {
  std::mutex mu;
  hipStream_t stream = nullptr;
  char *buf = nullptr;
  size_t cap = 0;  // bytes
};
std::mutex g_ctx_mu;
std::vector<HostCtx *> g_ctx;

HostCtx *ctx_for(int dev) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  if ((int)g_ctx.size() <= dev) g_ctx.resize(dev + 1, nullptr);
  if (!g_ctx[dev]) g_ctx[dev] = new HostCtx();  // lives for the process
  return g_ctx[dev];
}

struct DeviceGuard {
  int prev = -1;
  DeviceGuard() { (void)hipGetDevice(&prev); }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

constexpr size_t kStagingBytes = size_t(1) << 30;  // device staging per pass (1 GiB)

// One host array taking part in a host-pointer call: `bytes` per universe;
// src -> copied in before each chunk's launch, dst -> copied out after it
// (src == dst for in-place arrays).
struct HostIO {
  const void *src;
  void *dst;
  size_t bytes;
};
using ChunkFn = int (*)(void *const *dev, size_t m, hipStream_t s, const void *arg);

// Stages n universes through this device's reusable buffer in chunks of at
// most kStagingBytes: H2D, the stream-ordered *_dev entry point, D2H, sync.
int host_chunked(int dev, size_t n, const HostIO *io, int nio, ChunkFn fn, const void *arg) {
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return fail_hip(e, "hipSetDevice");
  HostCtx *c = ctx_for(dev);
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->stream) {
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) return fail_hip(e, "hipStreamCreate");
  }
  size_t per = 0;
  for (int k = 0; k < nio; ++k) per += (io[k].bytes + 255) & ~size_t(255);
  const size_t chunk = std::max<size_t>(1, std::min(n, kStagingBytes / per));
  size_t need = 0;
  for (int k = 0; k < nio; ++k) need += ((io[k].bytes * chunk + 255) & ~size_t(255));
  if (c->cap < need) {
    if (c->buf) (void)hipFree(c->buf);
    c->buf = nullptr;
    c->cap = 0;
    e = hipMalloc(&c->buf, need);
    if (e != hipSuccess) return fail_hip(e, "hipMalloc(staging)");
    c->cap = need;
  }
  void *d[8];
  for (size_t off = 0; off < n; off += chunk) {
    const size_t m = std::min(chunk, n - off);
    size_t pos = 0;
    for (int k = 0; k < nio; ++k) {
      d[k] = c->buf + pos;
      pos += (io[k].bytes * chunk + 255) & ~size_t(255);
      if (io[k].src) {
        e = hipMemcpyAsync(d[k], (const char *)io[k].src + off * io[k].bytes, m * io[k].bytes,
                           hipMemcpyHostToDevice, c->stream);
        if (e != hipSuccess) return fail_hip(e, "hipMemcpyAsync(H2D)");
      }
    }
    const int rc = fn(d, m, c->stream, arg);
    if (rc != LIFEAPI_OK) return rc;
    for (int k = 0; k < nio; ++k)
      if (io[k].dst) {
        e = hipMemcpyAsync((char *)io[k].dst + off * io[k].bytes, d[k], m * io[k].bytes,
                           hipMemcpyDeviceToHost, c->stream);
        if (e != hipSuccess) return fail_hip(e, "hipMemcpyAsync(D2H)");
      }
    e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return fail_hip(e, "hipStreamSynchronize");
  }
  return LIFEAPI_OK;
}

int host_device(int device) {
  const int ndev = lifeapi_device_count();
  if (ndev <= 0) return fail(LIFEAPI_E_NODEVICE, "no HIP device visible%s");
  if (device < 0) device = 0;
  if (device >= ndev) return fail(LIFEAPI_E_NODEVICE, "bad device index%s");
  return device;
}

int host_step_one_device(const uint64_t *in, uint64_t *out, size_t n, uint32_t gens, int dev) {
  const HostIO io[1] = {{in, out, 512}};
  return host_chunked(dev, n, io, 1,
                      [](void *const *d, size_t m, hipStream_t s, const void *arg) {
                        return lifeapi_step_batch_dev((const uint64_t *)d[0], (uint64_t *)d[0], m,
                                                      *(const uint32_t *)arg, s);
                      },
                      &gens);
}

}  // namespace

// ==========================================================================
// C ABI
// ==========================================================================

extern "C" {

int lifeapi_abi_version(void) { return LIFEAPI_ABI_VERSION; }

const char *lifeapi_last_error(void) { return g_err.c_str(); }

int lifeapi_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

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
    // bit, LDS exchange; state resident in VGPRs for all generations
    cfg->xchg = LIFEAPI_XCHG_LDS;
    cfg->rule = 6;
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

int lifeapi_pop_batch_dev(const uint64_t *d_states, uint32_t *d_pop, size_t n, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_states || !d_pop || !aligned8(d_states) || ((uintptr_t)d_pop & 3u))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_pop_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(k_pop, dim3(grid_for((n + kRedU - 1) / kRedU, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_states, d_pop, (uint64_t)n);
  return launched("k_pop launch");
}

int lifeapi_hash_batch_dev(const uint64_t *d_states, uint64_t *d_hash, size_t n, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_states || !d_hash || !aligned8(d_states) || !aligned8(d_hash))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_hash_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(k_hash, dim3(grid_for((n + kRedU - 1) / kRedU, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_states, d_hash, (uint64_t)n);
  return launched("k_hash launch");
}

int lifeapi_contains_batch_dev(const uint64_t *d_states, const uint64_t *d_wanted,
                               const uint64_t *d_unwanted, uint8_t *d_out, size_t n,
                               void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_states || !d_wanted || !d_unwanted || !d_out || !aligned8(d_states) ||
      !aligned8(d_wanted) || !aligned8(d_unwanted))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_contains_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(k_contains, dim3(grid_for((n + kRedU - 1) / kRedU, cus, 0)), dim3(kBlock), 0,
                     (hipStream_t)stream, d_states, d_wanted, d_unwanted, d_out, (uint64_t)n);
  return launched("k_contains launch");
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
    hipLaunchKernelGGL(k_step_contains_split<8>, dim3(grid_for((n + 3) / 4, cus, 0)), dim3(kBlock), 0,
                       (hipStream_t)stream, d_in, d_final, d_wanted, d_unwanted, d_first_gen,
                       (uint64_t)n, generations);
  } else {
    hipLaunchKernelGGL(k_step_contains, dim3(grid_for(n, cus, 0)), dim3(kBlock), 0,
                       (hipStream_t)stream, d_in, d_final, d_wanted, d_unwanted, d_first_gen,
                       (uint64_t)n, generations);
  }
  return launched("k_step_contains launch");
}

int lifeapi_rle_lengths_batch_dev(const uint64_t *d_states, uint32_t *d_len, size_t n, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_states || !d_len || !aligned8(d_states) || ((uintptr_t)d_len & 3u))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_rle_lengths_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(k_rle<false>, dim3(grid_for(n, cus, 8)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_states, d_len, nullptr, nullptr, (uint64_t)n);
  return launched("k_rle launch");
}

int lifeapi_rle_write_batch_dev(const uint64_t *d_states, const uint64_t *d_offsets, char *d_text,
                                size_t n, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_states || !d_offsets || !d_text || !aligned8(d_states) || !aligned8(d_offsets))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_rle_write_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(k_rle<true>, dim3(grid_for(n, cus, 8)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_states, nullptr, d_offsets, d_text, (uint64_t)n);
  return launched("k_rle launch");
}

int lifeapi_parse_rle_batch_dev(const char *d_text, const uint64_t *d_offsets, size_t n, uint64_t *d_out,
                                uint8_t *d_status, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_text || !d_offsets || !d_out || !d_status || !aligned8(d_offsets) || !aligned8(d_out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_parse_rle_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(k_parse_rle, dim3(grid_for(n, cus, 8)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_text, d_offsets, d_out, d_status, (uint64_t)n);
  return launched("k_parse_rle launch");
}

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
  hipLaunchKernelGGL(fn, dim3(grid_for(n, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream, d_in,
                     d_out, (uint64_t)n);
  return launched("k_counts launch");
}

int lifeapi_stable_pass_batch_dev(uint64_t *d_planes, uint8_t *d_flags, size_t n, int pass,
                                  uint32_t max_iters, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_planes || !d_flags || !aligned8(d_planes) || pass < 0 || pass > 4)
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_stable_pass_batch_dev%s");
  const uintptr_t a = (uintptr_t)d_planes, b = (uintptr_t)d_flags;
  if (b < a + n * 10 * 512 && a < b + n) return fail(LIFEAPI_E_INVALID, "flags overlap planes%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  using Fn = void (*)(uint64_t *, uint8_t *, uint64_t, uint32_t);
  const Fn fns[5] = {k_stable<0>, k_stable<1>, k_stable<2>, k_stable<3>, k_stable<4>};
  hipLaunchKernelGGL(fns[pass], dim3(grid_for(n, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_planes, d_flags, (uint64_t)n, max_iters ? max_iters : 1u << 20);
  return launched("k_stable launch");
}

int lifeapi_weld_step_batch_dev(uint64_t *d_welds, size_t n, uint32_t generations, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_welds || !aligned8(d_welds))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_weld_step_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(k_weld, dim3(grid_for(n, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_welds, (uint64_t)n, generations);
  return launched("k_weld launch");
}

int lifeapi_neighbour_count_batch_dev(const uint64_t *d_in, uint64_t *d_out, size_t n, void *stream) {
  return counts_launch(d_in, d_out, n, 0, stream);
}

int lifeapi_interaction_counts_batch_dev(const uint64_t *d_in, uint64_t *d_out, size_t n,
                                         int with_next, void *stream) {
  return counts_launch(d_in, d_out, n, with_next ? 2 : 1, stream);
}

int lifeapi_refined_step_batch_dev_cfg(const uint64_t *d_in, uint64_t *d_out, size_t n,
                                       void *stream, const lifeapi_launch_cfg *cfg) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_in || !d_out || !aligned8(d_in) || !aligned8(d_out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_refined_step_batch_dev%s");
  const uintptr_t a = (uintptr_t)d_in, b = (uintptr_t)d_out;
  if (a < b + n * 3 * 512 && b < a + n * 11 * 512)
    return fail(LIFEAPI_E_INVALID, "refined step input and output overlap%s");
  // cfg: universes_per_wave 1 = no prefetch, 2 = prefetch next universe;
  // blocks_per_cu = grid cap; rule = minimum waves per SIMD requested from the
  // register allocator (0 = none, 4, 6).  Default = the measured best
  // with the 192-op SOP network (profiles/r01/tune_c5.jsonl): prefetch the
  // next universe, one-shot grid, no occupancy bound -> 6.3 TB/s.
  int pf = 1, bpc = 0, occ = 0;
  if (cfg) {
    pf = cfg->universes_per_wave >= 2 ? 1 : 0;
    bpc = cfg->blocks_per_cu;
    occ = cfg->rule;
    if (occ != 0 && occ != 4 && occ != 6)
      return fail(LIFEAPI_E_INVALID, "unsupported refined cfg%s");
  }
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  using Fn = void (*)(const uint64_t *, uint64_t *, uint64_t);
  Fn fn = pf ? (occ == 4 ? (Fn)k_refined<1, 4> : occ == 6 ? (Fn)k_refined<1, 6> : (Fn)k_refined<1, 0>)
             : (occ == 4 ? (Fn)k_refined<0, 4> : occ == 6 ? (Fn)k_refined<0, 6> : (Fn)k_refined<0, 0>);
  hipLaunchKernelGGL(fn, dim3(grid_for(n, cus, bpc)), dim3(kBlock), 0, (hipStream_t)stream, d_in,
                     d_out, (uint64_t)n);
  return launched("k_refined launch");
}

int lifeapi_refined_step_batch_dev(const uint64_t *d_in, uint64_t *d_out, size_t n, void *stream) {
  return lifeapi_refined_step_batch_dev_cfg(d_in, d_out, n, stream, nullptr);
}

int lifeapi_fill_random_dev(uint64_t *d_out, size_t n, uint64_t seed, uint64_t first_universe,
                            int mode, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_out || !aligned8(d_out) || (mode != 0 && mode != 1))
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_fill_random_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const uint64_t words = (uint64_t)n * kWave;
  hipLaunchKernelGGL(k_fill, dim3(grid_for(words / kWave, cus, 0)), dim3(kBlock), 0,
                     (hipStream_t)stream, d_out, words, seed, first_universe * kWave, mode);
  return launched("k_fill launch");
}

int lifeapi_step_batch(const uint64_t *in, uint64_t *out, size_t n, uint32_t generations,
                       int device) {
  int rc = check_batch(in, out, n);
  if (rc != LIFEAPI_OK || n == 0) return rc;
  const int ndev = lifeapi_device_count();
  if (ndev <= 0) return fail(LIFEAPI_E_NODEVICE, "no HIP device visible%s");
  if (device >= ndev || device < -1) return fail(LIFEAPI_E_NODEVICE, "bad device index%s");
  if (device >= 0 || ndev == 1)
    return host_step_one_device(in, out, n, generations, device < 0 ? 0 : device);
  // every visible device, contiguous shards, one host thread each
  std::vector<int> rcs(ndev, LIFEAPI_OK);
  std::vector<std::string> errs(ndev);
  std::vector<std::thread> pool;
  for (int d = 0; d < ndev; ++d) {
    const size_t lo = n * d / ndev, hi = n * (d + 1) / ndev;
    pool.emplace_back([&, d, lo, hi] {
      if (hi > lo) rcs[d] = host_step_one_device(in + lo * 64, out + lo * 64, hi - lo, generations, d);
      errs[d] = g_err;
    });
  }
  for (auto &t : pool) t.join();
  for (int d = 0; d < ndev; ++d)
    if (rcs[d] != LIFEAPI_OK) {
      g_err = errs[d];
      return rcs[d];
    }
  return LIFEAPI_OK;
}

int lifeapi_pop_batch(const uint64_t *states, uint32_t *pop, size_t n, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!states || !pop || !aligned8(states)) return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_pop_batch%s");
  const int dev = host_device(device);
  if (dev < 0) return dev;
  const HostIO io[2] = {{states, nullptr, 512}, {nullptr, pop, 4}};
  return host_chunked(dev, n, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *) {
                        return lifeapi_pop_batch_dev((const uint64_t *)d[0], (uint32_t *)d[1], m, s);
                      },
                      nullptr);
}

int lifeapi_weld_step_batch(uint64_t *welds, size_t n, uint32_t generations, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!welds || !aligned8(welds)) return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_weld_step_batch%s");
  const int dev = host_device(device);
  if (dev < 0) return dev;
  const HostIO io[1] = {{welds, welds, 4 * 512}};
  return host_chunked(dev, n, io, 1,
                      [](void *const *d, size_t m, hipStream_t s, const void *arg) {
                        return lifeapi_weld_step_batch_dev((uint64_t *)d[0], m, *(const uint32_t *)arg, s);
                      },
                      &generations);
}

int lifeapi_stable_pass_batch(uint64_t *planes, uint8_t *flags, size_t n, int pass,
                              uint32_t max_iters, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!planes || !flags || !aligned8(planes) || pass < 0 || pass > 4)
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_stable_pass_batch%s");
  const int dev = host_device(device);
  if (dev < 0) return dev;
  const uint32_t arg[2] = {(uint32_t)pass, max_iters};
  const HostIO io[2] = {{planes, planes, 10 * 512}, {nullptr, flags, 1}};
  return host_chunked(dev, n, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *a) {
                        const uint32_t *p = (const uint32_t *)a;
                        return lifeapi_stable_pass_batch_dev((uint64_t *)d[0], (uint8_t *)d[1], m,
                                                             (int)p[0], p[1], s);
                      },
                      arg);
}

int lifeapi_neighbour_count_batch(const uint64_t *in, uint64_t *out, size_t n, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!in || !out || !aligned8(in) || !aligned8(out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_neighbour_count_batch%s");
  const int dev = host_device(device);
  if (dev < 0) return dev;
  const HostIO io[2] = {{in, nullptr, 512}, {nullptr, out, 4 * 512}};
  return host_chunked(dev, n, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *) {
                        return lifeapi_neighbour_count_batch_dev((const uint64_t *)d[0], (uint64_t *)d[1], m, s);
                      },
                      nullptr);
}

int lifeapi_interaction_counts_batch(const uint64_t *in, uint64_t *out, size_t n, int with_next,
                                     int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!in || !out || !aligned8(in) || !aligned8(out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_interaction_counts_batch%s");
  const int dev = host_device(device);
  if (dev < 0) return dev;
  const HostIO io[2] = {{in, nullptr, 512}, {nullptr, out, (with_next ? 4u : 3u) * 512}};
  return host_chunked(dev, n, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *a) {
                        return lifeapi_interaction_counts_batch_dev((const uint64_t *)d[0], (uint64_t *)d[1],
                                                                    m, *(const int *)a, s);
                      },
                      &with_next);
}

int lifeapi_refined_step_batch(const uint64_t *in, uint64_t *out, size_t n, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!in || !out || !aligned8(in) || !aligned8(out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_refined_step_batch%s");
  const int dev = host_device(device);
  if (dev < 0) return dev;
  const HostIO io[2] = {{in, nullptr, 11 * 512}, {nullptr, out, 3 * 512}};
  return host_chunked(dev, n, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *) {
                        return lifeapi_refined_step_batch_dev((const uint64_t *)d[0], (uint64_t *)d[1], m, s);
                      },
                      nullptr);
}

int lifeapi_contains_batch(const uint64_t *states, const uint64_t *wanted, const uint64_t *unwanted,
                           uint8_t *out, size_t n, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!states || !wanted || !unwanted || !out || !aligned8(states))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_contains_batch%s");
  const int dev = host_device(device);
  if (dev < 0) return dev;
  // the target rides along as a tiny device copy owned by this call
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return fail_hip(e, "hipSetDevice");
  uint64_t *dt = nullptr;
  if ((e = hipMalloc(&dt, 2 * 512)) != hipSuccess) return fail_hip(e, "hipMalloc(target)");
  int rc = LIFEAPI_OK;
  if ((e = hipMemcpy(dt, wanted, 512, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(dt + 64, unwanted, 512, hipMemcpyHostToDevice)) != hipSuccess)
    rc = fail_hip(e, "hipMemcpy(target)");
  if (rc == LIFEAPI_OK) {
    const HostIO io[2] = {{states, nullptr, 512}, {nullptr, out, 1}};
    rc = host_chunked(dev, n, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *a) {
                        const uint64_t *t = (const uint64_t *)a;
                        return lifeapi_contains_batch_dev((const uint64_t *)d[0], t, t + 64,
                                                          (uint8_t *)d[1], m, s);
                      },
                      dt);
  }
  (void)hipFree(dt);
  return rc;
}

}  // extern "C"

namespace {
// device buffers of one host-pointer RLE call, freed on every return path
struct DevBufs {
  std::vector<void *> p;
  template <class T>
  hipError_t get(T *&out, size_t bytes) {
    void *q = nullptr;
    const hipError_t e = hipMalloc(&q, bytes ? bytes : 1);
    if (e == hipSuccess) p.push_back(q);
    out = static_cast<T *>(q);
    return e;
  }
  ~DevBufs() {
    for (void *q : p) (void)hipFree(q);
  }
};
constexpr size_t kRleChunk = size_t(1) << 18;  // patterns per device pass
}  // namespace

extern "C" {

int lifeapi_rle_batch(const uint64_t *states, size_t n, char *text, size_t text_cap, uint64_t *offsets,
                      int device) {
  if (!offsets) return fail(LIFEAPI_E_INVALID, "null offsets to lifeapi_rle_batch%s");
  offsets[0] = 0;
  if (n == 0) return LIFEAPI_OK;
  if (!states || !aligned8(states)) return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_rle_batch%s");
  const int dev = host_device(device);
  if (dev < 0) return dev;
  std::vector<uint32_t> len(n);
  const HostIO io[2] = {{states, nullptr, 512}, {nullptr, len.data(), 4}};
  int rc = host_chunked(dev, n, io, 2,
                        [](void *const *d, size_t m, hipStream_t s, const void *) {
                          return lifeapi_rle_lengths_batch_dev((const uint64_t *)d[0], (uint32_t *)d[1], m, s);
                        },
                        nullptr);
  if (rc != LIFEAPI_OK) return rc;
  for (size_t u = 0; u < n; ++u) offsets[u + 1] = offsets[u] + len[u];
  if (!text) return LIFEAPI_OK;  // size query
  if (text_cap < offsets[n]) return fail(LIFEAPI_E_INVALID, "text buffer smaller than offsets[n]%s");
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return fail_hip(e, "hipSetDevice");
  for (size_t c = 0; c < n; c += kRleChunk) {
    const size_t m = std::min(kRleChunk, n - c);
    const uint64_t t0 = offsets[c], tb = offsets[c + m] - t0;
    std::vector<uint64_t> rel(m);
    for (size_t u = 0; u < m; ++u) rel[u] = offsets[c + u] - t0;
    DevBufs bufs;
    uint64_t *ds = nullptr, *doff = nullptr;
    char *dt = nullptr;
    if ((e = bufs.get(ds, m * 512)) != hipSuccess || (e = bufs.get(doff, m * 8)) != hipSuccess ||
        (e = bufs.get(dt, tb)) != hipSuccess)
      return fail_hip(e, "hipMalloc(rle)");
    if ((e = hipMemcpy(ds, states + c * 64, m * 512, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(doff, rel.data(), m * 8, hipMemcpyHostToDevice)) != hipSuccess)
      return fail_hip(e, "hipMemcpy(rle in)");
    if ((rc = lifeapi_rle_write_batch_dev(ds, doff, dt, m, nullptr)) != LIFEAPI_OK) return rc;
    if ((e = hipMemcpy(text + t0, dt, tb, hipMemcpyDeviceToHost)) != hipSuccess)
      return fail_hip(e, "hipMemcpy(rle out)");
  }
  return LIFEAPI_OK;
}

int lifeapi_parse_rle_batch(const char *text, const uint64_t *offsets, size_t n, uint64_t *out,
                            uint8_t *status, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!text || !offsets || !out || !status || !aligned8(out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_parse_rle_batch%s");
  for (size_t u = 0; u < n; ++u)
    if (offsets[u + 1] < offsets[u]) return fail(LIFEAPI_E_INVALID, "offsets must not decrease%s");
  const int dev = host_device(device);
  if (dev < 0) return dev;
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return fail_hip(e, "hipSetDevice");
  for (size_t c = 0; c < n; c += kRleChunk) {
    const size_t m = std::min(kRleChunk, n - c);
    const uint64_t t0 = offsets[c], tb = offsets[c + m] - t0;
    std::vector<uint64_t> rel(m + 1);
    for (size_t u = 0; u <= m; ++u) rel[u] = offsets[c + u] - t0;
    DevBufs bufs;
    uint64_t *doff = nullptr, *dout = nullptr;
    char *dt = nullptr;
    uint8_t *dst = nullptr;
    if ((e = bufs.get(dt, tb)) != hipSuccess || (e = bufs.get(doff, (m + 1) * 8)) != hipSuccess ||
        (e = bufs.get(dout, m * 512)) != hipSuccess || (e = bufs.get(dst, m)) != hipSuccess)
      return fail_hip(e, "hipMalloc(parse)");
    if ((e = hipMemcpy(dt, text + t0, tb, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(doff, rel.data(), (m + 1) * 8, hipMemcpyHostToDevice)) != hipSuccess)
      return fail_hip(e, "hipMemcpy(parse in)");
    int rc = lifeapi_parse_rle_batch_dev(dt, doff, m, dout, dst, nullptr);
    if (rc != LIFEAPI_OK) return rc;
    if ((e = hipMemcpy(out + c * 64, dout, m * 512, hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(status + c, dst, m, hipMemcpyDeviceToHost)) != hipSuccess)
      return fail_hip(e, "hipMemcpy(parse out)");
  }
  return LIFEAPI_OK;
}

}  // extern "C"
