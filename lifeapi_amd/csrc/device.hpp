// device.hpp -- lane-level building blocks shared by every kernel file.
//
// One 64-lane wavefront works on one universe at a time: lane x owns column x
// (the reference's state[x], LifeAPI.hpp:39-40) as two 32-bit VGPRs.  The
// vertical (in-column) neighbours are 1-bit rotates of the lane's own word; the
// horizontal neighbours are the adjacent lanes' columns, fetched with DPP
// wave_ror:1 / wave_rol:1 (64-lane rotates, so the torus wrap at columns 0/63
// is free), ds_bpermute or LDS.  Logic is gfx950's 3-input v_bitop3_b32.  No
// MFMA: the work is pure integer/bitwise.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace lifeapi_impl {

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

// (the numbering is the tuning build's LIFEAPI_XCHG_*, tools/tune/lifeapi_tune.h;
// the shipped kernels use XDPP and, in the assembly loop, LDS)
enum Xchg { XDPP = 0, XLDS = 1, XBPERM = 2, XMIX = 3, XMIX1 = 4, XMIX3 = 5, XLDSR = 6, XLDSR3 = 7, XASM = 8 };
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

// The 6-LUT tail (NET 6): the same inputs as the 7-LUT network, one v_bitop3
// fewer per 32-bit word (8 with the two h-layer LUTs, against 9).  Found by
// stochastic search over arbitrary 6-gate DAGs (tools/cgp_search.c) using the
// don't-cares of the centre row: its sum contains a, so (a = 1, sum 0) and
// (a = 0, sum 3) never occur.  No 5-gate network turned up, nor a 7-gate one
// with row- or row-pair-shared gates (tools/cgp_rows.c).
//   g1 = SB in {0,2,3}            = N1(h1, h1u, h1d)
//   g2 = maj(h1d, h1u, h0d)
//   g3 = SA in {1,2}              = Nae(h0d, h0u, h0)
//   g4 = N4(g3, g2, g1)
//   g5 = SA odd                   = xor3(h0, h0d, h0u)
//   next = g4 & (g5 | a)          = N6(g4, g5, a)
// Checked on all 512 neighbourhoods by tests/test_oracle.py::test_net6_truth.
constexpr uint32_t kN1 = 0xE9, kN4 = 0x52, kN6 = 0xE0;
__device__ __forceinline__ uint32_t life_tail6(uint32_t h0u, uint32_t h0, uint32_t h0d, uint32_t h1u,
                                               uint32_t h1, uint32_t h1d, uint32_t a) {
  const uint32_t g1 = lut3<kN1>(h1, h1u, h1d);
  const uint32_t g2 = lut3<kMaj>(h1d, h1u, h0d);
  const uint32_t g3 = lut3<kNae>(h0d, h0u, h0);
  const uint32_t g4 = lut3<kN4>(g3, g2, g1);
  const uint32_t g5 = lut3<kXor3>(h0, h0d, h0u);
  return lut3<kN6>(g4, g5, a);
}
// the 7-LUT tail above, per 32-bit word
__device__ __forceinline__ uint32_t life_tail7(uint32_t h0u, uint32_t h0, uint32_t h0d, uint32_t h1u,
                                               uint32_t h1, uint32_t h1d, uint32_t a) {
  const uint32_t s0 = lut3<kLe1>(h0u, h0, h0d), s1 = lut3<kNae>(h0u, h0, h0d);
  const uint32_t s2 = lut3<kLe1>(h1u, h1, h1d), s3 = lut3<kEven>(h1u, h1, h1d);
  const uint32_t t1 = lut3<kT1>(s0, s1, a);
  const uint32_t t2 = lut3<kT2>(s2, a, t1);
  return lut3<kT3>(s1, s3, t2);
}
template <int NET>
__device__ __forceinline__ uint32_t life_tail(uint32_t h0u, uint32_t h0, uint32_t h0d, uint32_t h1u,
                                              uint32_t h1, uint32_t h1d, uint32_t a) {
  static_assert(NET == 6 || NET == 7, "tails: 6 or 7 LUTs");
  if constexpr (NET == 6) return life_tail6(h0u, h0, h0d, h1u, h1, h1d, a);
  else return life_tail7(h0u, h0, h0d, h1u, h1, h1d, a);
}

// two adjacent 64-bit words: the unit of a 16-byte (dwordx4) access
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

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

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// Wave sums without the LDS crossbar (__shfl_xor is one ds_bpermute per
// step: a chain of six LDS round trips): four DPP adds sum each 16-lane row
// (quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror),
// then v_readlane of lanes 0/16/32/48 and scalar adds.  Wave-uniform result.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_mov64(uint64_t v) {
  return (uint64_t)dpp_mov<CTRL>((uint32_t)v) | ((uint64_t)dpp_mov<CTRL>((uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ uint32_t wave_sum_u32_dpp(uint32_t v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x141>(v);
  v += dpp_mov<0x140>(v);
  return (uint32_t)__builtin_amdgcn_readlane(v, 0) + (uint32_t)__builtin_amdgcn_readlane(v, 16) +
         (uint32_t)__builtin_amdgcn_readlane(v, 32) + (uint32_t)__builtin_amdgcn_readlane(v, 48);
}
// The lane index, re-derived (v_mbcnt in an opaque asm, so the compiler
// cannot CSE it with an earlier copy): kernels whose hand-allocated loops
// pin most of the VGPRs call it after the loop instead of keeping the lane
// (and addresses built from it) live across it.
__device__ __forceinline__ uint32_t lane_id_fresh() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n v_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// the OR of v over the wave, the same way (wave-uniform)
__device__ __forceinline__ uint32_t wave_or_u32_dpp(uint32_t v) {
  v |= dpp_mov<0xB1>(v);
  v |= dpp_mov<0x4E>(v);
  v |= dpp_mov<0x141>(v);
  v |= dpp_mov<0x140>(v);
  return (uint32_t)__builtin_amdgcn_readlane(v, 0) | (uint32_t)__builtin_amdgcn_readlane(v, 16) |
         (uint32_t)__builtin_amdgcn_readlane(v, 32) | (uint32_t)__builtin_amdgcn_readlane(v, 48);
}
__device__ __forceinline__ uint64_t wave_sum_u64_dpp(uint64_t v) {
  auto step = [&](auto mov) __attribute__((always_inline)) {
    v += (uint64_t)mov((uint32_t)v) | ((uint64_t)mov((uint32_t)(v >> 32)) << 32);
  };
  step(dpp_mov<0xB1>);
  step(dpp_mov<0x4E>);
  step(dpp_mov<0x141>);
  step(dpp_mov<0x140>);
  uint64_t t = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    t += (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, 16 * r) |  // (readlane
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), 16 * r) << 32);  // is int)
  return t;
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


// The block's place in the batch with each XCD dealt one contiguous run of
// it.  Blocks go to the 8 XCDs round-robin (MI355X_MICROARCH.md, workgroup
// dispatch: blocks b and b + 8 share one), so with blockIdx.x as the index an
// XCD touches every 8th stretch of the whole batch.  Numbering XCD x's i-th
// block x*q + min(x, r) + i (grid = 8q + r) is a bijection onto [0, grid)
// that gives XCD x one contiguous eighth: +5-11 % on the in-place LifeStable
// passes and +2-4 % on 8M-16M-universe steps (tools/ab/stable_xcd_ab.py,
// tools/ab/step_xcd_ab.py).
__device__ __forceinline__ uint64_t xcd_chunk_block() {
  const uint32_t b = blockIdx.x, nb = gridDim.x, q = nb >> 3, r = nb & 7u, x = b & 7u;
  return (uint64_t)x * q + (x < r ? x : r) + (b >> 3);
}
template <bool CHUNK>
__device__ __forceinline__ uint64_t block_index() {
  if constexpr (CHUNK) return xcd_chunk_block();
  else return blockIdx.x;
}

__device__ __forceinline__ uint64_t rotr64(uint64_t v, uint32_t k) {
  return (v >> k) | (v << ((64 - k) & 63));
}
// the smallest cyclic window [y0, y0 + h) of rows holding every set bit of
// rm (wave-uniform; h = 1 for an empty mask): the complement of the longest
// cyclic run of empty rows, found by binary lifting (run_k bit p = rows
// p .. p + k - 1 all empty) in a few dozen scalar instructions
__device__ __forceinline__ void care_window(uint64_t rm, uint32_t &y0, uint32_t &h) {
  y0 = 0;
  h = 1;
  if (rm == 0) return;
  uint64_t run[6];
  run[0] = ~rm;  // runs of 1
#pragma unroll
  for (int k = 1; k < 6; ++k) run[k] = run[k - 1] & rotr64(run[k - 1], 1u << (k - 1));  // runs of 2^k
  uint64_t cur = ~0ull;  // starts of runs of length len
  uint32_t len = 0;
#pragma unroll
  for (int k = 5; k >= 0; --k) {
    const uint64_t t = cur & rotr64(run[k], len);
    if (t) cur = t, len += 1u << k;
  }
  h = 64 - len;
  y0 = len ? ((uint32_t)__builtin_ctzll(cur) + len) & 63 : 0;
}
// s_waitcnt immediates (gfx9 encoding: vmcnt [3:0] + [15:14], expcnt [6:4],
// lgkmcnt [11:8]): at most N vector-memory ops outstanding, or no LDS op.
// "s_waitcnt vmcnt(N) waits until all but the wave's N youngest
// vector-memory operations are done.  Loads, stores, atomics and LDS-DMA
// count together, in issue order (flat_* excepted)" (MI355X_MICROARCH.md,
// the paragraph after the per-instruction cycle constants) -- so a wave waits
// for a global_load_lds by allowing the ops it issued after it to remain.
// (The compiler's own waitcnt pass treats a load followed by a store as out
// of order and, before a compiled LDS read after an LDS-DMA, inserts
// vmcnt(0): the counted waits below hold only where the reads are inline
// assembly or no compiled LDS access follows.  The shipped launches of the
// counted forms -- k_stable_dma with U = 1 and one chunk per wave in
// cone_wave_full_dma / cone_wave_rows_dma -- issue no store between a fetch and
// its wait except the chunk's answer store, the case vmcnt(1) covers; the
// tuning forms with U >= 2 rely on the ordering as cited.)
constexpr int kWaitVm0 = 0x0F70, kWaitVm1 = 0x0F71, kWaitVm5 = 0x0F75, kWaitVm6 = 0x0F76, kWaitVm9 = 0x0F79,
              kWaitVm11 = 0x0F7B, kWaitLgkm0 = 0xC07F;

// Contains(LifeTarget) (LifeTarget.hpp:44-51): (s ^ w) & (w | u) == 0 on all columns
__device__ __forceinline__ bool wave_contains(W s, W w, W u) {
  const uint32_t dlo = (s.lo ^ w.lo) & (w.lo | u.lo), dhi = (s.hi ^ w.hi) & (w.hi | u.hi);
  return __ballot((dlo | dhi) != 0u) == 0ull;
}


}  // namespace lifeapi_impl
