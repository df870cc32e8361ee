// split_layout.hpp -- register layouts of the iterated Step() (RULE 4..7):
// the even/odd row split and the S-way row splits with S/2 universes
// interleaved bit by bit, and one generation on them.
#pragma once

#include "device.hpp"

namespace lifeapi_impl {

// ---- even/odd row layout (RULE 4) ----
// A 64-bit column held as (E, O): E bit k = row 2k, O bit k = row 2k+1.  The
// vertical neighbours of row 2k are O bits k-1 and k; those of row 2k+1 are
// E bits k and k+1.  So a vertical triple costs one 32-bit rotate per plane
// and parity instead of two 64-bit rotates (four v_alignbit) per plane, and a
// v_alignbit issues at half rate on gfx950 (tools/ab/bank_probe.hip).
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

// One swap stage.  Stages 0 and 1 (16- and 8-bit shifts) move whole bytes:
// each register of a pair is one v_perm of the pair (the delta swap's five
// VALU -- shift, masked xor, xor, shift, xor -- become two).  Stages 2-4 write
// each register as a bit select between itself and its partner shifted into
// place: new B = (A >> s) & m | B & ~m, new A = (B << s) & (m << s) | A &
// ~(m << s) -- a shift and a v_bitop3 each, four VALU per pair.
template <int S>
__device__ __forceinline__ void split_swap(uint32_t (&x)[S], int stage) {
  constexpr uint32_t masks[5] = {0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
  constexpr uint32_t kSel = ((TA & TC) | (TB & ~TC)) & 0xFF;  // c ? a : b, bit by bit
  const int a = SplitNet<S>::a[stage], sh = 16 >> stage;
  const uint32_t m = masks[stage];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    if ((i >> a) & 1) continue;
    const int k = i | (1 << a);
    const uint32_t xi = x[i], xk = x[k];
    if (sh == 16) {  // A.hi16 <-> B.lo16
      x[i] = __builtin_amdgcn_perm(xk, xi, 0x05040100u);
      x[k] = __builtin_amdgcn_perm(xk, xi, 0x07060302u);
    } else if (sh == 8) {  // A bytes 1, 3 <-> B bytes 0, 2
      x[i] = __builtin_amdgcn_perm(xk, xi, 0x06020400u);
      x[k] = __builtin_amdgcn_perm(xk, xi, 0x07030501u);
    } else {
      x[k] = lut3<kSel>(xi >> sh, xk, m);
      x[i] = lut3<kSel>(xk << sh, xi, m << sh);
    }
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

// LDS exchange of m registers (m = 4a + 2b + c): planes of 4, then 2, then
// 1 words per lane, each at its natural lane stride (16 / 8 / 4 B), which
// keeps every ds_write / ds_read free of bank conflicts (a 32-B stride would
// be 2-way).  All writes first, then the reads of lanes x-1 and x+1: a wave's
// LDS operations complete in order, and the store and the loads may alias,
// so the compiler keeps their order.
template <int Q>
struct LdsVec {
  typedef uint32_t type __attribute__((ext_vector_type(Q)));
};
template <>
struct LdsVec<1> {
  typedef uint32_t type;
};
template <int Q>
__device__ __forceinline__ void lds_put(uint32_t *plane, const uint32_t *r, int lane) {
  typename LdsVec<Q>::type v;
  if constexpr (Q == 1) v = r[0];
  else {
#pragma unroll
    for (int q = 0; q < Q; ++q) v[q] = r[q];
  }
  reinterpret_cast<typename LdsVec<Q>::type *>(plane)[lane] = v;
}
template <int Q>
__device__ __forceinline__ void lds_get(const uint32_t *plane, uint32_t *out, int src) {
  const typename LdsVec<Q>::type v = reinterpret_cast<const typename LdsVec<Q>::type *>(plane)[src];
  if constexpr (Q == 1) out[0] = v;
  else {
#pragma unroll
    for (int q = 0; q < Q; ++q) out[q] = v[q];
  }
}
template <int M>
__device__ __forceinline__ void lds_exchange(const uint32_t *r, uint32_t *lv, uint32_t *rv, uint32_t *slot,
                                             int lane) {
  constexpr int A = M / 4, B = (M % 4) / 2, C = M % 2;
  const int xp = (lane + kWave - 1) & (kWave - 1), xn = (lane + 1) & (kWave - 1);
#pragma unroll
  for (int p = 0; p < A; ++p) lds_put<4>(slot + 4 * p * kWave, r + 4 * p, lane);
  if constexpr (B) lds_put<2>(slot + 4 * A * kWave, r + 4 * A, lane);
  if constexpr (C) lds_put<1>(slot + (4 * A + 2 * B) * kWave, r + 4 * A + 2 * B, lane);
#pragma unroll
  for (int p = 0; p < A; ++p) {
    lds_get<4>(slot + 4 * p * kWave, lv + 4 * p, xp);
    lds_get<4>(slot + 4 * p * kWave, rv + 4 * p, xn);
  }
  if constexpr (B) {
    lds_get<2>(slot + 4 * A * kWave, lv + 4 * A, xp);
    lds_get<2>(slot + 4 * A * kWave, rv + 4 * A, xn);
  }
  if constexpr (C) {
    lds_get<1>(slot + (4 * A + 2 * B) * kWave, lv + 4 * A + 2 * B, xp);
    lds_get<1>(slot + (4 * A + 2 * B) * kWave, rv + 4 * A + 2 * B, xn);
  }
}

// one generation of the P universes in r[] (the h-layer and a NET-LUT tail
// per register: NET 7 = the RULE 3 network, NET 6 = life_tail6).  The
// neighbour columns of registers 0..S-D-1 go through LDS, those of the last
// D registers by DPP wave_ror / wave_rol (VALU slots instead of LDS
// bandwidth: the two pipes balance the load).
template <int S, int NET = 7, int D = 0>
__device__ __forceinline__ void gen_split(uint32_t (&r)[S], uint32_t *slot, int lane) {
  constexpr int P = S / 2;
  static_assert(D >= 0 && D <= S, "DPP registers");
  uint32_t lv[S], rv[S];
  if constexpr (D < S) lds_exchange<S - D>(r, lv, rv, slot, lane);
#pragma unroll
  for (int j = S - D; j < S; ++j) lv[j] = dpp_prev(r[j]), rv[j] = dpp_next(r[j]);
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
    r[j] = life_tail<NET>(a0, h0[j], c0, a1, h1[j], c1, r[j]);
  }
}

// `gens` generations of gen_split<S, NET> (S % 4 == 0), software-pipelined
// across the LDS planes: a plane's four new registers are published, and the
// next generation's reads of that plane issued, as soon as its rows' tail is
// done, so those LDS round trips overlap the remaining planes' tails instead
// of stalling the wave at the top of each generation.  The reads for the
// generation after the last are issued too and simply dropped.
template <int S, int NET>
__device__ __forceinline__ void gens_split_pipe(uint32_t (&r)[S], uint32_t *slot, int lane, uint32_t gens) {
  constexpr int P = S / 2, NPL = S / 4;
  static_assert(S % 4 == 0, "planes of 4 registers");
  typedef uint32_t vec __attribute__((ext_vector_type(4)));
  vec *v = reinterpret_cast<vec *>(slot);
  const int xp = (lane + kWave - 1) & (kWave - 1), xn = (lane + 1) & (kWave - 1);
  vec L[NPL], R[NPL];
#pragma unroll
  for (int p = 0; p < NPL; ++p) {
    v[p * kWave + lane] = vec{r[4 * p], r[4 * p + 1], r[4 * p + 2], r[4 * p + 3]};
    L[p] = v[p * kWave + xp];
    R[p] = v[p * kWave + xn];
  }
  for (uint32_t it = 0; it < gens; ++it) {
    uint32_t h0[S], h1[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const uint32_t l = L[j / 4][j % 4], rr = R[j / 4][j % 4];
      h0[j] = lut3<kXor3>(l, r[j], rr);
      h1[j] = lut3<kMaj>(l, r[j], rr);
    }
    const uint32_t h0u = __builtin_amdgcn_alignbit(h0[S - 1], h0[S - 1], 32 - P);  // rotl P
    const uint32_t h1u = __builtin_amdgcn_alignbit(h1[S - 1], h1[S - 1], 32 - P);
    const uint32_t h0d = __builtin_amdgcn_alignbit(h0[0], h0[0], P);  // rotr P
    const uint32_t h1d = __builtin_amdgcn_alignbit(h1[0], h1[0], P);
#pragma unroll
    for (int p = 0; p < NPL; ++p) {
#pragma unroll
      for (int j = 4 * p; j < 4 * p + 4; ++j) {
        const uint32_t a0 = j == 0 ? h0u : h0[j - 1], c0 = j == S - 1 ? h0d : h0[j + 1];
        const uint32_t a1 = j == 0 ? h1u : h1[j - 1], c1 = j == S - 1 ? h1d : h1[j + 1];
        r[j] = life_tail<NET>(a0, h0[j], c0, a1, h1[j], c1, r[j]);
      }
      // a wave's LDS operations complete in order: this generation's reads
      // of plane p are done (consumed above), and the new reads see the new
      // words; the compiler keeps the order (the store and loads may alias)
      v[p * kWave + lane] = vec{r[4 * p], r[4 * p + 1], r[4 * p + 2], r[4 * p + 3]};
      L[p] = v[p * kWave + xp];
      R[p] = v[p * kWave + xn];
      // keep the machine scheduler from sinking these LDS operations below
      // the next plane's tail (it otherwise groups all of them at the end)
      if (p + 1 < NPL) __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// ------------------------------------------------------------------------
// Tile layouts (RULE 8: C = 4, RULE 9: C = 2 adjacent columns per lane)
// ------------------------------------------------------------------------
//
// The S-way row split of gen_split, but a lane owns C adjacent columns
// (x = C*i .. C*i + C-1 of its group's P universes), so a group of 64/C lanes
// holds P whole universes and a wave C*P of them.  Horizontal neighbours of
// the inner columns are the lane's own registers; only the two edge columns
// cross lanes.  Per generation a lane publishes columns 0 and C-1 and fetches
// column C-1 of lane i-1 and column 0 of lane i+1 (mod 64/C: the torus wrap).
// Against gen_split (C = 1) that is 2/C of the exchanged words per cell, which
// takes the LDS pipe off the critical path; with C = 4 a group is one 16-lane
// DPP row, so row_ror moves the edges with the wrap built in (XDPP), at 0.9
// VALU slot per word instead of LDS traffic (XLDS).
template <int S, int C, int X, int NET = 7>
__device__ __forceinline__ void gen_tile(uint32_t (&r)[C][S], uint32_t *slot, int lane) {
  constexpr int P = S / 2;
  uint32_t lv[S], rv[S];
  if constexpr (X == XDPP) {
    static_assert(C == 4, "row_ror rotates 16-lane rows: 4 columns per lane");
#pragma unroll
    for (int j = 0; j < S; ++j) {
      // row_ror:1 -> lane i reads lane i-1 of its row; row_ror:15 -> lane i+1
      lv[j] = (uint32_t)__builtin_amdgcn_mov_dpp((int)r[C - 1][j], 0x121, 0xF, 0xF, true);
      rv[j] = (uint32_t)__builtin_amdgcn_mov_dpp((int)r[0][j], 0x12F, 0xF, 0xF, true);
    }
  } else {
    static_assert(S % 4 == 0, "16-B LDS planes");
    constexpr int LPG = kWave / C;  // lanes per group
    constexpr int Q = S / 4;        // planes per edge column
    typedef uint32_t vec __attribute__((ext_vector_type(4)));
    vec *v = reinterpret_cast<vec *>(slot);
#pragma unroll
    for (int p = 0; p < Q; ++p) {
      v[p * kWave + lane] = vec{r[0][4 * p], r[0][4 * p + 1], r[0][4 * p + 2], r[0][4 * p + 3]};
      v[(Q + p) * kWave + lane] =
          vec{r[C - 1][4 * p], r[C - 1][4 * p + 1], r[C - 1][4 * p + 2], r[C - 1][4 * p + 3]};
    }
    // a wave's LDS operations complete in order; stores and loads may alias,
    // so the compiler keeps their order
    const int g0 = lane & ~(LPG - 1);
    const int xp = g0 | ((lane + LPG - 1) & (LPG - 1)), xn = g0 | ((lane + 1) & (LPG - 1));
#pragma unroll
    for (int p = 0; p < Q; ++p) {
      const vec l = v[(Q + p) * kWave + xp], rr = v[p * kWave + xn];
#pragma unroll
      for (int q = 0; q < 4; ++q) lv[4 * p + q] = l[q], rv[4 * p + q] = rr[q];
    }
  }
  // Order: h(0), h(1), out(0), h(2), out(1), ...  Column c's new state is
  // produced after h(c+1) has read its old one, so it can take the old
  // registers (no loop-carried copies).
  uint32_t h0[C][S], h1[C][S];
  auto hcol = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const uint32_t L = c == 0 ? lv[j] : r[c - 1][j], R = c == C - 1 ? rv[j] : r[c + 1][j];
      h0[c][j] = lut3<kXor3>(L, r[c][j], R);
      h1[c][j] = lut3<kMaj>(L, r[c][j], R);
    }
  };
  hcol(0);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    if (c + 1 < C) hcol(c + 1);
    const uint32_t h0u = __builtin_amdgcn_alignbit(h0[c][S - 1], h0[c][S - 1], 32 - P);  // rotl P
    const uint32_t h1u = __builtin_amdgcn_alignbit(h1[c][S - 1], h1[c][S - 1], 32 - P);
    const uint32_t h0d = __builtin_amdgcn_alignbit(h0[c][0], h0[c][0], P);  // rotr P
    const uint32_t h1d = __builtin_amdgcn_alignbit(h1[c][0], h1[c][0], P);
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const uint32_t a0 = j == 0 ? h0u : h0[c][j - 1], c0 = j == S - 1 ? h0d : h0[c][j + 1];
      const uint32_t a1 = j == 0 ? h1u : h1[c][j - 1], c1 = j == S - 1 ? h1d : h1[c][j + 1];
      r[c][j] = life_tail<NET>(a0, h0[c][j], c0, a1, h1[c][j], c1, r[c][j]);
    }
  }
}

}  // namespace lifeapi_impl
