// cone_split.hpp -- the iterated search filter (first hits only, 3-15
// generations; Step() LifeAPI.hpp:1196-1216 then Contains(LifeTarget)
// LifeTarget.hpp:44-51 after every generation) on a target whose light cone
// fits R = 32 or 16 rows: the row-split register layout of the iterated step
// (split_layout.hpp) inside that window.
//
// cone_wave_rows (step_kernels.hpp) packs each universe's window as one
// R-bit field of a 32-bit word and finds the vertical neighbours by 1-bit
// shifts: four shifts (1.8 issue slots each on gfx950) of the two h-planes
// per word and generation.  Here eight registers r[0..7] hold the window of
// 256 / R universes per lane: register j holds the window rows 8k + j, and
// the universes are interleaved bit by bit below the row group k
//   R = 32:  position 8k + u              (k = 0..3, u = 0..7)
//   R = 16:  position 16 h + 8k + v       (k = 0..1, universe 2 v + h)
// so the vertical neighbours of register j are registers j - 1 and j + 1,
// and only the ends of the register ring take a rotate by 8 positions (one
// row group): per word and generation two DPP moves, the two h-layer LUTs,
// the six-LUT tail and half a rotate, against the packed form's four shifts
// more.  The window's own edges wrap onto each other -- wrong data, which
// moves one row inwards per generation and never reaches a care row: the
// window starts `gens` rows above the care rows and ends at least `gens`
// rows below them (cone_rows), exactly as in the packed form.  The columns
// are cone_wave's: P lanes per universe from column xs, the 64-lane DPP
// rotate handing a group's edge lanes the neighbouring group's columns --
// wrong only in the `gens` margin columns.
//
// Layout change: the U = 256 / R cut words of a lane (R = 16: two per
// 32-bit word) are eight registers x[i] of (universe bits i | row bits
// j2 j1 j0 at positions 0-2); three delta swaps exchange register index bit
// b with position bit b (b = 0, 1, 2), after which register j holds rows
// with row bits j and the universe index sits in positions 0-2 -- 48 VALU
// per eight registers, once per set.
//
// The test: after every generation the differences (s ^ wanted) & care of
// the eight registers are OR-ed into one word, folded over the row groups
// to one bit per universe, and packed into an accumulator, 4 (R = 32) or 2
// (R = 16) generations per 32-bit word; the lane OR within each P-lane
// group (DPP) and a scalar test of the group's word run once per such
// batch.  A universe is clean at a generation iff its bit is 0 in the
// group's word; hits (rare) take a scalar slow path that records the first
// clean generation of every universe not yet found.
#pragma once

#include "step_kernels.hpp"

namespace lifeapi_impl {
namespace {

// the three index swaps of the window layout (register bit b <-> position
// bit b), as split_swap's select form
__device__ __forceinline__ void win_swap3(uint32_t (&x)[8]) {
  constexpr uint32_t kSel = ((TA & TC) | (TB & ~TC)) & 0xFF;  // c ? a : b
  constexpr uint32_t masks[3] = {0x55555555u, 0x33333333u, 0x0F0F0F0Fu};
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const int sh = 1 << b;
    const uint32_t m = masks[b];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if ((i >> b) & 1) continue;
      const int k = i | (1 << b);
      const uint32_t xi = x[i], xk = x[k];
      x[k] = lut3<kSel>(xi >> sh, xk, m);
      x[i] = lut3<kSel>(xk << sh, xi, m << sh);
    }
  }
}

// U cut words (R-row windows, in the low R bits) -> eight registers
template <int R>
__device__ __forceinline__ void win_pack(const uint32_t (&e)[256 / R], uint32_t (&x)[8]) {
  if constexpr (R == 32) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = e[i];
  } else {
    static_assert(R == 16, "windows of 32 or 16 rows");
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_perm(e[2 * i + 1], e[2 * i], 0x05040100u);  // e0 | e1 << 16
  }
  win_swap3(x);
}

// the universe (0 .. 256 / R - 1 within a group) of bit b of a batch word
template <int R>
__device__ __forceinline__ uint32_t win_universe(uint32_t b) {
  if constexpr (R == 32) return b & 7u;
  else return 2u * (b & 7u) + ((b >> 4) & 1u);
}
// the generation (0 .. 32 / DB - 1 within a batch) of bit b of a batch word
template <int R>
__device__ __forceinline__ uint32_t win_batch_gen(uint32_t b) {
  if constexpr (R == 32) return b >> 3;
  else return (b >> 3) & 1u;
}

// One wave's passes over universes u_first, u_first + u_step, ... (chunks of
// UPS = (64 / P) (256 / R) universes, one register set each).  out[u] = the
// first generation in 1..gens whose state contains the target, 0 = never.
// xs / K: the column window (K <= P), y0: the first window row (WRAP: the
// window crosses row 63), as cone_wave_rows.
template <int P, int R, bool WRAP, typename OutT>
__device__ __forceinline__ void cone_wave_split(const uint64_t *in, const uint64_t *__restrict__ wanted,
                                                const uint64_t *__restrict__ unwanted, OutT *__restrict__ out,
                                                uint64_t n, uint64_t u_first, uint64_t u_step, uint32_t gens,
                                                uint32_t xs, uint32_t K, uint32_t y0, int lane) {
  constexpr int GPS = kWave / P;                 // groups (universe columns) per wave
  constexpr int U = 256 / R;                     // universes per register per group
  constexpr int UPS = GPS * U;                   // universes per register set
  constexpr int GPB = R == 32 ? 4 : 2;           // generations per batch word
  constexpr uint32_t kRot = 8;                   // one row group
  static_assert(UPS <= kWave, "one answer per lane");
  static_assert(P >= 8 && P <= kWave, "8 .. 64 lanes per universe");
  constexpr uint32_t kDiff = ((TA ^ TB) & TC) & 0xFF;  // (s ^ wanted) & care
  constexpr uint32_t kOr3 = (TA | TB | TC) & 0xFF;
  constexpr uint32_t rmask = R == 32 ? ~0u : 0xFFFFu;
  const uint32_t j = (uint32_t)lane & (P - 1), q = (uint32_t)lane / P;
  const uint32_t col = (xs + j) & (kWave - 1);
  const bool live = j < K;
  const uint32_t sh = y0 & 31u;
  auto cut = [&](uint64_t v) __attribute__((always_inline)) {
    const W w = split(v);
    return (WRAP ? __builtin_amdgcn_alignbit(w.lo, w.hi, sh) : __builtin_amdgcn_alignbit(w.hi, w.lo, sh)) & rmask;
  };
  // the target in the same layout, replicated over the universes
  uint32_t tw[8], tm[8];
  {
    const uint64_t w64 = live ? wanted[col] : 0ull, m64 = live ? (w64 | unwanted[col]) : 0ull;
    uint32_t ew[U], em[U];
    const uint32_t cw = cut(w64), cm = cut(m64);
#pragma unroll
    for (int u = 0; u < U; ++u) ew[u] = cw, em[u] = cm;
    win_pack<R>(ew, tw);
    win_pack<R>(em, tm);
  }
  const uint32_t fold_mask = R == 32 ? 0xFFu : 0x00FF00FFu;  // one bit per universe after the fold
  for (uint64_t u0 = u_first; u0 < n; u0 += u_step) {
    uint32_t r[8];
    {
      uint32_t e[U];
      const uint64_t ub = u0 + (uint64_t)q * U;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t uu = ub + u;
        e[u] = (live && uu < n) ? cut(__builtin_nontemporal_load(in + uu * kWave + col)) : 0u;
      }
      win_pack<R>(e, r);
    }
    uint32_t mine = 0;      // lane L: the answer of universe u0 + L
    uint64_t found = 0;     // set-local universes already answered
    uint32_t foundrep[GPS];  // per group: the found universes' bits in a batch word
#pragma unroll
    for (int g = 0; g < GPS; ++g) foundrep[g] = 0;
    for (uint32_t g0 = 0; g0 < gens; g0 += GPB) {
      const uint32_t nb = gens - g0 < (uint32_t)GPB ? gens - g0 : (uint32_t)GPB;  // (wave-uniform)
      uint32_t acc = 0;
#pragma unroll
      for (int m = 0; m < GPB; ++m) {
        if ((uint32_t)m >= nb) break;
        uint32_t h0[8], h1[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const uint32_t L = dpp_prev(r[i]), Rt = dpp_next(r[i]);
          h0[i] = lut3<kXor3>(L, r[i], Rt);
          h1[i] = lut3<kMaj>(L, r[i], Rt);
        }
        const uint32_t h0u0 = __builtin_amdgcn_alignbit(h0[7], h0[7], 32 - kRot);  // rotl 8: row group k - 1
        const uint32_t h1u0 = __builtin_amdgcn_alignbit(h1[7], h1[7], 32 - kRot);
        const uint32_t h0d7 = __builtin_amdgcn_alignbit(h0[0], h0[0], kRot);       // rotr 8: row group k + 1
        const uint32_t h1d7 = __builtin_amdgcn_alignbit(h1[0], h1[0], kRot);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const uint32_t u0v = i ? h0[i - 1] : h0u0, d0v = i < 7 ? h0[i + 1] : h0d7;
          const uint32_t u1v = i ? h1[i - 1] : h1u0, d1v = i < 7 ? h1[i + 1] : h1d7;
          r[i] = life_tail6(u0v, h0[i], d0v, u1v, h1[i], d1v, r[i]);
        }
        uint32_t d[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) d[i] = lut3<kDiff>(r[i], tw[i], tm[i]);
        const uint32_t D = lut3<kOr3>(lut3<kOr3>(d[0], d[1], d[2]), lut3<kOr3>(d[3], d[4], d[5]), d[6] | d[7]);
        uint32_t f;
        if constexpr (R == 32) {
          f = D | __builtin_amdgcn_alignbit(D, D, 16);
          f = f | __builtin_amdgcn_alignbit(f, f, 8);
        } else {
          f = D | __builtin_amdgcn_alignbit(D, D, 8);
        }
        acc |= (f & fold_mask) << (8 * m);
      }
      // the OR over each group's P lanes: every lane of an 8-lane half
      // (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror), of a 16-lane row
      // (row_mirror), then the rows by v_readlane
      uint32_t v = acc;
      v |= dpp_mov<0xB1>(v);
      v |= dpp_mov<0x4E>(v);
      v |= dpp_mov<0x141>(v);
      if constexpr (P >= 16) v |= dpp_mov<0x140>(v);
      uint32_t vmask = 0;  // the batch word's bits of generations g0 + 1 .. g0 + nb
#pragma unroll
      for (int m = 0; m < GPB; ++m)
        if ((uint32_t)m < nb) vmask |= fold_mask << (8 * m);
#pragma unroll
      for (int g = 0; g < GPS; ++g) {
        uint32_t w = 0;
        if constexpr (P <= 16) {
          w = (uint32_t)__builtin_amdgcn_readlane((int)v, g * P);
        } else {
#pragma unroll
          for (int t = 0; t < P / 16; ++t) w |= (uint32_t)__builtin_amdgcn_readlane((int)v, g * P + 16 * t);
        }
        uint32_t c = ~w & vmask & ~foundrep[g];
        while (c) {  // (rare) hits: the first clean generation of each new universe
          const uint32_t b = (uint32_t)__builtin_ctz(c);
          const uint32_t uu = win_universe<R>(b), idx = (uint32_t)g * U + uu;
          if (!((found >> idx) & 1ull)) {
            found |= 1ull << idx;
            if ((uint32_t)lane == idx) mine = g0 + win_batch_gen<R>(b) + 1u;
            // this universe's bits in every generation of a batch word
            foundrep[g] |= R == 32 ? 0x01010101u << (b & 7u) : 0x0101u << (b & 0x17u);
          }
          c &= c - 1;
        }
      }
    }
    if (lane < UPS && u0 + (uint64_t)lane < n) out[u0 + lane] = (OutT)mine;
  }
}

}  // namespace
}  // namespace lifeapi_impl
