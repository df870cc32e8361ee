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
//
// Round 6 additions (cone_wave_split): the shrinking pass (two register sets
// merged onto half the lanes once the cone's columns fit them) and, on a
// whole board, chunks fetched by LDS-DMA while the last one steps.
#pragma once

#include <type_traits>

#include "device.hpp"

// A/B switches of the round-6 forms (the tuning probes' builds without them):
// LIFE_SHRINK_MASK bit i enables the i-th shrinking form of cone_split_pass
// (0: none; 1M universes, 4 x 4 block, alone: 8 / 13 generations 0.097 /
// 0.137 ms against 0.110 / 0.153, other targets within +-3 %,
// profiles/r06/shrink_ab/, tools/gpu_r06f.sh); LIFE_WIN_DMA=0 builds the
// whole-board window pass without its LDS-DMA chunks (tools/gpu_r06h.sh).
#ifndef LIFE_SHRINK_MASK
#define LIFE_SHRINK_MASK 31
#endif
#ifndef LIFE_WIN_DMA
#define LIFE_WIN_DMA 1
#endif

namespace lifeapi_impl {
namespace {

// One pass of the whole-board LDS form: the RB universes from ub on (RB * 512
// contiguous bytes; past n, universe n - 1 again: a valid address whose
// answer is never stored) into img by RB / 2 sixteen-byte-per-lane
// global_load_lds (lanes 0-31 one universe, 32-63 the next).
template <int RB>
__device__ __forceinline__ void dma_fetch_pass(const uint64_t *in, uint64_t n, uint64_t ub, int lane, uint64_t *img) {
#pragma unroll
  for (int i = 0; i < RB / 2; ++i) {
    uint64_t u = ub + 2 * i + (lane >> 5);
    if (u >= n) u = n - 1;
    const char *src = reinterpret_cast<const char *>(in + u * kWave) + (lane & 31) * 16;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)(img + i * 2 * kWave), 16, 0, 2);
  }
}

// The whole-board pass of the filter (FIRST, gens >= 1) when the target's care
// rows, widened by the light cone, fit FW = 32 / PK rows: rows y0 .. y0 + FW - 1
// of each universe's column are cut out by one v_alignbit (WRAP: the window
// crosses row 63), PK universes share one 32-bit register (v_perm, universe j
// of the word in bits j FW .. j FW + FW - 1), and the generation runs on the
// packed words with 1-bit shifts for the vertical neighbours.  The bits
// shifted in at a field's edges (the next field's, or zero) are wrong, and the
// error moves one row inwards per generation -- never onto a care row, which
// lies at least `gens` rows inside its field (cone_rows).  Columns are whole
// (the DPP rotate is the torus), so the care cells are exact.  Same passes,
// LDS image and answers as cone_wave_full_dma; a universe costs one cut, a
// share of the pack, 1 / PK of the network and its field's test.
template <int RB, int PK, bool WRAP, typename OutT, int SLEEP = 0>
__device__ __forceinline__ void cone_wave_rows_dma(const uint64_t *in, uint64_t w64, uint64_t m64,
                                                   OutT *__restrict__ out, uint64_t n, uint64_t u_first,
                                                   uint64_t u_step, uint32_t gens, uint32_t y0, int lane,
                                                   uint64_t *img, bool prefetched) {
  static_assert(RB % 2 == 0 && RB % PK == 0 && 2 * RB <= kWave, "passes of whole words and pairs of universes");
  static_assert(PK == 1 || PK == 2 || PK == 4, "fields of 32, 16 or 8 rows");
  constexpr int FW = 32 / PK, NW = RB / PK;
  constexpr uint32_t fmask = FW == 32 ? ~0u : (1u << FW) - 1u;
  constexpr uint32_t rep = PK == 1 ? 1u : PK == 2 ? 0x00010001u : 0x01010101u;
  const uint32_t sh = y0 & 31u;
  auto cut = [&](uint64_t v) __attribute__((always_inline)) {
    const W w = split(v);
    return WRAP ? __builtin_amdgcn_alignbit(w.lo, w.hi, sh) : __builtin_amdgcn_alignbit(w.hi, w.lo, sh);
  };
  const uint32_t tw = (cut(w64) & fmask) * rep, tm = (cut(m64) & fmask) * rep;
  constexpr uint32_t kDiff = ((TA ^ TB) & TC) & 0xFF;  // (s ^ wanted) & care
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
    uint32_t a[NW];
#pragma unroll
    for (int m = 0; m < NW; ++m) {
      uint32_t e[PK];
#pragma unroll
      for (int j = 0; j < PK; ++j) e[j] = cut(img[(m * PK + j) * kWave + lane]);
      if constexpr (PK == 1) {
        a[m] = e[0];
      } else if constexpr (PK == 2) {
        a[m] = __builtin_amdgcn_perm(e[1], e[0], 0x05040100u);  // low halves: e0 | e1 << 16
      } else {
        const uint32_t p01 = __builtin_amdgcn_perm(e[1], e[0], 0x0C0C0400u);  // e0.b0, e1.b0
        const uint32_t p23 = __builtin_amdgcn_perm(e[3], e[2], 0x0C0C0400u);  // e2.b0, e3.b0
        a[m] = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
      }
    }
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);  // read out before the next fetch lands
    const uint64_t nb = base(t + 1);
    if (nb < n) fetch(nb);
    if constexpr (SLEEP > 0) __builtin_amdgcn_s_sleep(SLEEP);  // (the tuning build's pacing probe)
    uint32_t res[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) res[k] = 0;
    for (uint32_t g = 1; g <= gens; ++g) {
#pragma unroll
      for (int m = 0; m < NW; ++m) {
        const uint32_t L = dpp_prev(a[m]), R = dpp_next(a[m]);
        const uint32_t h0 = lut3<kXor3>(L, a[m], R), h1 = lut3<kMaj>(L, a[m], R);
        a[m] = life_tail6(h0 << 1, h0, h0 >> 1, h1 << 1, h1, h1 >> 1, a[m]);
        const uint32_t d = lut3<kDiff>(a[m], tw, tm);
#pragma unroll
        for (int j = 0; j < PK; ++j) {
          const bool clean = __ballot((d & (fmask << (j * FW))) != 0u) == 0ull;
          if (res[m * PK + j] == 0 && clean) res[m * PK + j] = g;
        }
      }
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

// Generations g_begin + 1 .. g_end of one register set (P lanes per
// universe), the test after each: a universe's first clean generation goes
// to lane base + (its group) U + (its index) of `mine`, and `found` (bit =
// that lane) keeps it from being recorded again.
template <int P, int R>
__device__ __forceinline__ void win_gens(uint32_t (&r)[8], const uint32_t (&tw)[8], const uint32_t (&tm)[8],
                                         uint32_t g_begin, uint32_t g_end, uint32_t &mine, uint64_t &found,
                                         uint32_t base, int lane) {
  constexpr int GPS = kWave / P;
  constexpr int U = 256 / R;
  constexpr int GPB = R == 32 ? 4 : 2;  // generations per batch word
  constexpr uint32_t kRot = 8;          // one row group
  constexpr uint32_t kDiff = ((TA ^ TB) & TC) & 0xFF;  // (s ^ wanted) & care
  constexpr uint32_t kOr3 = (TA | TB | TC) & 0xFF;
  constexpr uint32_t fold_mask = R == 32 ? 0xFFu : 0x00FF00FFu;  // one bit per universe after the fold
  // per group: the bits of the universes answered before this call, in every
  // generation of a batch word (R = 32: universe u at u + 8 m; R = 16:
  // universe 2 v + h at 16 h + v + 8 m)
  uint32_t foundrep[GPS];
#pragma unroll
  for (int g = 0; g < GPS; ++g) {
    const uint32_t fu = (uint32_t)(found >> (base + (uint32_t)g * U)) & ((1u << U) - 1u);
    if constexpr (R == 32) {
      foundrep[g] = fu * 0x01010101u;
    } else {
      uint32_t rep = 0;
      for (uint32_t t = fu; t; t &= t - 1) {  // (rare)
        const uint32_t u = (uint32_t)__builtin_ctz(t);
        rep |= 0x0101u << (16u * (u & 1u) + (u >> 1));
      }
      foundrep[g] = rep;
    }
  }
  for (uint32_t g0 = g_begin; g0 < g_end; g0 += GPB) {
    const uint32_t nb = g_end - g0 < (uint32_t)GPB ? g_end - g0 : (uint32_t)GPB;  // (wave-uniform)
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
        const uint32_t idx = base + (uint32_t)g * U + win_universe<R>(b);
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
}

// One wave's passes over universes u_first, u_first + u_step, ... (chunks of
// UPS = (64 / P) (256 / R) universes, one register set each).  out[u] = the
// first generation in 1..gens whose state contains the target, 0 = never.
// xs / K: the column window (K <= P), y0: the first window row (WRAP: the
// window crosses row 63), as cone_wave_rows.
//
// SHRINK: the light cone narrows by two columns a generation; once the
// columns still needed, K - 2 g1, fit P / 2 lanes, two register sets become
// one: chunks of 2 UPS universes, each set stepped g1 generations and parked
// in the wave's LDS (`stash`, 4 KiB), then read back as one set of P / 2
// lanes per universe (lane j2 of new group 2 s + q takes lane q P + g1 + j2
// of set s -- the window's first g1 columns dropped) and stepped the rest:
// every later generation at half the issue slots.  The target is loaded
// again in each layout (a cached 512-byte read) rather than held twice.
//
// DMA (the whole board, P = 64 and R = 32: chunks of 8 universes = 4 KiB, a
// 16-byte aligned batch): the chunks arrive by LDS-DMA into `stash`
// (dma_fetch_pass), the next one fetched as soon as this one is read out, so
// its loads run under this chunk's generations instead of stalling the wave
// at every chunk's start.  1M universes, the one-row whole-board target
// (row windows of 32 rows), same box: 8 / 13 generations 0.197 / 0.280 ->
// 0.180 / 0.266 ms back to back; every other target within +-3 %
// (profiles/r06/win_dma_ab/).
template <int P, int R, bool WRAP, bool SHRINK, typename OutT, bool DMA = false>
__device__ __forceinline__ void cone_wave_split(const uint64_t *in, const uint64_t *__restrict__ wanted,
                                                const uint64_t *__restrict__ unwanted, OutT *__restrict__ out,
                                                uint64_t n, uint64_t u_first, uint64_t u_step, uint32_t gens,
                                                uint32_t xs, uint32_t K, uint32_t y0, int lane, uint32_t *stash) {
  constexpr int GPS = kWave / P;  // groups (universe columns) per wave
  constexpr int U = 256 / R;      // universes per register per group
  constexpr int UPS = GPS * U;    // universes per register set
  constexpr int CH = SHRINK ? 2 * UPS : UPS;  // universes per chunk
  static_assert(CH <= kWave, "one answer per lane");
  static_assert(P >= 8 && P <= kWave && (!SHRINK || P >= 16), "8 .. 64 lanes per universe");
  static_assert(!DMA || (P == kWave && R == 32 && !SHRINK), "the LDS-DMA form: whole columns, 8 universes");
  constexpr uint32_t rmask = R == 32 ? ~0u : 0xFFFFu;
  const uint32_t j = (uint32_t)lane & (P - 1), q = (uint32_t)lane / P;
  const uint32_t col = (xs + j) & (kWave - 1);
  const bool live = j < K;
  const uint32_t sh = y0 & 31u;
  auto cut = [&](uint64_t v) __attribute__((always_inline)) {
    const W w = split(v);
    return (WRAP ? __builtin_amdgcn_alignbit(w.lo, w.hi, sh) : __builtin_amdgcn_alignbit(w.hi, w.lo, sh)) & rmask;
  };
  // the target in the same layout, replicated over the universes: window
  // column jj in this lane
  auto target = [&](uint32_t jj, uint32_t (&tw_)[8], uint32_t (&tm_)[8]) __attribute__((always_inline)) {
    const uint32_t c = (xs + jj) & (kWave - 1);
    const uint64_t w64 = jj < K ? wanted[c] : 0ull, m64 = jj < K ? (w64 | unwanted[c]) : 0ull;
    uint32_t ew[U], em[U];
    const uint32_t cw = cut(w64), cm = cut(m64);
#pragma unroll
    for (int u = 0; u < U; ++u) ew[u] = cw, em[u] = cm;
    win_pack<R>(ew, tw_);
    win_pack<R>(em, tm_);
  };
  auto load_set = [&](uint64_t ub, uint32_t (&r)[8]) __attribute__((always_inline)) {
    uint32_t e[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t uu = ub + (uint64_t)q * U + u;
      e[u] = (live && uu < n) ? cut(__builtin_nontemporal_load(in + uu * kWave + col)) : 0u;
    }
    win_pack<R>(e, r);
  };
  uint32_t tw[8], tm[8];
  if constexpr (!SHRINK) target(j, tw, tm);
  if constexpr (DMA) {
    uint64_t *const img = reinterpret_cast<uint64_t *>(stash);  // universe m of the chunk: img[m * 64 + column]
    if (u_first < n) dma_fetch_pass<UPS>(in, n, u_first, lane, img);
    int after = 0;  // vector-memory ops issued after the pending fetch (the chunk's answer store)
    for (uint64_t u0 = u_first; u0 < n; u0 += u_step) {
      if (after) __builtin_amdgcn_s_waitcnt(kWaitVm1);
      else __builtin_amdgcn_s_waitcnt(kWaitVm0);
      uint32_t e[U];
#pragma unroll
      for (int u = 0; u < U; ++u) e[u] = cut(img[u * kWave + lane]);  // (past n: universe n - 1 again)
      __builtin_amdgcn_s_waitcnt(kWaitLgkm0);  // read out before the next fetch lands
      if (u0 + u_step < n) dma_fetch_pass<UPS>(in, n, u0 + u_step, lane, img);
      uint32_t r[8];
      win_pack<R>(e, r);
      uint32_t mine = 0;
      uint64_t found = 0;
      win_gens<P, R>(r, tw, tm, 0u, gens, mine, found, 0u, lane);
      if (lane < UPS && u0 + (uint64_t)lane < n) out[u0 + lane] = (OutT)mine;
      after = 1;  // (lane 0 stores: u0 < n)
    }
    return;
  }
  // SHRINK: the generation after which the needed columns fit P / 2 lanes
  const uint32_t g1 = SHRINK ? (K - P / 2 + 1) / 2 : gens;
  for (uint64_t u0 = u_first; u0 < n; u0 += u_step) {
    uint32_t mine = 0;   // lane L: the answer of universe u0 + L
    uint64_t found = 0;  // chunk-local universes already answered
    if constexpr (!SHRINK) {
      uint32_t r[8];
      load_set(u0, r);
      win_gens<P, R>(r, tw, tm, 0u, gens, mine, found, 0u, lane);
    } else {
      constexpr int P2 = P / 2;
      using V4 = __attribute__((ext_vector_type(4))) uint32_t;
      V4 *const st = reinterpret_cast<V4 *>(stash);  // set s, lane L: st[128 s + 2 L], [+ 1]
      {
        uint32_t jj = j;  // (opaque: loaded again per chunk, not held across the merged phase)
        asm volatile("" : "+v"(jj));
        target(jj, tw, tm);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        uint32_t r[8];
        load_set(u0 + (uint64_t)s * UPS, r);
        win_gens<P, R>(r, tw, tm, 0u, g1, mine, found, (uint32_t)(s * UPS), lane);
        st[128 * s + 2 * lane] = V4{r[0], r[1], r[2], r[3]};
        st[128 * s + 2 * lane + 1] = V4{r[4], r[5], r[6], r[7]};
      }
      // lane L of the merged set: group q2 = L / P2 (set q2 / GPS, its group
      // q2 % GPS), column j2 = L % P2 of the narrowed window
      const uint32_t q2 = (uint32_t)lane / P2, j2 = (uint32_t)lane & (P2 - 1);
      const uint32_t src = 128u * (q2 / GPS) + 2u * ((q2 % GPS) * P + g1 + j2);
      const V4 a = st[src], b = st[src + 1];
      uint32_t r2[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      target(g1 + j2, tw, tm);
      win_gens<P2, R>(r2, tw, tm, g1, gens, mine, found, 0u, lane);
    }
    if (lane < CH && u0 + (uint64_t)lane < n) out[u0 + lane] = (OutT)mine;
  }
}

template <typename OutT>
__device__ __forceinline__ void cone_split_pass(const uint64_t *in, const uint64_t *__restrict__ wanted,
                                                const uint64_t *__restrict__ unwanted, OutT *__restrict__ out,
                                                uint64_t n, uint64_t wave, uint64_t nw, uint32_t gens, uint32_t xs,
                                                uint32_t K, int pk, uint32_t y0, int lane,
                                                uint32_t *stash = nullptr, bool dma = false) {
  auto run4 = [&](auto p_c, auto r_c, auto s_c, auto d_c) __attribute__((always_inline)) {
    constexpr int Pc = decltype(p_c)::value, Rc = decltype(r_c)::value;
    constexpr bool Sc = decltype(s_c)::value, Dc = decltype(d_c)::value;
    constexpr uint64_t CH = (uint64_t)(kWave / Pc) * (256 / Rc) * (Sc ? 2 : 1);
    if (wave * CH >= n) return;
    if (y0 >= 32u)
      cone_wave_split<Pc, Rc, true, Sc, OutT, Dc>(in, wanted, unwanted, out, n, wave * CH, nw * CH, gens, xs, K, y0,
                                                  lane, stash);
    else
      cone_wave_split<Pc, Rc, false, Sc, OutT, Dc>(in, wanted, unwanted, out, n, wave * CH, nw * CH, gens, xs, K, y0,
                                                   lane, stash);
  };
  auto run = [&](auto p_c, auto r_c, auto s_c) __attribute__((always_inline)) {
    run4(p_c, r_c, s_c, std::false_type{});
  };
  using I8 = std::integral_constant<int, 8>;
  using I16 = std::integral_constant<int, 16>;
  using I32 = std::integral_constant<int, 32>;
  using I64 = std::integral_constant<int, 64>;
  using T = std::true_type;
  using F = std::false_type;
  // the columns fit half the lanes before the last generation: K - 2 g1 <=
  // P / 2 with g1 < gens (and 2 UPS answers fit the wave's 64 lanes); a
  // caller without a stash never shrinks
  auto shrinks = [&](uint32_t P, int bit) {
    return ((LIFE_SHRINK_MASK >> bit) & 1) && stash && K > P / 2 && (K - P / 2 + 1) / 2 < gens;
  };
  if (pk == 1) {
    if (K <= 8u) return run(I8{}, I32{}, F{});
    if (K <= 16u) return shrinks(16, 0) ? run(I16{}, I32{}, T{}) : run(I16{}, I32{}, F{});
    if (K <= 32u) return shrinks(32, 1) ? run(I32{}, I32{}, T{}) : run(I32{}, I32{}, F{});
    if (shrinks(64, 2)) return run(I64{}, I32{}, T{});
    // (dma: a 16-byte aligned batch with the stash; the whole board only,
    // whose chunks are 4 KiB)
    if (LIFE_WIN_DMA && dma && stash && K == (uint32_t)kWave) return run4(I64{}, I32{}, F{}, T{});
    return run(I64{}, I32{}, F{});
  }
  if (K <= 16u) return run(I16{}, I16{}, F{});
  if (K <= 32u) return shrinks(32, 3) ? run(I32{}, I16{}, T{}) : run(I32{}, I16{}, F{});
  return shrinks(64, 4) ? run(I64{}, I16{}, T{}) : run(I64{}, I16{}, F{});
}

}  // namespace
}  // namespace lifeapi_impl
