// tune_cone.hip -- TUNING build: shapes of the light-cone Contains / search
// filter (k_cone, lifeapi_amd/csrc/cone_kernels.hpp) for A/Bs.  Every shape
// computes the same answers as the shipped one.
#include "lifeapi_tune.h"
#include "cone_kernels.hpp"

using namespace lifeapi_impl;

namespace {

template <bool FIRST, typename OutT>
int cone_by_shape(const uint64_t *in, const uint64_t *w, const uint64_t *u, OutT *out, size_t n, uint32_t gens,
                  int upw, int rmax, int cus, hipStream_t st, int cap) {
#define LIFEAPI_CONE(U, R) \
  if (upw == U && rmax == R) return launch_cone<U, R, FIRST>(in, w, u, out, n, gens, cus, st, cap); \
  if (upw == U && rmax == R + 100) return launch_cone<U, R, FIRST, OutT, true>(in, w, u, out, n, gens, cus, st, cap);
  // upw 0: k_cone_adapt (64 universes per chunk for P <= 8, else 16), cap blocks per CU
  if (upw == 0 && rmax == 8) return launch_cone_adapt<8, FIRST>(in, w, u, out, n, gens, cus, st, cap);
  if (upw == 0 && rmax == 16) return launch_cone_adapt<16, FIRST>(in, w, u, out, n, gens, cus, st, cap);
  // upw 1: k_cone_adapt with the whole board through LDS (cone_wave_full_dma, rmax sets per pass)
  if (upw == 1 && rmax == 4) return launch_cone_adapt<4, FIRST, OutT, true>(in, w, u, out, n, gens, cus, st, cap);
  if (upw == 1 && rmax == 8) return launch_cone_adapt<8, FIRST, OutT, true>(in, w, u, out, n, gens, cus, st, cap);
  // upw 3: upw 1 with the whole-board grid capped at `cap` blocks per CU
  if (upw == 3 && rmax == 8)
    return launch_cone_adapt<8, FIRST, OutT, true>(in, w, u, out, n, gens, cus, st, 0, kWave, cap);
  // upw 10: upw 3 with the whole board's first pass fetched only after the
  // row-window search (EARLY = false)
  if (upw == 10 && rmax == 8)
    return launch_cone_adapt<8, FIRST, OutT, true, true, false, false>(in, w, u, out, n, gens, cus, st, 0, kWave, cap);
  // (upw 4, 5, 9: round 5's forms told the last launch report; removed with it)
  // upw 7: upw 0 (the capped form) without the row-window passes
  if (upw == 7 && rmax == 8)
    return launch_cone_adapt<8, FIRST, OutT, false, false>(in, w, u, out, n, gens, cus, st, cap);
  // upw 8: upw 0 (the capped form) with the window split layout (cone_split.hpp) for row windows
  if (upw == 8 && rmax == 8)
    return launch_cone_adapt<8, FIRST, OutT, false, true, true>(in, w, u, out, n, gens, cus, st, cap);
  // upw 2: upw 1 without the packed row-window pass (cone_wave_rows_dma): every whole-board target full
  if (upw == 2 && rmax == 8)
    return launch_cone_adapt<8, FIRST, OutT, true, false>(in, w, u, out, n, gens, cus, st, cap);
  LIFEAPI_CONE(8, 8)
  LIFEAPI_CONE(16, 4)
  LIFEAPI_CONE(16, 8)
  LIFEAPI_CONE(16, 16)
  LIFEAPI_CONE(32, 4)
  LIFEAPI_CONE(32, 8)
  LIFEAPI_CONE(32, 16)
  LIFEAPI_CONE(32, 32)
  LIFEAPI_CONE(64, 8)
  LIFEAPI_CONE(64, 16)
  LIFEAPI_CONE(64, 32)
#undef LIFEAPI_CONE
  return fail(LIFEAPI_E_INVALID, "cone shapes: upw 16/32/64 x rmax 4/8/16/32%s");
}

// The light cone's access shape with nothing else: LPU lanes per universe
// read LPU consecutive words of one 128-byte line of each 512-byte universe
// (16: the whole line; 4: words 8..11 of it, as the cone for a 4-column
// target loads them), 64 universes per wave with every load issued
// together, one uint32 out per universe (whether the words read are
// nonzero), one coalesced store per wave; one-shot grid.
template <int LPU>
__global__ __launch_bounds__(kBlock) void k_line_read(const uint64_t *in, uint32_t *__restrict__ out, uint64_t n,
                                                      uint32_t line) {
  constexpr int UPI = kWave / LPU, NL = 64 / UPI;  // universes per load instruction, loads per wave
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t u0 = wave * 64;
  if (u0 >= n) return;
  const uint32_t word = 16 * line + (LPU == 16 ? 0u : 8u) + (uint32_t)(lane & (LPU - 1));
  uint64_t v[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const uint64_t u = u0 + (uint64_t)UPI * k + lane / LPU;
    v[k] = u < n ? __builtin_nontemporal_load(in + u * kWave + word) : 0ull;
  }
  uint32_t mine = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const uint64_t nz = __ballot(v[k] != 0ull);
    const uint32_t rel = (uint32_t)lane - (uint32_t)(UPI * k);
    if (rel < (uint32_t)UPI) mine = (uint32_t)((nz >> (LPU * rel)) & ((1ull << LPU) - 1)) != 0u;
  }
  if (u0 + lane < n) out[u0 + lane] = mine;
}

// Pacing probe: the row-window pass (cone_wave_rows_dma, 4 universes per
// register) with no window search -- y0 given, the first pass fetched at
// once -- and s_sleep(SLEEP) after each next-pass fetch; uncapped grid of
// chunks of 16 universes.  For targets whose care rows, widened by gens, lie
// in rows y0 + gens .. y0 + 7 - gens (the caller's to ensure).
template <int SLEEP>
__global__ __launch_bounds__(kBlock) void k_rows_probe(const uint64_t *in, const uint64_t *__restrict__ wanted,
                                                       const uint64_t *__restrict__ unwanted, uint32_t *out,
                                                       uint64_t n, uint32_t gens, uint32_t y0) {
  __shared__ uint64_t img_all[kWavesPerBlock][8 * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t nw = (uint64_t)gridDim.x * kWavesPerBlock;
  if (wave * 16 >= n) return;
  uint64_t *img = img_all[__builtin_amdgcn_readfirstlane(threadIdx.x / kWave)];
  dma_fetch_pass<8>(in, n, wave * 16, lane, img);
  const uint64_t w64 = wanted[lane], m64 = w64 | unwanted[lane];
  if (y0 >= 32u)
    cone_wave_rows_dma<8, 4, true, uint32_t, SLEEP>(in, w64, m64, out, n, wave * 16, nw * 16, gens, y0, lane, img,
                                                      true);
  else
    cone_wave_rows_dma<8, 4, false, uint32_t, SLEEP>(in, w64, m64, out, n, wave * 16, nw * 16, gens, y0, lane, img,
                                                       true);
}

}  // namespace

extern "C" {

/* k_rows_probe with s_sleep `sleep` (0, 1, 2, 4, 8, 16) */
int lifeapi_tune_rows_probe(const uint64_t *d_in, const uint64_t *d_wanted, const uint64_t *d_unwanted,
                            uint32_t *d_out, size_t n, uint32_t gens, uint32_t y0, int sleep, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_in || !d_wanted || !d_unwanted || !d_out || !aligned16(d_in) || y0 > 63)
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_tune_rows_probe%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const dim3 grid(grid_for((n + 15) / 16, cus, 0));
  using Fn = void (*)(const uint64_t *, const uint64_t *, const uint64_t *, uint32_t *, uint64_t, uint32_t, uint32_t);
  Fn fn = sleep == 1 ? k_rows_probe<1> : sleep == 2 ? k_rows_probe<2> : sleep == 4 ? k_rows_probe<4>
        : sleep == 8 ? k_rows_probe<8> : sleep == 16 ? k_rows_probe<16> : k_rows_probe<0>;
  hipLaunchKernelGGL(fn, grid, dim3(kBlock), 0, (hipStream_t)stream, d_in, d_wanted, d_unwanted, d_out, (uint64_t)n,
                     gens, y0);
  return launched("k_rows_probe launch");
}

int lifeapi_tune_line_read(const uint64_t *d_in, uint32_t *d_out, size_t n, int line, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  // line + 4 * k: k = 0 the whole line (16 lanes per universe), 1 words 8..11 of it (4 lanes),
  // 2 words 8..15 (8 lanes)
  const int lpu = (line >> 2) == 1 ? 4 : (line >> 2) == 2 ? 8 : 16;
  line &= 3;
  if (!d_in || !d_out || line < 0) return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_tune_line_read%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const dim3 grid(grid_for((n + 63) / 64, cus, 0));
  if (lpu == 4)
    hipLaunchKernelGGL(k_line_read<4>, grid, dim3(kBlock), 0, (hipStream_t)stream, d_in, d_out, (uint64_t)n,
                       (uint32_t)line);
  else if (lpu == 8)
    hipLaunchKernelGGL(k_line_read<8>, grid, dim3(kBlock), 0, (hipStream_t)stream, d_in, d_out, (uint64_t)n,
                       (uint32_t)line);
  else
    hipLaunchKernelGGL(k_line_read<16>, grid, dim3(kBlock), 0, (hipStream_t)stream, d_in, d_out, (uint64_t)n,
                       (uint32_t)line);
  return launched("k_line_read launch");
}

/* rmax + 100: the pipelined pass (cone_wave PIPE).
 * first != 0: the search filter (d_out uint32 first generations, any gens;
 * every window, the whole board included);
 * first == 0: Contains (d_out uint8).  upw universes per wave, rmax register
 * sets per pass; upw + 1000 * c: a grid of at most c blocks per CU looping
 * over the batch (each wave finds the window once). */
int lifeapi_tune_cone(int first, const uint64_t *d_in, const uint64_t *d_wanted, const uint64_t *d_unwanted,
                      void *d_out, size_t n, uint32_t gens, int upw, int rmax, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_in || !d_wanted || !d_unwanted || !d_out)
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_tune_cone%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const int cap = upw / 1000;
  upw %= 1000;
  if (first)
    return cone_by_shape<true>(d_in, d_wanted, d_unwanted, (uint32_t *)d_out, n, gens, upw, rmax, cus,
                               (hipStream_t)stream, cap);
  return cone_by_shape<false>(d_in, d_wanted, d_unwanted, (uint8_t *)d_out, n, 0u, upw, rmax, cus,
                              (hipStream_t)stream, cap);
}

/* the iterated search loop without final states (gens > 2), round 4's first
 * form: the cone kernel launched alone (8 universes per wave, cones of <= 32
 * columns, grid capped at cone_cap blocks per CU, 0 = one-shot), then the
 * split pair (kContainsLo, kContainsHi) with each grid capped at split_cap
 * blocks per CU (0 = one-shot) -- whose kContainsLo now also steps the cone
 * (step_kernels.hpp), so the cone launch's waves have answered first and
 * Lo's rewrite the same values.  cone_cap < 0: no cone launch (the shipped
 * form, step.hip).                                                          */
int lifeapi_tune_search_iter(const uint64_t *d_in, const uint64_t *d_wanted, const uint64_t *d_unwanted,
                             uint32_t *d_first, size_t n, uint32_t gens, int cone_cap, int split_cap, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_in || !d_wanted || !d_unwanted || !d_first || gens <= 2 || split_cap < 0)
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_tune_search_iter%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  // cone_cap + 1000 * u: u universes per cone wave (8, 16, 32; 0 = 8)
  const int upw = cone_cap < 0 ? -1 : cone_cap / 1000;
  cone_cap %= 1000;
  const hipStream_t st = (hipStream_t)stream;
  const uint64_t *w = d_wanted, *u = d_unwanted;
  const uint32_t km = kConeIterColumns;
  if (upw == 16) rc = launch_cone<16, 8, true>(d_in, w, u, d_first, n, gens, cus, st, cone_cap, km);
  else if (upw == 32) rc = launch_cone<32, 8, true>(d_in, w, u, d_first, n, gens, cus, st, cone_cap, km);
  else if (upw == 8) rc = launch_cone<8, 8, true>(d_in, w, u, d_first, n, gens, cus, st, cone_cap, km);
  else if (upw == 0)
    rc = launch_cone<kConeIterUniverses, kConeSets, true>(d_in, w, u, d_first, n, gens, cus, st, cone_cap, km);
  if (rc != LIFEAPI_OK) return rc;
  const dim3 grid(grid_for((n + 3) / 4, cus, split_cap));
  hipLaunchKernelGGL((k_step_contains_split<8, kContainsNet, kContainsLo>), grid, dim3(kBlock), 0, (hipStream_t)stream,
                     d_in, (uint64_t *)nullptr, d_wanted, d_unwanted, d_first, (uint64_t)n, gens, kConeIterColumns);
  rc = launched("k_step_contains_split (tuning) launch");
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL((k_step_contains_split<8, kContainsNet, kContainsHi>), grid, dim3(kBlock), 0, (hipStream_t)stream,
                     d_in, (uint64_t *)nullptr, d_wanted, d_unwanted, d_first, (uint64_t)n, gens, kConeIterColumns);
  return launched("k_step_contains_split (tuning) launch");
}

}  // extern "C"
