// tune_stencils.hip -- TUNING build: the LifeStable kernels of the product
// (stable_kernels.hpp) launched on an explicit grid, for the grid-cap A/Bs
// behind stencils.hip's launch choices (tools/ab/stable_grid_ab.py); and the
// other streaming stencils (stencil_kernels.hpp) with an occupancy cap
// (tools/ab/stencil_occupancy_ab.py).
#include "lifeapi_tune.h"
#include "host.hpp"
#include "stable_kernels.hpp"
#include "stencil_kernels.hpp"
#include "step_kernels.hpp"

using namespace lifeapi_impl;

namespace {

// The prefetching loop (round 3, measured slower): each wave
// loops over the batch (a grid of at most the resident waves) and loads the
// next LifeStable's planes before it works on the current one.
template <int PASS>
__device__ __forceinline__ int stable_run(W (&p)[10], uint32_t max_iters) {
  W chg = W{0u, 0u};  // (this form stores every line)
  if constexpr (PASS == 0) return stable_sync(p, chg);
  else if constexpr (PASS == 1) return stable_options(p, chg);
  else if constexpr (PASS == 2) return stable_signal(p, chg);
  else if constexpr (PASS == 3) return stable_step(p, chg);
  int ever = 0;
  for (uint32_t it = 0; it < max_iters; ++it) {
    if constexpr (PASS == 5) {  // StabiliseOptions (LifeStable.hpp:677-693)
      const int k = stable_sync(p, chg);
      if (!(k & 1)) return 0;
      const int o = stable_options(p, chg);
      if (!(o & 1)) return 0;
      if (!((k | o) & 2)) return 1 | ever;
    } else {  // Propagate (LifeStable.hpp:718-729)
      const int s = stable_step(p, chg);
      if (!(s & 1)) return 0;
      if (!(s & 2)) return 1 | ever;
    }
    ever = 2;
  }
  return 1 | ever | 4;
}

template <int PASS>
__global__ __launch_bounds__(kBlock) void k_stable_pf(uint64_t *__restrict__ planes, uint8_t *__restrict__ flags,
                                                      uint64_t n, uint32_t max_iters, uint32_t mode) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  uint64_t k0 = (uint64_t)blockIdx.x * kWavesPerBlock + wib;
  if (k0 >= n) return;
  const bool rev = (mode & 1u) != 0;
  W p[10], pn[10];
  {
    const uint64_t *q = planes + (rev ? n - 1 - k0 : k0) * 10 * kWave + lane;
#pragma unroll
    for (int k = 0; k < 10; ++k) p[k] = ld<true>(q + k * kWave);
  }
  for (; k0 < n; k0 += stride) {
    const uint64_t u = rev ? n - 1 - k0 : k0, k1 = k0 + stride;
    if (k1 < n) {
      const uint64_t *qn = planes + (rev ? n - 1 - k1 : k1) * 10 * kWave + lane;
#pragma unroll
      for (int k = 0; k < 10; ++k) pn[k] = ld<true>(qn + k * kWave);
    }
    const int r = stable_run<PASS>(p, max_iters);
    uint64_t *q = planes + u * 10 * kWave + lane;
#pragma unroll
    for (int k = 0; k < 10; ++k) st<true>(q + k * kWave, p[k]);
    if (lane == 0) flags[u] = (uint8_t)r;
#pragma unroll
    for (int k = 0; k < 10; ++k) p[k] = pn[k];
  }
}

// The pass repeated `reps` times on each LifeStable's planes in VGPRs, each
// repetition on the input again (so every repetition does the same work),
// the last result stored: the pass's VALU side with its memory side paid
// once (a probe of the issue rate, tools/stable_valu_probe.py).
template <int PASS>
__global__ __launch_bounds__(kBlock) void k_stable_rep(uint64_t *__restrict__ planes, uint8_t *__restrict__ flags,
                                                       uint64_t n, uint32_t max_iters, uint32_t reps) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t u = xcd_chunk_block() * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  if (u >= n) return;
  uint64_t *q = planes + u * 10 * kWave + lane;
  W p0[10], p[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) p0[k] = ld<true>(q + k * kWave);
  int r = 0;
  for (uint32_t i = 0; i < reps; ++i) {
#pragma unroll
    for (int k = 0; k < 10; ++k) p[k] = p0[k];
    r = stable_run<PASS>(p, max_iters);
    // (keep p0 live and the repetitions distinct)
    p0[0].lo ^= (uint32_t)__builtin_amdgcn_readfirstlane((int)(r & 0x100));
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) st<true>(q + k * kWave, p[k]);
  if (lane == 0) flags[u] = (uint8_t)r;
}

}  // namespace

extern "C" {

int lifeapi_tune_stable_rep(uint64_t *d_planes, uint8_t *d_flags, size_t n, int pass, uint32_t reps, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_planes || !d_flags || pass < 0 || pass > 5) return fail(LIFEAPI_E_INVALID, "bad argument%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  using Fn = void (*)(uint64_t *, uint8_t *, uint64_t, uint32_t, uint32_t);
  const Fn fns[6] = {k_stable_rep<0>, k_stable_rep<1>, k_stable_rep<2>, k_stable_rep<3>, k_stable_rep<4>,
                     k_stable_rep<5>};
  hipLaunchKernelGGL(fns[pass], dim3(grid_for(n, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream, d_planes, d_flags,
                     (uint64_t)n, 1u << 20, reps);
  return launched("k_stable_rep launch");
}

int lifeapi_tune_stable_pass(uint64_t *d_planes, uint8_t *d_flags, size_t n, int pass, uint32_t max_iters,
                             int blocks_per_cu, void *stream, int reverse) {
  if (n == 0) return LIFEAPI_OK;
  // k_stable_dma on a grid of blocks_per_cu (0: all resident) per CU:
  // 16 + k: pass k, nt fetch, counted waits; 24 + k: plain fetch, counted;
  // 32 + k: nt fetch, counted, the changed lines stored 16 bytes per lane
  // through the image (U = 1 only); k in {0, 4} for the plain fetch
  // 38 / 39: StabiliseOptions / Propagate as 37 / 36 with the iterations
  // after the first on a 32-row window (PW = true; the product ships PW = false)
  if (pass >= 16 && pass <= 39) {
    if (!d_planes || !d_flags || !aligned8(d_planes)) return fail(LIFEAPI_E_INVALID, "bad argument%s");
    int cus = 0, rc = device_cus(cus);
    if (rc != LIFEAPI_OK) return rc;
    using Fn = void (*)(uint64_t *, uint8_t *, uint64_t, uint32_t, uint32_t);
    const Fn fns[24] = {k_stable_dma<0>, k_stable_dma<1>, k_stable_dma<2>, k_stable_dma<3>, k_stable_dma<4>,
                        k_stable_dma<5>, nullptr, nullptr,
                        k_stable_dma<0, 0>, nullptr, nullptr, nullptr, k_stable_dma<4, 0>, nullptr, nullptr, nullptr,
                        k_stable_dma<0, 2, true, true>, k_stable_dma<1, 2, true, true>,
                        k_stable_dma<2, 2, true, true>, k_stable_dma<3, 2, true, true>,
                        k_stable_dma<4, 2, true, true>, k_stable_dma<5, 2, true, true>,
                        k_stable_dma<5, 2, true, true, true>, k_stable_dma<4, 2, true, true, true>};
    if (!fns[pass - 16]) return fail(LIFEAPI_E_INVALID, "no such k_stable_dma variant%s");
    int res = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&res, fns[pass - 16], kBlock, 0);
    if (e != hipSuccess || res < 1) return fail(LIFEAPI_E_INVALID, "k_stable_dma cannot be resident%s");
    // reverse >> 8 = U > 0: ceil(n / U) waves of U LifeStables each (blocks_per_cu
    // then caps the resident blocks by unused LDS), else the looping grid
    const uint32_t upw = (uint32_t)reverse >> 8;
    uint64_t grid;
    unsigned lds = 0;
    if (upw) {
      grid = grid_for((n + upw - 1) / upw, cus, 0);
      if (blocks_per_cu > 0 && (rc = occupancy_lds((const void *)fns[pass - 16], blocks_per_cu, lds)) != LIFEAPI_OK)
        return rc;
    } else {
      const int bpc = blocks_per_cu > 0 ? std::min(blocks_per_cu, res) : res;
      grid = std::min<uint64_t>((uint64_t)cus * bpc, (n + kWavesPerBlock - 1) / kWavesPerBlock);
      grid = (grid + 7) & ~7ull;  // every XCD takes part: the eighths are dealt by blockIdx & 7
    }
    hipLaunchKernelGGL(fns[pass - 16], dim3((unsigned)grid), dim3(kBlock), lds, (hipStream_t)stream, d_planes,
                       d_flags, (uint64_t)n, max_iters ? max_iters : 1u << 20, (uint32_t)reverse);
    return launched("k_stable_dma (tuning) launch");
  }
  // pass 8 + k: pass k with the prefetching loop (k_stable_pf<k>)
  // pass 14 / 15: Propagate with every step on the whole columns / the steps
  // after the first on a 32-row window (k_stable<4, PW>; the product ships
  // PW = kPropagateWindow = true); pass 6 / 7: StabiliseOptions in k_stable
  // with every round on the whole columns / the rounds after the first on
  // the window, columns stashed in LDS (k_stable<5, PW, SW>)
  // pass 40: Propagate as 15, each plane's dirty line stored only where the
  // plane changed (k_stable<4, true, false, true>)
  if (!d_planes || !d_flags || !aligned8(d_planes) || pass < 0 || (pass > 15 && pass != 40))
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_tune_stable_pass%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  using Fn = void (*)(uint64_t *, uint8_t *, uint64_t, uint32_t, uint32_t);
  const Fn fns[17] = {k_stable<0>, k_stable<1>, k_stable<2>, k_stable<3>, k_stable<4>, k_stable<5>,
                      k_stable<5, true, false>, k_stable<5, true, true>,
                      k_stable_pf<0>, k_stable_pf<1>, k_stable_pf<2>, k_stable_pf<3>, k_stable_pf<4>, k_stable_pf<5>,
                      k_stable<4, false>, k_stable<4, true>, k_stable<4, true, false, true>};
  if (pass == 40) pass = 16;
  // blocks_per_cu < 0: uncapped grid, at most -blocks_per_cu blocks resident
  // per CU (unused dynamic LDS out of the CU's 160 KiB)
  unsigned lds = 0;
  if (blocks_per_cu < 0 && (rc = occupancy_lds((const void *)fns[pass], -blocks_per_cu, lds)) != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(fns[pass], dim3(grid_for(n, cus, blocks_per_cu > 0 ? blocks_per_cu : 0)), dim3(kBlock), lds,
                     (hipStream_t)stream, d_planes, d_flags, (uint64_t)n, max_iters ? max_iters : 1u << 20,
                     (uint32_t)reverse);
  return launched("k_stable (tuning) launch");
}

int lifeapi_tune_stable_vulnerable(const uint64_t *d_planes, uint64_t *d_out, size_t n, int blocks_per_cu,
                                   void *stream) {
  // blocks_per_cu + 1000: the XCD-chunked block mapping (k_stable_vulnerable<true>)
  const bool chunk = blocks_per_cu >= 500;
  if (chunk) blocks_per_cu -= 1000;
  if (n == 0) return LIFEAPI_OK;
  if (!d_planes || !d_out || !aligned8(d_planes) || !aligned8(d_out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_tune_stable_vulnerable%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const void *fn = chunk ? (const void *)k_stable_vulnerable<true> : (const void *)k_stable_vulnerable<false>;
  unsigned lds = 0;
  if (blocks_per_cu < 0 && (rc = occupancy_lds(fn, -blocks_per_cu, lds)) != LIFEAPI_OK) return rc;
  const dim3 grid(grid_for(n, cus, blocks_per_cu > 0 ? blocks_per_cu : 0));
  if (chunk)
    hipLaunchKernelGGL(k_stable_vulnerable<true>, grid, dim3(kBlock), lds, (hipStream_t)stream, d_planes, d_out,
                       (uint64_t)n);
  else
    hipLaunchKernelGGL(k_stable_vulnerable<false>, grid, dim3(kBlock), lds, (hipStream_t)stream, d_planes, d_out,
                       (uint64_t)n);
  return launched("k_stable_vulnerable (tuning) launch");
}

/* the product's streaming stencils with at most `resident` blocks per CU
 * (0 = as many as fit): kind 0..2 = k_counts<kind> (NeighbourCount,
 * InteractionCounts, ...AndNext; in = n universes, out = their planes),
 * 3 = k_weld one generation (in place on in = n LifeWelds), 4 = k_refined
 * (in = n x 11 planes, out = n x 3 planes); kind + 8: the same with the
 * XCD-chunked block mapping (CHUNK = true)                                  */
}  // extern "C"
template <bool C>
static int tune_stencil(int kind, const uint64_t *d_in, uint64_t *d_out, size_t n, int resident, void *stream) {
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  unsigned lds = 0;
  if (resident) {
    const void *fns[5] = {(const void *)k_counts<0, C>, (const void *)k_counts<1, C>, (const void *)k_counts<2, C>,
                          (const void *)k_weld<C>, (const void *)k_refined<1, 0, C>};
    rc = occupancy_lds(fns[kind], resident, lds);
    if (rc != LIFEAPI_OK) return rc;
  }
  const dim3 grid(grid_for(n, cus, 0));
  switch (kind) {
    case 0: hipLaunchKernelGGL((k_counts<0, C>), grid, dim3(kBlock), lds, (hipStream_t)stream, d_in, d_out, (uint64_t)n); break;
    case 1: hipLaunchKernelGGL((k_counts<1, C>), grid, dim3(kBlock), lds, (hipStream_t)stream, d_in, d_out, (uint64_t)n); break;
    case 2: hipLaunchKernelGGL((k_counts<2, C>), grid, dim3(kBlock), lds, (hipStream_t)stream, d_in, d_out, (uint64_t)n); break;
    case 3:
      // one order, nontemporal throughout (the launch before the product's order policy)
      hipLaunchKernelGGL(k_weld<C>, grid, dim3(kBlock), lds, (hipStream_t)stream, (uint64_t *)d_in, (uint64_t)n, 1u,
                         ~(uint64_t)0);
      break;
    default:
      hipLaunchKernelGGL((k_refined<1, 0, C>), grid, dim3(kBlock), lds, (hipStream_t)stream, d_in, d_out, (uint64_t)n);
  }
  return launched("stencil (tuning) launch");
}
extern "C" {
int lifeapi_tune_stencil(int kind, const uint64_t *d_in, uint64_t *d_out, size_t n, int resident, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  const int k = kind & 7;
  if (!d_in || kind < 0 || kind > 12 || k > 4 || resident < 0 || (k != 3 && !d_out))
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_tune_stencil%s");
  return kind >= 8 ? tune_stencil<true>(k, d_in, d_out, n, resident, stream)
                   : tune_stencil<false>(k, d_in, d_out, n, resident, stream);
}

/* resident blocks per CU of a shipped kernel under the occupancy cap
 * occupancy_lds sets for `want` (which: 0 = the streaming k_step, 1..6 =
 * k_stable<which-1>, 7 = k_stable_vulnerable): *got from the occupancy API */
int lifeapi_tune_capped_occupancy(int which, int want, int *got) {
  if (!got || which < 0 || which > 7 || want < 1) return fail(LIFEAPI_E_INVALID, "bad argument%s");
  const void *fns[8] = {(const void *)k_step<XDPP, 8, true, 3, true>,
                        (const void *)k_stable<0>, (const void *)k_stable<1>, (const void *)k_stable<2>,
                        (const void *)k_stable<3>, (const void *)k_stable<4>, (const void *)k_stable<5>,
                        (const void *)k_stable_vulnerable<false>};
  unsigned lds = 0;
  int rc = occupancy_lds(fns[which], want, lds);
  if (rc != LIFEAPI_OK) return rc;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(got, fns[which], kBlock, lds);
  return e == hipSuccess ? LIFEAPI_OK : fail_hip(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
}

/* the product's launch-order book (host.hpp launch_reverse): 1 = a launch
 * reading d_in (bytes) and writing d_out on the current device would take
 * the reverse order; records d_out, as the product's launchers do        */
int lifeapi_tune_order_probe(const void *d_in, const void *d_out, uint64_t bytes) {
  return launch_reverse(d_in, d_out, bytes) ? 1 : 0;
}

/* the book's note_forward_write: d_out (bytes) recorded as written forward */
void lifeapi_tune_order_note(const void *d_out, uint64_t bytes) { note_forward_write(d_out, bytes); }

/* k_weld one generation in place with u welds per wave (1, 2, 4), at most
 * `resident` blocks per CU (0 = all), each XCD a contiguous eighth if
 * `chunk`, nontemporal throughout, one order                                */
int lifeapi_tune_weld_u(uint64_t *d_welds, size_t n, int u, int resident, int chunk, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_welds || (u != 1 && u != 2 && u != 4) || resident < 0) return fail(LIFEAPI_E_INVALID, "bad argument%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  using Fn = void (*)(uint64_t *, uint64_t, uint32_t, uint64_t);
  const Fn fns[2][3] = {{k_weld<false, 1>, k_weld<false, 2>, k_weld<false, 4>},
                        {k_weld<true, 1>, k_weld<true, 2>, k_weld<true, 4>}};
  const Fn fn = fns[chunk ? 1 : 0][u == 1 ? 0 : u == 2 ? 1 : 2];
  unsigned lds = 0;
  if (resident && (rc = occupancy_lds((const void *)fn, resident, lds)) != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(grid_for((n + u - 1) / u, cus, 0)), dim3(kBlock), lds, (hipStream_t)stream, d_welds,
                     (uint64_t)n, 1u, ~(uint64_t)0);
  return launched("k_weld (u) launch");
}

/* k_weld one generation in place, the order reversed if `reverse`, the
 * welds taken from position n - plain_welds on loaded and stored plain     */
int lifeapi_tune_weld_order(uint64_t *d_welds, size_t n, int reverse, uint64_t plain_welds, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_welds) return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_tune_weld_order%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(k_weld<false>, dim3(grid_for(n, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream, d_welds, (uint64_t)n,
                     1u | (reverse ? kWeldReverse : 0u), plain_welds < n ? (uint64_t)n - plain_welds : (uint64_t)0);
  return launched("k_weld (order) launch");
}

}  // extern "C"
