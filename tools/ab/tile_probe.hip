// tile_probe.hip -- issue rate of the tile-layout generation loop (RULE 8) on
// gfx950: the generated bank-conflict-free loop with and without its LDS
// exchange (build/tile_probe.inc from tools/gen_tile_asm.py), next to the
// compiler-allocated LDS and DPP versions, on the config-3 shape (4096 waves
// = 4 per SIMD, 1024 generations).  Prints ns per VALU per SIMD and the
// in-kernel shader clock.  Results are garbage data; only the time matters.
// Build: see tools/ab/gpu_tile_probe.sh
#include "../lifeapi_amd/csrc/split_layout.hpp"

using namespace lifeapi_impl;

#include <cstdio>

#include "../build/tile_probe.inc"

namespace {

template <int MODE>
__global__ __launch_bounds__(kBlock) void probe(uint32_t *out, uint32_t gens, unsigned long long *clk) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), q0 = __builtin_amdgcn_s_memrealtime();
  __shared__ uint32_t lds[kWavesPerBlock * 1024];
  const int lane = threadIdx.x & 63;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  uint32_t *slot = lds + wib * 1024;
  uint32_t r[4][8];
  for (int c = 0; c < 4; ++c)
    for (int j = 0; j < 8; ++j) r[c][j] = (uint32_t)mix64(threadIdx.x * 977 + blockIdx.x * 31337 + c * 8 + j);
  const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)slot;
  const int g0 = lane & ~15;
  const uint32_t as = base + lane * 16u, ap = base + (g0 | ((lane + 15) & 15)) * 16u,
                 an = base + (g0 | ((lane + 1) & 15)) * 16u;
  if constexpr (MODE == 0) tile_full(r, gens, as, ap, an);
  if constexpr (MODE == 1) tile_nolds(r, gens, as, ap, an);
  if constexpr (MODE == 2)
    for (uint32_t i = 0; i < gens; ++i) gen_tile<8, 4, XLDS>(r, slot, lane);
  if constexpr (MODE == 3)
    for (uint32_t i = 0; i < gens; ++i) gen_tile<8, 4, XDPP>(r, slot, lane);
  uint32_t acc = 0;
  for (int c = 0; c < 4; ++c)
    for (int j = 0; j < 8; ++j) acc ^= r[c][j];
  out[blockIdx.x * kBlock + threadIdx.x] = acc;
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), q1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    atomicAdd(&clk[0], (unsigned long long)(t1 - t0));
    atomicAdd(&clk[1], (unsigned long long)(q1 - q0));
  }
}

template <int MODE>
void run(const char *name, uint32_t *d_out, unsigned long long *d_clk, int blocks, uint32_t gens, int valu) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e9;
  unsigned long long clk[2] = {0, 0};
  for (int rep = 0; rep < 6; ++rep) {
    hipMemset(d_clk, 0, 16);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(kBlock), 0, 0, d_out, gens, d_clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) {
      best = ms;
      hipMemcpy(clk, d_clk, 16, hipMemcpyDeviceToHost);
    }
  }
  const double waves_per_simd = blocks * 4.0 / 1024.0;
  const double ns_per_valu = best * 1e6 / (waves_per_simd * gens * valu);
  printf("{\"variant\": \"%s\", \"blocks\": %d, \"ms_best\": %.4f, \"valu_per_gen\": %d, "
         "\"ns_per_valu_per_simd\": %.4f, \"clock_GHz\": %.3f}\n",
         name, blocks, best, valu, ns_per_valu, clk[1] ? 0.1 * (double)clk[0] / (double)clk[1] : 0.0);
}

}  // namespace

int main() {
  uint32_t *d_out;
  unsigned long long *d_clk;
  hipMalloc(&d_out, 1 << 24);
  hipMalloc(&d_clk, 16);
  const uint32_t gens = 1024;
  for (int blocks : {1024, 512}) {
    run<0>("asm_lds", d_out, d_clk, blocks, gens, 304);
    run<1>("asm_no_lds", d_out, d_clk, blocks, gens, 304);
    run<2>("cc_lds", d_out, d_clk, blocks, gens, 304);
    run<3>("cc_dpp", d_out, d_clk, blocks, gens, 320);
  }
  return 0;
}
