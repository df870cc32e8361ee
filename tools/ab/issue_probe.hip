// issue_probe.hip -- VALU issue model of gfx950 for the config-3 loop: ns per
// VALU instruction per SIMD and the in-kernel clock for the probes of
// tools/ab/issue_probe.py, at 1, 2, 4 and 8 waves per SIMD (one 256-thread
// block = one wave per SIMD; resident blocks per CU capped by dynamic LDS;
// grid = one round), on zero and on random register data.
// Build: python tools/ab/issue_probe.py && hipcc --offload-arch=gfx950 -O3 -std=c++17 \
//        -o build/issue_probe tools/ab/issue_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../build/issue_probe.inc"

#define KERN(name)                                                                                   \
  __global__ __launch_bounds__(256) void k_##name(uint32_t iters, uint32_t rnd, uint64_t *stamps) {  \
    extern __shared__ uint32_t pad[];                                                                \
    const uint32_t lane = threadIdx.x & 63;                                                         \
    uint32_t seed = rnd ? (lane * 0x85EBCA6Bu + blockIdx.x * 0xC2B2AE35u + threadIdx.x) | 1u : 0u;  \
    if (iters == 0) pad[threadIdx.x] = seed;                                                         \
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), q0 = __builtin_amdgcn_s_memrealtime();       \
    probe_##name(iters, seed);                                                                       \
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), q1 = __builtin_amdgcn_s_memrealtime();       \
    if (threadIdx.x == 0) {                                                                          \
      stamps[2 * blockIdx.x] = t1 - t0;                                                              \
      stamps[2 * blockIdx.x + 1] = q1 - q0;                                                          \
    }                                                                                                \
  }
ISSUE_PROBES(KERN)

typedef void (*Kern)(uint32_t, uint32_t, uint64_t *);
struct P {
  const char *name;
  Kern k;
};
#define ENTRY(name) {#name, k_##name},
const P kProbes[] = {ISSUE_PROBES(ENTRY)};

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const size_t lds = prop.maxSharedMemoryPerMultiProcessor;
  uint64_t *d_st;
  (void)hipMalloc(&d_st, 8 * cus * 16);
  std::vector<uint64_t> h(2 * 8 * cus);
  const uint32_t iters = 4000;  // 256K VALU per wave
  // warm the clock
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 2.0) {
    hipLaunchKernelGGL(kProbes[0].k, dim3(cus * 8), dim3(256), 0, 0, iters, 1u, d_st);
    (void)hipDeviceSynchronize();
  }
  for (const P &p : kProbes)
    for (int w : {1, 2, 4, 8})
      for (uint32_t rnd : {0u, 1u}) {
        // w blocks resident per CU: dynamic LDS just over 1/(w+1) of the CU
        const size_t dyn = w == 8 ? 0 : (lds / (w + 1) + 1024) & ~(size_t)255;
        int occ = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, p.k, 256, dyn);
        std::vector<float> ms;
        std::vector<double> ghz;
        for (int rep = 0; rep < 5; ++rep) {
          hipEvent_t e0, e1;
          (void)hipEventCreate(&e0);
          (void)hipEventCreate(&e1);
          (void)hipEventRecord(e0);
          hipLaunchKernelGGL(p.k, dim3(cus * w), dim3(256), dyn, 0, iters, rnd, d_st);
          (void)hipEventRecord(e1);
          (void)hipEventSynchronize(e1);
          float t = 0;
          (void)hipEventElapsedTime(&t, e0, e1);
          ms.push_back(t);
          (void)hipMemcpy(h.data(), d_st, 16 * cus * w, hipMemcpyDeviceToHost);
          std::vector<double> c;
          for (int b = 0; b < cus * w; ++b)
            if (h[2 * b + 1]) c.push_back(0.1 * (double)h[2 * b] / (double)h[2 * b + 1]);
          std::sort(c.begin(), c.end());
          ghz.push_back(c[c.size() / 2]);
          (void)hipEventDestroy(e0);
          (void)hipEventDestroy(e1);
        }
        std::sort(ms.begin(), ms.end());
        std::sort(ghz.begin(), ghz.end());
        const double instr_per_simd = (double)w * iters * 64;
        const double ns = ms[2] * 1e6 / instr_per_simd;
        printf("{\"probe\": \"%s\", \"waves_per_simd\": %d, \"occupancy_blocks\": %d, \"data\": \"%s\", "
               "\"ms\": %.4f, \"ns_per_instr_per_simd\": %.4f, \"clock_GHz\": %.3f, \"clk_per_instr\": %.3f}\n",
               p.name, w, occ, rnd ? "random" : "zero", ms[2], ns, ghz[2], ns * ghz[2]);
      }
  return 0;
}
