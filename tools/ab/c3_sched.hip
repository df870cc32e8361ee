// c3_sched.hip -- same-process A/B of config-3 loop schedules
// (tools/ab/c3_sched.py -> build/c3_sched.inc): the shipped kernel's shape
// (64K universes, 4 per wave, 1024 generations) with each schedule, on the
// random input and on "ash" (the random input after 1024 generations), runs
// interleaved after >= 2.5 s of warm launches; median launch time and the
// in-kernel shader clock per (schedule, input).  One JSON line each.
// Build: python tools/ab/c3_sched.py && hipcc --offload-arch=gfx950 -O3 -std=c++17 \
//        -o build/c3_sched tools/ab/c3_sched.hip
#include "../lifeapi_amd/csrc/split_layout.hpp"

using namespace lifeapi_impl;

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../build/c3_sched.inc"

namespace {

#define C3_KERNEL(name)                                                                                         \
  __global__ __launch_bounds__(kBlock) void k_##name(const uint64_t *in, uint64_t *out, uint64_t n,             \
                                                     uint32_t gens, uint64_t *stamps) {                         \
    constexpr int S = 8, P = 4;                                                                                 \
    __shared__ uint32_t lds[kWavesPerBlock * S * kWave];                                                        \
    const int lane = threadIdx.x & (kWave - 1);                                                                 \
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);                                        \
    const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + wib;                                          \
    const uint64_t u0 = wave * P;                                                                               \
    if (u0 >= n) return;                                                                                        \
    uint32_t r[S];                                                                                              \
    W c[P];                                                                                                     \
    for (int u = 0; u < P; ++u) c[u] = ld<false>(in + (u0 + u) * kWave + lane);                                 \
    Split<S>::load(c, r);                                                                                       \
    const uint32_t base =                                                                                       \
        (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)(lds + wib * S * kWave);           \
    const uint32_t self = base + lane * 16u, prev = base + ((lane + kWave - 1) & (kWave - 1)) * 16u,            \
                   next = base + ((lane + 1) & (kWave - 1)) * 16u;                                              \
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), q0 = __builtin_amdgcn_s_memrealtime();                    \
    diag_##name(r, gens, self, prev, next);                                                                     \
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), q1 = __builtin_amdgcn_s_memrealtime();                    \
    Split<S>::store(r, c);                                                                                      \
    for (int u = 0; u < P; ++u) st<false>(out + (u0 + u) * kWave + lane, c[u]);                                 \
    if (lane == 0) {                                                                                            \
      stamps[wave * 2 + 0] = t1 - t0;                                                                           \
      stamps[wave * 2 + 1] = q1 - q0;                                                                           \
    }                                                                                                           \
  }
C3_SCHEDS(C3_KERNEL)

__global__ void k_fill(uint64_t *p, uint64_t words, uint64_t seed) {
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (uint64_t)gridDim.x * blockDim.x)
    p[w] = mix64(seed + (w + 1) * kGolden);
}

typedef void (*Kern)(const uint64_t *, uint64_t *, uint64_t, uint32_t, uint64_t *);
struct Sched {
  const char *name;
  Kern k;
};
#define C3_ENTRY(name) {#name, k_##name},
const Sched kScheds[] = {C3_SCHEDS(C3_ENTRY)};
constexpr int kN = sizeof(kScheds) / sizeof(kScheds[0]);

struct Run {
  float ms;
  double ghz;
};

Run launch(int s, const uint64_t *in, uint64_t *out, uint64_t n, uint32_t gens, uint64_t *d_st,
           std::vector<uint64_t> &h_st, bool stamp) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const uint64_t waves = n / 4;
  hipEventRecord(e0);
  hipLaunchKernelGGL(kScheds[s].k, dim3((unsigned)(waves / kWavesPerBlock)), dim3(kBlock), 0, 0, in, out, n, gens, d_st);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  double ghz = 0;
  if (stamp) {
    hipMemcpy(h_st.data(), d_st, waves * 16, hipMemcpyDeviceToHost);
    std::vector<double> r;
    for (uint64_t w = 0; w < waves; ++w)
      if (h_st[2 * w + 1]) r.push_back(0.1 * (double)h_st[2 * w] / (double)h_st[2 * w + 1]);
    std::nth_element(r.begin(), r.begin() + r.size() / 2, r.end());
    ghz = r[r.size() / 2];
  }
  return {ms, ghz};
}

}  // namespace

int main(int argc, char **argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1 << 16;  // a multiple of 1024
  const int reps = argc > 2 ? std::atoi(argv[2]) : 9;
  const uint32_t gens = 1024;
  const uint64_t words = n * 64;
  uint64_t *rnd, *ash, *out, *ref, *d_st;
  hipMalloc(&rnd, words * 8);
  hipMalloc(&ash, words * 8);
  hipMalloc(&out, words * 8);
  hipMalloc(&ref, words * 8);
  hipMalloc(&d_st, n / 4 * 16);
  std::vector<uint64_t> h_st(n / 4 * 2), h_ref(words), h_out(words);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, rnd, words, 3ull);
  launch(0, rnd, ash, n, gens, d_st, h_st, false);
  hipDeviceSynchronize();
  // every schedule must give the shipped one's result (bit-exact)
  launch(0, rnd, ref, n, 7, d_st, h_st, false);
  hipMemcpy(h_ref.data(), ref, words * 8, hipMemcpyDeviceToHost);
  std::vector<bool> same(kN);
  for (int s = 0; s < kN; ++s) {
    launch(s, rnd, out, n, 7, d_st, h_st, false);
    hipMemcpy(h_out.data(), out, words * 8, hipMemcpyDeviceToHost);
    same[s] = std::memcmp(h_out.data(), h_ref.data(), words * 8) == 0;
  }
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 2.5)
    for (int i = 0; i < 20; ++i)
      hipLaunchKernelGGL(kScheds[0].k, dim3((unsigned)(n / 4 / kWavesPerBlock)), dim3(kBlock), 0, 0, rnd, out, n,
                         gens, d_st);
  hipDeviceSynchronize();
  const uint64_t *inputs[2] = {rnd, ash};
  const char *names[2] = {"random", "ash"};
  std::vector<float> ms[kN][2];
  std::vector<double> ghz[kN][2];
  for (int rep = 0; rep < reps; ++rep)
    for (int s = 0; s < kN; ++s)
      for (int d = 0; d < 2; ++d) {
        for (int k = 0; k < 3; ++k) launch(s, inputs[d], out, n, gens, d_st, h_st, false);
        Run r = launch(s, inputs[d], out, n, gens, d_st, h_st, true);
        ms[s][d].push_back(r.ms);
        ghz[s][d].push_back(r.ghz);
      }
  for (int s = 0; s < kN; ++s)
    for (int d = 0; d < 2; ++d) {
      auto &m = ms[s][d];
      auto &g = ghz[s][d];
      std::sort(m.begin(), m.end());
      std::sort(g.begin(), g.end());
      const double kclk = m[reps / 2] * g[reps / 2] * 1e3;  // kilocycles at the held clock
      printf("{\"n\": %llu, \"sched\": \"%s\", \"input\": \"%s\", \"bit_exact\": %s, \"ms_median\": %.4f, \"ms_min\": %.4f, "
             "\"clock_GHz_median\": %.3f, \"kclk_median\": %.0f}\n",
             (unsigned long long)n, kScheds[s].name, names[d], same[s] ? "true" : "false", m[reps / 2], m[0],
             g[reps / 2], kclk);
    }
  return 0;
}
