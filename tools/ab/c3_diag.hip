// c3_diag.hip -- where does a generation of the shipped config-3 loop spend
// its time?  The shipped kernel's shape (k_step_split<8, 1, false, 6,
// kAsmLoop>: 64K universes, 4 per wave, 1024 generations) with the assembly
// loop replaced by diagnostic cuts of it (build/c3_diag.inc from
// tools/ab/c3_diag.py), on three inputs: uniform random, all zero, and "ash"
// (the random input after 1024 generations, what the loop mostly sees).
// Per (cut, input): median launch time and the in-kernel shader clock
// (s_memtime / s_memrealtime around the loop, MI355X_MICROARCH.md DVFS
// item 6) after >= 2 s of back-to-back launches.  One JSON line each.
// Build: python tools/ab/c3_diag.py && hipcc --offload-arch=gfx950 -O3 -std=c++17 \
//        -o build/c3_diag tools/ab/c3_diag.hip
#include "../lifeapi_amd/csrc/split_layout.hpp"

using namespace lifeapi_impl;

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../build/c3_diag.inc"

namespace {


template <int CUT>
__global__ __launch_bounds__(kBlock) void k_diag(const uint64_t *in, uint64_t *out, uint64_t n, uint32_t gens,
                                                 uint64_t *stamps) {
  constexpr int S = 8, P = 4;
  __shared__ uint32_t lds[kWavesPerBlock * S * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + wib;
  const uint64_t u0 = wave * P;
  if (u0 >= n) return;
  uint32_t r[S];
  W c[P];
#pragma unroll
  for (int u = 0; u < P; ++u) c[u] = ld<false>(in + (u0 + u) * kWave + lane);
  Split<S>::load(c, r);
  const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)(lds + wib * S * kWave);
  const uint32_t self = base + lane * 16u, prev = base + ((lane + kWave - 1) & (kWave - 1)) * 16u,
                 next = base + ((lane + 1) & (kWave - 1)) * 16u;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), q0 = __builtin_amdgcn_s_memrealtime();
  if constexpr (CUT == 0) diag_full(r, gens, self, prev, next);
  if constexpr (CUT == 1) diag_nolds(r, gens, self, prev, next);
  if constexpr (CUT == 2) diag_norot(r, gens, self, prev, next);
  if constexpr (CUT == 3) diag_valu_only(r, gens, self, prev, next);
  if constexpr (CUT == 4) diag_lds_only(r, gens, self, prev, next);
  if constexpr (CUT == 5) diag_half_write(r, gens, self, prev, next);
  if constexpr (CUT == 6) diag_half_read(r, gens, self, prev, next);
  if constexpr (CUT == 7) diag_no_write(r, gens, self, prev, next);
  if constexpr (CUT == 8) diag_no_read(r, gens, self, prev, next);
  if constexpr (CUT == 9) diag_b64(r, gens, self, prev, next);
  if constexpr (CUT == 10) diag_prio1(r, gens, self, prev, next);
  if constexpr (CUT == 11) diag_prio_e(r, gens, self, prev, next);
  if constexpr (CUT == 12) {  // odd blocks one priority class higher (static, guide "Two waves per SIMD" item 4)
    if (blockIdx.x & 1) diag_hi(r, gens, self, prev, next);
    else diag_full(r, gens, self, prev, next);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), q1 = __builtin_amdgcn_s_memrealtime();
  Split<S>::store(r, c);
#pragma unroll
  for (int u = 0; u < P; ++u) st<false>(out + (u0 + u) * kWave + lane, c[u]);
  if (lane == 0) {
    stamps[wave * 2 + 0] = t1 - t0;
    stamps[wave * 2 + 1] = q1 - q0;
  }
}

__global__ void k_fill(uint64_t *p, uint64_t words, uint64_t seed) {
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (uint64_t)gridDim.x * blockDim.x)
    p[w] = mix64(seed + (w + 1) * kGolden);
}

typedef void (*Kern)(const uint64_t *, uint64_t *, uint64_t, uint32_t, uint64_t *);
struct Cut {
  const char *name;
  Kern k;
  int upw;  // universes per wave
};
const Cut kCuts[] = {{"full", k_diag<0>, 4},      {"nolds", k_diag<1>, 4},      {"norot", k_diag<2>, 4},
                     {"valu_only", k_diag<3>, 4}, {"lds_only", k_diag<4>, 4},   {"half_write", k_diag<5>, 4},
                     {"half_read", k_diag<6>, 4}, {"no_write", k_diag<7>, 4},   {"no_read", k_diag<8>, 4},
                     {"b64", k_diag<9>, 4},       {"prio1", k_diag<10>, 4},     {"prio_e", k_diag<11>, 4},
                     {"odd_blocks_hi", k_diag<12>, 4}};
constexpr int kNCuts = sizeof(kCuts) / sizeof(kCuts[0]);

struct Run {
  float ms;
  double ghz;
};

Run launch(int cut, const uint64_t *in, uint64_t *out, uint64_t n, uint32_t gens, uint64_t *d_st,
           std::vector<uint64_t> &h_st, bool stamp) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const uint64_t waves = n / kCuts[cut].upw;
  hipEventRecord(e0);
  hipLaunchKernelGGL(kCuts[cut].k, dim3((unsigned)(waves / kWavesPerBlock)), dim3(kBlock), 0, 0, in, out, n, gens, d_st);
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
  const uint32_t gens = 1024;
  const uint64_t words = n * 64;
  uint64_t *rnd, *zero, *ash, *out, *d_st;
  hipMalloc(&rnd, words * 8);
  hipMalloc(&zero, words * 8);
  hipMalloc(&ash, words * 8);
  hipMalloc(&out, words * 8);
  hipMalloc(&d_st, n / 4 * 16);
  std::vector<uint64_t> h_st(n / 4 * 2);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, rnd, words, 3ull);
  hipMemset(zero, 0, words * 8);
  launch(0, rnd, ash, n, gens, d_st, h_st, false);
  hipDeviceSynchronize();
  // warm the clock: >= 2 s of back-to-back full launches on the random input
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 2.5)
    for (int i = 0; i < 20; ++i)
      hipLaunchKernelGGL(kCuts[0].k, dim3((unsigned)(n / 4 / kWavesPerBlock)), dim3(kBlock), 0, 0, rnd, out, n, gens, d_st);
  hipDeviceSynchronize();
  const uint64_t *inputs[3] = {rnd, zero, ash};
  const char *names[3] = {"random", "zero", "ash"};
  constexpr int kReps = 7;
  std::vector<float> ms[kNCuts][3];
  std::vector<double> ghz[kNCuts][3];
  for (int rep = 0; rep < kReps; ++rep)
    for (int cut = 0; cut < kNCuts; ++cut)
      for (int d = 0; d < 3; ++d) {
        for (int k = 0; k < 3; ++k) launch(cut, inputs[d], out, n, gens, d_st, h_st, false);  // settle
        Run r = launch(cut, inputs[d], out, n, gens, d_st, h_st, true);
        ms[cut][d].push_back(r.ms);
        ghz[cut][d].push_back(r.ghz);
      }
  for (int cut = 0; cut < kNCuts; ++cut)
    for (int d = 0; d < 3; ++d) {
      auto &m = ms[cut][d];
      auto &g = ghz[cut][d];
      std::sort(m.begin(), m.end());
      std::sort(g.begin(), g.end());
      printf("{\"n\": %llu, \"cut\": \"%s\", \"input\": \"%s\", \"ms_median\": %.4f, \"ms_min\": %.4f, \"clock_GHz_median\": %.3f, "
             "\"clock_GHz_min\": %.3f, \"clock_GHz_max\": %.3f}\n",
             (unsigned long long)n, kCuts[cut].name, names[d], m[kReps / 2], m[0], g[kReps / 2], g[0], g[kReps - 1]);
    }
  return 0;
}
