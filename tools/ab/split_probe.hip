// split_probe.hip -- where does a generation of the row-split loop spend its
// time?  The same loop as k_step_split<S, 1> with the LDS exchange and/or the
// bitop3 network switched off (MODE bit 0: exchange, bit 1: network), timed
// with HIP events on 64K universes x 1024 generations (config 3).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude tools/ab/split_probe.hip
//        -Llifeapi_amd -llifeapi_hip -Wl,-rpath,$PWD/lifeapi_amd
#include "../lifeapi_amd/csrc/split_layout.hpp"

using namespace lifeapi_impl;

#include <cstdio>

namespace {

template <int S, int MODE>
__global__ __launch_bounds__(kBlock) void probe(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                uint64_t n, uint32_t gens, uint64_t *clk) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  constexpr int P = S / 2;
  typedef uint32_t vec __attribute__((ext_vector_type(S)));
  __shared__ uint32_t lds[kWavesPerBlock * S * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wib) * P;
  if (u0 >= n) return;
  uint32_t r[S];
  W c[P];
  for (int u = 0; u < P; ++u) c[u] = ld<false>(in + (u0 + u) * kWave + lane);
  Split<S>::load(c, r);
  vec *v = reinterpret_cast<vec *>(lds + wib * S * kWave);
  for (uint32_t it = 0; it < gens; ++it) {
    uint32_t lv[S], rv[S];
    if constexpr (MODE & 1) {
      constexpr int Q = S < 4 ? S : 4;  // as gen_split: planes of <= 16 B per lane
      typedef uint32_t qv __attribute__((ext_vector_type(Q)));
      qv *w = reinterpret_cast<qv *>(v);
      for (int p = 0; p < S / Q; ++p) {
        qv m;
        for (int q = 0; q < Q; ++q) m[q] = r[p * Q + q];
        w[p * kWave + lane] = m;
      }
      for (int p = 0; p < S / Q; ++p) {
        const qv l = w[p * kWave + ((lane + kWave - 1) & (kWave - 1))], rr = w[p * kWave + ((lane + 1) & (kWave - 1))];
        for (int q = 0; q < Q; ++q) lv[p * Q + q] = l[q], rv[p * Q + q] = rr[q];
      }
    } else {
      for (int j = 0; j < S; ++j) lv[j] = r[j] ^ it, rv[j] = r[j] + it;
    }
    if constexpr (MODE & 2) {
      uint32_t h0[S], h1[S];
      for (int j = 0; j < S; ++j) {
        h0[j] = lut3<kXor3>(lv[j], r[j], rv[j]);
        h1[j] = lut3<kMaj>(lv[j], r[j], rv[j]);
      }
      const uint32_t h0u = __builtin_amdgcn_alignbit(h0[S - 1], h0[S - 1], 32 - P);
      const uint32_t h1u = __builtin_amdgcn_alignbit(h1[S - 1], h1[S - 1], 32 - P);
      const uint32_t h0d = __builtin_amdgcn_alignbit(h0[0], h0[0], P);
      const uint32_t h1d = __builtin_amdgcn_alignbit(h1[0], h1[0], P);
      for (int j = 0; j < S; ++j) {
        const uint32_t a0 = j == 0 ? h0u : h0[j - 1], c0 = j == S - 1 ? h0d : h0[j + 1];
        const uint32_t a1 = j == 0 ? h1u : h1[j - 1], c1 = j == S - 1 ? h1d : h1[j + 1];
        const uint32_t s0 = lut3<kLe1>(a0, h0[j], c0), s1 = lut3<kNae>(a0, h0[j], c0);
        const uint32_t s2 = lut3<kLe1>(a1, h1[j], c1), s3 = lut3<kEven>(a1, h1[j], c1);
        const uint32_t t1 = lut3<kT1>(s0, s1, r[j]);
        const uint32_t t2 = lut3<kT2>(s2, r[j], t1);
        r[j] = lut3<kT3>(s1, s3, t2);
      }
    } else {
      for (int j = 0; j < S; ++j) r[j] = lv[j] ^ rv[j];
    }
  }
  Split<S>::store(r, c);
  for (int u = 0; u < P; ++u) st<false>(out + (u0 + u) * kWave + lane, c[u]);
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {  // in-kernel clock: shader cycles per 100 MHz real-time tick
    atomicAdd((unsigned long long *)&clk[0], (unsigned long long)(t1 - t0));
    atomicAdd((unsigned long long *)&clk[1], (unsigned long long)(r1 - r0));
  }
}

template <int S, int MODE>
void run(const uint64_t *in, uint64_t *out, uint64_t n, uint32_t gens, const char *name) {
  constexpr int P = S / 2;
  const unsigned grid = (unsigned)((n / P + kWavesPerBlock - 1) / kWavesPerBlock);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  uint64_t *clk;
  (void)hipMalloc(&clk, 16);
  for (int w = 0; w < 3; ++w) probe<S, MODE><<<grid, kBlock>>>(in, out, n, gens, clk);
  (void)hipMemset(clk, 0, 16);
  float best = 1e30f;
  for (int rep = 0; rep < 7; ++rep) {
    (void)hipEventRecord(a);
    probe<S, MODE><<<grid, kBlock>>>(in, out, n, gens, clk);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  uint64_t h[2];
  (void)hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  (void)hipFree(clk);
  std::printf("{\"S\": %d, \"mode\": \"%s\", \"ms_best\": %.4f, \"ns_per_universe_gen_per_cu\": %.3f, "
              "\"clock_GHz\": %.3f}\n", S, name, best, best * 1e6 / ((double)n * gens / 256.0),
              (double)h[0] / (double)h[1] * 0.1);
}

}  // namespace

int main() {
  const uint64_t n = 1 << 16;
  const uint32_t gens = 1024;
  uint64_t *in, *out;
  (void)hipMalloc(&in, n * 512);
  (void)hipMalloc(&out, n * 512);
  (void)lifeapi_fill_random_dev(in, n, 2, 0, 0, nullptr);
  run<2, 3>(in, out, n, gens, "full");
  run<4, 3>(in, out, n, gens, "full");
  run<8, 3>(in, out, n, gens, "full");
  run<16, 3>(in, out, n, gens, "full");
  run<4, 1>(in, out, n, gens, "exchange_only");
  run<8, 1>(in, out, n, gens, "exchange_only");
  run<4, 2>(in, out, n, gens, "network_only");
  run<8, 2>(in, out, n, gens, "network_only");
  return 0;
}
