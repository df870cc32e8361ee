// valu_probe.hip -- where does the iterated (config-3) step loop spend its
// issue slots?  Measurement tool, not product code: variants of the same
// 32-instruction generation body that differ only in how the neighbour
// columns cross lanes.  V0 = DPP wave_ror/rol (the product kernel), V1 = DPP
// row_ror (16-lane rows: wrong answer, same instruction class), V2 = no
// cross-lane (plain copies: wrong answer), V3 = V0 with 2 universes
// interleaved per wave.  Also reports the in-kernel shader clock
// (s_memtime / s_memrealtime at 100 MHz) of a diagnostic run.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

struct W {
  uint32_t lo, hi;
};
template <uint32_t TT>
__device__ __forceinline__ W l3(W a, W b, W c) {
  return W{(uint32_t)__builtin_amdgcn_bitop3_b32(a.lo, b.lo, c.lo, TT),
           (uint32_t)__builtin_amdgcn_bitop3_b32(a.hi, b.hi, c.hi, TT)};
}
template <int V>
__device__ __forceinline__ uint32_t xl(uint32_t v) {
  if constexpr (V == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x121, 0xF, 0xF, true);  // row_ror:1
  else if constexpr (V == 2) return v ^ 0x1234567u;
  else return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xF, 0xF, true);
}
template <int V>
__device__ __forceinline__ uint32_t xr(uint32_t v) {
  if constexpr (V == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x12F, 0xF, 0xF, true);  // row_ror:15
  else if constexpr (V == 2) return v ^ 0x7654321u;
  else return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x134, 0xF, 0xF, true);
}
__device__ __forceinline__ W rup(W a) {
  return W{__builtin_amdgcn_alignbit(a.lo, a.hi, 31), __builtin_amdgcn_alignbit(a.hi, a.lo, 31)};
}
__device__ __forceinline__ W rdn(W a) {
  return W{__builtin_amdgcn_alignbit(a.hi, a.lo, 1), __builtin_amdgcn_alignbit(a.lo, a.hi, 1)};
}

template <int V>
__device__ __forceinline__ W gen(W a) {
  if constexpr (V >= 3) {  // row-first (the product's default rule): 4 DPP
    const W L{xl<0>(a.lo), xl<0>(a.hi)}, R{xr<0>(a.lo), xr<0>(a.hi)};
    const W h0 = l3<0x96>(L, a, R), h1 = l3<0xE8>(L, a, R);
    const W h0u = rup(h0), h0d = rdn(h0), h1u = rup(h1), h1d = rdn(h1);
    const W fs = l3<0x96>(h0u, h0, h0d), fc = l3<0xE8>(h0u, h0, h0d);
    const W cs = l3<0x96>(h1u, h1, h1d), cc = l3<0xE8>(h1u, h1, h1d);
    const W b2 = l3<0x78>(cc, fc, cs);
    const W p = l3<0x38>(fs, b2, a);
    const W q = l3<0x96>(fc, cs, b2);
    return W{p.lo & q.lo, p.hi & q.hi};
  }
  const W up{__builtin_amdgcn_alignbit(a.lo, a.hi, 31), __builtin_amdgcn_alignbit(a.hi, a.lo, 31)};
  const W dn{__builtin_amdgcn_alignbit(a.hi, a.lo, 1), __builtin_amdgcn_alignbit(a.lo, a.hi, 1)};
  const W c0 = l3<0x96>(up, dn, a), c1 = l3<0xE8>(up, dn, a);
  const W L0{xl<V>(c0.lo), xl<V>(c0.hi)}, R0{xr<V>(c0.lo), xr<V>(c0.hi)};
  const W L1{xl<V>(c1.lo), xl<V>(c1.hi)}, R1{xr<V>(c1.lo), xr<V>(c1.hi)};
  const W fs = l3<0x96>(L0, c0, R0), fc = l3<0xE8>(L0, c0, R0);
  const W cs = l3<0x96>(L1, c1, R1), cc = l3<0xE8>(L1, c1, R1);
  const W b2 = l3<0x78>(cc, fc, cs);
  const W p = l3<0x38>(fs, b2, a);  // (a^b)&(c|a) with a=fs,b=b2,c=a
  const W q = l3<0x96>(fc, cs, b2);
  return W{p.lo & q.lo, p.hi & q.hi};
}

template <int V, int U, bool STAMP>
__global__ __launch_bounds__(256) void k_iter(const uint64_t *in, uint64_t *out, uint64_t n,
                                              uint32_t gens, uint64_t *clk) {
  const int lane = threadIdx.x & 63;
  const uint64_t u0 = ((uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * U;
  if (u0 >= n) return;
  W a[U];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const uint64_t v = in[(u0 + k) * 64 + lane];
    a[k] = W{(uint32_t)v, (uint32_t)(v >> 32)};
  }
  uint64_t t0 = 0, r0 = 0;
  if (STAMP) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (V == 4) {  // row-first, generation loop unrolled x4
    uint32_t g = 0;
    for (; g + 4 <= gens; g += 4)
#pragma unroll
      for (int k = 0; k < U; ++k) a[k] = gen<V>(gen<V>(gen<V>(gen<V>(a[k]))));
    for (; g < gens; ++g)
#pragma unroll
      for (int k = 0; k < U; ++k) a[k] = gen<V>(a[k]);
  } else {
    for (uint32_t g = 0; g < gens; ++g)
#pragma unroll
      for (int k = 0; k < U; ++k) a[k] = gen<V>(a[k]);
  }
  if (STAMP && lane == 0 && (threadIdx.x >> 6) == 0) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
#pragma unroll
  for (int k = 0; k < U; ++k) out[(u0 + k) * 64 + lane] = (uint64_t)a[k].lo | ((uint64_t)a[k].hi << 32);
}

template <int V, int U, bool STAMP>
int run(const char *name, const uint64_t *in, uint64_t *out, uint64_t n, uint32_t gens, uint64_t *clk) {
  const unsigned blocks = (unsigned)((n / U + 3) / 4);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int r = 0; r < 8; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((k_iter<V, U, STAMP>), dim3(blocks), dim3(256), 0, 0, in, out, n, gens, clk);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float t;
    CHECK(hipEventElapsedTime(&t, e0, e1));
    if (r >= 2) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  double ghz = 0;
  if (STAMP) {
    std::vector<uint64_t> h(2 * blocks);
    CHECK(hipMemcpy(h.data(), clk, 16 * (size_t)blocks, hipMemcpyDeviceToHost));
    std::vector<double> f;
    for (unsigned b = 0; b < blocks; ++b)
      if (h[2 * b + 1]) f.push_back((double)h[2 * b] / h[2 * b + 1] * 0.1);
    std::sort(f.begin(), f.end());
    ghz = f[f.size() / 2];
  }
  const double med = ms[ms.size() / 2];
  std::printf("{\"variant\": \"%s\", \"U\": %d, \"stamp\": %d, \"ms_median\": %.4f, \"gen_per_s\": %.4g, "
              "\"wave_valu_per_s\": %.4g, \"clock_GHz\": %.3f}\n",
              name, U, (int)STAMP, med, n * gens / (med * 1e-3), 32.0 * n * gens / (med * 1e-3), ghz);
  return 0;
}

int main() {
  const uint64_t n = 1 << 16;
  const uint32_t gens = 1024;
  uint64_t *a, *b, *clk;
  CHECK(hipMalloc(&a, n * 512));
  CHECK(hipMalloc(&b, n * 512));
  CHECK(hipMalloc(&clk, n * 16));
  CHECK(hipMemset(a, 0x6b, n * 512));
  int rc = 0;
  for (int rep = 0; rep < 2; ++rep) {
    rc |= run<3, 1, false>("rowfirst", a, b, n, gens, clk);
    rc |= run<4, 1, false>("rowfirst_unroll4", a, b, n, gens, clk);
    rc |= run<3, 2, false>("rowfirst", a, b, n, gens, clk);
    rc |= run<4, 2, false>("rowfirst_unroll4", a, b, n, gens, clk);
    rc |= run<0, 1, false>("dpp_wave", a, b, n, gens, clk);
    rc |= run<1, 1, false>("dpp_row", a, b, n, gens, clk);
    rc |= run<2, 1, false>("no_xlane", a, b, n, gens, clk);
    rc |= run<0, 2, false>("dpp_wave", a, b, n, gens, clk);
    rc |= run<0, 1, true>("dpp_wave", a, b, n, gens, clk);
    rc |= run<2, 1, true>("no_xlane", a, b, n, gens, clk);
  }
  return rc;
}
