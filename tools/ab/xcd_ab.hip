// xcd_ab.hip -- does dealing each XCD a contiguous slice of the batch help
// the streaming kernels?  Blocks are dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH.md "Workgroup dispatch"), so with the plain mapping an
// XCD's blocks touch every 8th 8-KiB stripe of the whole batch; the chunked
// mapping hands block b the logical block (b mod 8) * (B / 8) + b / 8, so
// XCD k streams one contiguous eighth.  Two access shapes, each ping-pong or
// in place, 8-byte nontemporal loads and stores, one wave per group:
//   step   4 universes (4 x 512 B) per wave, in -> out
//   stable one LifeStable (10 planes, 5 KiB) per wave, in place
// at several batch sizes; median of 15 launches after 5, both mappings
// interleaved.  One JSON line per (shape, size, mapping).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build/xcd_ab tools/ab/xcd_ab.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

namespace {

constexpr int kWave = 64, kWaves = 4, kBlock = kWave * kWaves;

__device__ __forceinline__ uint64_t logical_block(bool chunk) {
  const uint64_t b = blockIdx.x, nb = gridDim.x;
  return chunk ? (b % 8) * (nb / 8) + b / 8 : b;
}

template <bool CHUNK>
__global__ __launch_bounds__(kBlock) void k_copy4(const uint64_t *in, uint64_t *out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t grp = logical_block(CHUNK) * kWaves + w;
  const uint64_t base = grp * 4 * kWave + lane;
  uint64_t v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(in + base + k * kWave);
#pragma unroll
  for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(v[k] ^ 1ull, out + base + k * kWave);
}

template <bool CHUNK>
__global__ __launch_bounds__(kBlock) void k_inplace10(uint64_t *p) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t obj = logical_block(CHUNK) * kWaves + w;
  uint64_t *q = p + obj * 10 * kWave + lane;
  uint64_t v[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) v[k] = __builtin_nontemporal_load(q + k * kWave);
#pragma unroll
  for (int k = 0; k < 10; ++k) __builtin_nontemporal_store(v[k] ^ 1ull, q + k * kWave);
}

float time_one(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

}  // namespace

int main() {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const uint64_t step_sizes[] = {1ull << 20, 1ull << 22, 1ull << 24};  // universes
  for (uint64_t n : step_sizes) {
    uint64_t *a, *b;
    if (hipMalloc(&a, n * 512) != hipSuccess || hipMalloc(&b, n * 512) != hipSuccess) return 1;
    hipMemset(a, 1, n * 512);
    hipMemset(b, 2, n * 512);
    const unsigned blocks = (unsigned)(n / 4 / kWaves);  // a multiple of 8
    std::vector<float> ms[2];
    for (int rep = 0; rep < 20; ++rep)
      for (int c = 0; c < 2; ++c) {
        hipEventRecord(e0);
        for (int k = 0; k < 4; ++k) {
          const uint64_t *src = (k & 1) ? b : a;
          uint64_t *dst = (k & 1) ? a : b;
          if (c) hipLaunchKernelGGL(k_copy4<true>, dim3(blocks), dim3(kBlock), 0, 0, src, dst);
          else hipLaunchKernelGGL(k_copy4<false>, dim3(blocks), dim3(kBlock), 0, 0, src, dst);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        if (rep >= 5) ms[c].push_back(time_one(e0, e1) / 4);
      }
    for (int c = 0; c < 2; ++c) {
      std::sort(ms[c].begin(), ms[c].end());
      const double m = ms[c][ms[c].size() / 2];
      printf("{\"shape\": \"step copy\", \"universes\": %llu, \"mapping\": \"%s\", \"ms_median\": %.4f, \"TBps\": %.3f}\n",
             (unsigned long long)n, c ? "xcd_chunk" : "plain", m, n * 1024.0 / m / 1e9);
    }
    hipFree(a);
    hipFree(b);
  }
  const uint64_t stable_sizes[] = {1ull << 18, 1ull << 20};  // LifeStables
  for (uint64_t n : stable_sizes) {
    uint64_t *p;
    if (hipMalloc(&p, n * 5120) != hipSuccess) return 1;
    hipMemset(p, 3, n * 5120);
    const unsigned blocks = (unsigned)(n / kWaves);
    std::vector<float> ms[2];
    for (int rep = 0; rep < 20; ++rep)
      for (int c = 0; c < 2; ++c) {
        hipEventRecord(e0);
        for (int k = 0; k < 4; ++k) {
          if (c) hipLaunchKernelGGL(k_inplace10<true>, dim3(blocks), dim3(kBlock), 0, 0, p);
          else hipLaunchKernelGGL(k_inplace10<false>, dim3(blocks), dim3(kBlock), 0, 0, p);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        if (rep >= 5) ms[c].push_back(time_one(e0, e1) / 4);
      }
    for (int c = 0; c < 2; ++c) {
      std::sort(ms[c].begin(), ms[c].end());
      const double m = ms[c][ms[c].size() / 2];
      printf("{\"shape\": \"stable in place\", \"objects\": %llu, \"mapping\": \"%s\", \"ms_median\": %.4f, \"TBps\": %.3f}\n",
             (unsigned long long)n, c ? "xcd_chunk" : "plain", m, n * 10240.0 / m / 1e9);
    }
    hipFree(p);
  }
  return 0;
}
