// reduce_kernels.hpp -- the per-universe reductions GetPop (LifeAPI.hpp:
// 290-298) and Contains(LifeTarget) (LifeTarget.hpp:44-51) as templates on
// the universes per wave; reduce.hip launches the shipped shape, the tuning
// build (tools/tune/tune_reduce.hip) the others for A/Bs.
#pragma once

#include "device.hpp"

namespace lifeapi_impl {
namespace {

// The per-universe reductions below take kRedU universes per wave, all loads
// issued before the first reduction (one wave per universe and a grid-stride
// loop left them latency-bound at 36-60 % of HBM, tools/rows_bench.py), and
// sum over the wave by DPP (wave_sum_*_dpp), not through ds_bpermute.
constexpr int kRedU = 4;  // (templates below take U; the launches pick it)

// The states are read once: nontemporal loads, and a grid of at most 32
// blocks per CU looping over the batch (full grids and plain loads were 6-20 %
// slower, profiles/r01/red_ab.jsonl).
constexpr int kRedBlocksPerCU = 32;

__device__ __forceinline__ uint64_t ld_state(const uint64_t *p) { return __builtin_nontemporal_load(p); }

// GetPop (LifeAPI.hpp:290-298): two universes' popcounts per 32-bit reduction
template <int U>
__global__ __launch_bounds__(kBlock) void k_pop(const uint64_t *__restrict__ s,
                                                uint32_t *__restrict__ pop, uint64_t n) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * U;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave) * U; u0 < n;
       u0 += stride) {
    uint32_t c[U];
#pragma unroll
    for (int k = 0; k < U; ++k) c[k] = u0 + k < n ? (uint32_t)__popcll(ld_state(s + (u0 + k) * kWave + lane)) : 0u;
#pragma unroll
    for (int k = 0; k < U; k += 2) {
      const uint32_t t = wave_sum_u32_dpp(c[k] | c[k + 1] << 16);  // each sum <= 4096
      if (lane == 0) {
        if (u0 + k < n) pop[u0 + k] = t & 0xFFFF;
        if (u0 + k + 1 < n) pop[u0 + k + 1] = t >> 16;
      }
    }
  }
}

template <int U>
__global__ __launch_bounds__(kBlock) void k_contains(const uint64_t *__restrict__ s,
                                                     const uint64_t *__restrict__ wanted,
                                                     const uint64_t *__restrict__ unwanted,
                                                     uint8_t *__restrict__ out, uint64_t n) {
  const int lane = threadIdx.x & (kWave - 1);
  const W w = split(wanted[lane]), uw = split(unwanted[lane]);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * U;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave) * U; u0 < n;
       u0 += stride) {
    W a[U];
#pragma unroll
    for (int k = 0; k < U; ++k) a[k] = u0 + k < n ? split(ld_state(s + (u0 + k) * kWave + lane)) : W{0u, 0u};
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const bool c = wave_contains(a[k], w, uw);
      if (lane == 0 && u0 + k < n) out[u0 + k] = c ? 1 : 0;
    }
  }
}

// The same two reductions with 16-byte loads: lane l reads words 2(l%32),
// 2(l%32)+1 of universe u0 + 2k + l/32 (one dwordx4 per lane = two universes
// per wave-instruction, against one with lane = column), so half the load
// instructions move the same bytes.  U (even) universes per wave.

template <int U>
__global__ __launch_bounds__(kBlock) void k_pop16(const uint64_t *__restrict__ s,
                                                  uint32_t *__restrict__ pop, uint64_t n) {
  static_assert(U % 2 == 0, "universes come in pairs");
  const int lane = threadIdx.x & (kWave - 1);
  const int half = lane >> 5, col = (lane & 31) * 2;
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * U;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave) * U; u0 < n;
       u0 += stride) {
    uint32_t c[U / 2];
#pragma unroll
    for (int k = 0; k < U / 2; ++k) {
      const uint64_t u = u0 + 2 * k + half;
      if (u < n) {
        const u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(s + u * kWave + col));
        c[k] = (uint32_t)(__popcll(v[0]) + __popcll(v[1])) << (16 * half);
      } else {
        c[k] = 0u;
      }
    }
#pragma unroll
    for (int k = 0; k < U / 2; ++k) {
      const uint32_t t = wave_sum_u32_dpp(c[k]);  // universe 2k in the low half, 2k+1 in the high
      if (lane == 0) {
        if (u0 + 2 * k < n) pop[u0 + 2 * k] = t & 0xFFFF;
        if (u0 + 2 * k + 1 < n) pop[u0 + 2 * k + 1] = t >> 16;
      }
    }
  }
}

template <int U>
__global__ __launch_bounds__(kBlock) void k_contains16(const uint64_t *__restrict__ s,
                                                       const uint64_t *__restrict__ wanted,
                                                       const uint64_t *__restrict__ unwanted,
                                                       uint8_t *__restrict__ out, uint64_t n) {
  static_assert(U % 2 == 0, "universes come in pairs");
  const int lane = threadIdx.x & (kWave - 1);
  const int half = lane >> 5, col = (lane & 31) * 2;
  const uint64_t w0 = wanted[col], w1 = wanted[col + 1];
  const uint64_t m0 = w0 | unwanted[col], m1 = w1 | unwanted[col + 1];
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * U;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave) * U; u0 < n;
       u0 += stride) {
    u64x2 v[U / 2];
#pragma unroll
    for (int k = 0; k < U / 2; ++k) {
      const uint64_t u = u0 + 2 * k + half;
      v[k] = u < n ? __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(s + u * kWave + col))
                   : u64x2{w0, w1};
    }
#pragma unroll
    for (int k = 0; k < U / 2; ++k) {
      const uint64_t d = ((v[k][0] ^ w0) & m0) | ((v[k][1] ^ w1) & m1);
      const uint64_t bad = __ballot(d != 0ull);  // lanes 0-31: universe 2k, 32-63: 2k+1
      if (lane == 0) {
        if (u0 + 2 * k < n) out[u0 + 2 * k] = (uint32_t)bad == 0u ? 1 : 0;
        if (u0 + 2 * k + 1 < n) out[u0 + 2 * k + 1] = (uint32_t)(bad >> 32) == 0u ? 1 : 0;
      }
    }
  }
}

}  // namespace
}  // namespace lifeapi_impl
