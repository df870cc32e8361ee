// tune_reduce.hip -- TUNING build: variants of the per-universe hash
// (lifeapi_hash_batch_dev's k_hash, reduce.hip) for A/Bs; same definition
// h_u = mix(sum_x mix(s[x] + (x+1)*G)), so every variant must equal the
// product kernel bit for bit.
//   0: as shipped -- 4 universes per wave, lane = column, DPP row sums +
//      v_readlane per universe;
//   1: the same with 8 universes per wave (more loads in flight);
//   2: lane = universe -- each lane reads its universe's 512 B as 32
//      dwordx4 loads and sums its own 64 mixes: no cross-lane work at all;
//   3: as 2 with nontemporal loads;
//   4: as 0, but the 4 universes' 64 lane values are transposed through
//      LDS so that each 16-lane DPP row sums one universe (4 values per
//      lane, then 4 row-butterfly levels): one tree for all 4 universes
//      instead of one per universe, and no v_readlane;
//   5: as 4 with 8 universes per wave (8 lanes and 8 values per universe,
//      3 butterfly levels).
#include "lifeapi_tune.h"
#include "device.hpp"
#include "host.hpp"
#include "reduce_kernels.hpp"

using namespace lifeapi_impl;

namespace {

template <int U>
__global__ __launch_bounds__(kBlock) void k_hash_lanecol(const uint64_t *__restrict__ s, uint64_t *__restrict__ h,
                                                         uint64_t n) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * U;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave) * U; u0 < n; u0 += stride) {
    uint64_t m[U];
#pragma unroll
    for (int k = 0; k < U; ++k) m[k] = u0 + k < n ? __builtin_nontemporal_load(s + (u0 + k) * kWave + lane) : 0ull;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t t = wave_sum_u64_dpp(mix64(m[k] + (uint64_t)(lane + 1) * kGolden));
      if (lane == 0 && u0 + k < n) h[u0 + k] = mix64(t);
    }
  }
}


// lane = universe: 64 universes per wave, each lane streams its own 512 B
template <bool NT>
__global__ __launch_bounds__(kBlock) void k_hash_laneuni(const uint64_t *__restrict__ s, uint64_t *__restrict__ h,
                                                         uint64_t n) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t u = (uint64_t)blockIdx.x * kBlock + threadIdx.x; u < n; u += stride) {
    const u64x2 *p = reinterpret_cast<const u64x2 *>(s + u * kWave);
    uint64_t acc = 0;
#pragma unroll 8
    for (int i = 0; i < kWave / 2; ++i) {
      const u64x2 v = NT ? __builtin_nontemporal_load(p + i) : p[i];
      acc += mix64(v[0] + (uint64_t)(2 * i + 1) * kGolden);
      acc += mix64(v[1] + (uint64_t)(2 * i + 2) * kGolden);
    }
    h[u] = mix64(acc);
  }
  (void)lane;
}


// U universes per wave; lane l sums universe l / (64/U) from LDS
template <int U>
__global__ __launch_bounds__(kBlock) void k_hash_lds(const uint64_t *__restrict__ s, uint64_t *__restrict__ h,
                                                     uint64_t n) {
  constexpr int LPU = kWave / U;  // lanes per universe
  constexpr int VPL = kWave / LPU;  // values each lane sums (= U)
  __shared__ uint64_t buf[kWavesPerBlock][U * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = threadIdx.x / kWave;
  uint64_t *b = buf[wib];
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * U;
  const uint64_t g = (uint64_t)(lane + 1) * kGolden;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wib) * U; u0 < n; u0 += stride) {
    uint64_t m[U];
#pragma unroll
    for (int k = 0; k < U; ++k) m[k] = u0 + k < n ? __builtin_nontemporal_load(s + (u0 + k) * kWave + lane) : 0ull;
#pragma unroll
    for (int k = 0; k < U; ++k) b[k * kWave + lane] = mix64(m[k] + g);
    __builtin_amdgcn_wave_barrier();
    const int u = lane / LPU, j = (lane % LPU) * VPL;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < VPL; ++k) acc += b[u * kWave + j + k];
    __builtin_amdgcn_wave_barrier();  // (the next iteration's writes come after these reads)
    acc += dpp_mov64<0xB1>(acc);   // quad_perm [1,0,3,2]
    acc += dpp_mov64<0x4E>(acc);   // quad_perm [2,3,0,1]
    acc += dpp_mov64<0x141>(acc);  // row_half_mirror: 8-lane sums in every lane
    if constexpr (LPU == 16) acc += dpp_mov64<0x140>(acc);  // row_mirror
    if (lane % LPU == 0 && u0 + u < n) h[u0 + u] = mix64(acc);
  }
}

// the seeded fill with 16-byte stores: two consecutive words per lane
__global__ __launch_bounds__(kBlock) void k_fill16(uint64_t *__restrict__ out, uint64_t nwords, uint64_t seed,
                                                   uint64_t first_word, int mode) {
  typedef uint64_t u64x2v __attribute__((ext_vector_type(2)));
  const uint64_t stride = (uint64_t)gridDim.x * kBlock * 2;
  for (uint64_t i = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 2; i < nwords; i += stride) {
    uint64_t v0 = mix64(seed + (first_word + i + 1) * kGolden), v1 = mix64(seed + (first_word + i + 2) * kGolden);
    if (mode == 1) {
      v0 = (v0 & ((1ULL << 61) - 1)) | (1ULL << 61);
      v1 = (v1 & ((1ULL << 61) - 1)) | (1ULL << 61);
    }
    __builtin_nontemporal_store(u64x2v{v0, v1}, reinterpret_cast<u64x2v *>(out + i));
  }
}

}  // namespace

extern "C" {

/* the seeded fill (lifeapi_fill_random_dev's definition) with 16-byte
 * stores; grid of one block per 512 words, capped at blocks_per_cu if > 0 */
int lifeapi_tune_fill16(uint64_t *d_out, size_t n, uint64_t seed, uint64_t first_universe, int mode,
                        int blocks_per_cu, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_out || ((uintptr_t)d_out & 15u) || (mode != 0 && mode != 1))
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_tune_fill16%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const uint64_t words = (uint64_t)n * kWave;
  hipLaunchKernelGGL(k_fill16, dim3(grid_for(words / (2 * kWave), cus, blocks_per_cu)), dim3(kBlock), 0,
                     (hipStream_t)stream, d_out, words, seed, first_universe * kWave, mode);
  return launched("k_fill16 launch");
}


int lifeapi_tune_hash(const uint64_t *d_states, uint64_t *d_hash, size_t n, int variant, int blocks_per_cu,
                      void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_states || !d_hash || !aligned8(d_states) || !aligned8(d_hash))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_tune_hash%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipStream_t st = (hipStream_t)stream;
  switch (variant) {
    case 0:
      hipLaunchKernelGGL(k_hash_lanecol<4>, dim3(grid_for((n + 3) / 4, cus, blocks_per_cu)), dim3(kBlock), 0, st,
                         d_states, d_hash, (uint64_t)n);
      break;
    case 1:
      hipLaunchKernelGGL(k_hash_lanecol<8>, dim3(grid_for((n + 7) / 8, cus, blocks_per_cu)), dim3(kBlock), 0, st,
                         d_states, d_hash, (uint64_t)n);
      break;
    case 2:
    case 3:
      hipLaunchKernelGGL(variant == 2 ? k_hash_laneuni<false> : k_hash_laneuni<true>,
                         dim3(grid_for((n + kWave - 1) / kWave, cus, blocks_per_cu)), dim3(kBlock), 0, st, d_states,
                         d_hash, (uint64_t)n);
      break;
    case 4:
      hipLaunchKernelGGL(k_hash_lds<4>, dim3(grid_for((n + 3) / 4, cus, blocks_per_cu)), dim3(kBlock), 0, st,
                         d_states, d_hash, (uint64_t)n);
      break;
    case 5:
      hipLaunchKernelGGL(k_hash_lds<8>, dim3(grid_for((n + 7) / 8, cus, blocks_per_cu)), dim3(kBlock), 0, st,
                         d_states, d_hash, (uint64_t)n);
      break;
    default:
      return fail(LIFEAPI_E_INVALID, "unknown hash variant%s");
  }
  return launched("k_hash (tuning) launch");
}

/* GetPop (kind 0, d_out = uint32 per universe) or Contains (kind 1, d_out =
 * uint8, target d_w / d_u) with `upw` universes per wave (2, 4, 8) and
 * blocks_per_cu > 0: grid cap, 0: none, -k: at most k blocks resident     */
int lifeapi_tune_reduce(int kind, const uint64_t *d_states, const uint64_t *d_w, const uint64_t *d_u, void *d_out,
                        size_t n, int upw, int blocks_per_cu, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_states || !d_out || ((kind & 1) && (!d_w || !d_u)) || kind < 0 || kind > 3)
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_tune_reduce%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const dim3 grid(grid_for((n + upw - 1) / upw, cus, blocks_per_cu > 0 ? blocks_per_cu : 0));
  const hipStream_t st = (hipStream_t)stream;
  unsigned lds = 0;
  if (kind == 0 || kind == 2) {
    using Fn = void (*)(const uint64_t *, uint32_t *, uint64_t);
    Fn fn = kind == 2 ? (upw == 2 ? (Fn)k_pop16<2> : upw == 4 ? (Fn)k_pop16<4> : upw == 8 ? (Fn)k_pop16<8> : nullptr)
                      : (upw == 2 ? (Fn)k_pop<2> : upw == 4 ? (Fn)k_pop<4> : upw == 8 ? (Fn)k_pop<8> : nullptr);
    if (!fn) return fail(LIFEAPI_E_INVALID, "universes per wave: 2, 4 or 8%s");
    if (blocks_per_cu < 0 && (rc = occupancy_lds((const void *)fn, -blocks_per_cu, lds)) != LIFEAPI_OK) return rc;
    hipLaunchKernelGGL(fn, grid, dim3(kBlock), lds, st, d_states, (uint32_t *)d_out, (uint64_t)n);
  } else {
    using Fn = void (*)(const uint64_t *, const uint64_t *, const uint64_t *, uint8_t *, uint64_t);
    Fn fn = kind == 3
                ? (upw == 2 ? (Fn)k_contains16<2> : upw == 4 ? (Fn)k_contains16<4> : upw == 8 ? (Fn)k_contains16<8>
                                                                                          : nullptr)
                : (upw == 2 ? (Fn)k_contains<2> : upw == 4 ? (Fn)k_contains<4> : upw == 8 ? (Fn)k_contains<8>
                                                                                    : nullptr);
    if (!fn) return fail(LIFEAPI_E_INVALID, "universes per wave: 2, 4 or 8%s");
    if (blocks_per_cu < 0 && (rc = occupancy_lds((const void *)fn, -blocks_per_cu, lds)) != LIFEAPI_OK) return rc;
    hipLaunchKernelGGL(fn, grid, dim3(kBlock), lds, st, d_states, d_w, d_u, (uint8_t *)d_out, (uint64_t)n);
  }
  return launched("reduce (tuning) launch");
}

}  // extern "C"
