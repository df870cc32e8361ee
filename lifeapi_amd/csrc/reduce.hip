// reduce.hip -- per-universe reductions and synthetic input: GetPop
// (LifeAPI.hpp:290-298), Contains(LifeTarget) (LifeTarget.hpp:44-51), the
// build-defined hash, and the seeded RandomState()-style fill.
#include "device.hpp"
#include "host.hpp"
#include "reduce_kernels.hpp"
#include "cone_kernels.hpp"

using namespace lifeapi_impl;

namespace {

// build-defined universe hash: mix(sum_x mix(s[x] + (x+1)*G)).  The
// per-word mix is heavy (four 64-bit multiplies), so the cross-lane sum must
// be cheap: kHashU = 8 universes per wave, loaded lane = column (coalesced),
// mixed, then transposed through LDS so that each 8-lane DPP group sums one
// universe (8 values per lane, then 3 butterfly levels) -- one tree for all 8
// universes instead of one per universe, and no v_readlane.  1M universes:
// 0.122 -> 0.082 ms (4.5 -> 6.6 TB/s); 16M: 1.85 -> 1.38 ms (4.7 -> 6.3 TB/s)
// against the per-universe DPP tree (profiles/r02/hash_ab.jsonl; one-shot
// grid, every capped grid measured slower).
constexpr int kHashU = 8;
__global__ __launch_bounds__(kBlock) void k_hash(const uint64_t *__restrict__ s, uint64_t *__restrict__ h,
                                                 uint64_t n) {
  constexpr int LPU = kWave / kHashU;  // lanes per universe in the sum
  __shared__ uint64_t buf[kWavesPerBlock][kHashU * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = threadIdx.x / kWave;
  uint64_t *b = buf[wib];
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock * kHashU;
  const uint64_t g = (uint64_t)(lane + 1) * kGolden;
  for (uint64_t u0 = ((uint64_t)blockIdx.x * kWavesPerBlock + wib) * kHashU; u0 < n; u0 += stride) {
    uint64_t m[kHashU];
#pragma unroll
    for (int k = 0; k < kHashU; ++k) m[k] = u0 + k < n ? ld_state(s + (u0 + k) * kWave + lane) : 0ull;
#pragma unroll
    for (int k = 0; k < kHashU; ++k) b[k * kWave + lane] = mix64(m[k] + g);
    __builtin_amdgcn_wave_barrier();
    const int u = lane / LPU, j = (lane % LPU) * kHashU;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < kHashU; ++k) acc += b[u * kWave + j + k];
    __builtin_amdgcn_wave_barrier();  // (the next iteration's writes come after these reads)
    acc += dpp_mov64<0xB1>(acc);   // quad_perm [1,0,3,2]
    acc += dpp_mov64<0x4E>(acc);   // quad_perm [2,3,0,1]
    acc += dpp_mov64<0x141>(acc);  // row_half_mirror: the 8-lane sum in every lane
    if (lane % LPU == 0 && u0 + u < n) h[u0 + u] = mix64(acc);
  }
}

__global__ __launch_bounds__(kBlock) void k_fill(uint64_t *__restrict__ out, uint64_t nwords,
                                                 uint64_t seed, uint64_t first_word, int mode) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nwords; i += stride) {
    uint64_t v = mix64(seed + (first_word + i + 1) * kGolden);
    if (mode == 1) v = (v & ((1ULL << 61) - 1)) | (1ULL << 61);
    __builtin_nontemporal_store(v, out + i);
  }
}

// the same words with 16-byte stores: two consecutive words per lane
__global__ __launch_bounds__(kBlock) void k_fill16(uint64_t *__restrict__ out, uint64_t nwords, uint64_t seed,
                                                   uint64_t first_word, int mode) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock * 2;
  for (uint64_t i = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 2; i < nwords; i += stride) {
    uint64_t v0 = mix64(seed + (first_word + i + 1) * kGolden), v1 = mix64(seed + (first_word + i + 2) * kGolden);
    if (mode == 1) {
      v0 = (v0 & ((1ULL << 61) - 1)) | (1ULL << 61);
      v1 = (v1 & ((1ULL << 61) - 1)) | (1ULL << 61);
    }
    __builtin_nontemporal_store(u64x2{v0, v1}, reinterpret_cast<u64x2 *>(out + i));
  }
}

}  // namespace

extern "C" {

int lifeapi_pop_batch_dev(const uint64_t *d_states, uint32_t *d_pop, size_t n, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_states || !d_pop || !aligned8(d_states) || ((uintptr_t)d_pop & 3u))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_pop_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  // 16-byte loads (two universes per wave-instruction), 8 universes per
  // wave, one-shot grid: 0.0820 ms on 1M against 0.0918 for the 8-byte
  // k_pop<4> on the 32-blocks-per-CU grid, same process (tools/ab/rows_ab.py,
  // profiles/r03/rows_ab.jsonl); batches that are only 8-byte aligned keep
  // the 8-byte kernel
  if (aligned16(d_states))
    hipLaunchKernelGGL(k_pop16<8>, dim3(grid_for((n + 7) / 8, cus, 0)), dim3(kBlock), 0, (hipStream_t)stream,
                       d_states, d_pop, (uint64_t)n);
  else
    hipLaunchKernelGGL(k_pop<kRedU>, dim3(grid_for((n + kRedU - 1) / kRedU, cus, kRedBlocksPerCU)), dim3(kBlock),
                       0, (hipStream_t)stream, d_states, d_pop, (uint64_t)n);
  return launched("k_pop launch");
}

int lifeapi_hash_batch_dev(const uint64_t *d_states, uint64_t *d_hash, size_t n, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_states || !d_hash || !aligned8(d_states) || !aligned8(d_hash))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_hash_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(k_hash, dim3(grid_for((n + kHashU - 1) / kHashU, cus, 0)), dim3(kBlock), 0,
                     (hipStream_t)stream, d_states, d_hash, (uint64_t)n);
  return launched("k_hash launch");
}

int lifeapi_contains_batch_dev(const uint64_t *d_states, const uint64_t *d_wanted,
                               const uint64_t *d_unwanted, uint8_t *d_out, size_t n,
                               void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_states || !d_wanted || !d_unwanted || !d_out || !aligned8(d_states) ||
      !aligned8(d_wanted) || !aligned8(d_unwanted))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_contains_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  // only the columns holding the target's care cells (cone_kernels.hpp)
  return launch_cone_adapt<kConeSets, false>(d_states, d_wanted, d_unwanted, d_out, n, 0u, cus,
                                             (hipStream_t)stream, kConeAdaptBlocksPerCU);
}

int lifeapi_fill_random_dev(uint64_t *d_out, size_t n, uint64_t seed, uint64_t first_universe,
                            int mode, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_out || !aligned8(d_out) || (mode != 0 && mode != 1))
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_fill_random_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  const uint64_t words = (uint64_t)n * kWave;
  note_forward_write(d_out, words * 8);
  // 16-byte stores (two words per lane): 0.0836 ms on 1M against 0.0862 for
  // 8-byte ones (tools/ab/rows_ab.py, profiles/r03/rows_ab.jsonl)
  if (aligned16(d_out))
    hipLaunchKernelGGL(k_fill16, dim3(grid_for(words / (2 * kWave), cus, 0)), dim3(kBlock), 0,
                       (hipStream_t)stream, d_out, words, seed, first_universe * kWave, mode);
  else
    hipLaunchKernelGGL(k_fill, dim3(grid_for(words / kWave, cus, 0)), dim3(kBlock), 0,
                       (hipStream_t)stream, d_out, words, seed, first_universe * kWave, mode);
  return launched("k_fill launch");
}

}  // extern "C"
