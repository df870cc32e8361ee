// membw.hip -- HBM streaming ceilings for the access shapes the step kernel
// can use (measurement tool, not product code).  Copies 2^20 universes (512
// MiB in + 512 MiB out) with wave-contiguous 512-B (dwordx2) or 1-KiB
// (dwordx4) accesses, U loads in flight per lane, plain or nontemporal, for
// several grid sizes, and prints one JSON line per variant.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

typedef unsigned long long u64;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

template <class T, int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const T *__restrict__ in, T *__restrict__ out,
                                              u64 nvec) {
  // a "row" = 64 lanes x sizeof(T); waves take U rows at a time, grid-strided
  const int lane = threadIdx.x & 63;
  const u64 wave = (u64)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 rows = nvec / 64, stride = (u64)gridDim.x * 4 * U;
  for (u64 r0 = wave * U; r0 < rows; r0 += stride) {
    T v[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (r0 + k < rows) v[k] = NT ? __builtin_nontemporal_load(in + (r0 + k) * 64 + lane)
                                   : in[(r0 + k) * 64 + lane];
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (r0 + k < rows) {
        if (NT) __builtin_nontemporal_store(v[k], out + (r0 + k) * 64 + lane);
        else out[(r0 + k) * 64 + lane] = v[k];
      }
  }
}

static bool g_calib = false;  // `membw calib`: only the step kernel's access shape

template <class T, int U, bool NT>
int run(const char *name, void *a, void *b, size_t bytes, int cus) {
  const u64 nvec = bytes / sizeof(T);
  const u64 rows = nvec / 64;
  for (int bpc : {2, 4, 8, 16, 32, 0}) {
    if (g_calib && bpc != 0) continue;
    u64 blocks = (rows / U + 3) / 4;
    if (bpc) blocks = std::min<u64>(blocks, (u64)cus * bpc);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<float> ms;
    for (int rep = 0; rep < 25; ++rep) {
      CHECK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL((k_copy<T, U, NT>), dim3(blocks), dim3(256), 0, 0, (const T *)a, (T *)b, nvec);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float t;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      if (rep >= 5) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double gbs_best = 2.0 * bytes / (ms.front() * 1e-3) / 1e9;
    const double gbs_med = 2.0 * bytes / (ms[ms.size() / 2] * 1e-3) / 1e9;
    std::printf("{\"variant\": \"%s\", \"U\": %d, \"nt\": %d, \"blocks_per_cu\": %d, \"blocks\": %llu, "
                "\"ms_best\": %.4f, \"ms_median\": %.4f, \"GBps_best\": %.1f, \"GBps_median\": %.1f}\n",
                name, U, (int)NT, bpc, blocks, ms.front(), ms[ms.size() / 2], gbs_best, gbs_med);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
  }
  return 0;
}

int main(int argc, char **argv) {
  g_calib = argc > 1 && std::string(argv[1]) == "calib";
  const size_t bytes = size_t(1) << 29;  // 2^20 universes x 512 B
  void *a, *b;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMemset(a, 0x5a, bytes));
  CHECK(hipMemset(b, 0, bytes));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  int rc = 0;
  if (g_calib) return run<u32x2, 4, true>("dwordx2", a, b, bytes, cus);
  rc |= run<u32x2, 1, false>("dwordx2", a, b, bytes, cus);
  rc |= run<u32x2, 4, false>("dwordx2", a, b, bytes, cus);
  rc |= run<u32x2, 4, true>("dwordx2", a, b, bytes, cus);
  rc |= run<u32x2, 8, true>("dwordx2", a, b, bytes, cus);
  rc |= run<u32x2, 8, false>("dwordx2", a, b, bytes, cus);
  rc |= run<u32x4, 1, false>("dwordx4", a, b, bytes, cus);
  rc |= run<u32x4, 2, false>("dwordx4", a, b, bytes, cus);
  rc |= run<u32x4, 2, true>("dwordx4", a, b, bytes, cus);
  rc |= run<u32x4, 4, true>("dwordx4", a, b, bytes, cus);
  rc |= run<u32x4, 4, false>("dwordx4", a, b, bytes, cus);
  return rc;
}
