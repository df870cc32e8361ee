// membw.hip -- HBM streaming ceilings for the access shapes the step kernel
// can use (measurement tool, not product code).  Copies 2^20 universes (512
// MiB in + 512 MiB out) with wave-contiguous 512-B (dwordx2) or 1-KiB
// (dwordx4) accesses, U loads in flight per lane, plain or nontemporal loads
// and stores, for several grid sizes; plus read-only and write-only streams
// of the same 512 MiB.  Prints one JSON line per variant.
//   membw         the full sweep
//   membw calib   only the step kernel's shape (dwordx2, U=4, nt, one-shot
//                 grid): the byte-counter calibration run for rocprofv3
//   membw pingpong <universes>
//                 the step kernel's shape as the bench runs it: ping-pong
//                 between two buffers of <universes> x 512 B (1M: 1 GiB
//                 footprint, partly served from the 256 MB Infinity Cache;
//                 16M: 16 GiB, not); with as many blocks resident per CU
//                 as fit and with at most 4, 5, 6 (unused dynamic LDS)
//   membw snake <universes>
//                 the same ping-pong with the group order reversed on every
//                 other launch (each launch first reads what the last one
//                 wrote last), against the same order, per nontemporal mode
//   membw inplace <objects> <planes>
//                 the LifeStable kernels' shape: one wave per object reads
//                 its <planes> x 512 B (contiguous) and writes them back in
//                 place (nontemporal, as k_stable), at grid caps 0 (one wave
//                 per object), 8 and 32 blocks per CU, and uncapped with the
//                 blocks per CU limited by unused dynamic LDS
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

// MODE bit 0: nontemporal loads, bit 1: nontemporal stores,
//      bit 2: read only (xor-reduce, one store per wave), bit 3: write only
template <class T, int U, int MODE>
__global__ __launch_bounds__(256) void k_copy(const T *__restrict__ in, T *__restrict__ out,
                                              u64 nvec) {
  // a "row" = 64 lanes x sizeof(T); waves take U rows at a time, grid-strided
  const int lane = threadIdx.x & 63;
  const u64 wave = (u64)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 rows = nvec / 64, stride = (u64)gridDim.x * 4 * U;
  T acc = T(0);
  for (u64 r0 = wave * U; r0 < rows; r0 += stride) {
    T v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (MODE & 8) v[k] = T((unsigned)(r0 + k));
      else if (r0 + k < rows)
        v[k] = (MODE & 1) ? __builtin_nontemporal_load(in + (r0 + k) * 64 + lane) : in[(r0 + k) * 64 + lane];
    }
    if constexpr ((MODE & 4) != 0) {
#pragma unroll
      for (int k = 0; k < U; ++k) acc ^= v[k];
    } else {
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (r0 + k < rows) {
          if (MODE & 2) __builtin_nontemporal_store(v[k], out + (r0 + k) * 64 + lane);
          else out[(r0 + k) * 64 + lane] = v[k];
        }
    }
  }
  if constexpr ((MODE & 4) != 0) out[wave * 64 + lane] = acc;  // keep the loads live
}

// read-modify-write in place of P planes of 512 B per object, one wave per
// object (grid-strided when the grid is capped)
template <int P>
__global__ __launch_bounds__(256) void k_inplace(u32x2 *buf, u64 n) {
  const int lane = threadIdx.x & 63;
  const u64 stride = (u64)gridDim.x * 4;
  for (u64 u = (u64)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); u < n; u += stride) {
    u32x2 *q = buf + u * P * 64 + lane;
    u32x2 v[P];
#pragma unroll
    for (int k = 0; k < P; ++k) v[k] = __builtin_nontemporal_load(q + k * 64);
#pragma unroll
    for (int k = 0; k < P; ++k) __builtin_nontemporal_store(v[k] ^ u32x2{1u, 0u}, q + k * 64);
  }
}

template <int P>
int inplace(u64 objects, int cus) {
  const size_t bytes = objects * P * 512;
  void *a;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMemset(a, 0x5a, bytes));
  // grid caps (bpc), then occupancy caps through unused dynamic LDS: at
  // most 160 KiB / lds blocks (of 4 waves) per CU
  const int caps[][2] = {{0, 0}, {8, 0}, {32, 0}, {0, 0}, {0, 20 << 10}, {0, 27 << 10}, {0, 40 << 10},
                         {0, 54 << 10}, {0, 80 << 10}};
  for (const auto &cap : caps) {
    const int bpc = cap[0], lds = cap[1];
    u64 blocks = (objects + 3) / 4;
    if (bpc) blocks = std::min<u64>(blocks, (u64)cus * bpc);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<float> ms;
    for (int rep = 0; rep < 20; ++rep) {
      CHECK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL((k_inplace<P>), dim3(blocks), dim3(256), lds, 0, (u32x2 *)a, objects);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float t;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      if (rep >= 5) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::printf("{\"variant\": \"inplace dwordx2 nt\", \"planes\": %d, \"objects\": %llu, \"blocks_per_cu\": %d, "
                "\"dyn_lds\": %d, \"ms_best\": %.4f, \"ms_median\": %.4f, \"GBps_best\": %.1f, \"GBps_median\": %.1f}\n",
                P, objects, bpc, lds, ms.front(), ms[ms.size() / 2], 2.0 * bytes / (ms.front() * 1e-3) / 1e9,
                2.0 * bytes / (ms[ms.size() / 2] * 1e-3) / 1e9);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
  }
  CHECK(hipFree(a));
  return 0;
}

static bool g_calib = false;

template <class T, int U, int MODE>
int run(const char *name, void *a, void *b, size_t bytes, int cus) {
  const u64 nvec = bytes / sizeof(T);
  const u64 rows = nvec / 64;
  const double moved = (MODE & 12) ? (double)bytes : 2.0 * bytes;
  for (int bpc : {4, 16, 0}) {
    if (g_calib && bpc != 0) continue;
    u64 blocks = (rows / U + 3) / 4;
    if (bpc) blocks = std::min<u64>(blocks, (u64)cus * bpc);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<float> ms;
    for (int rep = 0; rep < 25; ++rep) {
      CHECK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL((k_copy<T, U, MODE>), dim3(blocks), dim3(256), 0, 0, (const T *)a, (T *)b, nvec);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float t;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      if (rep >= 5) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::printf("{\"variant\": \"%s\", \"U\": %d, \"mode\": %d, \"blocks_per_cu\": %d, \"blocks\": %llu, "
                "\"ms_best\": %.4f, \"ms_median\": %.4f, \"GBps_best\": %.1f, \"GBps_median\": %.1f}\n",
                name, U, MODE, bpc, blocks, ms.front(), ms[ms.size() / 2], moved / (ms.front() * 1e-3) / 1e9,
                moved / (ms[ms.size() / 2] * 1e-3) / 1e9);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
  }
  return 0;
}

int pingpong(u64 universes) {
  const size_t bytes = universes * 512;
  void *a, *b;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMemset(a, 0x5a, bytes));
  CHECK(hipMemset(b, 0x3c, bytes));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const u64 nvec = bytes / sizeof(u32x2), rows = nvec / 64;
  const u64 blocks = (rows / 4 + 3) / 4;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // as many blocks resident per CU as fit, then at most 4 / 5 / 6 (unused
  // dynamic LDS), as the step kernel can be launched
  for (int resident : {0, 4, 5, 6}) {
    const unsigned lds = resident ? (unsigned)((p.maxSharedMemoryPerMultiProcessor / resident) & ~255ull)  /* round down: k blocks fit */ : 0u;
    std::vector<float> ms;
    for (int rep = 0; rep < 30; ++rep) {
      void *src = rep & 1 ? b : a, *dst = rep & 1 ? a : b;
      CHECK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL((k_copy<u32x2, 4, 3>), dim3(blocks), dim3(256), lds, 0, (const u32x2 *)src, (u32x2 *)dst,
                         nvec);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float t;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      if (rep >= 6) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::printf("{\"variant\": \"dwordx2 pingpong\", \"U\": 4, \"mode\": 3, \"universes\": %llu, "
                "\"resident_blocks\": %d, \"ms_best\": %.4f, \"ms_median\": %.4f, \"GBps_best\": %.1f, "
                "\"GBps_median\": %.1f}\n",
                universes, resident, ms.front(), ms[ms.size() / 2], 2.0 * bytes / (ms.front() * 1e-3) / 1e9,
                2.0 * bytes / (ms[ms.size() / 2] * 1e-3) / 1e9);
  }
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  return 0;
}

// One-shot copy (each wave one group of U rows) whose group order is reversed
// when `rev` is set: alternating it between ping-pong launches makes each
// launch read first what the previous one wrote last (the memory-side
// Infinity Cache may still hold it).
template <int U, int MODE>
__global__ __launch_bounds__(256) void k_copy_dir(const u32x2 *in, u32x2 *out, u64 groups, int rev) {
  const int lane = threadIdx.x & 63;
  u64 g = (u64)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (g >= groups) return;
  if (rev) g = groups - 1 - g;
  const u32x2 *p = in + g * U * 64 + lane;
  u32x2 *q = out + g * U * 64 + lane;
  u32x2 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) v[k] = (MODE & 1) ? __builtin_nontemporal_load(p + k * 64) : p[k * 64];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    if (MODE & 2) __builtin_nontemporal_store(v[k] ^ u32x2{1u, 0u}, q + k * 64);
    else q[k * 64] = v[k] ^ u32x2{1u, 0u};
  }
}

// ping-pong copies as the bench's step launches (1 KiB per universe per
// launch), same direction every launch vs alternating direction ("snake"),
// for each nontemporal mode, at most 6 blocks resident per CU or all
template <int MODE>
int snake_mode(void *a, void *b, u64 universes, const hipDeviceProp_t &p) {
  const size_t bytes = universes * 512;
  const u64 groups = universes / 4;  // a row of 64 x 8 B is one universe; 4 per wave
  const u64 blocks = (groups + 3) / 4;
  hipEvent_t ev[41];
  for (auto &e : ev) CHECK(hipEventCreate(&e));
  for (int resident : {0, 6}) {
    const unsigned lds = resident ? (unsigned)((p.maxSharedMemoryPerMultiProcessor / resident) & ~255ull)  /* round down: k blocks fit */ : 0u;
    for (int snake : {0, 1, 0, 1}) {
      for (int rep = 0; rep < 10; ++rep)  // warm
        hipLaunchKernelGGL((k_copy_dir<4, MODE>), dim3(blocks), dim3(256), lds, 0, (const u32x2 *)(rep & 1 ? b : a),
                           (u32x2 *)(rep & 1 ? a : b), groups, snake ? (rep & 1) : 0);
      CHECK(hipEventRecord(ev[0], 0));
      for (int rep = 0; rep < 40; ++rep) {
        hipLaunchKernelGGL((k_copy_dir<4, MODE>), dim3(blocks), dim3(256), lds, 0, (const u32x2 *)(rep & 1 ? b : a),
                           (u32x2 *)(rep & 1 ? a : b), groups, snake ? (rep & 1) : 0);
        CHECK(hipEventRecord(ev[rep + 1], 0));
      }
      CHECK(hipEventSynchronize(ev[40]));
      std::vector<float> ms;
      for (int rep = 0; rep < 40; ++rep) {
        float t;
        CHECK(hipEventElapsedTime(&t, ev[rep], ev[rep + 1]));
        ms.push_back(t);
      }
      float tot;
      CHECK(hipEventElapsedTime(&tot, ev[0], ev[40]));
      std::sort(ms.begin(), ms.end());
      std::printf("{\"variant\": \"dwordx2 pingpong snake\", \"mode\": %d, \"snake\": %d, \"universes\": %llu, "
                  "\"resident_blocks\": %d, \"ms_mean\": %.4f, \"ms_median\": %.4f, \"GBps_mean\": %.1f, "
                  "\"GBps_median\": %.1f}\n",
                  MODE, snake, universes, resident, tot / 40, ms[20], 2.0 * bytes / (tot / 40 * 1e-3) / 1e9,
                  2.0 * bytes / (ms[20] * 1e-3) / 1e9);
      std::fflush(stdout);
    }
  }
  for (auto &e : ev) CHECK(hipEventDestroy(e));
  return 0;
}

int snake(u64 universes) {
  if (universes % 4) return 1;
  const size_t bytes = universes * 512;
  void *a, *b;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMemset(a, 0x5a, bytes));
  CHECK(hipMemset(b, 0x3c, bytes));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  if (snake_mode<3>(a, b, universes, p) || snake_mode<1>(a, b, universes, p) ||
      snake_mode<0>(a, b, universes, p) || snake_mode<2>(a, b, universes, p))
    return 1;
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 2 && std::string(argv[1]) == "pingpong") return pingpong(std::stoull(argv[2]));
  if (argc > 2 && std::string(argv[1]) == "snake") return snake(std::stoull(argv[2]));
  if (argc > 3 && std::string(argv[1]) == "inplace") {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const u64 n = std::stoull(argv[2]);
    switch (std::stoi(argv[3])) {
      case 1: return inplace<1>(n, p.multiProcessorCount);
      case 4: return inplace<4>(n, p.multiProcessorCount);
      case 10: return inplace<10>(n, p.multiProcessorCount);
      case 11: return inplace<11>(n, p.multiProcessorCount);
      default: std::fprintf(stderr, "planes: 1, 4, 10 or 11\n"); return 2;
    }
  }
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
  if (g_calib) return run<u32x2, 4, 3>("dwordx2", a, b, bytes, cus);
  int rc = 0;
  rc |= run<u32x2, 4, 0>("dwordx2", a, b, bytes, cus);
  rc |= run<u32x2, 4, 1>("dwordx2", a, b, bytes, cus);
  rc |= run<u32x2, 4, 2>("dwordx2", a, b, bytes, cus);
  rc |= run<u32x2, 4, 3>("dwordx2", a, b, bytes, cus);
  rc |= run<u32x2, 8, 3>("dwordx2", a, b, bytes, cus);
  rc |= run<u32x2, 16, 3>("dwordx2", a, b, bytes, cus);
  rc |= run<u32x4, 2, 3>("dwordx4", a, b, bytes, cus);
  rc |= run<u32x4, 4, 3>("dwordx4", a, b, bytes, cus);
  rc |= run<u32x4, 8, 3>("dwordx4", a, b, bytes, cus);
  rc |= run<u32x2, 4, 5>("dwordx2-readonly", a, b, bytes, cus);
  rc |= run<u32x4, 4, 5>("dwordx4-readonly", a, b, bytes, cus);
  rc |= run<u32x2, 4, 10>("dwordx2-writeonly", a, b, bytes, cus);
  rc |= run<u32x4, 4, 10>("dwordx4-writeonly", a, b, bytes, cus);
  return rc;
}
