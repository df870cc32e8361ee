// host.hip -- host side of the C ABI: errors, device checks, launch
// geometry, the staging used by every host-pointer entry point, and those
// entry points that only stage data around a *_dev call.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "host.hpp"

namespace lifeapi_impl {

thread_local std::string g_err;

int fail(int code, const char *fmt, const char *arg) {
  char buf[512];
  std::snprintf(buf, sizeof buf, fmt, arg ? arg : "");
  g_err = buf;
  return code;
}
int fail_hip(hipError_t e, const char *what) {
  // the error is reported through our return code: consume HIP's sticky
  // per-thread copy, or the next launch's hipGetLastError() would return it
  (void)hipGetLastError();
  char buf[512];
  std::snprintf(buf, sizeof buf, "%s: %s (hipError %d)", what, hipGetErrorString(e), (int)e);
  g_err = buf;
  if (e == hipErrorNoBinaryForGpu || e == hipErrorInvalidDeviceFunction ||
      e == hipErrorInvalidImage || e == hipErrorSharedObjectInitFailed)
    return LIFEAPI_E_NOKERNEL;
  return (int)e;
}

struct DevInfo {
  int cus = 0;
  size_t lds_per_cu = 0;
  bool ok = false;
};
std::mutex g_info_mu;
std::vector<DevInfo> g_info;

static int device_info(DevInfo &out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return fail_hip(e, "hipGetDevice");
  std::lock_guard<std::mutex> lk(g_info_mu);
  if ((int)g_info.size() <= dev) g_info.resize(dev + 1);
  if (!g_info[dev].ok) {
    hipDeviceProp_t p;
    e = hipGetDeviceProperties(&p, dev);
    if (e != hipSuccess) return fail_hip(e, "hipGetDeviceProperties");
    if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
      return fail(LIFEAPI_E_NODEVICE, "device is %s, this library is built for gfx950 only",
                  p.gcnArchName);
    g_info[dev].cus = p.multiProcessorCount;
    g_info[dev].lds_per_cu = p.maxSharedMemoryPerMultiProcessor;
    g_info[dev].ok = true;
  }
  out = g_info[dev];
  return LIFEAPI_OK;
}

int device_cus(int &cus) {
  DevInfo d;
  const int rc = device_info(d);
  cus = d.cus;
  return rc;
}

// occupancy_lds results per (device, kernel, blocks per CU): the answer
// depends on nothing else, and computing it takes several occupancy queries
struct OccKey {
  int dev;
  const void *kernel;
  int blocks;
  bool operator<(const OccKey &o) const {
    return std::tie(dev, kernel, blocks) < std::tie(o.dev, o.kernel, o.blocks);
  }
};
std::mutex g_occ_mu;
std::map<OccKey, unsigned> g_occ;

static int occupancy_lds_uncached(const void *kernel, int blocks_per_cu, unsigned &bytes);

int occupancy_lds(const void *kernel, int blocks_per_cu, unsigned &bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return fail_hip(e, "hipGetDevice");
  const OccKey key{dev, kernel, blocks_per_cu};
  {
    std::lock_guard<std::mutex> lk(g_occ_mu);
    auto it = g_occ.find(key);
    if (it != g_occ.end()) {
      bytes = it->second;
      return LIFEAPI_OK;
    }
  }
  const int rc = occupancy_lds_uncached(kernel, blocks_per_cu, bytes);
  if (rc == LIFEAPI_OK) {
    std::lock_guard<std::mutex> lk(g_occ_mu);
    g_occ[key] = bytes;
  }
  return rc;
}

static int occupancy_lds_uncached(const void *kernel, int blocks_per_cu, unsigned &bytes) {
  DevInfo d;
  int rc = device_info(d);
  if (rc != LIFEAPI_OK) return rc;
  if (blocks_per_cu < 1) return fail(LIFEAPI_E_INVALID, "occupancy cap below one block per CU%s");
  hipFuncAttributes fa;
  hipError_t e = hipFuncGetAttributes(&fa, kernel);
  if (e != hipSuccess) return fail_hip(e, "hipFuncGetAttributes");
  int free_blocks = 0;  // what the kernel's registers and static LDS allow
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&free_blocks, kernel, kBlock, 0);
  if (e != hipSuccess) return fail_hip(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
  if (free_blocks < 1) return fail(LIFEAPI_E_INVALID, "kernel cannot be resident%s");
  const int want = std::min(blocks_per_cu, free_blocks);
  // round DOWN: k blocks of (static + dynamic) LDS must fit in the CU's LDS
  // (rounding up to the granule allowed one block fewer whenever k does not
  // divide it: 6 -> 5, 3 -> 2)
  const size_t per_block = d.lds_per_cu / (size_t)want;
  size_t dyn = per_block > fa.sharedSizeBytes ? (per_block - fa.sharedSizeBytes) & ~(size_t)255 : 0;
  for (;; dyn -= 256) {
    int got = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&got, kernel, kBlock, dyn);
    if (e != hipSuccess) return fail_hip(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    if (got >= want) break;  // the granule rounded us above the share: shrink
    if (dyn < 256) return fail(LIFEAPI_E_INVALID, "cannot set the occupancy cap%s");
  }
  bytes = (unsigned)dyn;
  return LIFEAPI_OK;
}

// ---- launch order keyed on the batch (host.hpp launch_reverse) ----
namespace {
constexpr int kOrderDevices = 64, kOrderSlots = 8;
struct OrderSlot {
  uintptr_t ptr = 0;
  uint64_t bytes = 0, tick = 0;
  bool reverse = false;
};
struct OrderBook {
  std::mutex mu;
  OrderSlot slot[kOrderSlots];
  uint64_t tick = 0;
};
OrderBook g_order[kOrderDevices];

OrderBook *order_book() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kOrderDevices) return nullptr;
  return &g_order[dev];
}

// forget every batch overlapping [p, p + bytes), then remember it written in
// order `rev` (the least recently written slot makes room); mu held
void order_record(OrderBook &b, uintptr_t p, uint64_t bytes, bool rev) {
  OrderSlot *victim = &b.slot[0];
  for (OrderSlot &s : b.slot) {
    if (s.bytes && s.ptr < p + bytes && p < s.ptr + s.bytes) s = OrderSlot{};
    if (!s.bytes || (victim->bytes && s.tick < victim->tick)) victim = &s;
  }
  *victim = OrderSlot{p, bytes, ++b.tick, rev};
}
}  // namespace

bool launch_reverse(const void *d_in, const void *d_out, uint64_t bytes) {
  OrderBook *b = order_book();
  if (!b || bytes == 0) return false;
  std::lock_guard<std::mutex> lk(b->mu);
  bool rev = false;
  for (const OrderSlot &s : b->slot)
    if (s.bytes == bytes && s.ptr == (uintptr_t)d_in) rev = !s.reverse;
  order_record(*b, (uintptr_t)d_out, bytes, rev);
  return rev;
}

void note_forward_write(const void *d_out, uint64_t bytes) {
  OrderBook *b = order_book();
  if (!b || bytes == 0) return;
  std::lock_guard<std::mutex> lk(b->mu);
  order_record(*b, (uintptr_t)d_out, bytes, false);
}

bool aligned8(const void *p) { return ((uintptr_t)p & 7u) == 0; }

int check_batch(const void *in, const void *out, size_t n) {
  if (n == 0) return LIFEAPI_OK;
  if (!in || !out) return fail(LIFEAPI_E_INVALID, "null universe pointer%s");
  if (!aligned8(in) || !aligned8(out)) return fail(LIFEAPI_E_INVALID, "universe pointers must be 8-byte aligned%s");
  if (n > (SIZE_MAX / 512)) return fail(LIFEAPI_E_INVALID, "n too large%s");
  const uintptr_t a = (uintptr_t)in, b = (uintptr_t)out, bytes = (uintptr_t)n * 512u;
  if (a != b && a < b + bytes && b < a + bytes)
    return fail(LIFEAPI_E_INVALID, "input and output batches overlap (only in == out is allowed)%s");
  return LIFEAPI_OK;
}

unsigned grid_for(uint64_t waves_needed, int cus, int blocks_per_cu) {
  uint64_t blocks = (waves_needed + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks_per_cu > 0) blocks = std::min<uint64_t>(blocks, (uint64_t)cus * blocks_per_cu);
  blocks = std::min<uint64_t>(blocks, 1u << 30);
  return (unsigned)std::max<uint64_t>(blocks, 1);
}

int launched(const char *what) {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? LIFEAPI_OK : fail_hip(e, what);
}

// ---- host-pointer staging: one context per device ----
// Chunks alternate between two streams, each with its own staging buffer,
// and everything is issued asynchronously before one final sync per call.
// Stream order alone protects a buffer's reuse (chunk k + 2 waits for chunk
// k's D2H on the same stream).  Chunk k's H2D also waits (event) for chunk
// k-1's H2D, so the two streams run one chunk apart and chunk k's D2H
// overlaps chunk k+1's H2D; without that they start in phase and both
// directions stay serialised.  That pays only for page-locked host arrays:
// the runtime serialises pageable copies in both directions.  So every call
// moving at least kPinMinBytes page-locks the caller's arrays itself for its
// duration (hipHostRegister, then hipHostUnregister): on MI355X that costs
// under 1 ms and takes 1M universes from 19.4 to 12.2-13.1 ms
// (profiles/r01/host_bench.jsonl).  Arrays the caller pinned already
// (lifeapi_host_register) or that cannot be pinned are used as they are.
constexpr int kLanes = 2;  // (the event chain below assumes two)
constexpr size_t kChunkBytes = size_t(64) << 20;  // staging per stream and pass
constexpr size_t kPinMinBytes = size_t(8) << 20;  // smaller calls stay pageable

// Ranges this library pinned, shared by every call in the process: a call
// whose array lies inside one takes a reference instead of registering again,
// so concurrent calls (other threads, the per-device shards of
// lifeapi_step_batch) never unpin memory another call is still copying.
struct PinRec {
  uintptr_t lo, hi;
  int refs;
};
std::mutex g_pin_mu;
std::vector<PinRec> g_pins;

// Adds to `keys` a reference on every range this library pinned that
// overlaps [p, p + bytes) -- whatever the call's size, so no other call can
// unpin memory this call's copies may DMA from, even where the ranges only
// partly overlap.  With no overlap, a call of at least kPinMinBytes pins the
// array itself (and references that); smaller calls, arrays the caller
// pinned and unpinnable memory are used as they are.  Each key goes back
// through pin_release.
void pin_acquire(const void *p, size_t bytes, std::vector<uintptr_t> &keys) {
  if (!p || !bytes) return;
  const uintptr_t lo = (uintptr_t)p, hi = lo + bytes;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  bool overlap = false;
  for (PinRec &r : g_pins)
    if (lo < r.hi && r.lo < hi) {
      ++r.refs;
      keys.push_back(r.lo);
      overlap = true;
    }
  if (overlap || bytes < kPinMinBytes) return;
  // Leave ranges the caller pinned alone: the runtime accepts a second
  // registration without counting it, so our unregister would undo theirs
  // (tools/ab/pin_probe.cpp; hipHostGetFlags fails on registered memory, the
  // pointer attributes report it as host memory).
  for (uintptr_t q : {lo, hi - 1}) {
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, (const void *)q);
    (void)hipGetLastError();
    if (e != hipSuccess || a.type != hipMemoryTypeUnregistered) return;
  }
  if (hipHostRegister((void *)lo, bytes, hipHostRegisterPortable) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  g_pins.push_back({lo, hi, 1});
  keys.push_back(lo);
}

void pin_release(uintptr_t key) {
  if (!key) return;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  for (size_t k = 0; k < g_pins.size(); ++k)
    if (g_pins[k].lo == key) {
      if (--g_pins[k].refs == 0) {
        if (hipHostUnregister((void *)key) != hipSuccess) (void)hipGetLastError();
        g_pins.erase(g_pins.begin() + k);
      }
      return;
    }
}

// Holds pin_acquire references for one call.
struct CallPins {
  std::vector<uintptr_t> keys;
  void add(const void *p, size_t bytes) { pin_acquire(p, bytes, keys); }
  ~CallPins() {
    for (uintptr_t k : keys) pin_release(k);
  }
};

struct HostCtx {
  std::mutex mu;
  hipStream_t stream[kLanes] = {};
  hipEvent_t h2d_done[kLanes] = {};
  char *buf[kLanes] = {};
  size_t cap = 0;  // bytes per stream
};
std::mutex g_ctx_mu;
std::vector<HostCtx *> g_ctx;

HostCtx *ctx_for(int dev) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  if ((int)g_ctx.size() <= dev) g_ctx.resize(dev + 1, nullptr);
  if (!g_ctx[dev]) g_ctx[dev] = new HostCtx();  // lives for the process
  return g_ctx[dev];
}

// Chunks are disjoint ranges of every array, so in-place arrays (src == dst)
// are safe.
int host_chunked(int dev, size_t n, const HostIO *io, int nio, ChunkFn fn, const void *arg) {
  if (nio > 8) return fail(LIFEAPI_E_INVALID, "too many arrays%s");
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return fail_hip(e, "hipSetDevice");
  HostCtx *c = ctx_for(dev);
  std::lock_guard<std::mutex> lk(c->mu);
  for (int l = 0; l < kLanes; ++l)
    if (!c->stream[l]) {
      e = hipStreamCreateWithFlags(&c->stream[l], hipStreamNonBlocking);
      if (e != hipSuccess) return fail_hip(e, "hipStreamCreate");
      e = hipEventCreateWithFlags(&c->h2d_done[l], hipEventDisableTiming);
      if (e != hipSuccess) return fail_hip(e, "hipEventCreate");
    }
  size_t per = 0;
  for (int k = 0; k < nio; ++k) per += (io[k].bytes + 255) & ~size_t(255);
  const size_t half = (n + kLanes - 1) / kLanes;
  const size_t chunk = std::max<size_t>(1, std::min(half, kChunkBytes / per));
  size_t need = 0;
  for (int k = 0; k < nio; ++k) need += ((io[k].bytes * chunk + 255) & ~size_t(255));
  if (c->cap < need) {
    for (int l = 0; l < kLanes; ++l) {
      if (c->buf[l]) (void)hipFree(c->buf[l]);
      c->buf[l] = nullptr;
    }
    c->cap = 0;
    for (int l = 0; l < kLanes; ++l) {
      e = hipMalloc(&c->buf[l], need);
      if (e != hipSuccess) return fail_hip(e, "hipMalloc(staging)");
    }
    c->cap = need;
  }
  // page-lock the caller's arrays for this call (see above)
  CallPins pins;
  for (int q = 0; q < nio; ++q) {
    pins.add(io[q].src, n * io[q].bytes);
    if (io[q].dst != io[q].src) pins.add(io[q].dst, n * io[q].bytes);
  }
  int rc = LIFEAPI_OK;
  void *d[8];
  for (size_t k = 0; k * chunk < n && rc == LIFEAPI_OK; ++k) {
    const int l = (int)(k % kLanes);
    hipStream_t st = c->stream[l];
    const size_t off = k * chunk, m = std::min(chunk, n - off);
    if (k > 0 && (e = hipStreamWaitEvent(st, c->h2d_done[1 - l], 0)) != hipSuccess) {
      rc = fail_hip(e, "hipStreamWaitEvent");
      break;
    }
    size_t pos = 0;
    for (int q = 0; q < nio && rc == LIFEAPI_OK; ++q) {
      d[q] = c->buf[l] + pos;
      pos += (io[q].bytes * chunk + 255) & ~size_t(255);
      if (io[q].src &&
          (e = hipMemcpyAsync(d[q], (const char *)io[q].src + off * io[q].bytes, m * io[q].bytes,
                              hipMemcpyHostToDevice, st)) != hipSuccess)
        rc = fail_hip(e, "hipMemcpyAsync(H2D)");
    }
    if (rc == LIFEAPI_OK && (e = hipEventRecord(c->h2d_done[l], st)) != hipSuccess)
      rc = fail_hip(e, "hipEventRecord");
    if (rc == LIFEAPI_OK) rc = fn(d, m, st, arg);
    for (int q = 0; q < nio && rc == LIFEAPI_OK; ++q)
      if (io[q].dst &&
          (e = hipMemcpyAsync((char *)io[q].dst + off * io[q].bytes, d[q], m * io[q].bytes,
                              hipMemcpyDeviceToHost, st)) != hipSuccess)
        rc = fail_hip(e, "hipMemcpyAsync(D2H)");
  }
  // drain both streams even after an error: nothing may still read or write
  // the caller's arrays once we return
  for (int l = 0; l < kLanes; ++l) {
    e = hipStreamSynchronize(c->stream[l]);
    if (e != hipSuccess && rc == LIFEAPI_OK) rc = fail_hip(e, "hipStreamSynchronize");
  }
  return rc;  // (both streams synchronised: the pins can go)
}

int host_device(int device) {
  const int ndev = lifeapi_device_count();
  if (ndev <= 0) return fail(LIFEAPI_E_NODEVICE, "no HIP device visible%s");
  if (device < 0) device = 0;
  if (device >= ndev) return fail(LIFEAPI_E_NODEVICE, "bad device index%s");
  return device;
}

// device >= 0: fn(0, n, device) on that device.  device -1: one contiguous
// shard per visible device, fn(lo, hi, dev) on one host thread each, with the
// given host ranges page-locked once for all shards (shard boundaries share
// pages).  LIFEAPI_HOST_SHARDS=k (1 <= k <= 64, else LIFEAPI_E_INVALID; empty = unset)
// overrides the shard count (at most n shards), shard s
// running on device s mod ndev: a rehearsal knob that runs the threaded path
// on a machine with fewer GPUs (tests/test_host_multidev.py).  The first
// failing shard's code and message are returned.
constexpr long kMaxHostShards = 64;
template <class F>
int over_devices(size_t n, int device, const std::pair<const void *, size_t> *ranges, int nranges, F &&fn) {
  const int ndev = lifeapi_device_count();
  if (ndev <= 0) return fail(LIFEAPI_E_NODEVICE, "no HIP device visible%s");
  if (device >= ndev || device < -1) return fail(LIFEAPI_E_NODEVICE, "bad device index%s");
  int shards = ndev;
  if (device < 0) {
    const char *e = std::getenv("LIFEAPI_HOST_SHARDS");
    if (e && *e) {  // (set but empty = unset, as `export LIFEAPI_HOST_SHARDS=` leaves it)
      char *end = nullptr;
      const long k = std::strtol(e, &end, 10);
      if (end == e || *end != '\0' || k < 1 || k > kMaxHostShards)
        return fail(LIFEAPI_E_INVALID, "LIFEAPI_HOST_SHARDS must be an integer in 1..64, not '%s'", e);
      shards = (int)k;
    }
    shards = (int)std::min<size_t>((size_t)shards, std::max<size_t>(n, 1));  // no empty shards
  }
  if (device >= 0 || shards == 1) return fn(0, n, device < 0 ? 0 : device);
  CallPins pins;
  for (int r = 0; r < nranges; ++r)
    if (ranges[r].first) pins.add(ranges[r].first, ranges[r].second);
  std::vector<int> rcs(shards, LIFEAPI_OK);
  std::vector<std::string> errs(shards);
  std::vector<std::thread> pool;
  for (int k = 0; k < shards; ++k) {
    const size_t lo = n * k / shards, hi = n * (k + 1) / shards;
    pool.emplace_back([&, k, lo, hi] {
      if (hi > lo) rcs[k] = fn(lo, hi, k % ndev);
      errs[k] = g_err;
    });
  }
  for (auto &t : pool) t.join();
  for (int k = 0; k < shards; ++k)
    if (rcs[k] != LIFEAPI_OK) {
      g_err = errs[k];
      return rcs[k];
    }
  return LIFEAPI_OK;
}

// host_chunked over device(s): device >= 0 one device, -1 every visible one
// (over_devices), each shard's arrays offset by its first universe
int host_batch(size_t n, int device, const HostIO *io, int nio, ChunkFn fn, const void *arg) {
  std::pair<const void *, size_t> ranges[8];
  int nr = 0;
  for (int i = 0; i < nio && nr < 7; ++i) {
    if (io[i].src) ranges[nr++] = {io[i].src, n * io[i].bytes};
    if (io[i].dst && io[i].dst != io[i].src) ranges[nr++] = {io[i].dst, n * io[i].bytes};
  }
  return over_devices(n, device, ranges, nr, [&](size_t lo, size_t hi, int dev) {
    HostIO sh[4];
    for (int i = 0; i < nio; ++i)
      sh[i] = {io[i].src ? (const char *)io[i].src + lo * io[i].bytes : nullptr,
               io[i].dst ? (char *)io[i].dst + lo * io[i].bytes : nullptr, io[i].bytes};
    return host_chunked(dev, hi - lo, sh, nio, fn, arg);
  });
}

int host_step_one_device(const uint64_t *in, uint64_t *out, size_t n, uint32_t gens, int dev) {
  const HostIO io[1] = {{in, out, 512}};
  return host_chunked(dev, n, io, 1,
                      [](void *const *d, size_t m, hipStream_t s, const void *arg) {
                        return lifeapi_step_batch_dev((const uint64_t *)d[0], (uint64_t *)d[0], m,
                                                      *(const uint32_t *)arg, s);
                      },
                      &gens);
}

}  // namespace lifeapi_impl

using namespace lifeapi_impl;

extern "C" {

int lifeapi_abi_version(void) { return LIFEAPI_ABI_VERSION; }

const char *lifeapi_last_error(void) { return g_err.c_str(); }

int lifeapi_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int lifeapi_step_batch(const uint64_t *in, uint64_t *out, size_t n, uint32_t generations,
                       int device) {
  int rc = check_batch(in, out, n);
  if (rc != LIFEAPI_OK || n == 0) return rc;
  const std::pair<const void *, size_t> ranges[2] = {{in, n * 512}, {out != in ? out : nullptr, n * 512}};
  return over_devices(n, device, ranges, 2, [&](size_t lo, size_t hi, int dev) {
    return host_step_one_device(in + lo * 64, out + lo * 64, hi - lo, generations, dev);
  });
}

int lifeapi_host_register(void *p, size_t bytes) {
  if (!p || bytes == 0) return fail(LIFEAPI_E_INVALID, "null or empty range to lifeapi_host_register%s");
  if (lifeapi_device_count() <= 0) return fail(LIFEAPI_E_NODEVICE, "no HIP device visible%s");
  const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterPortable);
  return e == hipSuccess ? LIFEAPI_OK : fail_hip(e, "hipHostRegister");
}

int lifeapi_host_unregister(void *p) {
  if (!p) return fail(LIFEAPI_E_INVALID, "null pointer to lifeapi_host_unregister%s");
  if (lifeapi_device_count() <= 0) return fail(LIFEAPI_E_NODEVICE, "no HIP device visible%s");
  const hipError_t e = hipHostUnregister(p);
  return e == hipSuccess ? LIFEAPI_OK : fail_hip(e, "hipHostUnregister");
}

int lifeapi_pop_batch(const uint64_t *states, uint32_t *pop, size_t n, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!states || !pop || !aligned8(states)) return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_pop_batch%s");
  const HostIO io[2] = {{states, nullptr, 512}, {nullptr, pop, 4}};
  return host_batch(n, device, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *) {
                        return lifeapi_pop_batch_dev((const uint64_t *)d[0], (uint32_t *)d[1], m, s);
                      },
                      nullptr);
}

int lifeapi_weld_step_batch(uint64_t *welds, size_t n, uint32_t generations, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!welds || !aligned8(welds)) return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_weld_step_batch%s");
  const HostIO io[1] = {{welds, welds, 4 * 512}};
  return host_batch(n, device, io, 1,
                      [](void *const *d, size_t m, hipStream_t s, const void *arg) {
                        return lifeapi_weld_step_batch_dev((uint64_t *)d[0], m, *(const uint32_t *)arg, s);
                      },
                      &generations);
}

int lifeapi_stable_pass_batch(uint64_t *planes, uint8_t *flags, size_t n, int pass,
                              uint32_t max_iters, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!planes || !flags || !aligned8(planes) || pass < 0 || pass > 5)
    return fail(LIFEAPI_E_INVALID, "bad argument to lifeapi_stable_pass_batch%s");
  const uint32_t arg[2] = {(uint32_t)pass, max_iters};
  const HostIO io[2] = {{planes, planes, 10 * 512}, {nullptr, flags, 1}};
  return host_batch(n, device, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *a) {
                        const uint32_t *p = (const uint32_t *)a;
                        return lifeapi_stable_pass_batch_dev((uint64_t *)d[0], (uint8_t *)d[1], m,
                                                             (int)p[0], p[1], s);
                      },
                      arg);
}

int lifeapi_stable_vulnerable_batch(const uint64_t *planes, uint64_t *out, size_t n, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!planes || !out || !aligned8(planes) || !aligned8(out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_stable_vulnerable_batch%s");
  const HostIO io[2] = {{planes, nullptr, 10 * 512}, {nullptr, out, 512}};
  return host_batch(n, device, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *) {
                        return lifeapi_stable_vulnerable_batch_dev((const uint64_t *)d[0], (uint64_t *)d[1],
                                                                   m, s);
                      },
                      nullptr);
}

int lifeapi_neighbour_count_batch(const uint64_t *in, uint64_t *out, size_t n, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!in || !out || !aligned8(in) || !aligned8(out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_neighbour_count_batch%s");
  const HostIO io[2] = {{in, nullptr, 512}, {nullptr, out, 4 * 512}};
  return host_batch(n, device, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *) {
                        return lifeapi_neighbour_count_batch_dev((const uint64_t *)d[0], (uint64_t *)d[1], m, s);
                      },
                      nullptr);
}

int lifeapi_interaction_counts_batch(const uint64_t *in, uint64_t *out, size_t n, int with_next,
                                     int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!in || !out || !aligned8(in) || !aligned8(out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_interaction_counts_batch%s");
  const HostIO io[2] = {{in, nullptr, 512}, {nullptr, out, (with_next ? 4u : 3u) * 512}};
  return host_batch(n, device, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *a) {
                        return lifeapi_interaction_counts_batch_dev((const uint64_t *)d[0], (uint64_t *)d[1],
                                                                    m, *(const int *)a, s);
                      },
                      &with_next);
}

int lifeapi_refined_step_batch(const uint64_t *in, uint64_t *out, size_t n, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!in || !out || !aligned8(in) || !aligned8(out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_refined_step_batch%s");
  const HostIO io[2] = {{in, nullptr, 11 * 512}, {nullptr, out, 3 * 512}};
  return host_batch(n, device, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *) {
                        return lifeapi_refined_step_batch_dev((const uint64_t *)d[0], (uint64_t *)d[1], m, s);
                      },
                      nullptr);
}

static int host_contains_one_device(const uint64_t *states, const uint64_t *wanted, const uint64_t *unwanted,
                                    uint8_t *out, size_t n, int dev) {
  // the target rides along as a tiny device copy owned by this call
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return fail_hip(e, "hipSetDevice");
  uint64_t *dt = nullptr;
  if ((e = hipMalloc(&dt, 2 * 512)) != hipSuccess) return fail_hip(e, "hipMalloc(target)");
  int rc = LIFEAPI_OK;
  if ((e = hipMemcpy(dt, wanted, 512, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(dt + 64, unwanted, 512, hipMemcpyHostToDevice)) != hipSuccess)
    rc = fail_hip(e, "hipMemcpy(target)");
  if (rc == LIFEAPI_OK) {
    const HostIO io[2] = {{states, nullptr, 512}, {nullptr, out, 1}};
    rc = host_chunked(dev, n, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *a) {
                        const uint64_t *t = (const uint64_t *)a;
                        return lifeapi_contains_batch_dev((const uint64_t *)d[0], t, t + 64,
                                                          (uint8_t *)d[1], m, s);
                      },
                      dt);
  }
  (void)hipFree(dt);
  return rc;
}

int lifeapi_contains_batch(const uint64_t *states, const uint64_t *wanted, const uint64_t *unwanted,
                           uint8_t *out, size_t n, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!states || !wanted || !unwanted || !out || !aligned8(states))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_contains_batch%s");
  const std::pair<const void *, size_t> ranges[2] = {{states, n * 512}, {out, n}};
  return over_devices(n, device, ranges, 2, [&](size_t lo, size_t hi, int dev) {
    return host_contains_one_device(states + lo * 64, wanted, unwanted, out + lo, hi - lo, dev);
  });
}

static int host_step_contains_one_device(const uint64_t *in, uint64_t *final_states, const uint64_t *wanted,
                                         const uint64_t *unwanted, uint32_t *first_gen, size_t n,
                                         uint32_t generations, int dev) {
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return fail_hip(e, "hipSetDevice");
  uint64_t *dt = nullptr;  // the target, a tiny device copy owned by this call
  if ((e = hipMalloc(&dt, 2 * 512)) != hipSuccess) return fail_hip(e, "hipMalloc(target)");
  int rc = LIFEAPI_OK;
  if ((e = hipMemcpy(dt, wanted, 512, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(dt + 64, unwanted, 512, hipMemcpyHostToDevice)) != hipSuccess)
    rc = fail_hip(e, "hipMemcpy(target)");
  if (rc == LIFEAPI_OK) {
    struct Arg {
      const uint64_t *t;
      uint32_t gens;
      bool keep;
    } arg{dt, generations, final_states != nullptr};
    // the states' staging slot doubles as the device final buffer (in place)
    const HostIO io[2] = {{in, final_states, 512}, {nullptr, first_gen, 4}};
    rc = host_chunked(dev, n, io, 2,
                      [](void *const *d, size_t m, hipStream_t s, const void *a) {
                        const Arg *g = (const Arg *)a;
                        return lifeapi_step_contains_batch_dev((const uint64_t *)d[0],
                                                               g->keep ? (uint64_t *)d[0] : nullptr,
                                                               g->t, g->t + 64, (uint32_t *)d[1], m,
                                                               g->gens, s);
                      },
                      &arg);
  }
  (void)hipFree(dt);
  return rc;
}

int lifeapi_step_contains_batch(const uint64_t *in, uint64_t *final_states, const uint64_t *wanted,
                                const uint64_t *unwanted, uint32_t *first_gen, size_t n,
                                uint32_t generations, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!in || !wanted || !unwanted || !first_gen || !aligned8(in))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_step_contains_batch%s");
  if (final_states) {
    const int rc = check_batch(in, final_states, n);
    if (rc != LIFEAPI_OK) return rc;
  }
  const std::pair<const void *, size_t> ranges[3] = {
      {in, n * 512}, {final_states != in ? final_states : nullptr, n * 512}, {first_gen, n * 4}};
  return over_devices(n, device, ranges, 3, [&](size_t lo, size_t hi, int dev) {
    return host_step_contains_one_device(in + lo * 64, final_states ? final_states + lo * 64 : nullptr, wanted,
                                         unwanted, first_gen + lo, hi - lo, generations, dev);
  });
}

}  // extern "C"
