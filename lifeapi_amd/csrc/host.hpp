// host.hpp -- host-side helpers shared by the kernel files (host.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

#include "common.hpp"
#include "lifeapi_hip.h"

namespace lifeapi_impl {

extern thread_local std::string g_err;  // lifeapi_last_error()

// set g_err (fmt has one %s for arg) and return code
int fail(int code, const char *fmt, const char *arg = nullptr);
// set g_err from a HIP error; missing code objects map to LIFEAPI_E_NOKERNEL
int fail_hip(hipError_t e, const char *what);
// CUs of the current device, which must be a gfx950
int device_cus(int &cus);
// unused dynamic LDS per block that leaves exactly min(blocks_per_cu, what
// the kernel's registers allow) blocks of `kernel` resident per CU of the
// current device (an occupancy cap), checked against the occupancy API
int occupancy_lds(const void *kernel, int blocks_per_cu, unsigned &bytes);
// Launch order keyed on the batch (the order never changes a result): true
// = take the groups in reverse.  Reverse exactly when d_in is a batch of
// `bytes` that an earlier order-keyed launch on this device wrote in forward
// order (and forward when it wrote it in reverse), so that each launch starts
// on what the launch that wrote its input wrote last, which the memory-side
// Infinity Cache may still hold; any other input runs forward.  Records d_out
// as written in the order returned.  A few batches are remembered per device,
// so interleaved loops over several batches keep the alternation.
bool launch_reverse(const void *d_in, const void *d_out, uint64_t bytes);
// Records d_out (bytes) as written in forward order by a launch that does not
// alternate (so a stale entry for that range cannot reverse a later reader).
void note_forward_write(const void *d_out, uint64_t bytes);
bool aligned8(const void *p);
inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }
// n universes in / out: non-null, 8-byte aligned, equal or disjoint
int check_batch(const void *in, const void *out, size_t n);
// blocks for `waves_needed` waves, capped at cus * blocks_per_cu (0 = no cap)
unsigned grid_for(uint64_t waves_needed, int cus, int blocks_per_cu);
// the launch's error state as a return code
int launched(const char *what);

struct DeviceGuard {  // restores the caller's current device
  int prev = -1;
  DeviceGuard() { (void)hipGetDevice(&prev); }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// One host array taking part in a host-pointer call: `bytes` per universe;
// src -> copied in before each chunk's launch, dst -> copied out after it
// (src == dst for in-place arrays).
struct HostIO {
  const void *src;
  void *dst;
  size_t bytes;
};
using ChunkFn = int (*)(void *const *dev, size_t m, hipStream_t s, const void *arg);

// Stages n universes through this device's reusable buffers in chunks that
// alternate between two streams: H2D, the stream-ordered *_dev entry point,
// D2H, all asynchronous, then one sync of both streams.
int host_chunked(int dev, size_t n, const HostIO *io, int nio, ChunkFn fn, const void *arg);
// the device a host-pointer call runs on (-1 = device 0), or an error code
int host_device(int device);

}  // namespace lifeapi_impl
