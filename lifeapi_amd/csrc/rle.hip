// rle.hip -- RLE batch I/O: LifeState::Parse and LifeState::RLE()
// (Parsing.hpp:8-63,143-204) over many patterns, one wave per pattern.
#include <algorithm>
#include <vector>

#include "device.hpp"
#include "host.hpp"

using namespace lifeapi_impl;

namespace {

// ------------------------------------------------------------------------
// RLE batch I/O (Parsing.hpp:143-204), one wave per pattern
// ------------------------------------------------------------------------

// LifeState::RLE() prints row y = (j + 32) & 63 as output row j, cells from
// x = 32 (GenericRLE, Parsing.hpp:13-16).  Lane j gets output row j with bit
// i = cell x = (i + 32) & 63: a 64x64 bit transpose by 64 ballots.
__device__ __forceinline__ uint64_t rle_row(uint64_t col, int lane) {
  uint64_t mine = 0;
  for (int j = 0; j < kWave; ++j) {
    const uint64_t m = __ballot((col >> ((j + 32) & 63)) & 1);
    if (lane == j) mine = (m >> 32) | (m << 32);
  }
  return mine;
}

// One output row's tokens (GenericRLE's loop body, Parsing.hpp:18-50): "<k>$"
// before the row's first live cell (k = rows since the last flush, omitted
// when 1), then "<n>o" / "<n>b" runs (n omitted when 1), a dead run that
// ends the row dropped.  Counts are at most 64, so at most two digits.
// Returns the byte count; writes them when WRITE.
template <bool WRITE>
__device__ uint32_t rle_row_tokens(uint64_t r, uint32_t eol, char *out) {
  uint32_t n = 0;
  auto count = [&](uint32_t c) {
    if (c <= 1) return;
    if (c >= 10) {
      if (WRITE) out[n] = (char)('0' + c / 10);
      ++n;
    }
    if (WRITE) out[n] = (char)('0' + c % 10);
    ++n;
  };
  if (r == 0) return 0;
  if (eol) {
    count(eol);
    if (WRITE) out[n] = '$';
    ++n;
  }
  uint32_t pos = 0, v = (uint32_t)(r & 1);
  while (pos < 64) {
    const uint64_t rest = r >> pos;
    const uint64_t ends = v ? ~rest : rest;  // first cell of the other value
    const uint32_t len = ends ? (uint32_t)__builtin_ctzll(ends) : 64u - pos;
    const uint32_t run = len < 64u - pos ? len : 64u - pos;
    if (!v && pos + run >= 64) break;  // dead run to the end of the row
    count(run);
    if (WRITE) out[n] = v ? 'o' : 'b';
    ++n;
    pos += run;
    v ^= 1u;
  }
  return n;
}

// longest RLE() of a 64x64 board: per row at most a 3-byte "<k>$" and 64
// bytes of runs (a run of n cells costs at most n bytes), then "!"
constexpr uint32_t kRleMaxBytes = 64 * (3 + 64) + 1 + 63;

// WRITE = false: len[u] = strlen(RLE()); WRITE = true: RLE() at text + offs[u]
template <bool WRITE>
__global__ __launch_bounds__(kBlock) void k_rle(const uint64_t *__restrict__ s, uint32_t *__restrict__ len,
                                                const uint64_t *__restrict__ offs, char *__restrict__ text,
                                                uint64_t n) {
  // the pattern is assembled in LDS and then copied out 64 consecutive bytes
  // per store (the rows' tokens land at scattered offsets)
  __shared__ char stage_all[WRITE ? kWavesPerBlock : 1][WRITE ? kRleMaxBytes : 1];
  char *stage = stage_all[WRITE ? threadIdx.x / kWave : 0];
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t u = (uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave; u < n; u += stride) {
    const uint64_t r = rle_row(s[u * kWave + lane], lane);
    // rows since the previous live row (or since the top): GenericRLE's eol_count
    const int prev = last_set(__ballot(r != 0) & below_lane(lane));
    const uint32_t eol = (uint32_t)(lane - (prev < 0 ? 0 : prev));
    const uint32_t mine = rle_row_tokens<false>(r, eol, nullptr);
    if constexpr (!WRITE) {
      const uint32_t total = wave_sum_u32(mine) + 1;  // + "!"
      if (lane == 0) len[u] = total;
    } else {
      const uint32_t at = wave_excl_scan(mine, lane);
      rle_row_tokens<true>(r, eol, stage + at);
      if (lane == kWave - 1) stage[at + mine] = '!';
      const uint32_t total = __shfl(at + mine, kWave - 1, kWave) + 1;
      char *base = text + offs[u];
      for (uint32_t i = lane; i < total; i += kWave) base[i] = stage[i];
    }
  }
}

// LifeState::Parse (GenericParse, Parsing.hpp:143-198) of text[offs[u],
// offs[u+1]), 64 bytes per step, one byte per lane:
//  * a line whose first byte is 'x' is dropped (:148-151); '\n' goes with it
//    (getline), '\r' and ' ' are skipped (:181-182);
//  * a decimal count accumulates across skipped bytes and lines (:164-166);
//  * '$' moves down count rows (0 -> 1), a count of 129 ends the parse
//    (:171-173); '!' ends it (:178-179);
//  * any other byte is a run of count cells (0 -> 1), live iff 'o' (:196).
// Per step: ballots give the line starts, kept bytes, digit and tag masks;
// each tag's count comes from the digit bit planes; wave scans give every
// tag's (x, y); every 'o' run ORs its cells into its row in LDS (one
// ds_or_b64 for all runs of the step), and the rows are turned into
// columns at the end.  status[u] bit 0: a live cell fell off the 64x64 board and was
// dropped (the reference writes out of bounds there); bit 1: stopped by a
// "$" count of 129.
__global__ __launch_bounds__(kBlock) void k_parse_rle(const char *__restrict__ text,
                                                      const uint64_t *__restrict__ offs,
                                                      uint64_t *__restrict__ out, uint8_t *__restrict__ status,
                                                      uint64_t n) {
  __shared__ uint64_t board[kWavesPerBlock][kWave];  // row y of this wave's pattern
  const int lane = threadIdx.x & (kWave - 1);
  uint64_t *rows = board[threadIdx.x / kWave];
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t u = (uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave; u < n; u += stride) {
    const uint64_t b = offs[u], e = offs[u + 1] > b ? offs[u + 1] : b;
    rows[lane] = 0;
    int64_t x = 0, y = 0;
    uint32_t cnt = 0, st = 0;
    bool line_start = true, header = false, done = false, off_board = false;
    for (uint64_t p0 = b; p0 < e && !done; p0 += kWave) {
      const uint64_t p = p0 + lane;
      const bool valid = p < e;
      const uint32_t c = valid ? (uint32_t)(uint8_t)text[p] : 0u;
      // header lines: first byte of my line
      const int nl_before = last_set(__ballot(valid && c == '\n') & below_lane(lane));
      const uint32_t first = __shfl(c, nl_before < 0 ? 0 : nl_before + 1, kWave);
      const bool hdr = nl_before >= 0 ? first == 'x' : (line_start ? first == 'x' : header);
      const bool kept = valid && c != '\n' && !hdr && c != '\r' && c != ' ';
      const bool dig = kept && c >= '0' && c <= '9';
      const bool tag = kept && !dig;
      const uint64_t D = __ballot(dig), T = __ballot(tag);
      const uint32_t dv = dig ? c - '0' : 0u;
      const uint64_t d0 = __ballot(dv & 1), d1 = __ballot(dv & 2), d2 = __ballot(dv & 4), d3 = __ballot(dv & 8);
      auto digits_value = [&](uint64_t m, uint32_t v) {  // digits in m, ascending, after v
        for (; m; m &= m - 1) {
          const int k = __builtin_ctzll(m);
          v = v * 10u + (uint32_t)(((d0 >> k) & 1) | ((d1 >> k) & 1) << 1 | ((d2 >> k) & 1) << 2 |
                                   ((d3 >> k) & 1) << 3);
        }
        return v;
      };
      auto after = [](int k) { return k < 0 ? ~0ull : ~((2ull << k) - 1); };
      // this tag's count: digits since the previous tag (or carried in)
      const int pt = last_set(T & below_lane(lane));
      uint32_t v = 0;
      if (tag) v = digits_value(D & below_lane(lane) & after(pt), pt < 0 ? cnt : 0u);
      const uint32_t cv = v == 0 ? 1u : v;
      const uint64_t S = __ballot(tag && (c == '!' || (c == '$' && cv == 129)));
      const uint64_t live_tags = S ? T & below_lane(__builtin_ctzll(S)) : T;
      const bool active = (live_tags >> lane) & 1;
      const bool dollar = active && c == '$';
      const bool cell = active && c != '$';
      const uint32_t dy = dollar ? cv : 0u, dx = cell ? cv : 0u;
      const uint32_t ey = wave_excl_scan(dy, lane), ex = wave_excl_scan(dx, lane);
      const uint64_t Dl = __ballot(dollar);
      const int ld = last_set(Dl & below_lane(lane));
      const uint32_t ex_ld = __shfl(ex, ld < 0 ? 0 : ld, kWave);
      const int64_t my_y = y + ey;
      const int64_t my_x = ld < 0 ? x + ex : (int64_t)(ex - ex_ld);
      if (cell && c == 'o') {  // each 'o' run ORs its cells into its row of the board
        if (my_y < 0 || my_y >= 64 || my_x < 0 || my_x + cv > 64) off_board = true;
        if (my_y >= 0 && my_y < 64 && my_x >= 0 && my_x < 64) {
          const uint64_t end = my_x + cv < 64 ? my_x + cv : 64;
          const uint64_t hi = end == 64 ? ~0ull : (1ull << end) - 1;
          __hip_atomic_fetch_or(&rows[my_y], hi & ~((1ull << my_x) - 1), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      // carry to the next 64 bytes
      const uint32_t ey_all = __shfl(ey + dy, kWave - 1, kWave), ex_all = __shfl(ex + dx, kWave - 1, kWave);
      const int lda = last_set(Dl);
      y += ey_all;
      x = lda < 0 ? x + ex_all : (int64_t)(ex_all - __shfl(ex, lda < 0 ? 0 : lda, kWave));
      if (S) {
        done = true;
        const int k = __builtin_ctzll(S);
        if (__shfl(c, k, kWave) == '$') st |= 2u;
      } else {
        const int lt = last_set(T);
        cnt = digits_value(D & after(lt), lt < 0 ? cnt : 0u);
      }
      line_start = __shfl(c, kWave - 1, kWave) == '\n';
      header = __shfl((uint32_t)hdr, kWave - 1, kWave) != 0;
    }
    // rows -> columns: lane x collects bit x of every row
    uint64_t word = 0;
#pragma unroll 8
    for (int r = 0; r < kWave; ++r) word |= ((rows[r] >> lane) & 1ull) << r;
    if (__ballot(off_board)) st |= 1u;
    out[u * kWave + lane] = word;
    if (lane == 0) status[u] = (uint8_t)st;
  }
}


// device buffers of one host-pointer RLE call, freed on every return path
struct DevBufs {
  std::vector<void *> p;
  template <class T>
  hipError_t get(T *&out, size_t bytes) {
    void *q = nullptr;
    const hipError_t e = hipMalloc(&q, bytes ? bytes : 1);
    if (e == hipSuccess) p.push_back(q);
    out = static_cast<T *>(q);
    return e;
  }
  ~DevBufs() {
    for (void *q : p) (void)hipFree(q);
  }
};
constexpr size_t kRleChunk = size_t(1) << 18;  // patterns per device pass

}  // namespace

extern "C" {

int lifeapi_rle_lengths_batch_dev(const uint64_t *d_states, uint32_t *d_len, size_t n, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_states || !d_len || !aligned8(d_states) || ((uintptr_t)d_len & 3u))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_rle_lengths_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(k_rle<false>, dim3(grid_for(n, cus, 8)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_states, d_len, nullptr, nullptr, (uint64_t)n);
  return launched("k_rle launch");
}

int lifeapi_rle_write_batch_dev(const uint64_t *d_states, const uint64_t *d_offsets, char *d_text,
                                size_t n, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_states || !d_offsets || !d_text || !aligned8(d_states) || !aligned8(d_offsets))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_rle_write_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  hipLaunchKernelGGL(k_rle<true>, dim3(grid_for(n, cus, 8)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_states, nullptr, d_offsets, d_text, (uint64_t)n);
  return launched("k_rle launch");
}

int lifeapi_parse_rle_batch_dev(const char *d_text, const uint64_t *d_offsets, size_t n, uint64_t *d_out,
                                uint8_t *d_status, void *stream) {
  if (n == 0) return LIFEAPI_OK;
  if (!d_text || !d_offsets || !d_out || !d_status || !aligned8(d_offsets) || !aligned8(d_out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_parse_rle_batch_dev%s");
  int cus = 0, rc = device_cus(cus);
  if (rc != LIFEAPI_OK) return rc;
  note_forward_write(d_out, (uint64_t)n * 512);
  hipLaunchKernelGGL(k_parse_rle, dim3(grid_for(n, cus, 8)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_text, d_offsets, d_out, d_status, (uint64_t)n);
  return launched("k_parse_rle launch");
}

int lifeapi_rle_batch(const uint64_t *states, size_t n, char *text, size_t text_cap, uint64_t *offsets,
                      int device) {
  if (!offsets) return fail(LIFEAPI_E_INVALID, "null offsets to lifeapi_rle_batch%s");
  offsets[0] = 0;
  if (n == 0) return LIFEAPI_OK;
  if (!states || !aligned8(states)) return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_rle_batch%s");
  const int dev = host_device(device);
  if (dev < 0) return dev;
  std::vector<uint32_t> len(n);
  const HostIO io[2] = {{states, nullptr, 512}, {nullptr, len.data(), 4}};
  int rc = host_chunked(dev, n, io, 2,
                        [](void *const *d, size_t m, hipStream_t s, const void *) {
                          return lifeapi_rle_lengths_batch_dev((const uint64_t *)d[0], (uint32_t *)d[1], m, s);
                        },
                        nullptr);
  if (rc != LIFEAPI_OK) return rc;
  for (size_t u = 0; u < n; ++u) offsets[u + 1] = offsets[u] + len[u];
  if (!text) return LIFEAPI_OK;  // size query
  if (text_cap < offsets[n]) return fail(LIFEAPI_E_INVALID, "text buffer smaller than offsets[n]%s");
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return fail_hip(e, "hipSetDevice");
  for (size_t c = 0; c < n; c += kRleChunk) {
    const size_t m = std::min(kRleChunk, n - c);
    const uint64_t t0 = offsets[c], tb = offsets[c + m] - t0;
    std::vector<uint64_t> rel(m);
    for (size_t u = 0; u < m; ++u) rel[u] = offsets[c + u] - t0;
    DevBufs bufs;
    uint64_t *ds = nullptr, *doff = nullptr;
    char *dt = nullptr;
    if ((e = bufs.get(ds, m * 512)) != hipSuccess || (e = bufs.get(doff, m * 8)) != hipSuccess ||
        (e = bufs.get(dt, tb)) != hipSuccess)
      return fail_hip(e, "hipMalloc(rle)");
    if ((e = hipMemcpy(ds, states + c * 64, m * 512, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(doff, rel.data(), m * 8, hipMemcpyHostToDevice)) != hipSuccess)
      return fail_hip(e, "hipMemcpy(rle in)");
    if ((rc = lifeapi_rle_write_batch_dev(ds, doff, dt, m, nullptr)) != LIFEAPI_OK) return rc;
    if ((e = hipMemcpy(text + t0, dt, tb, hipMemcpyDeviceToHost)) != hipSuccess)
      return fail_hip(e, "hipMemcpy(rle out)");
  }
  return LIFEAPI_OK;
}

int lifeapi_parse_rle_batch(const char *text, const uint64_t *offsets, size_t n, uint64_t *out,
                            uint8_t *status, int device) {
  if (n == 0) return LIFEAPI_OK;
  if (!text || !offsets || !out || !status || !aligned8(out))
    return fail(LIFEAPI_E_INVALID, "bad pointer to lifeapi_parse_rle_batch%s");
  for (size_t u = 0; u < n; ++u)
    if (offsets[u + 1] < offsets[u]) return fail(LIFEAPI_E_INVALID, "offsets must not decrease%s");
  const int dev = host_device(device);
  if (dev < 0) return dev;
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return fail_hip(e, "hipSetDevice");
  for (size_t c = 0; c < n; c += kRleChunk) {
    const size_t m = std::min(kRleChunk, n - c);
    const uint64_t t0 = offsets[c], tb = offsets[c + m] - t0;
    std::vector<uint64_t> rel(m + 1);
    for (size_t u = 0; u <= m; ++u) rel[u] = offsets[c + u] - t0;
    DevBufs bufs;
    uint64_t *doff = nullptr, *dout = nullptr;
    char *dt = nullptr;
    uint8_t *dst = nullptr;
    if ((e = bufs.get(dt, tb)) != hipSuccess || (e = bufs.get(doff, (m + 1) * 8)) != hipSuccess ||
        (e = bufs.get(dout, m * 512)) != hipSuccess || (e = bufs.get(dst, m)) != hipSuccess)
      return fail_hip(e, "hipMalloc(parse)");
    if ((e = hipMemcpy(dt, text + t0, tb, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(doff, rel.data(), (m + 1) * 8, hipMemcpyHostToDevice)) != hipSuccess)
      return fail_hip(e, "hipMemcpy(parse in)");
    int rc = lifeapi_parse_rle_batch_dev(dt, doff, m, dout, dst, nullptr);
    if (rc != LIFEAPI_OK) return rc;
    if ((e = hipMemcpy(out + c * 64, dout, m * 512, hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(status + c, dst, m, hipMemcpyDeviceToHost)) != hipSuccess)
      return fail_hip(e, "hipMemcpy(parse out)");
  }
  return LIFEAPI_OK;
}

}  // extern "C"
