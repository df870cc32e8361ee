// lifeapi/LifeState.hpp -- standalone, source-compatible subset of the
// reference's LifeState / LifeTarget (scorbiclife/LifeAPI, LifeAPI.hpp,
// LifeTarget.hpp) covering the Step() hot path, plus the batched GPU entry
// points in lifeapi/batch.hpp.
//
// Same layout (uint64_t state[64], aligned(64); word x = column x, bit y =
// row y: LifeAPI.hpp:39-40,131) and the same member names and semantics for
// the hot path, so loops written against the reference recompile against
// lifeapi::LifeState unchanged.  Single-universe Step() runs on the CPU (a
// ~50 ns operation cannot amortise a GPU launch); batches go to the GPU via
// lifeapi::StepBatch.  Code that keeps the reference's own LifeAPI.hpp can
// use lifeapi/batch.hpp directly on ::LifeState instead of this header.
#pragma once

#include <array>
#include <bit>
#include <cstdint>
#include <string>
#include <utility>

namespace lifeapi {

inline constexpr int N = 64;  // LifeAPI.hpp:12

constexpr unsigned torus_wrap(int x) { return unsigned(x) & (N - 1); }  // LifeAPI.hpp:14-16

enum class InitializedTag { UNINITIALIZED };  // LifeAPI.hpp:37

struct alignas(64) LifeState {
  uint64_t state[N];

  constexpr LifeState() : state{} {}
  explicit constexpr LifeState(InitializedTag) {}

  // ---- access (LifeAPI.hpp:131-146)
  void Set(unsigned x, unsigned y) { state[x] |= uint64_t(1) << y; }
  void Erase(unsigned x, unsigned y) { state[x] &= ~(uint64_t(1) << y); }
  void Set(unsigned x, unsigned y, bool v) { v ? Set(x, y) : Erase(x, y); }
  bool Get(unsigned x, unsigned y) const { return (state[x] >> y) & 1; }
  void SetSafe(int x, int y, bool v) { Set(torus_wrap(x), torus_wrap(y), v); }
  bool GetSafe(int x, int y) const { return Get(torus_wrap(x), torus_wrap(y)); }
  void Set(std::pair<int, int> c) { Set(c.first, c.second); }
  bool Get(std::pair<int, int> c) const { return Get(c.first, c.second); }
  constexpr uint64_t &operator[](unsigned i) { return state[i]; }
  constexpr uint64_t operator[](unsigned i) const { return state[i]; }

  static LifeState Cell(std::pair<int, int> c) {
    LifeState r;
    r.Set(c.first, c.second);
    return r;
  }

  // ---- value semantics (LifeAPI.hpp:213-275)
  bool operator==(const LifeState &o) const {
    uint64_t d = 0;
    for (int i = 0; i < N; ++i) d |= state[i] ^ o.state[i];
    return d == 0;
  }
  bool operator!=(const LifeState &o) const { return !(*this == o); }
#define LIFEAPI_BINOP(op)                                                   \
  LifeState operator op(const LifeState &o) const {                         \
    LifeState r(InitializedTag::UNINITIALIZED);                             \
    for (int i = 0; i < N; ++i) r.state[i] = state[i] op o.state[i];        \
    return r;                                                               \
  }                                                                         \
  LifeState &operator op##=(const LifeState &o) {                           \
    for (int i = 0; i < N; ++i) state[i] = state[i] op o.state[i];          \
    return *this;                                                           \
  }
  LIFEAPI_BINOP(&)
  LIFEAPI_BINOP(|)
  LIFEAPI_BINOP(^)
#undef LIFEAPI_BINOP
  LifeState operator~() const {
    LifeState r(InitializedTag::UNINITIALIZED);
    for (int i = 0; i < N; ++i) r.state[i] = ~state[i];
    return r;
  }

  // ---- queries (LifeAPI.hpp:281-298)
  bool IsEmpty() const {
    uint64_t a = 0;
    for (int i = 0; i < N; ++i) a |= state[i];
    return a == 0;
  }
  unsigned GetPop() const {
    unsigned p = 0;
    for (int i = 0; i < N; ++i) p += std::popcount(state[i]);
    return p;
  }
  bool Contains(const LifeState &pat) const {  // LifeAPI.hpp:388-397
    uint64_t d = 0;
    for (int i = 0; i < N; ++i) d |= (state[i] & pat[i]) ^ pat[i];
    return d == 0;
  }
  bool AreDisjoint(const LifeState &pat) const {  // LifeAPI.hpp:377-386
    uint64_t d = 0;
    for (int i = 0; i < N; ++i) d |= state[i] & pat[i];
    return d == 0;
  }
  // the offset forms (LifeAPI.hpp:399-421): target column i against state
  // column i + dx rotated right by dy
  bool Contains(const LifeState &pat, int dx, int dy) const {
    const int y = int(torus_wrap(dy));
    for (int i = 0; i < N; ++i)
      if ((std::rotr(state[torus_wrap(i + dx)], y) & pat[i]) != pat[i]) return false;
    return true;
  }
  bool AreDisjoint(const LifeState &pat, int dx, int dy) const {
    const int y = int(torus_wrap(dy));
    for (int i = 0; i < N; ++i)
      if ((std::rotr(state[torus_wrap(i + dx)], y) & pat[i]) != 0) return false;
    return true;
  }
  inline bool Contains(const struct LifeTarget &t) const;
  inline bool Contains(const struct LifeTarget &t, int dx, int dy) const;

  // ---- ZOI (LifeAPI.hpp:521-538): the 3x3 dilation on the torus, and the
  // cells next to the pattern but not in it
  LifeState ZOI() const {
    LifeState v(InitializedTag::UNINITIALIZED), r(InitializedTag::UNINITIALIZED);
    for (int i = 0; i < N; ++i) v.state[i] = state[i] | std::rotl(state[i], 1) | std::rotr(state[i], 1);
    for (int i = 0; i < N; ++i)
      r.state[i] = v.state[(i + N - 1) & (N - 1)] | v.state[i] | v.state[(i + 1) & (N - 1)];
    return r;
  }
  LifeState GetBoundary() const { return ZOI() & ~*this; }

  // ---- Move / Moved (LifeAPI.hpp:682-735): cell (x, y) -> (x + dx, y + dy) on the torus
  void Move(int dx, int dy) { *this = Moved(dx, dy); }
  void Move(std::pair<int, int> v) { Move(v.first, v.second); }
  LifeState Moved(int dx, int dy) const {
    LifeState r(InitializedTag::UNINITIALIZED);
    const int y = int(torus_wrap(dy));
    for (int i = 0; i < N; ++i) r.state[torus_wrap(i + dx)] = std::rotl(state[i], y);
    return r;
  }
  LifeState Moved(std::pair<int, int> v) const { return Moved(v.first, v.second); }

  // ---- bitsliced adders (LifeAPI.hpp:822-833)
  static void HalfAdd(uint64_t &out0, uint64_t &out1, uint64_t a, uint64_t b) {
    out0 = a ^ b;
    out1 = a & b;
  }
  static void FullAdd(uint64_t &out0, uint64_t &out1, uint64_t a, uint64_t b, uint64_t c) {
    const uint64_t h = a ^ b;
    out0 = h ^ c;
    out1 = (a & b) | (c & h);
  }

  // ---- stepping (LifeAPI.hpp:866-907,1196-1254), CPU, single universe
  void CountRows(LifeState &__restrict__ bit0, LifeState &__restrict__ bit1) const {
    for (int i = 0; i < N; ++i) {
      const uint64_t a = state[i], l = std::rotl(a, 1), r = std::rotr(a, 1);
      bit0.state[i] = l ^ r ^ a;
      bit1.state[i] = ((l ^ r) & a) | (l & r);
    }
  }
  // Rokicki form of the B3/S23 rule (LifeAPI.hpp:837-848): the centre column
  // plus the 2-bit vertical sums of the columns above (u) and below (b)
  static uint64_t Rokicki(uint64_t a, uint64_t u0, uint64_t u1, uint64_t b0, uint64_t b1) {
    const uint64_t aw = std::rotl(a, 1), ae = std::rotr(a, 1);
    const uint64_t s0 = aw ^ ae, s1 = aw & ae;
    const uint64_t ts0 = b0 ^ u0;
    const uint64_t ts1 = (b0 & u0) | (ts0 & s0);
    return (b1 ^ u1 ^ ts1 ^ s1) & ((b1 | u1) ^ (ts1 | s1)) & ((ts0 ^ s0) | a);
  }
  // Step() (LifeAPI.hpp:1196-1216).  The torus wrap is peeled out of the
  // loop (columns 0 and 63), so the 62 interior columns are straight-line
  // code the compiler unrolls and vectorises like the reference's
  // `unroll(full)` loop.
  void Step() {
    LifeState c0(InitializedTag::UNINITIALIZED), c1(InitializedTag::UNINITIALIZED);
    CountRows(c0, c1);
    state[0] = Rokicki(state[0], c0.state[N - 1], c1.state[N - 1], c0.state[1], c1.state[1]);
#if defined(__clang__)
#pragma clang loop unroll(full)
#elif defined(__GNUC__)
#pragma GCC unroll 64
#endif
    for (int i = 1; i < N - 1; ++i)
      state[i] = Rokicki(state[i], c0.state[i - 1], c1.state[i - 1], c0.state[i + 1], c1.state[i + 1]);
    state[N - 1] = Rokicki(state[N - 1], c0.state[N - 2], c1.state[N - 2], c0.state[0], c1.state[0]);
  }
  void StepAlt() {
    LifeState c0(InitializedTag::UNINITIALIZED), c1(InitializedTag::UNINITIALIZED);
    CountRows(c0, c1);
    for (int i = 0; i < N; ++i) {
      const int u = (i + N - 1) & (N - 1), b = (i + 1) & (N - 1);
      uint64_t fs, fc, cs, cc;
      FullAdd(fs, fc, c0[u], c0[i], c0[b]);
      FullAdd(cs, cc, c1[u], c1[i], c1[b]);
      cc ^= fc & cs;
      state[i] = (fs ^ cc) & (fc ^ cs ^ cc) & (state[i] | fs);
    }
  }
  void Step(unsigned n) {
    for (unsigned g = 0; g < n; ++g) Step();
  }
  LifeState Stepped() const {
    LifeState c = *this;
    c.Step();
    return c;
  }
  LifeState Stepped(unsigned n) const {
    LifeState c = *this;
    c.Step(n);
    return c;
  }

  // ---- parsing (Parsing.hpp:143-198 semantics: header lines starting with
  // 'x' skipped; bare '$' = 1; non-'o' cell chars are dead; no wrapping)
  static LifeState Parse(const std::string &rle) {
    LifeState r;
    int cnt = 0, x = 0, y = 0;
    bool at_line_start = true, skip_line = false;
    for (char ch : rle) {
      if (at_line_start) {
        skip_line = ch == 'x';
        at_line_start = false;
      }
      if (ch == '\n') {
        at_line_start = true;
        continue;
      }
      if (skip_line) continue;
      if (ch >= '0' && ch <= '9') {
        cnt = cnt * 10 + (ch - '0');
      } else if (ch == '$') {
        if (cnt == 0) cnt = 1;
        if (cnt == 129) return r;
        y += cnt;
        x = 0;
        cnt = 0;
      } else if (ch == '!') {
        break;
      } else if (ch == '\r' || ch == ' ') {
        continue;
      } else {
        if (cnt == 0) cnt = 1;
        for (int j = 0; j < cnt; ++j, ++x)
          if (ch == 'o' && x >= 0 && x < N && y >= 0 && y < N) r.Set(x, y);
        cnt = 0;
      }
    }
    return r;
  }

  // LifeState::RLE() (Parsing.hpp:8-63,200-204): printed from x = y = 32 like
  // the reference, so Parse(s.RLE()) is s moved by (32, 32)
  std::string RLE() const {
    std::string out;
    auto count = [&](unsigned c) {
      if (c > 1) out += std::to_string(c);
    };
    unsigned rows = 0;
    for (int j = 0; j < N; ++j) {
      const int y = (j + 32) & (N - 1);
      bool last = Get(32, y);
      unsigned run = 0;
      for (int i = 0; i < N; ++i) {
        const bool v = Get((i + 32) & (N - 1), y);
        if (v && rows) {
          count(rows);
          out += '$';
          rows = 0;
        }
        if (v != last) {
          count(run);
          out += last ? 'o' : 'b';
          run = 0;
        }
        ++run;
        last = v;
      }
      if (last) {
        count(run);
        out += 'o';
      }
      ++rows;
    }
    return out + '!';
  }

  // Seeded counterpart of RandomState() (LifeAPI.hpp:18-23,63-69): each column
  // uniform on [2^61, 2^62) (row 61 on, rows 62-63 off), from a splitmix64
  // stream instead of the reference's random_device-seeded mt19937_64.
  static LifeState RandomState(uint64_t &seed) {
    LifeState r;
    for (int i = 0; i < N; ++i) {
      uint64_t z = (seed += 0x9E3779B97F4A7C15ULL);
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
      z ^= z >> 31;
      r.state[i] = (z & ((uint64_t(1) << 61) - 1)) | (uint64_t(1) << 61);
    }
    return r;
  }
};

static_assert(sizeof(LifeState) == 512 && alignof(LifeState) == 64, "LifeAPI.hpp:39-40 layout");

// LifeTarget.hpp:5-36 (the search-loop subset; no Transform)
struct LifeTarget {
  LifeState wanted;
  LifeState unwanted;
  LifeTarget() = default;
  // the pattern and its boundary: the cells around it must be dead (:10-13)
  explicit LifeTarget(const LifeState &state) : wanted(state), unwanted(state.GetBoundary()) {}
  LifeTarget(const LifeState &w, const LifeState &u) : wanted(w), unwanted(u) {}
  LifeTarget Moved(std::pair<int, int> v) const {  // :33-35
    return LifeTarget(wanted.Moved(v), unwanted.Moved(v));
  }
};

// LifeTarget.hpp:44-51
inline bool LifeState::Contains(const LifeTarget &t) const {
  uint64_t d = 0;
  for (int i = 0; i < N; ++i) d |= (state[i] ^ t.wanted[i]) & (t.wanted[i] | t.unwanted[i]);
  return d == 0;
}
// LifeTarget.hpp:38-42
inline bool LifeState::Contains(const LifeTarget &t, int dx, int dy) const {
  return Contains(t.wanted, dx, dy) && AreDisjoint(t.unwanted, dx, dy);
}

// NeighbourCount.hpp:7-102 (hot-path subset): inclusive 3x3 count 0..9 as
// four bit planes, same member order as the reference.
struct NeighbourCount {
  LifeState bit3, bit2, bit1, bit0;

  NeighbourCount() = default;
  explicit NeighbourCount(const LifeState &s) {
    LifeState c0(InitializedTag::UNINITIALIZED), c1(InitializedTag::UNINITIALIZED);
    s.CountRows(c0, c1);
    for (int i = 0; i < N; ++i) {
      const int u = (i + N - 1) & (N - 1), d = (i + 1) & (N - 1);
      uint64_t fs, fc, cs, cc;
      LifeState::FullAdd(fs, fc, c0[u], c0[i], c0[d]);
      LifeState::FullAdd(cs, cc, c1[u], c1[i], c1[d]);
      bit0[i] = fs;
      bit1[i] = fc ^ cs;
      bit2[i] = cc ^ (fc & cs);
      bit3[i] = cc & fc & cs;
    }
  }
  LifeState WithExactly(unsigned n) const {
    LifeState r = ~LifeState();
    r &= (n & 1) ? bit0 : ~bit0;
    r &= (n & 2) ? bit1 : ~bit1;
    r &= (n & 4) ? bit2 : ~bit2;
    r &= (n & 8) ? bit3 : ~bit3;
    return r;
  }
};

// LifeWeld.hpp:18-186 (hot-path subset): a state plus a frozen 3-bit
// neighbour count added when stepping.
struct LifeWeld {
  LifeState state, frozen2, frozen1, frozen0;

  bool operator==(const LifeWeld &o) const {
    return state == o.state && frozen2 == o.frozen2 && frozen1 == o.frozen1 && frozen0 == o.frozen0;
  }
  void Step() {  // LifeWeld.hpp:169-186
    const NeighbourCount c(state);
    for (int i = 0; i < N; ++i) {
      uint64_t s0, k0, s1, k1, s2, k2;
      LifeState::HalfAdd(s0, k0, c.bit0[i], frozen0[i]);
      LifeState::FullAdd(s1, k1, c.bit1[i], frozen1[i], k0);
      LifeState::FullAdd(s2, k2, c.bit2[i], frozen2[i], k1);
      state[i] = (s0 ^ s2) & (s1 ^ s2) & (state[i] | s0);
    }
  }
};

// LifeStable.hpp:41-53: the ten planes of the stable-search state (options
// stored as "1 = ruled out").  Propagation runs on the GPU:
// lifeapi::PropagateStepBatch / PropagateBatch in lifeapi/batch.hpp.
struct LifeStable {
  LifeState state, unknown;
  LifeState live2, live3;
  LifeState dead0, dead1, dead2, dead4, dead5, dead6;
};

}  // namespace lifeapi

#include "batch.hpp"
