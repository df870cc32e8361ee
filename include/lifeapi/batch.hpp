// lifeapi/batch.hpp -- batched GPU Step() for any LifeState-layout type.
//
// Works on the reference's own ::LifeState (LifeAPI.hpp:39-40: uint64_t
// state[64], aligned(64), trivially copyable) as well as lifeapi::LifeState:
// an existing search loop keeps #include "LifeAPI.hpp" and adds
//
//     #include <lifeapi/batch.hpp>
//     std::vector<LifeState> candidates = ...;
//     lifeapi::StepBatch(std::span(candidates), 4);   // == c.Step(4) for each c
//
// Semantics mirror LifeState::Step(unsigned) / Stepped(unsigned)
// (LifeAPI.hpp:877-886) element-wise.  The reference's Step() cannot fail;
// a GPU call can, so failures throw lifeapi::Error (code = the C ABI's
// return value, see lifeapi_hip.h).  Link with -llifeapi_hip.
#pragma once

#include <bit>
#include <cstdint>
#include <span>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "../lifeapi_hip.h"

namespace lifeapi {

template <class S>
concept LifeStateLayout = sizeof(S) == 64 * sizeof(uint64_t) && alignof(S) >= alignof(uint64_t) &&
                          std::is_trivially_copyable_v<S> && std::is_standard_layout_v<S>;

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &what) : std::runtime_error(what), code(c) {}
};

inline void check(int rc) {
  if (rc != LIFEAPI_OK) throw Error(rc, std::string("lifeapi: ") + lifeapi_last_error());
}

inline const uint64_t *words(const void *p) { return static_cast<const uint64_t *>(p); }
inline uint64_t *words(void *p) { return static_cast<uint64_t *>(p); }

// In place: states[i].Step(generations) for every i.  device = -1 shards the
// batch over every visible GPU.
template <LifeStateLayout S>
void StepBatch(std::span<S> states, unsigned generations = 1, int device = 0) {
  check(lifeapi_step_batch(words(states.data()), words(states.data()), states.size(), generations,
                           device));
}

// out[i] = in[i].Stepped(generations)
template <LifeStateLayout S>
void SteppedBatch(std::span<const S> in, std::span<S> out, unsigned generations = 1,
                  int device = 0) {
  if (out.size() != in.size()) throw Error(LIFEAPI_E_INVALID, "lifeapi: size mismatch");
  check(lifeapi_step_batch(words(in.data()), words(out.data()), in.size(), generations, device));
}

// pops[i] = states[i].GetPop()
template <LifeStateLayout S>
std::vector<uint32_t> GetPopBatch(std::span<const S> states, int device = 0) {
  std::vector<uint32_t> pops(states.size());
  check(lifeapi_pop_batch(words(states.data()), pops.data(), states.size(), device));
  return pops;
}

// ---- the other per-generation kernels, on the reference's own types ----
//
// Each concept pins the reference struct's byte layout: N LifeStates in
// member order, nothing else.
template <class T, size_t Planes>
concept PlaneLayout = sizeof(T) == Planes * 64 * sizeof(uint64_t) && std::is_trivially_copyable_v<T> &&
                      std::is_standard_layout_v<T>;
// LifeWeld {state, frozen2, frozen1, frozen0}           LifeWeld.hpp:18-20
template <class T> concept LifeWeldLayout = PlaneLayout<T, 4>;
// LifeStable {state, unknown, live2 .. dead6}            LifeStable.hpp:41-53
template <class T> concept LifeStableLayout = PlaneLayout<T, 10>;
// NeighbourCount {bit3, bit2, bit1, bit0}                NeighbourCount.hpp:7-11
template <class T> concept NeighbourCountLayout = PlaneLayout<T, 4>;
// LifeTarget {wanted, unwanted}                          LifeTarget.hpp:5-7
template <class T> concept LifeTargetLayout = PlaneLayout<T, 2>;

// welds[i].Step() `generations` times (LifeWeld.hpp:169-186)
template <LifeWeldLayout W>
void WeldStepBatch(std::span<W> welds, unsigned generations = 1, int device = 0) {
  check(lifeapi_weld_step_batch(words(welds.data()), welds.size(), generations, device));
}

// LifeStable::PropagateResult (LifeStable.hpp:123-126)
struct PropagateResult {
  bool consistent;
  bool changed;
};

namespace detail {
template <LifeStableLayout S>
std::vector<PropagateResult> stable_pass(std::span<S> s, int pass, unsigned max_iters, int device) {
  std::vector<uint8_t> f(s.size());
  check(lifeapi_stable_pass_batch(words(s.data()), f.data(), s.size(), pass, max_iters, device));
  std::vector<PropagateResult> r(s.size());
  for (size_t i = 0; i < s.size(); ++i) r[i] = {(f[i] & 1) != 0, (f[i] & 2) != 0};
  return r;
}
}  // namespace detail

// s[i].PropagateStep() / s[i].Propagate() (LifeStable.hpp:695-729), in place
template <LifeStableLayout S>
std::vector<PropagateResult> PropagateStepBatch(std::span<S> s, int device = 0) {
  return detail::stable_pass(s, 3, 0, device);
}
template <LifeStableLayout S>
std::vector<PropagateResult> PropagateBatch(std::span<S> s, int device = 0) {
  return detail::stable_pass(s, 4, 0, device);
}
// s[i].StabiliseOptions() (LifeStable.hpp:677-693), in place
template <LifeStableLayout S>
std::vector<PropagateResult> StabiliseOptionsBatch(std::span<S> s, int device = 0) {
  return detail::stable_pass(s, 5, 0, device);
}

// out[i] = s[i].Vulnerable()  (LifeStable.hpp:366-412)
template <LifeStableLayout S, LifeStateLayout L>
void VulnerableBatch(std::span<const S> s, std::span<L> out, int device = 0) {
  if (out.size() != s.size()) throw Error(LIFEAPI_E_INVALID, "lifeapi: size mismatch");
  check(lifeapi_stable_vulnerable_batch(words(s.data()), words(out.data()), s.size(), device));
}

// out[i] = NeighbourCount(in[i])  (NeighbourCount.hpp:40-70)
template <LifeStateLayout S, NeighbourCountLayout C>
void NeighbourCountBatch(std::span<const S> in, std::span<C> out, int device = 0) {
  if (out.size() != in.size()) throw Error(LIFEAPI_E_INVALID, "lifeapi: size mismatch");
  check(lifeapi_neighbour_count_batch(words(in.data()), words(out.data()), in.size(), device));
}

// r[i] = in[i].Contains(target)  (LifeTarget.hpp:44-51)
template <LifeStateLayout S, LifeTargetLayout T>
std::vector<uint8_t> ContainsBatch(std::span<const S> in, const T &target, int device = 0) {
  std::vector<uint8_t> r(in.size());
  const uint64_t *t = words(&target);
  check(lifeapi_contains_batch(words(in.data()), t, t + 64, r.data(), in.size(), device));
  return r;
}

// The target as the offset forms of the reference test it:
//     s.Contains(target, dx, dy) = s.Contains(target.wanted, dx, dy) && s.AreDisjoint(target.unwanted, dx, dy)
// (LifeTarget.hpp:38-42) reads s at column i+dx rotated right by dy against
// target column i (LifeAPI.hpp:399-421): on the torus that is the unshifted
// test against the target Moved(dx, dy) (LifeAPI.hpp:682-696).  Returns false
// when some cell is both wanted and unwanted: no state passes the offset form
// then, where the unshifted Contains(target) asks such a cell to be alive.
namespace detail {
inline bool moved_target(const uint64_t *t, int dx, int dy, uint64_t *out) {
  const unsigned x = (unsigned)dx & 63u, y = (unsigned)dy & 63u;
  uint64_t clash = 0;
  for (unsigned i = 0; i < 64; ++i) {
    clash |= t[i] & t[64 + i];
    out[(i + x) & 63u] = std::rotl(t[i], (int)y);
    out[64 + ((i + x) & 63u)] = std::rotl(t[64 + i], (int)y);
  }
  return clash == 0;
}
}  // namespace detail

// r[i] = in[i].Contains(target, dx, dy)  (LifeTarget.hpp:38-42)
template <LifeStateLayout S, LifeTargetLayout T>
std::vector<uint8_t> ContainsBatch(std::span<const S> in, const T &target, int dx, int dy, int device = 0) {
  uint64_t t[128];
  if (!detail::moved_target(words(&target), dx, dy, t)) return std::vector<uint8_t>(in.size(), 0);
  std::vector<uint8_t> r(in.size());
  check(lifeapi_contains_batch(words(in.data()), t, t + 64, r.data(), in.size(), device));
  return r;
}

// The pattern tests (LifeAPI.hpp:377-421) are targets with one plane empty:
//     s.Contains(pat)          == s.Contains(LifeTarget{pat, {}})
//     s.AreDisjoint(pat)       == s.Contains(LifeTarget{{}, pat})
// and their (dx, dy) forms the same against pat Moved(dx, dy).  All run the
// batched Contains, which reads only the columns the pattern occupies.
namespace detail {
template <LifeStateLayout S>
std::vector<uint8_t> pattern_batch(std::span<const S> in, const uint64_t *pat, bool disjoint, int dx, int dy,
                                   int device) {
  uint64_t t[128] = {};
  const unsigned x = (unsigned)dx & 63u, y = (unsigned)dy & 63u;
  uint64_t *plane = t + (disjoint ? 64 : 0);
  for (unsigned i = 0; i < 64; ++i) plane[(i + x) & 63u] = std::rotl(pat[i], (int)y);
  std::vector<uint8_t> r(in.size());
  check(lifeapi_contains_batch(words(in.data()), t, t + 64, r.data(), in.size(), device));
  return r;
}
}  // namespace detail

// r[i] = in[i].Contains(pat)  (LifeAPI.hpp:388-397)
template <LifeStateLayout S, LifeStateLayout P>
std::vector<uint8_t> ContainsBatch(std::span<const S> in, const P &pat, int device = 0) {
  return detail::pattern_batch(in, words(&pat), false, 0, 0, device);
}
// r[i] = in[i].Contains(pat, dx, dy)  (LifeAPI.hpp:399-409)
template <LifeStateLayout S, LifeStateLayout P>
std::vector<uint8_t> ContainsBatch(std::span<const S> in, const P &pat, int dx, int dy, int device = 0) {
  return detail::pattern_batch(in, words(&pat), false, dx, dy, device);
}
// r[i] = in[i].AreDisjoint(pat)  (LifeAPI.hpp:377-386)
template <LifeStateLayout S, LifeStateLayout P>
std::vector<uint8_t> AreDisjointBatch(std::span<const S> in, const P &pat, int device = 0) {
  return detail::pattern_batch(in, words(&pat), true, 0, 0, device);
}
// r[i] = in[i].AreDisjoint(pat, dx, dy)  (LifeAPI.hpp:411-421)
template <LifeStateLayout S, LifeStateLayout P>
std::vector<uint8_t> AreDisjointBatch(std::span<const S> in, const P &pat, int dx, int dy, int device = 0) {
  return detail::pattern_batch(in, words(&pat), true, dx, dy, device);
}

// The search-loop idiom over a batch, in place (LifeAPI.hpp:1196-1216,
// LifeTarget.hpp:44-51):
//     for (unsigned g = 1; g <= gens; ++g) { s.Step(); if (!first && s.Contains(target)) first = g; }
// returns first (0 = never) per state; the states end Stepped(gens).
template <LifeStateLayout S, LifeTargetLayout T>
std::vector<uint32_t> StepContainsBatch(std::span<S> states, const T &target, unsigned gens, int device = 0) {
  std::vector<uint32_t> first(states.size());
  const uint64_t *t = words(&target);
  check(lifeapi_step_contains_batch(words(states.data()), words(states.data()), t, t + 64, first.data(),
                                    states.size(), gens, device));
  return first;
}

// The search loop with the offset test s.Contains(target, dx, dy)
// (LifeTarget.hpp:38-42) in place of s.Contains(target).
template <LifeStateLayout S, LifeTargetLayout T>
std::vector<uint32_t> StepContainsBatch(std::span<S> states, const T &target, int dx, int dy, unsigned gens,
                                        int device = 0) {
  uint64_t t[128];
  std::vector<uint32_t> first(states.size());
  if (!detail::moved_target(words(&target), dx, dy, t)) {  // never contained: step only
    check(lifeapi_step_batch(words(states.data()), words(states.data()), states.size(), gens, device));
    return first;
  }
  check(lifeapi_step_contains_batch(words(states.data()), words(states.data()), t, t + 64, first.data(),
                                    states.size(), gens, device));
  return first;
}

// LifeState::Parse of every string (Parsing.hpp:143-198).  status (optional)
// gets lifeapi_parse_rle_batch's per-pattern bits: 1 = a live cell off the
// 64x64 board was dropped (the reference writes out of bounds there), 2 =
// stopped at a "$" count of 129.
template <LifeStateLayout S>
std::vector<S> ParseBatch(std::span<const std::string> rles, std::vector<uint8_t> *status = nullptr,
                          int device = 0) {
  std::vector<uint64_t> offs(rles.size() + 1, 0);
  std::string blob;
  for (size_t i = 0; i < rles.size(); ++i) {
    blob += rles[i];
    offs[i + 1] = blob.size();
  }
  std::vector<S> out(rles.size());
  std::vector<uint8_t> st(rles.size());
  check(lifeapi_parse_rle_batch(blob.c_str(), offs.data(), rles.size(), words(out.data()), st.data(),
                                device));
  if (status) *status = std::move(st);
  return out;
}

// s.RLE() for every state (Parsing.hpp:8-63,200-204)
template <LifeStateLayout S>
std::vector<std::string> RLEBatch(std::span<const S> states, int device = 0) {
  std::vector<uint64_t> offs(states.size() + 1, 0);
  check(lifeapi_rle_batch(words(states.data()), states.size(), nullptr, 0, offs.data(), device));
  std::string text(offs.back(), '\0');
  check(lifeapi_rle_batch(words(states.data()), states.size(), text.data(), text.size(), offs.data(),
                          device));
  std::vector<std::string> out(states.size());
  for (size_t i = 0; i < states.size(); ++i) out[i] = text.substr(offs[i], offs[i + 1] - offs[i]);
  return out;
}

inline int DeviceCount() { return lifeapi_device_count(); }

// Page-locks a caller-owned array for its lifetime (lifeapi_host_register).
// Calls moving 8 MiB or more pin pageable arrays themselves; a HostPin holds
// the pin across the calls of a search loop and covers smaller batches.
class HostPin {
 public:
  HostPin(void *p, size_t bytes) : p_(p) { check(lifeapi_host_register(p, bytes)); }
  template <class T>
  explicit HostPin(std::span<T> s) : HostPin(static_cast<void *>(s.data()), s.size_bytes()) {}
  HostPin(const HostPin &) = delete;
  HostPin &operator=(const HostPin &) = delete;
  ~HostPin() { (void)lifeapi_host_unregister(p_); }

 private:
  void *p_;
};

}  // namespace lifeapi
