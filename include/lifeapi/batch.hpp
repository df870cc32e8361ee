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

inline int DeviceCount() { return lifeapi_device_count(); }

}  // namespace lifeapi
