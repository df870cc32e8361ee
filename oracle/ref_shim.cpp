// ref_shim.cpp -- extern "C" entry points around the REFERENCE's own code.
//
// TEST INFRASTRUCTURE ONLY.  Compiled by oracle/Makefile (target `ref`)
// directly against the headers where they lie under /root/reference; the
// result goes to oracle/_ref/ (git-ignored).  Used to (1) pin the C
// restatement in lifeapi_oracle.c, (2) generate tests/golden/ fixtures, and
// (3) time the reference's CPU Step() as bench.py's cpu_baseline
// ("kind": "reference").  Nothing here is shipped in the product.
#include "LifeAPI.hpp"
#include "NeighbourCount.hpp"
#include "LifeTarget.hpp"
#include "Parsing.hpp"

static_assert(sizeof(LifeState) == 512 && alignof(LifeState) == 64,
              "LifeState layout (LifeAPI.hpp:39-40)");

static inline LifeState load(const uint64_t *p) {
  LifeState s;
  std::memcpy(s.state, p, sizeof s.state);
  return s;
}
static inline void store(const LifeState &s, uint64_t *p) {
  std::memcpy(p, s.state, sizeof s.state);
}

extern "C" {

// LifeState::Step()  LifeAPI.hpp:1196-1216
void ref_step(uint64_t *s) { LifeState t = load(s); t.Step(); store(t, s); }
// LifeState::StepAlt()  LifeAPI.hpp:1218-1254
void ref_step_alt(uint64_t *s) { LifeState t = load(s); t.StepAlt(); store(t, s); }
// NeighbourCount(state).WithExactly(3) | (state & WithExactly(4))  NeighbourCount.hpp:40-102
void ref_step_nc(uint64_t *s) {
  LifeState t = load(s);
  NeighbourCount nc(t);
  LifeState next = nc.WithExactly(3) | (t & nc.WithExactly(4));
  store(next, s);
}
// LifeState::Step(unsigned)  LifeAPI.hpp:877-881
void ref_step_n(uint64_t *s, unsigned gens) { LifeState t = load(s); t.Step(gens); store(t, s); }

// LifeState::CountNeighbourhood  LifeAPI.hpp:909-952
void ref_count_neighbourhood(const uint64_t *s, uint64_t *b3, uint64_t *b2, uint64_t *b1, uint64_t *b0) {
  LifeState t = load(s), o3, o2, o1, o0;
  t.CountNeighbourhood(o3, o2, o1, o0);
  store(o3, b3); store(o2, b2); store(o1, b1); store(o0, b0);
}
// NeighbourCount ctor  NeighbourCount.hpp:40-70
void ref_neighbour_count(const uint64_t *s, uint64_t *b3, uint64_t *b2, uint64_t *b1, uint64_t *b0) {
  NeighbourCount nc(load(s));
  store(nc.bit3, b3); store(nc.bit2, b2); store(nc.bit1, b1); store(nc.bit0, b0);
}
// LifeState::GetPop  LifeAPI.hpp:290-298
unsigned ref_pop(const uint64_t *s) { return load(s).GetPop(); }
// LifeState::Contains(const LifeTarget&)  LifeTarget.hpp:44-51
int ref_contains_target(const uint64_t *s, const uint64_t *wanted, const uint64_t *unwanted) {
  LifeTarget t(load(wanted), load(unwanted));
  return load(s).Contains(t) ? 1 : 0;
}
// LifeState::Parse  Parsing.hpp:192-198
void ref_parse(const char *rle, uint64_t *out) { store(LifeState::Parse(std::string(rle)), out); }
// LifeState::RandomState  LifeAPI.hpp:63-69 (non-deterministic, random_device seeded)
void ref_random_state(uint64_t *out) { store(LifeState::RandomState(), out); }

// Batched Stepped(gens) (LifeAPI.hpp:882-886) over independent universes, one
// contiguous slice per std::thread: the reference algorithm on host cores.
void ref_step_batch(const uint64_t *in, uint64_t *out, size_t n, unsigned gens, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  auto work = [=](size_t lo, size_t hi) {
    for (size_t u = lo; u < hi; ++u) {
      LifeState t = load(in + u * 64);
      t.Step(gens);
      store(t, out + u * 64);
    }
  };
  if (nthreads == 1) { work(0, n); return; }
  std::vector<std::thread> pool;
  for (int k = 0; k < nthreads; ++k)
    pool.emplace_back(work, n * k / nthreads, n * (k + 1) / nthreads);
  for (auto &th : pool) th.join();
}

}  // extern "C"
