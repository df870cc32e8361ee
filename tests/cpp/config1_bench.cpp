// config1_bench.cpp -- BASELINE.json configs[0]: one 64x64 universe, the
// R-pentomino, 1103 generations of single-universe Step() on the CPU, timed
// for the drop-in facade (lifeapi::LifeState::Step, include/lifeapi/
// LifeState.hpp) and for the REFERENCE's own ::LifeState::Step()
// (LifeAPI.hpp:1196-1216) in the same binary, same compiler, same flags,
// 1 thread.  The pattern is the StepAltTest path's single-universe Step()
// (tests/StepAltTest.cpp:5-13) on the R-pentomino of SURVEY.md 8(c).
//
// Built by oracle/Makefile (target ref, into oracle/_ref/) where
// /root/reference exists; the binary travels to the GPU box prebuilt and is
// run by bench.py's CPU-baseline leg.  Prints one JSON line.
#include <lifeapi/LifeState.hpp>  // first: ref_prelude.hpp defines `constexpr` away

#include "ref_prelude.hpp"

#include "LifeAPI.hpp"
#include "Parsing.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>

namespace {

constexpr unsigned kGens = 1103;

template <class S>
double best_ns_per_gen(const S &start, int reps, S &final_state) {
  double best = 1e30;
  for (int r = 0; r < reps; ++r) {
    S s = start;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned g = 0; g < kGens; ++g) {
      s.Step();
      asm volatile("" : : "r"(&s) : "memory");  // keep every generation
    }
    const auto t1 = std::chrono::steady_clock::now();
    const double ns = std::chrono::duration<double, std::nano>(t1 - t0).count() / kGens;
    if (ns < best) best = ns;
    final_state = s;
  }
  return best;
}

}  // namespace

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;

  ::LifeState ref = ::LifeState::Parse("b2o$2o$bo!");
  lifeapi::LifeState fac = lifeapi::LifeState::Parse("b2o$2o$bo!");
  bool same_input = true;
  for (int i = 0; i < 64; ++i) same_input &= ref.state[i] == fac.state[i];

  // interleave the two so clock and cache state drift hit both alike
  double ref_ns = 1e30, fac_ns = 1e30;
  ::LifeState ref_out;
  lifeapi::LifeState fac_out;
  for (int k = 0; k < rounds; ++k) {
    const double r = best_ns_per_gen(ref, reps, ref_out);
    const double f = best_ns_per_gen(fac, reps, fac_out);
    if (r < ref_ns) ref_ns = r;
    if (f < fac_ns) fac_ns = f;
  }
  bool same_output = true;
  for (int i = 0; i < 64; ++i) same_output &= ref_out.state[i] == fac_out.state[i];
  const unsigned pop = fac_out.GetPop();

  std::printf("{\"workload\": \"config1: R-pentomino, %u generations of single-universe Step() on the CPU, "
              "1 thread\", \"reference_ns_per_gen\": %.2f, \"facade_ns_per_gen\": %.2f, "
              "\"facade_over_reference\": %.4f, \"reference_gens_per_s\": %.4g, \"facade_gens_per_s\": %.4g, "
              "\"pop_final\": %u, \"bit_exact\": %s, \"reps\": %d, \"rounds\": %d, "
              "\"timing\": \"best of reps x rounds runs of 1103 gens, interleaved\"}\n",
              kGens, ref_ns, fac_ns, fac_ns / ref_ns, 1e9 / ref_ns, 1e9 / fac_ns, pop,
              (same_input && same_output && pop == 113) ? "true" : "false", reps, rounds);
  return (same_input && same_output && pop == 113) ? 0 : 1;
}
