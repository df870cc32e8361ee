// ref_shim.cpp -- extern "C" entry points around the REFERENCE's own code.
//
// TEST INFRASTRUCTURE ONLY.  Compiled by oracle/Makefile (target `ref`)
// directly against the headers where they lie under /root/reference; the
// result goes to oracle/_ref/ (git-ignored).  Used to (1) pin the C
// restatement in lifeapi_oracle.c, (2) generate tests/golden/ fixtures, and
// (3) time the reference's CPU Step() as bench.py's cpu_baseline
// ("kind": "reference").  Nothing here is shipped in the product.
#include <cstring>
#include <thread>
#include <vector>

#include "LifeAPI.hpp"
#include "NeighbourCount.hpp"
#include "LifeTarget.hpp"
#include "Parsing.hpp"
#include "LifeWeld.hpp"

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
// LifeState::InteractionCountsAndNext  LifeAPI.hpp:997-1040 (and
// InteractionCounts :956-993, which must agree on the first three planes)
void ref_interaction_counts(const uint64_t *s, uint64_t *o1, uint64_t *o2, uint64_t *om, uint64_t *nx) {
  LifeState t = load(s), a1, a2, am, an, b1, b2, bm;
  t.InteractionCountsAndNext(a1, a2, am, an);
  t.InteractionCounts(b1, b2, bm);
  if (!(a1 == b1 && a2 == b2 && am == bm)) std::abort();
  store(a1, o1); store(a2, o2); store(am, om); store(an, nx);
}
// LifeWeld::Step  LifeWeld.hpp:169-186, `gens` times, in place on
// {state, frozen2, frozen1, frozen0} (4 x 64 words, the struct's member order)
void ref_weld_step(uint64_t *w, unsigned gens) {
  LifeWeld weld(load(w), load(w + 64), load(w + 128), load(w + 192));
  for (unsigned g = 0; g < gens; ++g) weld.Step();
  store(weld.state, w);
  store(weld.frozen2, w + 64);
  store(weld.frozen1, w + 128);
  store(weld.frozen0, w + 192);
}
// LifeWeld::FromRequired  LifeWeld.hpp:133-159 (tests/LifeWeldTest.cpp:19-33
// shape, with Parse instead of the `$`-buggy ConstantParse)
void ref_weld_from_required(const char *state_rle, const char *required_rle, int dx, int dy,
                            uint64_t *w) {
  LifeWeld weld = LifeWeld::FromRequired(LifeState::Parse(std::string(state_rle)),
                                         LifeState::Parse(std::string(required_rle)).Moved(dx, dy));
  store(weld.state, w);
  store(weld.frozen2, w + 64);
  store(weld.frozen1, w + 128);
  store(weld.frozen0, w + 192);
}
// ---- LifeStable passes (LifeStable.hpp:41-53,526-729): 10 planes in the
// class's member order {state, unknown, live2, live3, dead0, dead1, dead2,
// dead4, dead5, dead6}; options stored as "1 = ruled out".
static LifeStable load_stable(const uint64_t *p) {
  LifeStable s;
  s.state = load(p);
  s.unknown = load(p + 64);
  s.live2 = load(p + 128);
  s.live3 = load(p + 192);
  s.dead0 = load(p + 256);
  s.dead1 = load(p + 320);
  s.dead2 = load(p + 384);
  s.dead4 = load(p + 448);
  s.dead5 = load(p + 512);
  s.dead6 = load(p + 576);
  return s;
}
static void store_stable(const LifeStable &s, uint64_t *p) {
  store(s.state, p);
  store(s.unknown, p + 64);
  store(s.live2, p + 128);
  store(s.live3, p + 192);
  store(s.dead0, p + 256);
  store(s.dead1, p + 320);
  store(s.dead2, p + 384);
  store(s.dead4, p + 448);
  store(s.dead5, p + 512);
  store(s.dead6, p + 576);
}
// which: 0 SynchroniseStateKnown (:526-556), 1 UpdateOptions (:558-615),
// 2 SignalNeighbours (:617-675), 3 PropagateStep (:695-716),
// 4 Propagate (:718-729), 5 StabiliseOptions (:677-693).  Returns consistent | changed << 1.
int ref_stable_pass(uint64_t *planes, int which) {
  LifeStable s = load_stable(planes);
  LifeStable::PropagateResult r{};
  switch (which) {
    case 0: r = s.SynchroniseStateKnown(); break;
    case 1: r = s.UpdateOptions(); break;
    case 2: r = s.SignalNeighbours(); break;
    case 3: r = s.PropagateStep(); break;
    case 5: r = s.StabiliseOptions(); break;
    default: r = s.Propagate(); break;
  }
  store_stable(s, planes);
  return (r.consistent ? 1 : 0) | (r.changed ? 2 : 0);
}
// The two espresso fragments the passes include, evaluated on 64 cells.
// stable_count.hpp (included at LifeStable.hpp:591): 9 inputs -> 9 outputs
void ref_stable_count_frag(const uint64_t *in, uint64_t *out) {
  const uint64_t on2 = in[0], on1 = in[1], on0 = in[2], off3 = in[3], off2 = in[4], off1 = in[5],
                 off0 = in[6], known_on = in[7], known_off = in[8];
  uint64_t abort = 0, l2 = 0, l3 = 0, d0 = 0, d1 = 0, d2 = 0, d4 = 0, d5 = 0, d6 = 0;
#include "bitslicing/stable_count.hpp"
  const uint64_t r[9] = {l2, l3, d0, d1, d2, d4, d5, d6, abort};
  std::memcpy(out, r, sizeof r);
}
// stable_signal.hpp (included at LifeStable.hpp:654): 17 inputs -> 4 outputs
void ref_stable_signal_frag(const uint64_t *in, uint64_t *out) {
  const uint64_t l2 = in[0], l3 = in[1], d0 = in[2], d1 = in[3], d2 = in[4], d4 = in[5], d5 = in[6],
                 d6 = in[7], s2 = in[8], s1 = in[9], s0 = in[10], m3 = in[11], m2 = in[12],
                 m1 = in[13], m0 = in[14], stateon = in[15], stateunk = in[16];
  uint64_t signaloff = 0, signalon = 0, centeroff = 0, centeron = 0;
#include "bitslicing/stable_signal.hpp"
  const uint64_t r[4] = {signaloff, signalon, centeroff, centeron};
  std::memcpy(out, r, sizeof r);
}
// stable_vulnerable.hpp (included at LifeStable.hpp:400): 15 inputs -> 4 outputs
void ref_stable_vulnerable_frag(const uint64_t *in, uint64_t *out) {
  const uint64_t l2 = in[0], l3 = in[1], d0 = in[2], d1 = in[3], d2 = in[4], d4 = in[5], d5 = in[6],
                 d6 = in[7], s2 = in[8], s1 = in[9], s0 = in[10], unk3 = in[11], unk2 = in[12],
                 unk1 = in[13], unk0 = in[14];
  uint64_t vulnerable_on = 0, vulnerable_off = 0, vulnerable_center_on = 0, vulnerable_center_off = 0;
#include "bitslicing/stable_vulnerable.hpp"
  const uint64_t r[4] = {vulnerable_on, vulnerable_off, vulnerable_center_on, vulnerable_center_off};
  std::memcpy(out, r, sizeof r);
}
// LifeStable::Vulnerable()  LifeStable.hpp:366-412
void ref_stable_vulnerable(const uint64_t *planes, uint64_t *out) {
  store(load_stable(planes).Vulnerable(), out);
}
// LifeState::GetPop  LifeAPI.hpp:290-298
unsigned ref_pop(const uint64_t *s) { return load(s).GetPop(); }
// LifeState::Contains(const LifeTarget&)  LifeTarget.hpp:44-51
int ref_contains_target(const uint64_t *s, const uint64_t *wanted, const uint64_t *unwanted) {
  LifeTarget t(load(wanted), load(unwanted));
  return load(s).Contains(t) ? 1 : 0;
}
// LifeState::Contains(const LifeTarget&) over a batch: out[u] = 0/1
void ref_contains_batch(const uint64_t *s, size_t n, const uint64_t *wanted, const uint64_t *unwanted,
                        uint8_t *out) {
  const LifeTarget t(load(wanted), load(unwanted));
  for (size_t u = 0; u < n; ++u) out[u] = load(s + u * 64).Contains(t) ? 1 : 0;
}
// The pattern tests over a batch (LifeAPI.hpp:378-422, LifeTarget.hpp:38-42):
// kind 0 Contains(pat), 1 AreDisjoint(pat), 2 Contains(pat, dx, dy),
// 3 AreDisjoint(pat, dx, dy), 4 Contains(LifeTarget{pat, pat2}, dx, dy)
void ref_pattern_batch(const uint64_t *s, size_t n, const uint64_t *pat, const uint64_t *pat2, int kind, int dx,
                       int dy, uint8_t *out) {
  const LifeState p = load(pat), p2 = load(pat2);
  const LifeTarget t(p, p2);
  for (size_t u = 0; u < n; ++u) {
    const LifeState a = load(s + u * 64);
    bool r = false;
    switch (kind) {
      case 0: r = a.Contains(p); break;
      case 1: r = a.AreDisjoint(p); break;
      case 2: r = a.Contains(p, dx, dy); break;
      case 3: r = a.AreDisjoint(p, dx, dy); break;
      default: r = a.Contains(t, dx, dy); break;
    }
    out[u] = r ? 1 : 0;
  }
}
// LifeTarget(const LifeState&) (LifeTarget.hpp:10-13) and Moved (:33-35):
// the unwanted plane GetBoundary() (LifeAPI.hpp:521-538) of the moved target
void ref_target_from_state(const uint64_t *state, int dx, int dy, uint64_t *wanted, uint64_t *unwanted) {
  const LifeTarget t = LifeTarget(load(state)).Moved({dx, dy});
  store(t.wanted, wanted);
  store(t.unwanted, unwanted);
}
// LifeState::Parse  Parsing.hpp:192-198
void ref_parse(const char *rle, uint64_t *out) { store(LifeState::Parse(std::string(rle)), out); }
// LifeState::RLE  Parsing.hpp:8-63,200-204: writes at most cap bytes, returns the length
size_t ref_rle(const uint64_t *s, char *out, size_t cap) {
  const std::string r = load(s).RLE();
  std::memcpy(out, r.data(), r.size() < cap ? r.size() : cap);
  return r.size();
}
// LifeState::RandomState  LifeAPI.hpp:63-69 (non-deterministic, random_device seeded)
void ref_random_state(uint64_t *out) { store(LifeState::RandomState(), out); }

// ---- config 5: bitslicing/unknown_step_refined.hpp (the espresso fragment)
// Inputs in the fragment's own variable names, 64 cells per word, in the
// order of bitslicing/unknown_step_refined.py:105-113 (innames) with the
// older live-count encoding on2..on0 (bits 2..0 of the inclusive live count,
// :99) that this fragment was generated from.
void ref_unknown_step_refined(const uint64_t *in16, uint64_t *out3) {
  const uint64_t l2 = in16[0], l3 = in16[1], d0 = in16[2], d1 = in16[3], d2 = in16[4],
                 d4 = in16[5], d5 = in16[6], d6 = in16[7], current_unknown = in16[8],
                 current_on = in16[9], s2 = in16[10], s1 = in16[11], s0 = in16[12],
                 on2 = in16[13], on1 = in16[14], on0 = in16[15];
  uint64_t next_on = 0, next_unknown = 0, next_unknown_stable = 0;
#include "bitslicing/unknown_step_refined.hpp"
  out3[0] = next_on;
  out3[1] = next_unknown;
  out3[2] = next_unknown_stable;
}

// Config-5 harness (build-defined; the reference has no consumer of this
// fragment).  Per universe, 11 input planes of 64 words:
//   0 stable.state  1 current.state (ON)  2 current.unknown
//   3..10 live2 live3 dead0 dead1 dead2 dead4 dead5 dead6 (LifeStable.hpp:44-53,
//         1 = ruled out)
// s2..s0  = bits 2..0 of NeighbourCount(stable.state)    (NeighbourCount.hpp:40-70)
// on2..on0 = bits 2..0 of NeighbourCount(current.state)
// Output per universe, 3 planes: next_on, next_unknown, next_unknown_stable.
void ref_refined_step_batch(const uint64_t *in, uint64_t *out, size_t n) {
  for (size_t u = 0; u < n; ++u) {
    const uint64_t *p = in + u * 11 * 64;
    uint64_t *o = out + u * 3 * 64;
    NeighbourCount ns(load(p + 0 * 64)), nc(load(p + 1 * 64));
    for (unsigned i = 0; i < 64; ++i) {
      const uint64_t in16[16] = {p[3 * 64 + i], p[4 * 64 + i], p[5 * 64 + i], p[6 * 64 + i],
                                 p[7 * 64 + i], p[8 * 64 + i], p[9 * 64 + i], p[10 * 64 + i],
                                 p[2 * 64 + i], p[1 * 64 + i],
                                 ns.bit2[i], ns.bit1[i], ns.bit0[i],
                                 nc.bit2[i], nc.bit1[i], nc.bit0[i]};
      uint64_t r[3];
      ref_unknown_step_refined(in16, r);
      o[0 * 64 + i] = r[0];
      o[1 * 64 + i] = r[1];
      o[2 * 64 + i] = r[2];
    }
  }
}

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

// The search-loop idiom on the reference's own types: Step() then
// Contains(LifeTarget) after every generation (LifeAPI.hpp:1196-1216,
// LifeTarget.hpp:44-51); first[u] = the first generation (1..gens) whose
// state contains the target, 0 = none; out (may be NULL) = Stepped(gens).
void ref_step_contains_batch(const uint64_t *in, uint64_t *out, size_t n, unsigned gens, const uint64_t *wanted,
                             const uint64_t *unwanted, uint32_t *first, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  const LifeTarget target(load(wanted), load(unwanted));
  auto work = [=, &target](size_t lo, size_t hi) {
    for (size_t u = lo; u < hi; ++u) {
      LifeState t = load(in + u * 64);
      uint32_t f = 0;
      for (unsigned g = 1; g <= gens; ++g) {
        t.Step();
        if (!f && t.Contains(target)) f = g;
      }
      first[u] = f;
      if (out) store(t, out + u * 64);
    }
  };
  if (nthreads == 1) { work(0, n); return; }
  std::vector<std::thread> pool;
  for (int k = 0; k < nthreads; ++k)
    pool.emplace_back(work, n * k / nthreads, n * (k + 1) / nthreads);
  for (auto &th : pool) th.join();
}

}  // extern "C"
