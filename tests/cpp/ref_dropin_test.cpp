// ref_dropin_test.cpp -- the drop-in claim, checked with the REFERENCE's own
// types: a search loop keeps #include "LifeAPI.hpp" (and friends) and adds
// <lifeapi/batch.hpp>; the batched GPU calls on ::LifeState, ::LifeTarget,
// ::LifeWeld, ::NeighbourCount and ::LifeStable must give exactly what the
// reference's own member functions give.
//
// Built by oracle/Makefile (target ref, into oracle/_ref/) only where
// /root/reference exists (this container): the reference headers are compiled
// in, from where they lie, with oracle/ref_prelude.hpp (see oracle/Makefile
// for the two image gaps it bridges).  The binary travels to the GPU box with
// oracle/_ref/; nothing reads /root/reference at run time.  Run by
// tests/test_cpp_facade.py.  Exit status = number of failed checks.
#include <lifeapi/LifeState.hpp>  // first: ref_prelude.hpp defines `constexpr` away
#include <lifeapi/batch.hpp>

#include "ref_prelude.hpp"

#include "LifeAPI.hpp"
#include "LifeStable.hpp"
#include "LifeTarget.hpp"
#include "LifeWeld.hpp"
#include "NeighbourCount.hpp"
#include "Parsing.hpp"

#include <cstdio>
#include <cstring>
#include <span>
#include <vector>

static int g_failures = 0, g_checks = 0;
#define EXPECT_TRUE(c)                                                                  \
  do {                                                                                  \
    ++g_checks;                                                                         \
    if (!(c)) {                                                                         \
      ++g_failures;                                                                     \
      if (g_failures < 20) std::fprintf(stderr, "%s:%d: %s failed\n", __FILE__, __LINE__, #c); \
    }                                                                                   \
  } while (0)

// tests/StepAltTest.cpp:5-13 on the reference's own RandomState(), batched:
// StepBatch == Step() == StepAlt() for every state
static void StepAltTest_Random() {
  std::vector<LifeState> batch(10000), cpu, alt;
  for (auto &s : batch) s = LifeState::RandomState();
  cpu = alt = batch;
  for (size_t i = 0; i < batch.size(); ++i) {
    cpu[i].Step();
    alt[i].StepAlt();
  }
  lifeapi::StepBatch(std::span(batch), 1);
  for (size_t i = 0; i < batch.size(); ++i) {
    EXPECT_TRUE(batch[i] == cpu[i]);
    EXPECT_TRUE(cpu[i] == alt[i]);
  }
}

// Stepped(n) (LifeAPI.hpp:882-886) into a second span, and GetPop()
static void Stepped_And_Pop() {
  std::vector<LifeState> in(3000), out(3000);
  for (auto &s : in) s = LifeState::RandomState();
  lifeapi::SteppedBatch(std::span<const LifeState>(in), std::span(out), 37);
  const std::vector<uint32_t> pops = lifeapi::GetPopBatch(std::span<const LifeState>(out));
  for (size_t i = 0; i < in.size(); ++i) {
    EXPECT_TRUE(out[i] == in[i].Stepped(37));
    EXPECT_TRUE(pops[i] == (uint32_t)out[i].GetPop());
  }
}

// R-pentomino (BASELINE config 1) to generation 1103
static void RPentomino() {
  std::vector<LifeState> one{LifeState::Parse("b2o$2o$bo!")};
  LifeState cpu = one[0];
  cpu.Step(1103);
  lifeapi::StepBatch(std::span(one), 1103);
  EXPECT_TRUE(one[0] == cpu);
  EXPECT_TRUE(one[0].GetPop() == 113);
}

// LifeState::Contains(const LifeTarget&) (LifeTarget.hpp:44-51)
static void Contains_Target() {
  const LifeState block = LifeState::Parse("2o$2o!");
  const LifeTarget target(block, block.ZOI() & ~block);
  std::vector<LifeState> s(2000);
  for (size_t i = 0; i < s.size(); ++i) {
    s[i] = LifeState::RandomState();
    if (i % 3 == 0) s[i] = (s[i] & ~block.ZOI()) | block;
  }
  const std::vector<uint8_t> hit = lifeapi::ContainsBatch(std::span<const LifeState>(s), target);
  int hits = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    EXPECT_TRUE((hit[i] != 0) == s[i].Contains(target));
    hits += hit[i] != 0;
  }
  EXPECT_TRUE(hits >= 600);
}

// LifeState::Contains(const LifeTarget&, dx, dy) (LifeTarget.hpp:38-42):
// offsets on both sides of the torus seam and beyond +-64, and a target with
// a cell both wanted and unwanted (never contained by the offset form)
static void Contains_TargetOffset() {
  const LifeState loaf = LifeState::Parse("b2o$o2bo$bobo$2bo!");
  const LifeTarget target(loaf, loaf.ZOI() & ~loaf);
  LifeTarget clash = target;
  clash.unwanted.Set(1, 0);  // (1, 0) is alive in the loaf
  const int offs[][2] = {{0, 0}, {5, -3}, {-7, 60}, {63, 63}, {-64, 1}, {130, -200}};
  for (const auto &o : offs) {
    const int dx = o[0], dy = o[1];
    std::vector<LifeState> s(1500);
    for (size_t i = 0; i < s.size(); ++i) {
      s[i] = LifeState::RandomState();
      // plant the loaf where the offset test looks for it: state column
      // i + dx rotated right by dy is matched against target column i
      const LifeState at = loaf.Moved(dx, dy), zoi = loaf.ZOI().Moved(dx, dy);
      if (i % 3 == 0) s[i] = (s[i] & ~zoi) | at;
    }
    const std::vector<uint8_t> hit = lifeapi::ContainsBatch(std::span<const LifeState>(s), target, dx, dy);
    const std::vector<uint8_t> none = lifeapi::ContainsBatch(std::span<const LifeState>(s), clash, dx, dy);
    int hits = 0;
    for (size_t i = 0; i < s.size(); ++i) {
      EXPECT_TRUE((hit[i] != 0) == s[i].Contains(target, dx, dy));
      EXPECT_TRUE((none[i] != 0) == s[i].Contains(clash, dx, dy));
      hits += hit[i] != 0;
    }
    EXPECT_TRUE(hits >= 400);
  }
}

// the search loop with the offset test
static void StepContains_Offset() {
  const LifeState block = LifeState::Parse("2o$2o!");
  const LifeTarget target(block, block.ZOI() & ~block);
  const int dx = -20, dy = 45;
  std::vector<LifeState> s(2000);
  for (size_t i = 0; i < s.size(); ++i) {
    s[i] = LifeState::RandomState() & LifeState::RandomState();
    if (i % 4 == 0) s[i] = (s[i] & ~block.ZOI().Moved(dx, dy)) | block.Moved(dx, dy);
  }
  std::vector<LifeState> cpu = s, s2 = s;
  std::vector<uint32_t> want(s.size(), 0);
  for (size_t i = 0; i < s.size(); ++i)
    for (unsigned g = 1; g <= 12; ++g) {
      cpu[i].Step();
      if (!want[i] && cpu[i].Contains(target, dx, dy)) want[i] = g;
    }
  const std::vector<uint32_t> got = lifeapi::StepContainsBatch(std::span(s), target, dx, dy, 12);
  LifeTarget clash = target;
  clash.wanted.Set(7, 7);
  clash.unwanted.Set(7, 7);
  const std::vector<uint32_t> none = lifeapi::StepContainsBatch(std::span(s2), clash, dx, dy, 12);
  int hits = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    EXPECT_TRUE(got[i] == want[i]);
    EXPECT_TRUE(none[i] == 0);
    EXPECT_TRUE(s[i] == cpu[i] && s2[i] == cpu[i]);
    hits += want[i] != 0;
  }
  EXPECT_TRUE(hits > 0);
}

// the search-loop idiom: step, then Contains(target), first hit per state
static void StepContains_SearchLoop() {
  const LifeState block = LifeState::Parse("2o$2o!").Moved(30, 30);
  const LifeTarget target(block, block.ZOI() & ~block);
  std::vector<LifeState> s(3000);
  for (size_t i = 0; i < s.size(); ++i) {
    s[i] = LifeState::RandomState() & LifeState::RandomState();
    if (i % 4 == 0) s[i] = (s[i] & ~block.ZOI()) | block;
  }
  std::vector<LifeState> cpu = s;
  std::vector<uint32_t> want(s.size(), 0);
  for (size_t i = 0; i < s.size(); ++i)
    for (unsigned g = 1; g <= 20; ++g) {
      cpu[i].Step();
      if (!want[i] && cpu[i].Contains(target)) want[i] = g;
    }
  const std::vector<uint32_t> got = lifeapi::StepContainsBatch(std::span(s), target, 20);
  int hits = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    EXPECT_TRUE(got[i] == want[i]);
    EXPECT_TRUE(s[i] == cpu[i]);
    hits += want[i] != 0;
  }
  EXPECT_TRUE(hits > 0);
}

// the standalone facade (lifeapi/LifeState.hpp) against the reference
static lifeapi::LifeState facade(const LifeState &s) {
  lifeapi::LifeState r;
  std::memcpy(r.state, s.state, sizeof r.state);
  return r;
}
static bool same(const lifeapi::LifeState &a, const LifeState &b) {
  return std::memcmp(a.state, b.state, sizeof a.state) == 0;
}

// LifeTarget(const LifeState&) (LifeTarget.hpp:10-13: unwanted =
// GetBoundary(), LifeAPI.hpp:521-538), Moved (:33-35, LifeAPI.hpp:699-735),
// and the single-state pattern tests (LifeAPI.hpp:377-421, LifeTarget.hpp:38-42)
static void Facade_TargetAndPatternTests() {
  const int offs[][2] = {{0, 0}, {1, 0}, {0, -1}, {5, -3}, {-7, 60}, {63, 63}, {-64, 1}, {130, -200}};
  for (int k = 0; k < 200; ++k) {
    const LifeState pat = LifeState::RandomState() & LifeState::RandomState() & LifeState::RandomState() &
                          LifeState::Parse("8o$8o$8o$8o$8o$8o!").Moved(k % 64, (7 * k) % 64);
    const LifeTarget want(pat);
    const lifeapi::LifeTarget got(facade(pat));
    EXPECT_TRUE(same(got.wanted, want.wanted) && same(got.unwanted, want.unwanted));
    EXPECT_TRUE(same(facade(pat).ZOI(), pat.ZOI()) && same(facade(pat).GetBoundary(), pat.GetBoundary()));
    for (const auto &o : offs) {
      const LifeTarget wm = want.Moved({o[0], o[1]});
      const lifeapi::LifeTarget gm = got.Moved({o[0], o[1]});
      EXPECT_TRUE(same(gm.wanted, wm.wanted) && same(gm.unwanted, wm.unwanted));
      EXPECT_TRUE(same(facade(pat).Moved(o[0], o[1]), pat.Moved(o[0], o[1])));
      LifeState s = LifeState::RandomState() & LifeState::RandomState();
      if (k % 2) s = (s & ~pat.ZOI().Moved(o[0], o[1])) | pat.Moved(o[0], o[1]);
      const lifeapi::LifeState fs = facade(s);
      EXPECT_TRUE(fs.Contains(facade(pat), o[0], o[1]) == s.Contains(pat, o[0], o[1]));
      EXPECT_TRUE(fs.AreDisjoint(facade(pat), o[0], o[1]) == s.AreDisjoint(pat, o[0], o[1]));
      EXPECT_TRUE(fs.AreDisjoint(facade(pat)) == s.AreDisjoint(pat));
      EXPECT_TRUE(fs.Contains(got, o[0], o[1]) == s.Contains(want, o[0], o[1]));
      EXPECT_TRUE(fs.Contains(gm) == s.Contains(wm));
    }
  }
}

// the batched pattern tests on the reference's own ::LifeState:
// Contains(pat), Contains(pat, dx, dy), AreDisjoint(pat), AreDisjoint(pat, dx, dy)
static void PatternBatches() {
  const LifeState glider = LifeState::Parse("bo$2bo$3o!");
  const int offs[][2] = {{0, 0}, {30, 30}, {62, 5}, {-3, -3}, {100, -70}};
  for (const auto &o : offs) {
    std::vector<LifeState> s(3000);
    for (size_t i = 0; i < s.size(); ++i) {
      s[i] = LifeState::RandomState() & LifeState::RandomState();
      if (i % 3 == 0) s[i] |= glider.Moved(o[0], o[1]);
      if (i % 3 == 1) s[i] &= ~glider.Moved(o[0], o[1]);
    }
    const std::span<const LifeState> in(s);
    const auto c = lifeapi::ContainsBatch(in, glider), co = lifeapi::ContainsBatch(in, glider, o[0], o[1]);
    const auto d = lifeapi::AreDisjointBatch(in, glider), dd = lifeapi::AreDisjointBatch(in, glider, o[0], o[1]);
    int hits = 0, apart = 0;
    for (size_t i = 0; i < s.size(); ++i) {
      EXPECT_TRUE((c[i] != 0) == s[i].Contains(glider));
      EXPECT_TRUE((co[i] != 0) == s[i].Contains(glider, o[0], o[1]));
      EXPECT_TRUE((d[i] != 0) == s[i].AreDisjoint(glider));
      EXPECT_TRUE((dd[i] != 0) == s[i].AreDisjoint(glider, o[0], o[1]));
      hits += co[i] != 0;
      apart += dd[i] != 0;
    }
    EXPECT_TRUE(hits >= 1000 && apart >= 1000);
  }
}

// A search loop written against the standalone facade with LifeTarget(pattern)
// (it did not compile before the constructor existed), against the
// reference's own loop on the same states
static void Facade_SearchLoopWithPatternTarget() {
  const LifeState block = LifeState::Parse("2o$2o!").Moved(40, 9);
  std::vector<LifeState> ref(2000);
  for (size_t i = 0; i < ref.size(); ++i) {
    ref[i] = LifeState::RandomState() & LifeState::RandomState();
    // clear two cells around the block: then nothing can be born in its ring
    if (i % 4 == 0) ref[i] = (ref[i] & ~block.ZOI().ZOI()) | block;
  }
  std::vector<lifeapi::LifeState> fs(ref.size());
  for (size_t i = 0; i < ref.size(); ++i) fs[i] = facade(ref[i]);
  const lifeapi::LifeTarget target(facade(block));
  const std::vector<uint32_t> got = lifeapi::StepContainsBatch(std::span(fs), target, 1);
  const std::vector<uint32_t> got6 = lifeapi::StepContainsBatch(std::span(fs), target, 6);
  const LifeTarget want_t(block);
  int hits = 0;
  for (size_t i = 0; i < ref.size(); ++i) {
    LifeState t = ref[i];
    uint32_t w1 = 0, w6 = 0;
    t.Step();
    if (t.Contains(want_t)) w1 = 1;
    for (unsigned g = 2; g <= 7; ++g) {
      t.Step();
      if (!w6 && t.Contains(want_t)) w6 = g - 1;
    }
    EXPECT_TRUE(got[i] == w1 && got6[i] == w6 && same(fs[i], t));
    hits += w1 != 0;
  }
  EXPECT_TRUE(hits >= 300);
}

// NeighbourCount(state) (NeighbourCount.hpp:40-70)
static void NeighbourCount_Planes() {
  std::vector<LifeState> s(1000);
  for (auto &x : s) x = LifeState::RandomState();
  std::vector<NeighbourCount> nc(s.size(), NeighbourCount(LifeState()));
  lifeapi::NeighbourCountBatch(std::span<const LifeState>(s), std::span(nc));
  for (size_t i = 0; i < s.size(); ++i) {
    const NeighbourCount want(s[i]);
    EXPECT_TRUE(nc[i].bit3 == want.bit3 && nc[i].bit2 == want.bit2 && nc[i].bit1 == want.bit1 &&
                nc[i].bit0 == want.bit0);
  }
}

// LifeWeld::Step() (LifeWeld.hpp:169-186) on welds from FromRequired
// (tests/LifeWeldTest.cpp:19-33 shape, Parse for the `$`-safe patterns)
static void LifeWeld_Step() {
  const LifeState eater = LifeState::Parse("2o$obo$2bo$2b2o!");
  std::vector<LifeWeld> w;
  for (int k = 0; k < 300; ++k) {
    const LifeState junk = LifeState::RandomState() & LifeState::Parse("8o$8o$8o$8o!").Moved(20, 20);
    w.push_back(LifeWeld::FromRequired(eater | junk, eater));
  }
  std::vector<LifeWeld> cpu = w;
  for (auto &x : cpu) {
    x.Step();
    x.Step();
  }
  lifeapi::WeldStepBatch(std::span(w), 2);
  for (size_t i = 0; i < w.size(); ++i) EXPECT_TRUE(w[i].state == cpu[i].state);
}

// LifeStable::Propagate() (LifeStable.hpp:718-729) on partially unknown still
// lifes: every plane and the PropagateResult
static std::vector<LifeStable> partly_unknown_still_lifes() {
  std::vector<LifeStable> s;
  const LifeState block = LifeState::Parse("2o$2o!");
  for (int k = 0; k < 200; ++k) {
    LifeStable c;
    LifeState st;
    for (int b = 0; b < 5; ++b) st |= block.Moved(13 * ((k + 3 * b) % 5), 11 * ((k * 7 + b) % 5));
    LifeState unk = LifeState::Parse("6o$6o$6o$6o$6o$6o!").Moved((k * 5) % 50, (k * 3) % 50);
    c.state = st & ~unk;
    c.unknown = unk;
    s.push_back(c);
  }
  return s;
}

static void LifeStable_Propagate() {
  std::vector<LifeStable> s = partly_unknown_still_lifes();
  std::vector<LifeStable> cpu = s;
  std::vector<LifeStable::PropagateResult> want;
  for (auto &x : cpu) want.push_back(x.Propagate());
  const std::vector<lifeapi::PropagateResult> got = lifeapi::PropagateBatch(std::span(s));
  for (size_t i = 0; i < s.size(); ++i) {
    EXPECT_TRUE(got[i].consistent == want[i].consistent && got[i].changed == want[i].changed);
    EXPECT_TRUE(s[i] == cpu[i]);  // every plane (LifeStable::operator==, LifeStable.hpp:55)
  }
}

// LifeStable::StabiliseOptions() (LifeStable.hpp:677-693) through the
// host-pointer form (lifeapi_stable_pass_batch, pass 5), after one
// SynchroniseStateKnown so the counts are in sync as the reference assumes
// (LifeStable.hpp:133-134): every plane and the PropagateResult
static void LifeStable_StabiliseOptions() {
  std::vector<LifeStable> s = partly_unknown_still_lifes();
  for (auto &x : s) x.SynchroniseStateKnown();
  std::vector<LifeStable> cpu = s;
  std::vector<LifeStable::PropagateResult> want;
  for (auto &x : cpu) want.push_back(x.StabiliseOptions());
  const std::vector<lifeapi::PropagateResult> got = lifeapi::StabiliseOptionsBatch(std::span(s));
  int changed = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    EXPECT_TRUE(got[i].consistent == want[i].consistent && got[i].changed == want[i].changed);
    EXPECT_TRUE(s[i] == cpu[i]);
    changed += want[i].changed;
  }
  EXPECT_TRUE(changed > 0);  // the case exercises the pass, not just a no-op
}

// LifeState::Parse / RLE() (Parsing.hpp:143-204), batched
static void Rle_RoundTrip() {
  std::vector<LifeState> s(500);
  for (auto &x : s) x = LifeState::RandomState() & LifeState::RandomState();
  const std::vector<std::string> rle = lifeapi::RLEBatch(std::span<const LifeState>(s));
  const std::vector<LifeState> back = lifeapi::ParseBatch<LifeState>(std::span<const std::string>(rle));
  for (size_t i = 0; i < s.size(); ++i) {
    EXPECT_TRUE(rle[i] == s[i].RLE());
    EXPECT_TRUE(back[i] == LifeState::Parse(rle[i]));
  }
}

int main() {
  StepAltTest_Random();
  Stepped_And_Pop();
  RPentomino();
  Contains_Target();
  Contains_TargetOffset();
  StepContains_Offset();
  StepContains_SearchLoop();
  Facade_TargetAndPatternTests();
  PatternBatches();
  Facade_SearchLoopWithPatternTarget();
  NeighbourCount_Planes();
  LifeWeld_Step();
  LifeStable_Propagate();
  LifeStable_StabiliseOptions();
  Rle_RoundTrip();
  std::printf("%d checks, %d failures\n", g_checks, g_failures);
  return g_failures == 0 ? 0 : 1;
}
