// step_batch_test.cpp -- C++ facade tests, written like the reference's gtest
// files (tests/StepAltTest.cpp:5-13, tests/InteractionTest.cpp:7-27) but
// against lifeapi::LifeState and the batched GPU path.  Needs a GPU; run by
// tests/test_cpp_facade.py.  Exit status = number of failed checks.
#include <lifeapi/LifeState.hpp>

#include <cstdio>
#include <span>
#include <vector>

using lifeapi::LifeState;

static int g_failures = 0, g_checks = 0;
#define EXPECT_TRUE(c)                                                          \
  do {                                                                          \
    ++g_checks;                                                                 \
    if (!(c)) {                                                                 \
      ++g_failures;                                                             \
      std::fprintf(stderr, "%s:%d: EXPECT_TRUE(%s) failed\n", __FILE__, __LINE__, #c); \
    }                                                                           \
  } while (0)
#define EXPECT_EQ(a, b) EXPECT_TRUE((a) == (b))

// StepAltTest.Random, batched: GPU StepBatch == CPU Step() == CPU StepAlt()
static void StepAltTest_Random() {
  uint64_t seed = 12345;
  std::vector<LifeState> batch(10000), cpu(10000), alt(10000);
  for (unsigned i = 0; i < batch.size(); i++) {
    batch[i] = LifeState::RandomState(seed);
    cpu[i] = batch[i];
    alt[i] = batch[i];
    cpu[i].Step();
    alt[i].StepAlt();
  }
  lifeapi::StepBatch(std::span(batch), 1);
  for (unsigned i = 0; i < batch.size(); i++) {
    EXPECT_EQ(batch[i], cpu[i]);
    EXPECT_EQ(cpu[i], alt[i]);
  }
}

// Iterated batch on device == serial Step(n) on the CPU
static void SteppedBatch_Iterated() {
  uint64_t seed = 7;
  std::vector<LifeState> in(3001), out(3001);
  for (auto &s : in) s = LifeState::RandomState(seed);
  lifeapi::SteppedBatch(std::span<const LifeState>(in), std::span(out), 37);
  for (unsigned i = 0; i < in.size(); i += 7) EXPECT_EQ(out[i], in[i].Stepped(37));
}

// R-pentomino on the 64x64 torus: population 113 at generation 1103
static void RPentomino_KnownAnswer() {
  std::vector<LifeState> one{LifeState::Parse("b2o$2o$bo!")};
  lifeapi::StepBatch(std::span(one), 1103);
  EXPECT_EQ(one[0].GetPop(), 113u);
  EXPECT_EQ(one[0], LifeState::Parse("b2o$2o$bo!").Stepped(1103));
  auto pops = lifeapi::GetPopBatch(std::span<const LifeState>(one));
  EXPECT_EQ(pops[0], 113u);
}

// Eater pair at every offset (InteractionTest.cpp:7-27 shape): the batched
// step agrees with the single-universe CPU step on all 400 configurations
static void Interaction_BatchMatchesCpu() {
  LifeState eater = LifeState::Parse("2b2o$bobo$bo$2o!");
  std::vector<LifeState> together;
  for (int i = -10; i < 10; i++)
    for (int j = -10; j < 10; j++) {
      LifeState moved;
      for (int x = 0; x < 64; ++x)
        for (int y = 0; y < 64; ++y)
          if (eater.Get(x, y)) moved.SetSafe(x + i, y + j, true);
      together.push_back(eater | moved);
    }
  std::vector<LifeState> stepped = together;
  lifeapi::StepBatch(std::span(stepped), 1);
  for (size_t k = 0; k < together.size(); ++k) EXPECT_EQ(stepped[k], together[k].Stepped());
}

// Glider moves (+1, +1) every 4 generations, across both torus seams
static void Glider_Translation() {
  LifeState g = LifeState::Parse("bo$2bo$3o!");
  std::vector<LifeState> b{g};
  lifeapi::StepBatch(std::span(b), 4 * 64);  // full lap around the torus
  EXPECT_EQ(b[0], g);
  b[0] = g;
  lifeapi::StepBatch(std::span(b), 4);
  LifeState moved;
  for (int x = 0; x < 64; ++x)
    for (int y = 0; y < 64; ++y)
      if (g.Get(x, y)) moved.SetSafe(x + 1, y + 1, true);
  EXPECT_EQ(b[0], moved);
}

// all visible devices (device = -1) give the same answer as device 0
static void MultiDevice_Shards() {
  uint64_t seed = 99;
  std::vector<LifeState> a(5003), b;
  for (auto &s : a) s = LifeState::RandomState(seed);
  b = a;
  lifeapi::StepBatch(std::span(a), 3, 0);
  lifeapi::StepBatch(std::span(b), 3, -1);
  for (size_t i = 0; i < a.size(); ++i) EXPECT_EQ(a[i], b[i]);
}

// a page-locked batch (lifeapi::HostPin) stepped many chunks at a time gives
// the CPU's answer, as the pageable batch does
static void HostPin_ManyChunks() {
  uint64_t seed = 7;
  std::vector<LifeState> a(300000), want;
  for (auto &s : a) s = LifeState::RandomState(seed);
  want = a;
  for (size_t i = 0; i < 2000; ++i) want[i].Step(2);
  {
    lifeapi::HostPin pin{std::span(a)};
    lifeapi::StepBatch(std::span(a), 2);
  }
  for (size_t i = 0; i < 2000; ++i) EXPECT_EQ(a[i], want[i]);
  lifeapi::StepBatch(std::span(want).subspan(2000), 2);
  for (size_t i = 2000; i < a.size(); ++i) EXPECT_EQ(a[i], want[i]);
}

// LifeWeldTest.StableTest (tests/LifeWeldTest.cpp:6-17), batched: a weld of a
// still life with nothing frozen is invariant; random welds match the CPU
static void LifeWeld_StableAndRandom() {
  std::vector<lifeapi::LifeWeld> w(2);
  w[0].state = LifeState::Parse("2b2o$bobo$bo$2o!");
  w[1].state = LifeState::Parse("2o$2o!");
  auto copy = w;
  lifeapi::WeldStepBatch(std::span(w), 1);
  EXPECT_TRUE(w[0] == copy[0] && w[1] == copy[1]);
  uint64_t seed = 4242;
  std::vector<lifeapi::LifeWeld> r(1001);
  for (auto &x : r) {
    x.state = LifeState::RandomState(seed);
    x.frozen0 = LifeState::RandomState(seed) & LifeState::RandomState(seed);
    x.frozen1 = LifeState::RandomState(seed) & LifeState::RandomState(seed) & LifeState::RandomState(seed);
  }
  auto cpu = r;
  for (auto &x : cpu) {
    x.Step();
    x.Step();
  }
  lifeapi::WeldStepBatch(std::span(r), 2);
  for (size_t i = 0; i < r.size(); ++i) EXPECT_TRUE(r[i] == cpu[i]);
}

// NeighbourCount / Contains batches vs the CPU facade
static void Counts_And_Contains() {
  uint64_t seed = 777;
  std::vector<LifeState> s(513);
  for (auto &x : s) x = LifeState::RandomState(seed);
  std::vector<lifeapi::NeighbourCount> nc(s.size());
  lifeapi::NeighbourCountBatch(std::span<const LifeState>(s), std::span(nc));
  for (size_t i = 0; i < s.size(); i += 5) {
    const lifeapi::NeighbourCount c(s[i]);
    EXPECT_TRUE(nc[i].bit0 == c.bit0 && nc[i].bit1 == c.bit1 && nc[i].bit2 == c.bit2 && nc[i].bit3 == c.bit3);
    // Life == WithExactly(3) | (s & WithExactly(4)) (the NeighbourCount rule)
    EXPECT_EQ(c.WithExactly(3) | (s[i] & c.WithExactly(4)), s[i].Stepped());
  }
  lifeapi::LifeTarget t(s[3], ~s[3]);
  auto hit = lifeapi::ContainsBatch(std::span<const LifeState>(s), t);
  for (size_t i = 0; i < s.size(); ++i) EXPECT_EQ(hit[i] != 0, s[i].Contains(t));
  EXPECT_TRUE(hit[3] != 0);
}

// the pattern tests and LifeTarget(pattern) on the standalone facade: the
// batch forms against the facade's own single-state members
static void Pattern_Batches() {
  uint64_t seed = 4242;
  const LifeState loaf = LifeState::Parse("b2o$o2bo$bobo$2bo!");
  const lifeapi::LifeTarget t(loaf);  // unwanted = loaf.GetBoundary()
  EXPECT_TRUE(t.unwanted == (loaf.ZOI() & ~loaf) && t.unwanted.GetPop() == 23u);  // 30 cells in the ZOI, 7 live
  std::vector<LifeState> s(1500);
  for (size_t i = 0; i < s.size(); ++i) {
    s[i] = LifeState::RandomState(seed) & LifeState::RandomState(seed);
    if (i % 3 == 0) s[i] = (s[i] & ~loaf.ZOI().Moved(9, -4)) | loaf.Moved(9, -4);
  }
  const std::span<const LifeState> in(s);
  const auto c = lifeapi::ContainsBatch(in, loaf, 9, -4), d = lifeapi::AreDisjointBatch(in, loaf, 9, -4);
  const auto c0 = lifeapi::ContainsBatch(in, loaf), d0 = lifeapi::AreDisjointBatch(in, loaf);
  const auto tm = lifeapi::ContainsBatch(in, t.Moved({9, -4}));
  int hits = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    EXPECT_EQ(c[i] != 0, s[i].Contains(loaf, 9, -4));
    EXPECT_EQ(d[i] != 0, s[i].AreDisjoint(loaf, 9, -4));
    EXPECT_EQ(c0[i] != 0, s[i].Contains(loaf));
    EXPECT_EQ(d0[i] != 0, s[i].AreDisjoint(loaf));
    EXPECT_EQ(tm[i] != 0, s[i].Contains(t, 9, -4));
    hits += tm[i] != 0;
  }
  EXPECT_TRUE(hits >= 500);
}

// LifeStable propagation: a block field with an unknown window stays
// consistent and fills in; an inconsistent (unstable) known region is flagged
static void Stable_Propagate() {
  std::vector<lifeapi::LifeStable> st(2);
  for (int k = 0; k < 4; ++k) {
    st[0].state |= LifeState::Parse("2o$2o!");
    for (auto &w : st[0].state.state) w = std::rotl(w, 16);
  }
  for (int x = 20; x < 30; ++x) st[0].unknown[x] = 0xFFFull << 20;
  st[1].state = LifeState::Parse("3o!");  // a blinker is not still: inconsistent
  auto r = lifeapi::PropagateBatch(std::span(st));
  EXPECT_TRUE(r[0].consistent);
  EXPECT_TRUE(!r[1].consistent);
}

// RLE batch I/O: RLEBatch == RLE() per state, ParseBatch(RLE) == state moved
// by (32, 32), ParseBatch == Parse on hand-written strings
static void Rle_Batch() {
  uint64_t seed = 31337;
  std::vector<LifeState> s(777);
  for (auto &x : s) x = LifeState::RandomState(seed) & LifeState::RandomState(seed);
  s[0] = LifeState();
  s[1] = LifeState::Parse("bo$2bo$3o!");
  const auto rles = lifeapi::RLEBatch(std::span<const LifeState>(s));
  for (size_t i = 0; i < s.size(); i += 7) EXPECT_EQ(rles[i], s[i].RLE());
  EXPECT_EQ(rles[0], std::string("!"));
  std::vector<uint8_t> st;
  const auto back = lifeapi::ParseBatch<LifeState>(std::span<const std::string>(rles), &st);
  for (size_t i = 0; i < s.size(); ++i) {
    LifeState moved;
    for (int x = 0; x < 64; ++x)
      for (int y = 0; y < 64; ++y)
        if (s[i].Get(x, y)) moved.SetSafe(x + 32, y + 32, true);
    EXPECT_TRUE(back[i] == moved && st[i] == 0);
  }
  const std::vector<std::string> hand{"x = 3, y = 3\nbo$2bo$3o!", "2b2o$bobo$bo$2o!", "1 2o!", "70o!"};
  const auto p = lifeapi::ParseBatch<LifeState>(std::span<const std::string>(hand), &st);
  for (size_t i = 0; i + 1 < hand.size(); ++i) EXPECT_TRUE(p[i] == LifeState::Parse(hand[i]) && st[i] == 0);
  EXPECT_EQ(st[3], 1u);
}

// errors surface as lifeapi::Error (the reference has no failure path)
static void Errors_Throw() {
  std::vector<LifeState> a(4);
  bool threw = false;
  try {
    lifeapi::StepBatch(std::span(a), 1, 1 << 20);
  } catch (const lifeapi::Error &e) {
    threw = e.code == LIFEAPI_E_NODEVICE;
  }
  EXPECT_TRUE(threw);
}

int main() {
  StepAltTest_Random();
  SteppedBatch_Iterated();
  RPentomino_KnownAnswer();
  Interaction_BatchMatchesCpu();
  Glider_Translation();
  MultiDevice_Shards();
  HostPin_ManyChunks();
  LifeWeld_StableAndRandom();
  Counts_And_Contains();
  Pattern_Batches();
  Stable_Propagate();
  Rle_Batch();
  Errors_Throw();
  std::printf("%d checks, %d failures\n", g_checks, g_failures);
  return g_failures == 0 ? 0 : 1;
}
