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
  Errors_Throw();
  std::printf("%d checks, %d failures\n", g_checks, g_failures);
  return g_failures == 0 ? 0 : 1;
}
