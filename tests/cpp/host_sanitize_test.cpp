// host_sanitize_test.cpp -- the host-side code under AddressSanitizer and
// UndefinedBehaviorSanitizer (the reference has no sanitizers;
// the build adds them for its host code).  CPU only: the facade's CPU members
// (lifeapi/LifeState.hpp) against the C oracle (oracle/lifeapi_oracle.c),
// both compiled with -fsanitize=address,undefined by tests/test_sanitize.py.
// Exit status = number of failed checks.
#include <lifeapi/LifeState.hpp>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../oracle/lifeapi_oracle.h"

using lifeapi::LifeState;

static int g_failures = 0, g_checks = 0;
#define EXPECT_TRUE(c)                                                                    \
  do {                                                                                    \
    ++g_checks;                                                                           \
    if (!(c)) {                                                                           \
      ++g_failures;                                                                       \
      std::fprintf(stderr, "%s:%d: EXPECT_TRUE(%s) failed\n", __FILE__, __LINE__, #c); \
    }                                                                                     \
  } while (0)

static bool same(const LifeState &s, const uint64_t *w) { return std::memcmp(s.state, w, 512) == 0; }

int main() {
  // Step / StepAlt / Stepped(n) / GetPop / NeighbourCount rule vs the oracle
  std::vector<uint64_t> buf(64 * 512);
  oracle_fill(buf.data(), 512, 99, 0, 0);
  for (int u = 0; u < 512; ++u) {
    LifeState s;
    std::memcpy(s.state, &buf[64 * u], 512);
    uint64_t w[64];
    std::memcpy(w, s.state, 512);
    oracle_step(w);
    LifeState a = s, b = s;
    a.Step();
    b.StepAlt();
    EXPECT_TRUE(same(a, w));
    EXPECT_TRUE(a == b);
    const lifeapi::NeighbourCount nc(s);
    LifeState rule = nc.WithExactly(3) | (s & nc.WithExactly(4));
    EXPECT_TRUE(rule == a);
    std::memcpy(w, s.state, 512);
    oracle_step_n(w, 7);
    EXPECT_TRUE(same(s.Stepped(7), w));
    EXPECT_TRUE(s.GetPop() == oracle_pop(s.state));
  }
  // Contains(LifeTarget)
  for (int u = 0; u + 2 < 512; u += 3) {
    LifeState s, wa, un;
    std::memcpy(s.state, &buf[64 * u], 512);
    std::memcpy(wa.state, &buf[64 * u + 64], 512);
    std::memcpy(un.state, &buf[64 * u + 128], 512);
    LifeState w2 = s & wa, u2 = ~s & un;
    EXPECT_TRUE(s.Contains(lifeapi::LifeTarget(w2, u2)) ==
                (bool)oracle_contains_target(s.state, w2.state, u2.state));
    EXPECT_TRUE(s.Contains(lifeapi::LifeTarget(wa, un)) ==
                (bool)oracle_contains_target(s.state, wa.state, un.state));
  }
  // LifeWeld::Step (LifeWeld.hpp:169-186)
  for (int u = 0; u + 4 < 512; u += 4) {
    lifeapi::LifeWeld wd;
    std::memcpy(&wd, &buf[64 * u], sizeof wd);
    uint64_t w[256];
    std::memcpy(w, &wd, sizeof w);
    wd.Step();
    oracle_weld_step(w, 1);
    EXPECT_TRUE(std::memcmp(&wd, w, sizeof w) == 0);
  }
  // Parse / RLE (Parsing.hpp:8-63,143-204), including the edge strings
  const char *rles[] = {"b2o$2o$bo!", "bo$2bo$3o!", "x = 3, y = 3, rule = B3/S23\r\nbo$2bo$3o!",
                        "3o$$$3o!", "64o!", "2o128$2o!", "2o129$2o!", "o 2 3bo!", "", "!", "5$",
                        "12b3o$o10bo!", "#C comment\nobo!"};
  for (const char *r : rles) {
    uint64_t w[64];
    const int rc = oracle_parse_rle(r, w);
    const LifeState p = LifeState::Parse(r);
    if (rc == 0) EXPECT_TRUE(same(p, w));
    char text[70000];
    const size_t len = oracle_rle(p.state, text, sizeof text);  // (not NUL-terminated)
    EXPECT_TRUE(p.RLE() == std::string(text, len));
  }
  for (int u = 0; u < 64; ++u) {
    LifeState s;
    std::memcpy(s.state, &buf[64 * u], 512);
    char text[70000];
    const size_t len = oracle_rle(s.state, text, sizeof text);
    const std::string r = s.RLE();
    EXPECT_TRUE(r == std::string(text, len));
    // Parse(RLE(s)) is s moved by (32, 32)
    const LifeState back = LifeState::Parse(r);
    bool ok = true;
    for (int x = 0; x < 64; ++x)
      for (int y = 0; y < 64; ++y) ok &= back.Get(x, y) == s.Get((x + 32) & 63, (y + 32) & 63);
    EXPECT_TRUE(ok);
  }
  std::printf("%d checks, %d failures\n", g_checks, g_failures);
  return g_failures;
}
