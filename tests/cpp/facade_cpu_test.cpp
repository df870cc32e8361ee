// facade_cpu_test.cpp -- the standalone facade's single-state members
// (include/lifeapi/LifeState.hpp) against the REFERENCE's own, on the CPU:
// Step / StepAlt, ZOI / GetBoundary, Move / Moved, Contains / AreDisjoint
// with and without (dx, dy), Contains(LifeTarget[, dx, dy]), LifeTarget(state)
// and LifeTarget::Moved (LifeAPI.hpp:377-421,521-538,682-735,1196-1254;
// LifeTarget.hpp:10-51).  No GPU: the batch calls are not used.
//
// Built by oracle/Makefile (target ref, into oracle/_ref/) where
// /root/reference exists, like ref_dropin_test.cpp; run by
// tests/test_cpp_facade.py in the CPU suite.  Exit status 0 = all equal.
#include <lifeapi/LifeState.hpp>  // first: ref_prelude.hpp defines `constexpr` away

#include "ref_prelude.hpp"

#include "LifeAPI.hpp"
#include "LifeTarget.hpp"
#include "Parsing.hpp"

#include <cstdio>
#include <cstring>

static int g_failures = 0, g_checks = 0;
#define EXPECT_TRUE(c)                                                                   \
  do {                                                                                   \
    ++g_checks;                                                                          \
    if (!(c)) {                                                                          \
      ++g_failures;                                                                      \
      if (g_failures < 20) std::fprintf(stderr, "%s:%d: %s failed\n", __FILE__, __LINE__, #c); \
    }                                                                                    \
  } while (0)

static lifeapi::LifeState facade(const LifeState &s) {
  lifeapi::LifeState r;
  std::memcpy(r.state, s.state, sizeof r.state);
  return r;
}
static bool same(const lifeapi::LifeState &a, const LifeState &b) {
  return std::memcmp(a.state, b.state, sizeof a.state) == 0;
}

int main() {
  const int offs[][2] = {{0, 0}, {1, 0}, {0, -1}, {5, -3}, {-7, 60}, {63, 63}, {-64, 1}, {130, -200}};
  for (int k = 0; k < 300; ++k) {
    const LifeState a = LifeState::RandomState() & LifeState::RandomState();
    const LifeState pat = LifeState::RandomState() & LifeState::RandomState() & LifeState::RandomState() &
                          LifeState::Parse("8o$8o$8o$8o$8o$8o!").Moved(k % 64, (7 * k) % 64);
    const lifeapi::LifeState fa = facade(a), fp = facade(pat);
    // stepping
    LifeState s1 = a, s2 = a;
    lifeapi::LifeState f1 = fa, f2 = fa;
    s1.Step();
    f1.Step();
    s2.StepAlt();
    f2.StepAlt();
    EXPECT_TRUE(same(f1, s1) && same(f2, s2));
    // ZOI, boundary, targets
    EXPECT_TRUE(same(fp.ZOI(), pat.ZOI()) && same(fp.GetBoundary(), pat.GetBoundary()));
    const LifeTarget rt(pat);
    const lifeapi::LifeTarget ft(fp);
    EXPECT_TRUE(same(ft.wanted, rt.wanted) && same(ft.unwanted, rt.unwanted));
    EXPECT_TRUE(fa.Contains(fp) == a.Contains(pat) && fa.AreDisjoint(fp) == a.AreDisjoint(pat));
    EXPECT_TRUE(fa.Contains(ft) == a.Contains(rt));
    for (const auto &o : offs) {
      EXPECT_TRUE(same(fp.Moved(o[0], o[1]), pat.Moved(o[0], o[1])));
      EXPECT_TRUE(same(fp.Moved({o[0], o[1]}), pat.Moved(std::make_pair(o[0], o[1]))));
      lifeapi::LifeState fm = fp;
      LifeState rm = pat;
      fm.Move(o[0], o[1]);
      rm.Move(o[0], o[1]);
      EXPECT_TRUE(same(fm, rm));
      const LifeTarget rtm = rt.Moved({o[0], o[1]});
      const lifeapi::LifeTarget ftm = ft.Moved({o[0], o[1]});
      EXPECT_TRUE(same(ftm.wanted, rtm.wanted) && same(ftm.unwanted, rtm.unwanted));
      // plant the pattern where the offset test looks for it in half the cases
      LifeState b = a;
      if (k % 2) b = (b & ~pat.ZOI().Moved(o[0], o[1])) | pat.Moved(o[0], o[1]);
      const lifeapi::LifeState fb = facade(b);
      EXPECT_TRUE(fb.Contains(fp, o[0], o[1]) == b.Contains(pat, o[0], o[1]));
      EXPECT_TRUE(fb.AreDisjoint(fp, o[0], o[1]) == b.AreDisjoint(pat, o[0], o[1]));
      EXPECT_TRUE(fb.Contains(ft, o[0], o[1]) == b.Contains(rt, o[0], o[1]));
      EXPECT_TRUE(fb.Contains(ftm) == b.Contains(rtm));
    }
  }
  std::printf("%d checks, %d failures\n", g_checks, g_failures);
  return g_failures == 0 ? 0 : 1;
}
