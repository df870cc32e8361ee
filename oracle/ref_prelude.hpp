// ref_prelude.hpp -- forced-include prelude for building the REFERENCE's own
// headers (/root/reference/*.hpp) in this image.  Test infrastructure only.
//
// Why: LifeAPI.hpp:1185,1190 declare `constexpr LifeState corona =
// LifeState::ConstantParse("...")`, which needs a constexpr std::string.
// The image's only C++ standard library is libstdc++ 11, which has none, so
// the header does not compile as shipped.  Those two lines are off the Step()
// path.  We pre-include every standard header the reference (and this shim)
// uses, then define `constexpr` away for the rest of the translation unit;
// the reference's functions keep their run-time semantics (constexpr only
// permits compile-time evaluation).  No reference source is copied or edited.
#pragma once
#include <algorithm>
#include <array>
#include <bit>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <iostream>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <utility>
#include <vector>
#define constexpr
