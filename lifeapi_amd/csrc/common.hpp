// common.hpp -- launch geometry shared by the device and host sides.
#pragma once

#include <cstdint>

namespace lifeapi_impl {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ULL;

}  // namespace lifeapi_impl
