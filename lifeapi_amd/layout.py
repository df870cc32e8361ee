"""LifeState layout constants (LifeAPI.hpp:12,39-40)."""

N = 64                 # const int N = 64           LifeAPI.hpp:12
UNIVERSE_WORDS = N     # uint64_t state[N]          LifeAPI.hpp:40
UNIVERSE_BYTES = 8 * N  # 512 B, aligned(64)        LifeAPI.hpp:39
