"""Build-defined batch digest (checksum of checksums) for result collection.

The per-universe 64-bit hash is computed on the GPU (lifeapi_hash_batch_dev):
    h_u = mix(sum_x mix(state[x] + (x+1)*G))
and folded here on the host into an order-sensitive, shard-additive digest:
    D = sum_u mix(h_u + (u_global+1)*G)  mod 2^64
with mix = the splitmix64 finaliser and G = 0x9E3779B97F4A7C15.  Because D is
a sum, shard digests add up to the global one, so ranks can check their own
slice against a reference digest without gathering states.
"""
from __future__ import annotations

import numpy as np

G = np.uint64(0x9E3779B97F4A7C15)


def mix64(z: np.ndarray) -> np.ndarray:
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def batch_digest(hashes: np.ndarray, first_universe: int = 0) -> int:
    h = np.ascontiguousarray(hashes).view(np.uint64).ravel()
    idx = np.arange(first_universe + 1, first_universe + 1 + h.size, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return int(mix64(h + idx * G).sum(dtype=np.uint64))


def combine(digests) -> int:
    return int(sum(int(d) for d in digests) % (1 << 64))
