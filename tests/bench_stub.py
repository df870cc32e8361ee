"""TEST INFRASTRUCTURE ONLY: a CPU stand-in for ``lifeapi_amd.hip`` with which
tests/test_bench_ranks.py rehearses bench.py's rank logic (rank spawning,
barrier + MAX timing, per-shard first-launch verification, hash all-gather)
on a machine without a GPU, through tests/bench_rank_runner.py (which swaps
it in for bench.py's kernel loader; bench.py never loads it).
The compute is the oracle's C port (oracle/lifeapi_oracle.c), so the digests
it produces are checked against the reference-generated golden digests,
exactly as the GPU ranks' are.  Never a measurement.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from oracle.oracle import Port

P = Port()


class _Event:
    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other) -> float:
        return (other.t - self.t) * 1e3

    def synchronize(self):
        pass


class Runtime:
    kind = "oracle-port stub"

    def __init__(self, local_rank: int):
        self.device = torch.device("cpu")
        self.stream = None
        self.neutral_error = None

    @staticmethod
    def neutral(states, out, generations=1, reverse=False, nts=True, resident=0, upw=4, plain_bytes=0,
                stream=None, xcd_chunk=False):
        """stand-in for the tuning build's fixed-order launcher (same result)"""
        return step(states, out=out, generations=generations)

    def sync(self):
        pass

    @staticmethod
    def event():
        return _Event()


def step_kernel_name(generations: int = 1, n: int | None = None) -> str:
    return "stub: oracle C port on the CPU"


def _u64(t: torch.Tensor) -> np.ndarray:
    return np.ascontiguousarray(t.numpy()).view(np.uint64)


def fill_random(n, seed, first_universe=0, mode=0, out=None, device=None, stream=None):
    x = torch.from_numpy(P.fill(n, seed=seed, first_universe=first_universe, mode=mode).view(np.int64).copy())
    if out is not None:
        out.copy_(x)
        return out
    return x


def step(states, out=None, generations=1, stream=None):
    r = torch.from_numpy(P.step_batch(_u64(states), generations).view(np.int64))
    if out is None:
        return r.clone()
    out.copy_(r)
    return out


def hashes(states, stream=None):
    return torch.from_numpy(P.hashes(_u64(states)).view(np.int64).copy())
