"""TEST INFRASTRUCTURE ONLY: runs bench.py's own main() -- rank spawning,
barrier + MAX timing, per-shard first-launch verification, hash all-gather --
with the HIP kernels replaced by the oracle-backed CPU stand-in
tests/bench_stub.py, for tests/test_bench_ranks.py on a machine without a
GPU.  bench.py itself has no such path: this script swaps its
load_kernels() before calling main(), and bench.py's rank spawner re-runs
this script (sys.argv[0]) for every rank.  Refuses to run where a GPU is
visible, and every line it prints says STUB."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import bench  # noqa: E402
import bench_stub  # noqa: E402


def _stub_kernels(backend, local_rank, world):
    if torch.cuda.is_available():
        raise RuntimeError("tests/bench_rank_runner.py is for GPU-less rank rehearsals only")
    return bench_stub, bench_stub.Runtime(local_rank)


if __name__ == "__main__":
    bench.load_kernels = _stub_kernels
    bench.main()
