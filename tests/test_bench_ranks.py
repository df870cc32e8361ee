"""CPU, gloo: bench.py's own multi-rank path, end to end.

`python bench.py --gpus 2` (no torch.distributed environment) must start two
ranks itself, shard the problem, run the timed region with its barrier and
MAX over ranks, verify every rank's shard of the first launch against the
reference-generated digests (tests/golden/golden.json, *_small entries) and
all-gather the per-universe hashes.  tests/bench_rank_runner.py runs
bench.py's main() with the HIP kernels replaced by the oracle-backed CPU
stand-in tests/bench_stub.py (bench.py itself has no such path); everything
else is the code the GPU ranks run.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = dict(os.environ, LIFEAPI_BENCH_BACKEND="gloo", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="",
               MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "bench_rank_runner.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0]), r.stderr


def _expected_collect(total, seed, gens_done):
    from lifeapi_amd.digest import batch_digest
    from oracle.oracle import Port
    P = Port()
    x = P.fill(total, seed=seed)
    return f"{batch_digest(P.hashes(P.step_batch(x, gens_done)).view(np.int64)):016x}"


def test_bench_gpus2_strong_config4_spawns_two_ranks():
    line, err = _bench("--gpus", "2", "--config", "4", "--universes", str(1 << 14),
                       "--steps", "3", "--warmup", "2", "--no-cpu-baseline")
    assert "torch.distributed.run" in err and "bench_rank_runner.py" in err  # bench.py's spawner started the ranks
    assert line["n_gpus"] == 2 and line["collective_world_size"] == 2
    assert line["scaling"] == "strong"
    assert line["config"]["global_universes"] == 1 << 14
    assert [p["universes"] for p in line["per_rank"]] == [1 << 13, 1 << 13]
    v = line["verified"]
    assert v["ok"] is True and v["per_rank_ok"] == [True, True] and v["global_ok"] is True
    assert "config4_small" in v["against"]
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert "STUB" in line["kernel_backend"]
    # per rank: the shipped figure and the cache-neutral one (same kernel,
    # fixed order, all stores nontemporal), and live copy ceilings
    for p in line["per_rank"]:
        assert p["GBps"] > 0 and p["GBps_cache_neutral"] > 0
        assert p["kernel_ms_cache_neutral"] > 0 and p["copy_GBps"] > 0 and p["copy_GBps_cache_neutral"] > 0
    r = line["roofline"]
    assert r["aggregate_GBps_cache_neutral"] > 0 and r["cache_neutral"]["achieved"] > 0
    assert r["frac_kind"].startswith("effective") and r["copy_ceiling_GBps"] > 0
    assert line["value_cache_neutral"] > 0
    # result collection: 1 warmup launch + (warmup-1) + steps generations in all
    c = line["collect"]
    assert c["universes_gathered"] == 1 << 14
    assert c["final_digest"] == _expected_collect(1 << 14, 4, 1 + 1 + 3)


def test_bench_gpus8_strong_config4_rehearsal():
    """The N the scaling target names (8 GPUs, config 4: one 16M problem
    strong-split), rehearsed at 16K universes: 8 ranks spawned by bench.py
    itself, each shard on the golden chunk grid (2K universes per rank = one
    config4_small chunk), every shard verified against the reference-generated
    digest, all 16K hashes gathered."""
    line, err = _bench("--gpus", "8", "--config", "4", "--universes", str(1 << 14),
                       "--steps", "2", "--warmup", "1", "--no-cpu-baseline", timeout=600)
    assert "torch.distributed.run" in err
    assert line["n_gpus"] == 8 and line["collective_world_size"] == 8 and line["scaling"] == "strong"
    assert [p["universes"] for p in line["per_rank"]] == [1 << 11] * 8
    v = line["verified"]
    assert v["ok"] is True and v["per_rank_ok"] == [True] * 8 and v["global_ok"] is True
    assert "config4_small" in v["against"]
    assert line["value"] > 0 and line["value_cache_neutral"] > 0
    assert all(p["GBps_cache_neutral"] > 0 for p in line["per_rank"])
    c = line["collect"]
    assert c["universes_gathered"] == 1 << 14
    assert c["final_digest"] == _expected_collect(1 << 14, 4, 1 + 0 + 2)


def test_bench_gpus2_weak_config2():
    line, _ = _bench("--gpus", "2", "--config", "2", "--universes", str(1 << 11),
                     "--steps", "2", "--warmup", "1", "--no-cpu-baseline")
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["global_universes"] == 1 << 12
    v = line["verified"]
    assert v["ok"] is True and v["per_rank_ok"] == [True, True] and v["global_ok"] is True
    assert line["collect"]["final_digest"] == _expected_collect(1 << 12, 2, 1 + 0 + 2)


def test_bench_gpus4_ragged_strong_split():
    # 4 ranks over 16K + 4 universes: shard edges off the golden chunk grid, so
    # per-rank checks are unknown but the global digest still has to match
    # the single-process answer
    line, _ = _bench("--gpus", "4", "--config", "4", "--universes", str((1 << 14) + 4),
                     "--steps", "1", "--warmup", "1", "--no-cpu-baseline")
    assert line["n_gpus"] == 4
    assert sum(p["universes"] for p in line["per_rank"]) == (1 << 14) + 4
    from lifeapi_amd.digest import batch_digest
    from oracle.oracle import Port
    P = Port()
    x = P.fill((1 << 14) + 4, seed=4)
    assert line["verified"]["global_digest"] == f"{batch_digest(P.hashes(P.step_batch(x, 1)).view(np.int64)):016x}"
    assert len(line["per_rank"]) == 4 and all(p["GBps_cache_neutral"] > 0 for p in line["per_rank"])
    assert line["roofline"]["aggregate_GBps_cache_neutral"] > 0
    assert line["collect"]["final_digest"] == _expected_collect((1 << 14) + 4, 4, 2)


def test_bench_single_rank_default_is_config2():
    line, err = _bench("--gpus", "1", "--universes", str(1 << 11), "--steps", "2", "--warmup", "1",
                       "--no-cpu-baseline", "--no-secondary")
    assert "torch.distributed.run" not in err
    assert line["n_gpus"] == 1 and line["scaling"] == "weak"
    assert line["config"]["workload"].startswith("config2")
    assert line["verified"]["ok"] is True


@pytest.mark.parametrize("cfg", ["2", "4"])
def test_bench_refuses_stub_marking(cfg):
    # the stub line must never pass for a measurement
    line, _ = _bench("--gpus", "1", "--config", cfg, "--universes", str(1 << 11 if cfg == "2" else 1 << 14),
                     "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-secondary")
    assert "STUB" in line["kernel_backend"]
