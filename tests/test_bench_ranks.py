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
    # per rank: the shipped figure, the HBM-only one (the launch after a scrub
    # plus its deferred write-backs), and live copy ceilings
    for p in line["per_rank"]:
        assert p["GBps"] > 0 and p["GBps_hbm_only"] > 0 and p["GBps_launch_after_scrub"] > 0
        assert p["kernel_ms_hbm_only"] > 0 and p["copy_GBps"] > 0 and p["copy_GBps_cache_neutral"] > 0
    r = line["roofline"]
    assert r["aggregate_GBps_hbm_only"] > 0 and r["hbm_only"]["achieved"] > 0
    assert r["frac_kind"].startswith("effective") and r["copy_ceiling_GBps"] > 0
    assert line["value_hbm_only"] > 0
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
    assert line["value"] > 0 and line["value_hbm_only"] > 0
    assert all(p["GBps_hbm_only"] > 0 for p in line["per_rank"])
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
    assert len(line["per_rank"]) == 4 and all(p["GBps_hbm_only"] > 0 for p in line["per_rank"])
    assert line["roofline"]["aggregate_GBps_hbm_only"] > 0
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


def test_bench_one_rank_under_launcher_takes_the_collective_path():
    """One rank started by torch.distributed.run (WORLD_SIZE=1, MASTER_PORT set)
    opens a process group and runs the N > 1 lines' collective code: barrier,
    MAX of the timed region, the digest all-gather and the hash all-gather
    (tests/test_rccl.py runs the same with the nccl backend on the GPU)."""
    env = dict(os.environ, LIFEAPI_BENCH_BACKEND="gloo", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="",
               OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr=127.0.0.1", f"--master-port={port}",
                        os.path.join(ROOT, "tests", "bench_rank_runner.py"), "--gpus", "1", "--config", "4",
                        "--universes", str(1 << 14), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                        "--no-secondary"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert line["n_gpus"] == 1 and line["collective_world_size"] == 1
    assert line["verified"]["ok"] is True
    c = line["collect"]
    assert c["universes_gathered"] == 1 << 14 and "gloo" in c["op"]
    assert c["final_digest"] == _expected_collect(1 << 14, 4, 1 + 0 + 2)


def test_bench_line_is_compact_with_summary_last():
    """The printed line leaves the per-launch series and long prose to the
    detail file, and ends with the flat secondary_summary, so a 2000-character
    tail of stdout holds the summary whole."""
    import bench
    sec = {"config3": {"kernel_ms": 1.3, "kernel_ms_all": [1.3] * 20, "verified": True,
                       "roofline": {"frac": 0.66, "definition": "x" * 300},
                       "search_loop": {"kernel_ms": 1.4, "verified": True, "kernel_ms_all": [1.4] * 20}},
           "config5": {"kernel_ms": 0.3, "verified": True, "roofline": {"frac": 0.8, "hbm_only": {"frac": 0.7}}},
           "filter": {"targets": {"block": {"verified": True, "filter_1gen": {"kernel_ms": 0.01,
                                                                              "roofline": {"frac": 0.5}},
                                            "contains": {"kernel_ms": 0.01, "roofline": {"frac": 0.6}}}}}}
    line = {"metric": "m", "value": 1.0, "kernel_ms_avg": 0.16, "roofline": {"frac": 0.85, "hbm_only": {"frac": 0.7}},
            "verified": {"ok": True}, "secondary": sec}
    out = bench.compact_line(line)
    assert "kernel_ms_all" not in out["secondary"]["config3"]
    assert "definition" not in out["secondary"]["config3"]["roofline"]
    out["secondary_summary"] = bench.secondary_summary(out, sec, {"config1": {"facade_ns_per_gen": 31.0}})
    s = out["secondary_summary"]
    assert s["c3_kernel_ms"] == 1.3 and s["c3_verified"] is True and s["c3_search_verified"] is True
    assert s["c5_verified"] is True and s["c2_frac_hbm_only"] == 0.7 and s["filter_block_verified"] is True
    assert list(out)[-1] == "secondary_summary" and len(json.dumps(s)) < 1900
