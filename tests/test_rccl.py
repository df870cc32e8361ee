"""GPU: the RCCL (torch.distributed "nccl") path bench.py's N > 1 lines take,
exercised on the one GPU of the box before the driver's 8-GPU run needs it.

* a world-1 "nccl" process group created as bench.py creates it
  (`init_process_group("nccl", device_id=...)`), driven through bench.py's
  own collective calls: barrier, all_reduce(MAX) of the timed region,
  all_gather of the per-rank figures and digests, and gather_hashes'
  all_gather_into_tensor (taken at world 1 because a group exists);
* bench.py itself started by torch.distributed.run with one rank and the
  nccl backend: the whole N > 1 code path, first-launch verification
  included, on the real kernel.
Universes are independent (LifeAPI.hpp:1196-1216), so these collectives
carry results only, never the data path.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


_WORKER = r'''
import json, os, sys
sys.path.insert(0, os.environ["ROOT"])
import numpy as np, torch, torch.distributed as dist
import bench
import lifeapi_amd.hip as hip
from lifeapi_amd.digest import batch_digest
from lifeapi_amd.shard import gather_hashes
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
bench.COLL_DEV = dev
out = {"backend": dist.get_backend(), "world": dist.get_world_size()}
dist.barrier()
t = torch.tensor([3.5], dtype=torch.float64, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
out["max"] = float(t.item())
out["ints"] = bench.all_gather_ints([5, (1 << 64) - 1], 1)
x = hip.fill_random(1 << 16, seed=4, device=dev)
y = hip.step(x)
h = hip.hashes(y)
g = gather_hashes(h, 1, [h.numel()])
torch.cuda.synchronize()
out["gathered_is_copy"] = g.data_ptr() != h.data_ptr()
out["gathered_equal"] = bool(torch.equal(g, h))
out["digest"] = f"{batch_digest(g.cpu().numpy()):016x}"
dist.destroy_process_group()
print("RESULT " + json.dumps(out), flush=True)
'''


def _env():
    env = dict(os.environ, ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()),
               WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    env.pop("LIFEAPI_BENCH_BACKEND", None)
    return env


def test_world1_nccl_group_runs_bench_collectives():
    r = subprocess.run([sys.executable, "-c", _WORKER], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][0][7:])
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["max"] == 3.5 and res["ints"] == [[5, (1 << 64) - 1]]
    assert res["gathered_is_copy"] and res["gathered_equal"]
    from oracle.oracle import Ref
    if Ref.available():
        from oracle.oracle import Port
        P = Port()
        want = P.digest(P.hashes(Ref().step_batch(P.fill(1 << 16, seed=4), 1, nthreads=8)))
        assert res["digest"] == f"{want:016x}"


def test_bench_one_rank_rccl_end_to_end():
    """bench.py under torch.distributed.run, one rank, nccl: config 4's 16M
    problem as ONE shard (the N = 1 point of the strong split), every
    collective of the N > 1 line over RCCL, first launch verified against the
    reference-generated digest, 16M hashes gathered."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR", "LIFEAPI_BENCH_BACKEND"):
        env.pop(k, None)
    env["LIFEAPI_BENCH_DETAIL"] = os.path.join(ROOT, "gpurun_out", "rccl_bench_detail.json")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
                        "--gpus", "1", "--config", "4", "--steps", "5", "--warmup", "2", "--no-secondary",
                        "--no-cpu-baseline"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert line["collective_world_size"] == 1 and "kernel_backend" not in line
    assert line["verified"]["ok"] is True and line["verified"]["global_ok"] is True
    c = line["collect"]
    assert "RCCL" in c["op"] and c["universes_gathered"] == 1 << 24
    assert line["value"] > 0 and line["roofline"]["hbm_only"]["frac"] > 0
