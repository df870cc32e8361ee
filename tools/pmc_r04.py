"""Kernel driver for round 4's rocprofv3 --pmc passes (tools/gpu_r04_prof.sh):
a few launches of one kernel, each after a 768 MiB scrub (bench.py Scrub),
so that every launch reads from HBM and the counters per dispatch are those
of one cold launch.

  step N      the shipped 1-generation step on N universes (ping-pong)
  cone        the search filter (1 gen) and Contains on 1M config-2
              universes, for bench.py's two targets (golden.json
              digests.config2_filter): block first, then whole_board
  stable      Propagate on 1M LifeStables, each launch on a fresh copy: 3
              launches on tools/rows_bench.py's still lifes around an
              unknown window (every column changes), then 3 on a search's
              next node (rows_bench.stable_next_node: a few columns change):
              the bytes the changed-line stores write
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import lifeapi_amd.hip as hip  # noqa: E402


class RT:
    kind = "hip"

    def __init__(self):
        self.device = torch.device("cuda", 0)
        self.stream = torch.cuda.current_stream()


def main():
    rt = RT()
    scrub = bench.Scrub(rt)
    reps = 3
    if sys.argv[1] == "step":
        n = int(sys.argv[2])
        a = hip.fill_random(n, seed=4)
        b = torch.empty_like(a)
        for k in range(reps):
            scrub()
            hip.step(a if k % 2 == 0 else b, out=b if k % 2 == 0 else a, generations=1)
    elif sys.argv[1] == "stable":
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from rows_bench import stable_inputs, stable_next_node
        st = stable_inputs(1 << 20)
        nxt = stable_next_node(st)
        w = st.clone()
        for src in (st, nxt):
            for _ in range(reps):
                w.copy_(src)
                scrub()
                hip.stable_pass(w, "propagate")
    else:
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            gold = json.load(f)["digests"]["config2_filter"]
        x = hip.fill_random(gold["universes"], seed=gold["seed"])
        for name in ("block", "whole_board"):
            t = gold["targets"][name]
            tw, tu = (torch.from_numpy(np.array([[int(v, 16) for v in t[k]]], dtype=np.uint64).view(np.int64))
                      .cuda() for k in ("wanted", "unwanted"))
            for _ in range(reps):
                scrub()
                hip.step_contains(x, tw, tu, 1)
            for _ in range(reps):
                scrub()
                hip.contains(x, tw, tu)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
