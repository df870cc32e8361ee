"""Fused Step + Contains (lifeapi_step_contains_batch_dev) vs plain Step on the
config-3 shape (64K universes x 1024 generations); one JSON line per case."""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import lifeapi_amd.hip as hip  # noqa: E402


def timed(fn, reps=7):
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b))
    return sorted(ms)[len(ms) // 2]


def main():
    n, g = 1 << 16, 1024
    x = hip.fill_random(n, seed=3)
    out = torch.empty_like(x)
    w = torch.zeros((1, 64), dtype=torch.int64, device="cuda")
    w[0, 10] = w[0, 11] = 3 << 40                       # a block ...
    u = torch.zeros((1, 64), dtype=torch.int64, device="cuda")
    for c in (9, 10, 11, 12):
        u[0, c] = 15 << 39
    u &= ~w                                              # ... and its empty ring
    t_step = timed(lambda: hip.step(x, out=out, generations=g))
    t_fin = timed(lambda: hip.step_contains(x, w, u, g, final=out))
    t_nofin = timed(lambda: hip.step_contains(x, w, u, g))
    hits = int((hip.step_contains(x, w, u, g)[0] > 0).sum().item())
    print(json.dumps({"universes": n, "generations": g, "step_ms": t_step, "step_contains_final_ms": t_fin,
                      "step_contains_first_only_ms": t_nofin, "universes_with_hit": hits,
                      "step_contains_universe_gen_per_s": n * g / t_fin * 1e3}), flush=True)


if __name__ == "__main__":
    main()
