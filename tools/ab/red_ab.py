"""A/B of the per-universe reductions (k_pop, k_hash, k_contains): one JSON
line per kernel, median of 15 event-timed calls on 1M universes, plus a digest
of the results.  profiles/r01/red_ab.jsonl holds the sweep that chose their
launch (a temporary build read LIFEAPI_RED_BPC = blocks per CU, 0 = full grid,
and LIFEAPI_RED_NT = nontemporal loads from the environment)."""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import lifeapi_amd.hip as hip  # noqa: E402
from rows_bench import timed  # noqa: E402


def main():
    n = 1 << 20
    x = hip.fill_random(n, seed=7)
    w = x[:1].clone()
    ref = (hip.pop(x).cpu(), hip.hashes(x).cpu(), hip.contains(x, w, w).cpu())
    for name, nbytes, fn in (("k_pop", 516, lambda: hip.pop(x)), ("k_hash", 520, lambda: hip.hashes(x)),
                             ("k_contains", 513, lambda: hip.contains(x, w, w))):
        ms = timed(fn, reps=15)
        print(json.dumps({"kernel": name, "ms": ms,
                          "hbm_frac": n * nbytes / (ms / 1e3) / 8e12}), flush=True)
    print(json.dumps({"digest": [int(t.double().sum()) for t in ref]}), flush=True)


if __name__ == "__main__":
    main()
