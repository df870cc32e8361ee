"""A/B: the LifeStable passes with the next LifeStable fetched into LDS while
the wave works on the current one (k_stable_dma, tuning build) against the
shipped k_stable, same process, 1M LifeStables (--n), three inputs:
  still      rows_bench.stable_inputs: still lifes around an unknown window
             with fresh options (every column changes);
  next       rows_bench.stable_next_node: the same propagated, then one
             unknown cell decided (a search's next node; a few columns change);
  random     random planes (every pass changes most lines).
Forms (nt fetch, waits counted so the stores stay in flight): dma_loop, the
looping grid; dma_uU, a grid of n / U waves, each a contiguous run of U
LifeStables; wide_u1: U = 1 with the changed lines stored 16 bytes per lane
through the LDS image; _capC: at most C blocks resident per CU.
Per (input, pass, form): 4 launches back to back, each on its own fresh copy,
between one pair of events (/ 4), median of 7; results checked bit for bit
against the shipped pass (planes and flags).  One JSON line per row."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip  # noqa: E402
from rows_bench import stable_inputs, stable_next_node  # noqa: E402


def timed(run, src, works, reps=7):
    ms = []
    for _ in range(reps):
        for w in works:
            w.copy_(src)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for w in works:
            run(w)
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b) / len(works))
    return sorted(ms)[len(ms) // 2]


def main():
    n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 1 << 20
    # forms: label -> (tuning pass offset, blocks per CU cap, passes it exists for)
    # forms: label -> (tuning pass offset, blocks per CU cap, LifeStables per wave (0: looping grid), passes)
    forms = {"dma_u1": (16, 0, 1, range(6)), "dma_u2": (16, 0, 2, range(6)),
             "wide_u1": (32, 0, 1, range(6)), "wide_u1_cap3": (32, 3, 1, range(6)), "wide_u1_cap5": (32, 5, 1, range(6))}
    passes = sys.argv[sys.argv.index("--passes") + 1].split(",") if "--passes" in sys.argv else list(hip.STABLE_PASSES)
    st = stable_inputs(n)
    inputs = {"still": st, "next": stable_next_node(st),
              "random": hip.fill_random(10 * n, seed=31).view(n, 640)}
    works = [torch.empty_like(st) for _ in range(4)]
    chk = torch.empty_like(st)
    for iname, src in inputs.items():
        for pname in passes:
            w = hip.STABLE_PASSES.index(pname)
            chk.copy_(src)
            want_flags = hip.stable_pass(chk, pname)
            want = chk.clone()
            row = {"input": iname, "pass": pname, "objects": n}
            row["shipped_ms"] = timed(lambda x: hip.stable_pass(x, pname), src, works)
            for label, (off, cap, upw, which) in forms.items():
                if w not in which:
                    continue
                chk.copy_(src)
                f = tune_hip.stable_pass(chk, off + w, cap, upw=upw)
                torch.cuda.synchronize()
                ok = bool(torch.equal(chk, want)) and bool(torch.equal(f, want_flags))
                row[f"{label}_ms"] = timed(lambda x: tune_hip.stable_pass(x, off + w, cap, upw=upw), src, works)
                row[f"{label}_exact"] = ok
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
