"""Same-process, interleaved A/B for batches above 4M universes: the shipped
large-batch launch (4 universes per wave, at most 7 blocks per CU, each XCD
a contiguous eighth, one order, nontemporal) against the same with 8
universes per wave (and with 6 blocks), at 4M (where the small-batch
alternating form ships), 8M and 16M; back to back (20 ping-pong launches) in
7 interleaved rounds, plus a read-only-scrubbed single launch per round.
Medians; TB/s on 1024 algorithmic bytes."""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import bench  # noqa: E402
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip as tune  # noqa: E402


class RT:
    kind = "hip"

    def __init__(self):
        self.device = torch.device("cuda", 0)
        self.stream = torch.cuda.current_stream()

    @staticmethod
    def event():
        return torch.cuda.Event(enable_timing=True)


def main():
    rt = RT()
    scrub = bench.Scrub(rt)
    for n in (1 << 22, 1 << 23, 1 << 24):
        a = hip.fill_random(n, seed=4)
        b = torch.empty_like(a)
        forms = {"shipped": lambda x, y: hip.step(x, out=y, generations=1)}
        for upw, res in ((4, 7), (8, 7), (8, 6)):
            forms[f"upw{upw} res{res} xcd"] = (lambda x, y, upw=upw, res=res: tune.step_order(
                x, y, generations=1, reverse=False, nts=True, resident=res, upw=upw, plain_bytes=0, xcd_chunk=True))
        eq = {}
        for name, fn in forms.items():
            want = hip.step(a, generations=1)
            fn(a, b)
            torch.cuda.synchronize()
            eq[name] = bool((b == want).all().item())
        res = {k: {"b2b": [], "scr": []} for k in forms}
        for _ in range(7):
            for name, fn in forms.items():
                res[name]["b2b"].append(bench.back_to_back_ms(rt, fn, a, b, repeats=1))
                res[name]["scr"].append(bench.scrubbed_ms(rt, fn, a, b, scrub, reps=3, warm=1)[0])
        gb = lambda ms: n * 1024 / (ms / 1e3) / 1e9  # noqa: E731
        for name in forms:
            m, s = statistics.median(res[name]["b2b"]), statistics.median(res[name]["scr"])
            print(json.dumps({"universes": n, "form": name, "b2b_ms": m, "b2b_GBps": gb(m), "scrubbed_ms": s,
                              "scrubbed_GBps": gb(s), "b2b_all": res[name]["b2b"], "equal": eq[name]}), flush=True)
        del a, b, want
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
