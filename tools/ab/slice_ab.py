"""Does the 16M batch's lower HBM rate (7-8 % below 1M from
2 GiB per buffer on) follow the launch's footprint?  The 1-generation step on
16M universes as one launch (shipped) against back-to-back launches over
contiguous slices of the same buffers (512K / 1M / 2M / 4M universes each),
through the product (slices of <= 4M take the small-batch launch) and through
the large-batch kernel's code on every slice (tuning build step_order: 8 per
wave, 7 blocks per CU, XCD-chunked, nontemporal); each step timed alone after
a 768 MiB read-only scrub (median of 10) and back to back (20 ping-pong
steps, median of 3).  Results equal across forms.  One JSON line per form;
TB/s on 1024 algorithmic bytes per universe."""
import json
import os
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
    a = hip.fill_random(n, seed=4)
    b = torch.empty_like(a)
    gb = lambda ms: n * 1024 / (ms / 1e3) / 1e9  # noqa: E731

    def sliced(s, big):
        def fn(x, y):
            for k in range(0, n, s):
                if big:
                    tune.step_order(x[k:k + s], y[k:k + s], generations=1, reverse=False, nts=True, resident=7,
                                    upw=8, plain_bytes=0, xcd_chunk=True)
                else:
                    hip.step(x[k:k + s], out=y[k:k + s], generations=1)
        return fn

    forms = [("one launch (shipped)", lambda x, y: hip.step(x, out=y, generations=1))]
    for s in (1 << 19, 1 << 20, 1 << 21, 1 << 22):
        forms.append((f"slices of {s >> 10}K, product", sliced(s, False)))
        forms.append((f"slices of {s >> 10}K, large-batch code", sliced(s, True)))
    for name, fn in forms:
        want = hip.step(a, generations=1)  # (the timings ping-pong a and b: a changes form to form)
        fn(a, b)
        torch.cuda.synchronize()
        same = bool((b == want).all().item())
        scr, _ = bench.scrubbed_ms(rt, fn, a, b, scrub)
        b2b = bench.back_to_back_ms(rt, fn, a, b)
        print(json.dumps({"universes": n, "form": name, "scrubbed_ms": scr, "scrubbed_GBps": gb(scr),
                          "b2b_ms": b2b, "b2b_GBps": gb(b2b), "equal": same}), flush=True)


if __name__ == "__main__":
    main()
