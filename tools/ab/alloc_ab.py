"""Is the 16M step's lower HBM rate a property of the large allocation?
(tools/ab/slice_ab.py: 1M-universe slices of the 8 GiB buffers run at the
16M rate, 6.0-6.1 TB/s, where a 1M batch in its own 512 MiB buffers runs
at 6.8.)  The same 16M universes as one launch on one pair of 8 GiB buffers,
as launches over its 1M-universe slices, and as launches over 16 pairs of
separately allocated 512 MiB buffers (one hipMalloc each); each step timed
alone after a 768 MiB read-only scrub (median of 10) and back to back (20
ping-pong steps, median of 3).  One JSON line per form; TB/s on 1024
algorithmic bytes per universe."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import lifeapi_amd.hip as hip  # noqa: E402


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
    n, s = 1 << 24, 1 << 20
    gb = lambda ms: n * 1024 / (ms / 1e3) / 1e9  # noqa: E731
    a = hip.fill_random(n, seed=4)
    b = torch.empty_like(a)
    # 16 pairs of separate buffers holding the same universes
    pa = [a[k:k + s].clone() for k in range(0, n, s)]
    pb = [torch.empty_like(t) for t in pa]

    def one(x, y):
        hip.step(x, out=y, generations=1)

    def sliced(x, y):
        for k in range(0, n, s):
            hip.step(x[k:k + s], out=y[k:k + s], generations=1)

    def separate(x, y):
        for xs, ys in zip(x, y):
            hip.step(xs, out=ys, generations=1)

    for name, fn, x, y in (("one launch, 8 GiB buffers", one, a, b), ("1M slices, 8 GiB buffers", sliced, a, b),
                           ("1M launches, 16 pairs of 512 MiB buffers", separate, pa, pb)):
        scr, _ = bench.scrubbed_ms(rt, fn, x, y, scrub)
        b2b = bench.back_to_back_ms(rt, fn, x, y)
        print(json.dumps({"universes": n, "form": name, "scrubbed_ms": scr, "scrubbed_GBps": gb(scr),
                          "b2b_ms": b2b, "b2b_GBps": gb(b2b)}), flush=True)
    # results: the separate buffers step the same universes
    want = hip.step(a, generations=1)
    sep = torch.cat([hip.step(t, generations=1) for t in [a[k:k + s].clone() for k in range(0, n, s)]])
    print(json.dumps({"equal": bool((sep == want).all().item())}), flush=True)


if __name__ == "__main__":
    main()
