"""LifeWeld::Step one generation in place (k_weld, LifeWeld.hpp:169-186) with
1, 2 or 4 welds per wave, with and without the 7-blocks-per-CU cap and the
XCD-chunked mapping, same process, 1M welds (rows_bench's random welds):
back to back (20 launches in place, median of 3) and alone after a 768 MiB
scrub (median of 10).  Every variant's output after one step equals the
shipped entry point's.  One JSON line per variant; GB/s on 2560 algorithmic
bytes per weld (2048 read, 512 written)."""
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
    n = 1 << 20
    welds = torch.cat([hip.fill_random(n, seed=s).view(n, 1, 64) for s in (11, 12, 13, 14)], 1).reshape(n, 256)
    welds[:, 64:] &= hip.fill_random(3 * n, seed=15).view(n, 192)
    want = hip.weld_step(welds.clone(), 1)
    rt = RT()
    scrub = bench.Scrub(rt)
    cases = [("shipped", lambda w: hip.weld_step(w, 1))]
    for u in (1, 2, 4):
        for res in (0, 7):
            for chunk in (False, True):
                cases.append((f"u{u} res{res}{' xcd' if chunk else ''}",
                              lambda w, u=u, res=res, chunk=chunk: tune.weld_u(w, u, res, chunk)))
    for name, fn in cases:
        w = welds.clone()
        fn(w)
        torch.cuda.synchronize()
        same = bool((w == want).all().item())
        w = welds.clone()
        b2b = bench.back_to_back_ms(rt, lambda a, b: fn(a), w, w)
        scr, _ = bench.scrubbed_ms(rt, lambda a, b: fn(a), w, w, scrub)
        gb = lambda ms: n * 2560 / (ms / 1e3) / 1e9  # noqa: E731
        print(json.dumps({"variant": name, "welds": n, "b2b_ms": b2b, "b2b_frac": gb(b2b) / 8000,
                          "scrubbed_ms": scr, "scrubbed_frac": gb(scr) / 8000, "equal_to_shipped": same}),
              flush=True)


if __name__ == "__main__":
    main()
