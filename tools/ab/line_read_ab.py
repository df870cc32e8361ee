"""The small-target light cone against its access shape alone: Contains and
the 1-generation filter (product) on 1M universes for the rows_bench 2x2
block + ring target (one 128-byte line per universe), next to the tuning
build's k_line_read (the same line of every universe read, a uint32
written, nothing computed) on lines 0 and 1; each timed alone after a 768
MiB read-only scrub (median of 10) and back to back (median of 3 x 20).
One JSON line per kernel; TB/s on the bytes moved (128 read + 4 or 1
written per universe)."""
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
    n = 1 << 20
    x = hip.fill_random(n, seed=7)
    w = x[:1].clone()
    bw, bu = torch.zeros_like(w), torch.zeros_like(w)
    bw[0, 10] = bw[0, 11] = 3 << 40
    bu[0, 9:13] = 15 << 39
    bu &= ~bw
    rows = [("k_line_read line 0, 16 lanes per universe", 132, lambda a, b: tune.line_read(x, 0)),
            ("k_line_read line 0, 4 lanes per universe", 132, lambda a, b: tune.line_read(x, 4)),
            ("k_line_read line 1, 4 lanes per universe", 132, lambda a, b: tune.line_read(x, 5)),
            ("Contains, block + ring (product)", 129, lambda a, b: hip.contains(x, bw, bu)),
            ("filter 1 gen, block + ring (product)", 132, lambda a, b: hip.step_contains(x, bw, bu, 1))]
    for name, nbytes, fn in rows:
        scr, _ = bench.scrubbed_ms(rt, fn, x, x, scrub)
        b2b = bench.back_to_back_ms(rt, fn, x, x)
        print(json.dumps({"kernel": name, "objects": n, "bytes_per_object": nbytes, "scrubbed_ms": scr,
                          "scrubbed_GBps": n * nbytes / scr / 1e6, "b2b_ms": b2b,
                          "b2b_GBps": n * nbytes / b2b / 1e6}), flush=True)


if __name__ == "__main__":
    main()
