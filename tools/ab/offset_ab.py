"""Does the distance between the ping-pong pair matter at large batches?
The shipped 1-generation step ping-ponged between `a` and `b`, where `b`
starts `off` KiB past the end of `a` inside one allocation (off = 0: the two
buffers are adjacent), at 1M and 16M universes; each launch alone after a
768 MiB read-only scrub (median of 10) and back to back (20 launches, median
of 3).  If the read and write streams share DRAM banks at some distances,
the rate moves with `off`.  One JSON line per (size, offset)."""
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
    for n in (1 << 20, 1 << 24):
        for off_kib in (0, 1, 2, 4, 8, 64, 1024, 4096, 32768):
            extra = off_kib * 2  # universes of 512 B
            buf = torch.empty(((2 * n + extra), 64), dtype=torch.int64, device="cuda")
            a, b = buf[:n], buf[n + extra: 2 * n + extra]
            hip.fill_random(n, seed=4, out=a)
            fn = lambda x, y: hip.step(x, out=y, generations=1)  # noqa: E731
            scr, _ = bench.scrubbed_ms(rt, fn, a, b, scrub)
            b2b = bench.back_to_back_ms(rt, fn, a, b)
            gb = lambda ms: n * 1024 / (ms / 1e3) / 1e9  # noqa: E731
            print(json.dumps({"universes": n, "offset_KiB": off_kib, "scrubbed_GBps": gb(scr), "b2b_GBps": gb(b2b),
                              "scrubbed_ms": scr, "b2b_ms": b2b}), flush=True)
            del buf, a, b
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
