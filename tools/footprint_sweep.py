"""What the 1-generation step's "cache-neutral" figure measures, by footprint
(VERDICT r3, next #2): for n = 256K .. 16M universes, one process, the
shipped launch (lifeapi_step_batch_dev)
  b2b       ping-pong, 20 launches back to back, median of 3 runs (the timed
            region's method);
  scrubbed  the same launch alone after a 768 MiB read-only scrub (bench.py
            Scrub), events around the launch only, median of 10 -- HBM only;
  scrub_rw  the same after a read + write scrub (round 4's first form), which
            leaves dirty lines in the cache for the launch to write back;
  fixed     round 3's cache-neutral form: the kernel's code in one fixed
            order with every store nontemporal (tools/tune step_order), b2b;
  fixed_scr the fixed form after a scrub.
One JSON line per size, GB/s on 1024 algorithmic bytes per universe."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
    scrub_rw = bench.Scrub(rt, mode="rw")
    sizes = [1 << k for k in range(18, 25)]
    if "--sizes" in sys.argv:
        sizes = [int(v) for v in sys.argv[sys.argv.index("--sizes") + 1].split(",")]
    for n in sizes:
        a = hip.fill_random(n, seed=4)
        b = torch.empty_like(a)
        big = n > (1 << 22)

        def shipped(x, y):
            hip.step(x, out=y, generations=1)

        def fixed(x, y):
            tune.step_order(x, y, generations=1, reverse=False, nts=True, resident=7 if big else 0,
                            upw=8 if big else 4,
                            plain_bytes=0, xcd_chunk=big)

        gb = lambda ms: n * 1024 / (ms / 1e3) / 1e9  # noqa: E731
        row = {"universes": n, "MiB_per_buffer": n * 512 >> 20, "kernel": hip.step_kernel_name(1, n)}
        row["b2b_ms"] = bench.back_to_back_ms(rt, shipped, a, b)
        row["scrubbed_ms"], row["scrubbed_all"] = bench.scrubbed_ms(rt, shipped, a, b, scrub)
        row["scrub_rw_ms"], _ = bench.scrubbed_ms(rt, shipped, a, b, scrub_rw)
        row["fixed_b2b_ms"] = bench.back_to_back_ms(rt, fixed, a, b)
        row["fixed_scrubbed_ms"], _ = bench.scrubbed_ms(rt, fixed, a, b, scrub)
        for k in ("b2b", "scrubbed", "scrub_rw", "fixed_b2b", "fixed_scrubbed"):
            row[k + "_GBps"] = gb(row[k + "_ms"])
        print(json.dumps(row), flush=True)
        del a, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
