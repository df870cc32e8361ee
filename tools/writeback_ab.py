"""Where the 1M-16M gap of the step's HBM-only rate goes: a
launch timed alone after a scrub can leave up to 256 MiB of its writes dirty
in the memory-side Infinity Cache, written back to HBM only after its end
event.  For n = 1M .. 16M universes, one process, the shipped 1-generation
step (ping-pong buffers):
  launch_ms       the launch alone after a 768 MiB read-only scrub (bench.py
                  scrubbed_ms's method);
  scrub_after_ms  the next scrub, timed: it evicts whatever the launch left
                  dirty, so it pays those write-backs;
  scrub_clean_ms  the same scrub after a scrub (nothing dirty), the baseline;
  inclusive_ms    launch_ms + scrub_after_ms - scrub_clean_ms: the launch with
                  its deferred write-backs.
Medians of 10.  One JSON line per size, GB/s on 1024 algorithmic bytes."""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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


def timed(rt, fn):
    e0, e1 = rt.event(), rt.event()
    e0.record(rt.stream)
    fn()
    e1.record(rt.stream)
    return e0, e1


def main():
    rt = RT()
    scrub = bench.Scrub(rt)
    sizes = [1 << k for k in (20, 21, 22, 23, 24)]
    if len(sys.argv) > 1:
        sizes = [int(v) for v in sys.argv[1].split(",")]
    for n in sizes:
        bufs = [hip.fill_random(n, seed=4), hip.empty_universes(n)]
        launch, after, clean = [], [], []
        for k in range(13):
            x, y = bufs[k % 2], bufs[1 - k % 2]
            scrub()
            s0 = timed(rt, scrub)  # a scrub after a scrub: nothing dirty
            l0 = timed(rt, lambda: hip.step(x, out=y, generations=1))
            a0 = timed(rt, scrub)  # evicts what the launch left dirty
            a0[1].synchronize()
            if k >= 3:
                clean.append(s0[0].elapsed_time(s0[1]))
                launch.append(l0[0].elapsed_time(l0[1]))
                after.append(a0[0].elapsed_time(a0[1]))
        lm, am, cm = (statistics.median(v) for v in (launch, after, clean))
        inc = lm + am - cm
        gb = lambda ms: n * 1024 / (ms / 1e3) / 1e9  # noqa: E731
        print(json.dumps({"universes": n, "kernel": hip.step_kernel_name(1, n), "launch_ms": lm,
                          "scrub_after_ms": am, "scrub_clean_ms": cm, "inclusive_ms": inc,
                          "deferred_MiB_at_launch_rate": (am - cm) * n * 1024 / lm / 2**20,
                          "launch_GBps": gb(lm), "inclusive_GBps": gb(inc)}), flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
