"""The 1-generation step at large batches (16M within 5 %
of the scrubbed 1M rate?): the streaming kernel's code (tuning build
step_order, k_step_ab) at 2M, 4M and 16M universes with 4 or 8 universes per
wave, at most 5 / 6 / 7 / 8 blocks per CU or uncapped, plain or XCD-chunked
block mapping, one order, every store nontemporal; each timed alone after a
768 MiB read-only scrub (median of 10) and back to back (20 ping-pong
launches, median of 3).  Results equal across forms (checked once per size).
One JSON line per (size, form); TB/s on 1024 algorithmic bytes."""
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
    sizes = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1 << 21, 1 << 22, 1 << 24]
    for n in sizes:
        a = hip.fill_random(n, seed=4)
        b = torch.empty_like(a)
        gb = lambda ms: n * 1024 / (ms / 1e3) / 1e9  # noqa: E731
        forms = [("shipped", lambda x, y: hip.step(x, out=y, generations=1))]
        for upw in (4, 8):
            for res in (0, 5, 6, 7, 8):
                for chunk in (False, True):
                    forms.append((f"upw{upw} res{res}{' xcd' if chunk else ''}",
                                  lambda x, y, upw=upw, res=res, chunk=chunk: tune.step_order(
                                      x, y, generations=1, reverse=False, nts=True, resident=res, upw=upw,
                                      plain_bytes=0, xcd_chunk=chunk)))
        for name, fn in forms:
            want = hip.step(a, generations=1)
            fn(a, b)
            torch.cuda.synchronize()
            same = bool((b == want).all().item())
            scr, _ = bench.scrubbed_ms(rt, fn, a, b, scrub)
            b2b = bench.back_to_back_ms(rt, fn, a, b)
            print(json.dumps({"universes": n, "form": name, "scrubbed_ms": scr, "scrubbed_GBps": gb(scr),
                              "b2b_ms": b2b, "b2b_GBps": gb(b2b), "equal": same}), flush=True)
        del a, b, want
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
