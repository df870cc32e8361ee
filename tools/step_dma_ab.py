"""A/B: the 1-generation streaming step with its universes moved through LDS
(k_step_dma, tuning build upw 64 + U: 16-byte global_load_lds in, 8-byte
stores; 96 + U: 16-byte stores through the image too) against the shipped
k_step, same process, ping-pong as bench.py's timed region: 1M universes
(the batch-keyed alternating order, the last min(256 MiB, half) stored plain,
every slot) and 16M (one order, nontemporal, 8 per wave, 7 blocks per CU, XCD
chunks) -- each form with the shipped launch policy of that size.  Per form:
back to back (20 launches, median of 5 runs) and HBM-only (bench.py
hbm_only_ms: alone after a scrub, deferred write-backs included); results
checked against the shipped launch.  One JSON line per (size, form)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import bench  # noqa: E402
import lifeapi_amd.hip as hip  # noqa: E402
import tune_hip  # noqa: E402


class RT:
    kind = "hip"
    device = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()

    @staticmethod
    def event():
        return torch.cuda.Event(enable_timing=True)


def main():
    rt = RT()
    scrub = bench.Scrub(rt)
    for n in (1 << 20, 1 << 24):
        big = n > (1 << 22)
        a0 = hip.fill_random(n, seed=4)
        a = a0.clone()
        b = torch.empty_like(a)
        want = hip.step(a0)
        forms = {"shipped": None}
        for code, name in ((64, "dma"), (96, "dma_wide")):
            forms[name] = code + (8 if big else 4)
        flip = [False]
        for name, code in forms.items():
            if code is None:
                fn = lambda x, y: hip.step(x, out=y, generations=1)  # noqa: E731
            else:
                def fn(x, y, code=code):
                    if big:
                        tune_hip.step_order(x, y, 1, reverse=False, nts=True, resident=7, upw=code, plain_bytes=0,
                                            xcd_chunk=True)
                    else:
                        rev = flip[0]
                        flip[0] = not flip[0]
                        tune_hip.step_order(x, y, 1, reverse=rev, nts=True, resident=0, upw=code,
                                            plain_bytes=min(256 << 20, n * 512 // 2))
            a.copy_(a0)  # (the timings below ping-pong a and b)
            got = torch.empty_like(a)
            fn(a, got)
            torch.cuda.synchronize()
            exact = bool(torch.equal(got, want))
            b2b = sorted(bench.back_to_back_ms(rt, fn, a, b, reps=20, warm=5, repeats=1) for _ in range(5))[2]
            h = bench.hbm_only_ms(rt, fn, a, b, scrub)
            gb = lambda ms: n * 1024 / (ms / 1e3) / 1e9  # noqa: E731
            print(json.dumps({"universes": n, "form": name, "exact": exact, "b2b_ms": b2b, "b2b_frac": gb(b2b) / 8000,
                              "hbm_only_ms": h["inclusive_ms"], "hbm_only_frac": gb(h["inclusive_ms"]) / 8000,
                              "launch_after_scrub_ms": h["launch_ms"]}), flush=True)
        del a, a0, b, want
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
