"""Throughput of the RLE batch I/O kernels (k_rle lengths + write, k_parse_rle)
on 256K universes of three densities; prints one JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lifeapi_amd.hip as hip  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b))
    return sorted(ms)[len(ms) // 2]


def main():
    n = 1 << 18
    for name, k in (("density 0.5", 1), ("density 0.125", 3), ("density 0.0039", 8)):
        x = hip.fill_random(n, seed=90)
        for j in range(1, k):
            x &= hip.fill_random(n, seed=90 + j)
        text, offs = hip.rle(x)
        t_rle = timed(lambda: hip.rle(x))
        t_parse = timed(lambda: hip.parse_rle(text, offs))
        nbytes = text.numel()
        print(json.dumps({"case": name, "universes": n, "text_bytes": nbytes,
                          "rle_ms": t_rle, "rle_patterns_per_s": n / t_rle * 1e3,
                          "rle_text_GBps": nbytes / t_rle / 1e6,
                          "parse_ms": t_parse, "parse_patterns_per_s": n / t_parse * 1e3,
                          "parse_text_GBps": nbytes / t_parse / 1e6}), flush=True)


if __name__ == "__main__":
    main()
