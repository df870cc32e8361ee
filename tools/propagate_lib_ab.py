"""Propagate and StabiliseOptions through the product ABI of whichever
library LIFEAPI_HIP_LIB names (tools/gpu_r06p.sh runs it on two builds in
alternation): 1M LifeStables, a search's next node and fresh options
(rows_bench.stable_inputs / stable_next_node), each launch on its own fresh
copy, back to back (4 per timing, median of 7) and alone after a 768 MiB scrub
(median of 8), plus a checksum of the result planes and flags so that two
builds' answers can be compared.  One JSON line per input."""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
import lifeapi_amd.hip as hip  # noqa: E402
from rows_bench import stable_inputs, stable_next_node  # noqa: E402


class RT:
    kind = "hip"

    def __init__(self):
        self.device = torch.device("cuda", 0)
        self.stream = torch.cuda.current_stream()


def checksum(planes, flags):
    w = planes.view(torch.int64).reshape(-1)
    k = torch.arange(1, w.numel() + 1, device=w.device, dtype=torch.int64)
    return int((w * k).sum().item()) ^ int((flags.to(torch.int64) * k[: flags.numel()]).sum().item())


def main():
    n = int(os.environ.get("N", str(1 << 20)))
    scrub = bench.Scrub(RT())
    st = stable_inputs(n)
    lib = os.path.basename(os.environ.get("LIFEAPI_HIP_LIB") or hip.LIB_PATH)
    for which, src in (("next node", stable_next_node(st)), ("fresh options", st)):
        row = {"lib": lib, "input": which, "objects": n}
        works = [src.clone() for _ in range(4)]
        for name in ("propagate", "stabilise"):
            works[0].copy_(src)
            flags = hip.stable_pass(works[0], name)
            torch.cuda.synchronize()
            row[f"{name}_checksum"] = checksum(works[0], flags)
            ms = []
            for _ in range(7):
                for wk in works:
                    wk.copy_(src)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for wk in works:
                    hip.stable_pass(wk, name)
                b.record()
                b.synchronize()
                ms.append(a.elapsed_time(b) / len(works))
            alone = []
            for k in range(10):
                works[0].copy_(src)
                scrub()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                hip.stable_pass(works[0], name)
                b.record()
                b.synchronize()
                if k >= 2:
                    alone.append(a.elapsed_time(b))
            row[name] = {"ms": statistics.median(ms), "ms_alone": statistics.median(alone)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
