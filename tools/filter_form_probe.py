"""Which launch form the shipped search filter takes, call by call, on a
whole-board target (bench.py secondary.filter's timing: each launch alone
after a scrub): run under `rocprofv3 --kernel-trace` and read the
k_cone_adapt instantiations in order (DMA form: template arguments ending
`true, true>`).  Prints the per-call times."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import lifeapi_amd.hip as hip  # noqa: E402


class RT:
    kind = "hip"
    device = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()

    @staticmethod
    def event():
        return torch.cuda.Event(enable_timing=True)


def main():
    rt = RT()
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        t = json.load(f)["digests"]["config2_filter"]["targets"]["whole_board"]
    x = hip.fill_random(1 << 20, seed=2)
    tw, tu = (torch.from_numpy(np.array([[int(v, 16) for v in t[k]]], dtype=np.uint64).view(np.int64)).cuda()
              for k in ("wanted", "unwanted"))
    scrub = bench.Scrub(rt)
    for rnd in range(3):
        ms, allms = bench.scrubbed_ms(rt, lambda a, b: hip.step_contains(a, tw, tu, 1, stream=rt.stream), x, x, scrub)
        print(json.dumps({"round": rnd, "median_ms": ms, "all": allms}), flush=True)


if __name__ == "__main__":
    main()
