#!/usr/bin/env python3
"""Host-pointer path (lifeapi_step_batch on pageable numpy arrays, the C++
facade's StepBatch) against the PCIe copy rates torch gets for the same
bytes (pageable and pinned, each direction).  One JSON line per case."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lifeapi_amd.hip as hip  # noqa: E402


def wall(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    rng = np.random.default_rng(5)
    x = rng.integers(0, 2**63, size=(n, 64), dtype=np.uint64)
    nbytes = x.nbytes
    dev = torch.empty(n * 64, dtype=torch.int64, device="cuda")
    out = np.zeros_like(x)  # touched: no page faults inside the timed calls
    for gens in (1, 1024):
        if gens == 1024 and n > (1 << 16):
            continue
        for case, kw in (("step_host", {"out": out}), ("step_host_inplace", {"out": x}),
                         ("step_host_fresh_out", {})):
            t = wall(lambda: hip.step_host(x, generations=gens, **kw))
            print(json.dumps({"case": case, "universes": n, "gens": gens, "s": t,
                              "universe_gen_per_s": n * gens / t,
                              "GBps_round_trip": 2 * nbytes / t / 1e9}), flush=True)
        def pin_each_call():  # registration inside the timed call, as a library-side pin would
            with hip.host_pinned(x, out):
                hip.step_host(x, generations=gens, out=out)
        t = wall(pin_each_call)
        print(json.dumps({"case": "step_host_register_per_call", "universes": n, "gens": gens, "s": t,
                          "universe_gen_per_s": n * gens / t}), flush=True)
        with hip.host_pinned(x, out):  # page-locked once (lifeapi_host_register)
            for case, o in (("step_host_pinned", out), ("step_host_pinned_inplace", x)):
                t = wall(lambda: hip.step_host(x, generations=gens, out=o))
                print(json.dumps({"case": case, "universes": n, "gens": gens, "s": t,
                                  "universe_gen_per_s": n * gens / t,
                                  "GBps_round_trip": 2 * nbytes / t / 1e9}), flush=True)
    xt = torch.from_numpy(x.view(np.int64).reshape(-1))
    pin = xt.pin_memory()
    for name, src, dst in (("h2d_pageable", xt, dev), ("h2d_pinned", pin, dev),
                           ("d2h_pageable", dev, xt), ("d2h_pinned", dev, pin)):
        t = wall(lambda: dst.copy_(src, non_blocking=True))
        print(json.dumps({"case": name, "bytes": nbytes, "s": t, "GBps": nbytes / t / 1e9}), flush=True)
    # both directions at once on two streams: is the link full duplex?
    dev2 = torch.empty_like(dev)
    pin2 = torch.empty_like(pin).pin_memory()
    xt2 = xt.clone()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    cases = [("duplex_pinned", pin, pin2), ("duplex_pageable", xt, xt2)]
    for name, a, b in cases:
        def both():
            with torch.cuda.stream(s1):
                dev.copy_(a, non_blocking=True)
            with torch.cuda.stream(s2):
                b.copy_(dev2, non_blocking=True)
        t = wall(both)
        print(json.dumps({"case": name, "bytes_each_way": nbytes, "s": t,
                          "GBps_total": 2 * nbytes / t / 1e9}), flush=True)


    # the same duplex copy on hipHostRegister-ed (not hipHostMalloc-ed) memory
    with hip.host_pinned(xt.numpy(), xt2.numpy()):
        t = wall(both_fn(dev, dev2, xt, xt2, s1, s2))
        print(json.dumps({"case": "duplex_registered", "bytes_each_way": nbytes, "s": t,
                          "GBps_total": 2 * nbytes / t / 1e9}), flush=True)
    # step_host on hipHostMalloc-ed arrays (torch pinned tensors)
    pa, pb = pin.numpy().view(np.uint64), pin2.numpy().view(np.uint64)
    t = wall(lambda: hip.step_host(pa, generations=1, out=pb))
    print(json.dumps({"case": "step_host_hostmalloc", "universes": n, "s": t,
                      "universe_gen_per_s": n / t, "GBps_round_trip": 2 * nbytes / t / 1e9}), flush=True)


def both_fn(dev, dev2, a, b, s1, s2):
    def both():
        with torch.cuda.stream(s1):
            dev.copy_(a, non_blocking=True)
        with torch.cuda.stream(s2):
            b.copy_(dev2, non_blocking=True)
    return both


if __name__ == "__main__":
    main()
