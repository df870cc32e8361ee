#!/usr/bin/env python3
"""Iterated LifeWeld::Step: this build's library against a previous build's
(build/ab/liblifeapi_hip_prev.so, natural-layout k_weld for every gens), same
inputs, HIP-event timing; checks both give the same state.  One JSON line per
(library, gens)."""
import ctypes
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # tools/ab: its sibling A/Bs
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/: the live scripts

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import lifeapi_amd.hip as hip  # noqa: E402


def main():
    libs = {"current": hip.lib, "previous": ctypes.CDLL(os.path.join(ROOT, "build", "ab", "liblifeapi_hip_prev.so"))}
    for L in libs.values():
        L.lifeapi_weld_step_batch_dev.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p]
    n = 1 << 18
    w = torch.cat([hip.fill_random(n, seed=s).view(n, 1, 64) for s in (11, 12, 13, 14)], 1).reshape(n, 256)
    w[:, 64:] &= hip.fill_random(3 * n, seed=15).view(n, 192)
    stream = torch.cuda.current_stream().cuda_stream
    for gens in (3, 8, 12, 16, 32, 256):
        outs = {}
        for name, L in libs.items():
            d = w.clone()
            assert L.lifeapi_weld_step_batch_dev(d.data_ptr(), n, gens, stream) == 0
            outs[name] = d
            ms = []
            for _ in range(7):
                x = w.clone()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                L.lifeapi_weld_step_batch_dev(x.data_ptr(), n, gens, stream)
                b.record()
                b.synchronize()
                ms.append(a.elapsed_time(b))
            t = sorted(ms)[3]
            print(json.dumps({"lib": name, "welds": n, "gens": gens, "ms": t,
                              "weld_gen_per_s": n * gens / t * 1e3}), flush=True)
        assert torch.equal(outs["current"], outs["previous"]), gens


if __name__ == "__main__":
    main()
