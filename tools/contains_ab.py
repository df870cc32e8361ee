#!/usr/bin/env python3
"""Fused Step + Contains on the config-3 shape: this build's library against a
previous build's (build/ab/liblifeapi_hip_prev.so), same inputs and process,
HIP-event timing; checks both give the same first generations and states."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import lifeapi_amd.hip as hip  # noqa: E402


def main():
    libs = {"current": hip.lib, "previous": ctypes.CDLL(os.path.join(ROOT, "build", "ab", "liblifeapi_hip_prev.so"))}
    vp = ctypes.c_void_p
    for L in libs.values():
        L.lifeapi_step_contains_batch_dev.argtypes = [vp, vp, vp, vp, vp, ctypes.c_size_t, ctypes.c_uint32, vp]
    n, g = 1 << 16, 1024
    x = hip.fill_random(n, seed=3)
    w = x[0:1].clone()  # a target that occurs: universe 0's own start state
    u = torch.zeros_like(w)
    stream = torch.cuda.current_stream().cuda_stream
    res = {}
    for rnd in range(3):
        for name, L in libs.items():
            first = torch.empty(n, dtype=torch.int32, device="cuda")
            fin = torch.empty_like(x)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            assert L.lifeapi_step_contains_batch_dev(x.data_ptr(), fin.data_ptr(), w.data_ptr(), u.data_ptr(),
                                                     first.data_ptr(), n, g, stream) == 0
            b.record()
            b.synchronize()
            res.setdefault(name, []).append(a.elapsed_time(b))
            res[name + "_out"] = (first, fin)
    assert torch.equal(res["current_out"][0], res["previous_out"][0])
    assert torch.equal(res["current_out"][1], res["previous_out"][1])
    for name in libs:
        ms = sorted(res[name])[1]
        print(json.dumps({"lib": name, "universes": n, "gens": g, "ms_median": ms,
                          "universe_gen_per_s": n * g / ms * 1e3}), flush=True)


if __name__ == "__main__":
    main()
