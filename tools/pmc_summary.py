#!/usr/bin/env python3
"""Turns the rocprofv3 --pmc passes of tools/gpu_profile.sh into
profiles/pmc_traffic.json (HBM bytes per k_step launch, corrected).

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reads ½
of the bytes of a wide coalesced streaming read, and other access widths are
uncalibrated, so both counters are calibrated on a copy kernel with the SAME
access shape as the step kernel (dwordx2, 4 x 512 B per wave, nontemporal;
tools/membw.hip `calib`) whose byte counts are known exactly (512 MiB read +
512 MiB written per launch).  FETCH_SIZE / WRITE_SIZE are in KiB.
"""
from __future__ import annotations

import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mean_counter(path: str, name_sub: str, counter: str) -> tuple[float, int]:
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if name_sub in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {name_sub} in {path}")
    return statistics.mean(vals), len(vals)


def main(prof_dir: str, out_json: str, universes: int = 1 << 20):
    p = lambda *a: os.path.join(prof_dir, *a)  # noqa: E731
    known = 1 << 29  # calib copy: 2^20 universes x 512 B each way
    cf, ncf = mean_counter(p("calib_FETCH_SIZE", "calib_counter_collection.csv"), "k_copy", "FETCH_SIZE")
    cw, ncw = mean_counter(p("calib_WRITE_SIZE", "calib_counter_collection.csv"), "k_copy", "WRITE_SIZE")
    ff, wf = known / (cf * 1024), known / (cw * 1024)

    def entry(name_sub, label, algo, run="pmc", out="bench"):
        sf, nsf = mean_counter(p(f"{run}_FETCH_SIZE", f"{out}_counter_collection.csv"), name_sub, "FETCH_SIZE")
        sw, nsw = mean_counter(p(f"{run}_WRITE_SIZE", f"{out}_counter_collection.csv"), name_sub, "WRITE_SIZE")
        fetch_b, write_b = sf * 1024 * ff, sw * 1024 * wf
        return {"kernel": label, "kernel_name_match": name_sub,
                "raw": {"FETCH_SIZE_KiB_mean": sf, "WRITE_SIZE_KiB_mean": sw, "dispatches": [nsf, nsw]},
                "hbm_read_bytes_per_launch": fetch_b, "hbm_write_bytes_per_launch": write_b,
                "hbm_bytes_per_launch": fetch_b + write_b, "algorithmic_bytes_per_launch": algo,
                "traffic_over_algorithmic": (fetch_b + write_b) / algo}

    c2 = entry("k_step<0, 4, true, 3, true>", "k_step<DPP, U=4, nt loads, nt stores but the last 256 MiB plain, alternating order, rule 3> (config 2: 1M universes x 1 gen)",
               universes * 1024)
    d = dict(c2)
    d["universes"] = universes
    d["calibration"] = {"kernel": "tools/membw.hip calib: dwordx2 U=4 nt copy, 512 MiB each way",
                        "FETCH_SIZE_KiB_mean": cf, "WRITE_SIZE_KiB_mean": cw,
                        "fetch_factor": ff, "write_factor": wf, "dispatches": [ncf, ncw]}
    try:  # config 3: 1024 generations in VGPRs, HBM touched once per universe
        # (its own passes over tools/c3_once.py when present, else the bench's)
        run, out = ("c3", "c3") if os.path.isdir(p("c3_FETCH_SIZE")) else ("pmc", "bench")
        d["config3"] = entry("k_step_split<8, 1, false, 6, -3,",
                             "k_step_split<S=8, G=1, NET 6, asm loop> (rule 11; config 3: 64K universes x 1024 gens)",
                             (1 << 16) * 1024, run, out)
    except (SystemExit, OSError):
        pass
    try:  # config 5 (present when the bench ran its secondaries under the PMC passes)
        d["config5"] = entry("k_refined<1, 0>", "k_refined (config 5: 256K universes, 11 planes in, 3 out)",
                             (1 << 18) * 7168)
    except (SystemExit, OSError):
        pass
    with open(out_json, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    prof = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "prof")
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "pmc_traffic.json")
    main(prof, out)
