#!/usr/bin/env python3
"""Round-4 box summary: copies what a `tools/gpu_r04_final.sh` run left under
gpurun_out/<tag>/ into profiles/r04/<tag>/ (bench line, rows, footprint
sweep, rehearsal, pytest tail, rocprofv3 stats and PMC csvs) and writes
profiles/r04/<tag>/summary.json with the figures DESIGN.md §5.5 quotes.

PMC conventions (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is reported in
KiB and reads 1/2 of the bytes of a wide streaming read on gfx950 (doubled
here, as `fetch_bytes_x2`); TCC_EA0_RDREQ_{64B,128B} count the fabric read
requests by size, so bytes_by_request = 128 * n128 + 64 * n64 +
32 * (n - n64 - n128) does not depend on that calibration.

Usage: python tools/r04_summary.py <tag>"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    """{kernel short name: {counter: [values per dispatch]}} from a counter_collection.csv"""
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            k = k.split("::")[-1]
            out.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return out


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", "r04", tag)
    os.makedirs(dst, exist_ok=True)
    for name in ("bench.json", "rows_bench.jsonl", "footprint.jsonl", "dist_rehearsal.json", "smoke.log",
                 "trace_c2_bench.json"):
        if os.path.exists(os.path.join(src, name)):
            shutil.copy(os.path.join(src, name), dst)
    summ = {"tag": tag}
    log = os.path.join(src, "pytest_gpu.log")
    if os.path.exists(log):
        tail = open(log).read().strip().splitlines()[-1]
        summ["pytest_gpu"] = tail
        with open(os.path.join(dst, "pytest_gpu_tail.txt"), "w") as f:
            f.write(tail + "\n")
    for stats in glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True):
        rel = os.path.relpath(stats, src).replace(os.sep, "_")
        shutil.copy(stats, os.path.join(dst, rel))
    pmc = {}
    for cc in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        run = os.path.basename(os.path.dirname(cc))
        rel = os.path.relpath(cc, src).replace(os.sep, "_")
        shutil.copy(cc, os.path.join(dst, rel))
        per = {}
        for k, cs in counters(cc).items():
            d = {c: statistics.mean(v) for c, v in cs.items()}
            d["per_dispatch"] = {c: v for c, v in cs.items()}
            d["dispatches"] = max(len(v) for v in cs.values())
            if "FETCH_SIZE" in d:
                d["fetch_bytes_x2"] = d["FETCH_SIZE"] * 1024 * 2
            if "TCC_EA0_RDREQ_sum" in d and "TCC_EA0_RDREQ_128B_sum" in d:
                n, n64, n128 = d["TCC_EA0_RDREQ_sum"], d["TCC_EA0_RDREQ_64B_sum"], d["TCC_EA0_RDREQ_128B_sum"]
                d["bytes_by_request"] = 128 * n128 + 64 * n64 + 32 * (n - n64 - n128)
            if "WRITE_SIZE" in d:
                d["write_bytes"] = d["WRITE_SIZE"] * 1024
            per[k] = d
        pmc[run] = per
    summ["pmc"] = pmc
    b = os.path.join(src, "bench.json")
    if os.path.exists(b):
        line = json.loads(open(b).read().strip().splitlines()[-1])
        r, s = line["roofline"], line.get("secondary") or {}
        summ["bench"] = {
            "value": line["value"], "ms_per_step": line["ms_per_step"], "frac": r["frac"],
            "cache_neutral_frac": (r.get("cache_neutral") or {}).get("frac"),
            "fixed_order_nt_frac": (r.get("fixed_order_nt_back_to_back") or {}).get("frac"),
            "verified": (line.get("verified") or {}).get("ok"),
            "cpu": {k: (line.get("cpu_baseline") or {}).get(k) for k in ("value", "value_1thread", "cores")},
            "config1": {k: ((line.get("cpu_baseline") or {}).get("config1") or {}).get(k)
                        for k in ("reference_ns_per_gen", "facade_ns_per_gen")},
            "config3": {k: (s.get("config3") or {}).get(k) for k in ("kernel_ms", "verified")},
            "config3_frac": ((s.get("config3") or {}).get("roofline") or {}).get("frac"),
            "config3_search_over_plain": ((s.get("config3") or {}).get("search_loop") or {}).get("over_plain_step"),
            "config4": {"kernel_ms": (s.get("config4") or {}).get("kernel_ms"),
                        "frac": ((s.get("config4") or {}).get("roofline") or {}).get("frac"),
                        "cache_neutral_frac": (((s.get("config4") or {}).get("roofline") or {})
                                               .get("cache_neutral") or {}).get("frac"),
                        "verified": (s.get("config4") or {}).get("verified")},
            "config5": {"kernel_ms": (s.get("config5") or {}).get("kernel_ms"),
                        "frac": ((s.get("config5") or {}).get("roofline") or {}).get("frac"),
                        "single_launch_frac": ((s.get("config5") or {}).get("roofline") or {})
                        .get("single_launch_frac"),
                        "cache_neutral_frac": (((s.get("config5") or {}).get("roofline") or {})
                                               .get("cache_neutral") or {}).get("frac")},
            "filter": {t: {op: {"kernel_ms": v[op]["kernel_ms"], "kernel_ms_b2b": v[op]["kernel_ms_b2b"],
                                "objects_per_s": v[op]["objects_per_s"], "frac": v[op]["roofline"]["frac"]}
                           for op in ("filter_1gen", "contains")} | {"verified": v["verified"]}
                       for t, v in ((s.get("filter") or {}).get("targets") or {}).items()},
        }
    rows = os.path.join(src, "rows_bench.jsonl")
    if os.path.exists(rows):
        summ["rows"] = [{k: d.get(k) for k in ("kernel", "objects", "ms", "hbm_frac", "scrubbed_ms",
                                                 "scrubbed_hbm_frac", "objects_per_s", "scrubbed_objects_per_s")}
                        for d in map(json.loads, open(rows)) if "kernel" in d]
    fp = os.path.join(src, "footprint.jsonl")
    if os.path.exists(fp):
        summ["footprint"] = [{k: d[k] for k in ("universes", "b2b_GBps", "scrubbed_GBps", "fixed_b2b_GBps",
                                                "fixed_scrubbed_GBps")} for d in map(json.loads, open(fp))]
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(summ, f, indent=1)
    print(json.dumps(summ, indent=1)[:6000])


if __name__ == "__main__":
    main(sys.argv[1])
