"""PMC of the LifeStable rows: the bytes each pass really moves and the VALU
it issues, per LifeStable, so that tools/rows_bench.py prices every LifeStable
row on measured bytes.

  python tools/pmc_rows.py run
      the kernel driver, run under rocprofv3 (tools/gpu_r05_pmc.sh): on 1M
      LifeStables, each pass (sync, options, signal, step, propagate,
      stabilise) on the two rows_bench inputs (still: fresh options on still
      lifes, every column changes; next: a search's next node, a few columns
      change) and Vulnerable(), 3 launches each, every one on a fresh copy
      and after a 768 MiB scrub (bench.py Scrub), so each dispatch's counters
      are those of one cold launch.  Prints its manifest (one JSON line per
      workload, in dispatch order).
  python tools/pmc_rows.py summarize FETCH_DIR WRITE_DIR SQ_DIR MANIFEST
      the rocprofv3 CSVs of three passes (FETCH_SIZE; WRITE_SIZE; SQ_INSTS_VALU
      + SQ_WAVES) -> one JSON object: per workload the fetched and written
      bytes and the VALU instructions per LifeStable.

Corrections: FETCH_SIZE x 2 and WRITE_SIZE x 1 (MI355X_MICROARCH.md, HBM;
the same factors the dwordx2 nt calibration copy of profiles/pmc_traffic.json
measured: 1.9999 and 1.0000 -- the passes' loads and stores are that shape).
Both counters count L2-to-fabric bytes, so Infinity Cache hits count too; the
scrub before every launch keeps those to the launch's own re-reads."""
import csv
import glob
import re
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FETCH_FACTOR, WRITE_FACTOR = 2.0, 1.0
N = 1 << 20
REPS = 3


def run():
    import torch
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench
    import lifeapi_amd.hip as hip
    from rows_bench import stable_inputs, stable_next_node

    class RT:
        kind = "hip"
        device = torch.device("cuda", 0)
        stream = torch.cuda.current_stream()

    scrub = bench.Scrub(RT())
    st = stable_inputs(N)
    inputs = {"still": st, "next": stable_next_node(st)}
    w = torch.empty_like(st)
    torch.cuda.synchronize()
    for iname, src in inputs.items():
        for pname in hip.STABLE_PASSES:
            for _ in range(REPS):
                w.copy_(src)
                scrub()
                hip.stable_pass(w, pname)
            print(json.dumps({"workload": f"k_stable {pname} ({iname})", "match": r"k_stable(_dma)?<",
                              "dispatches": REPS, "objects": N}), flush=True)
    for _ in range(REPS):
        scrub()
        hip.stable_vulnerable(st)
    print(json.dumps({"workload": "k_stable_vulnerable (still)", "match": r"k_stable_vulnerable",
                      "dispatches": REPS, "objects": N}), flush=True)
    torch.cuda.synchronize()


def _rows(d):
    paths = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not paths:
        raise SystemExit(f"no counter_collection.csv under {d}")
    by_disp = {}
    with open(paths[0]) as f:
        for r in csv.DictReader(f):
            k = int(r["Dispatch_Id"])
            e = by_disp.setdefault(k, {"name": r["Kernel_Name"], "ctr": {}})
            e["ctr"][r["Counter_Name"]] = e["ctr"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [by_disp[k] for k in sorted(by_disp)]


def _assign(rows, manifest):
    """per workload, the counters of its dispatches: walk the dispatches in
    order, each workload taking the next `dispatches` whose name matches"""
    out, i = [], 0
    for m in manifest:
        got = []
        while len(got) < m["dispatches"]:
            if i >= len(rows):
                raise SystemExit(f"ran out of dispatches at {m['workload']}")
            r = rows[i]
            i += 1
            if re.search(m["match"], r["name"]):
                got.append(r["ctr"])
        out.append(got)
    return out


def summarize(fetch_dir, write_dir, sq_dir, manifest_path):
    with open(manifest_path) as f:
        manifest = [json.loads(ln) for ln in f if ln.startswith("{")]
    fetch, write, sq = (_assign(_rows(d), manifest) for d in (fetch_dir, write_dir, sq_dir))
    res = {"source": "tools/pmc_rows.py (rocprofv3 --pmc, one counter group per run; each launch alone after a "
                     "768 MiB scrub, on a fresh copy)",
           "corrections": {"FETCH_SIZE": FETCH_FACTOR, "WRITE_SIZE": WRITE_FACTOR,
                           "why": "MI355X_MICROARCH.md HBM: FETCH_SIZE reads half the bytes of wide streaming "
                                  "reads; the dwordx2 nt calibration copy (profiles/pmc_traffic.json) measured "
                                  "1.9999 / 1.0000"},
           "objects": N, "rows": {}}
    for m, fe, wr, s in zip(manifest, fetch, write, sq):
        n = m["objects"]
        fb = statistics.median(c["FETCH_SIZE"] for c in fe) * 1024 * FETCH_FACTOR / n
        wb = statistics.median(c["WRITE_SIZE"] for c in wr) * 1024 * WRITE_FACTOR / n
        valu = statistics.median(c["SQ_INSTS_VALU"] for c in s) / n
        waves = statistics.median(c["SQ_WAVES"] for c in s)
        res["rows"][m["workload"]] = {"fetch_bytes_per_object": fb, "write_bytes_per_object": wb,
                                      "hbm_bytes_per_object": fb + wb, "valu_per_object": valu,
                                      "waves_per_launch": waves, "dispatches": m["dispatches"]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(*sys.argv[2:6])
