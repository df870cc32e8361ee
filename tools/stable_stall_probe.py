"""Where a LifeStable pass's wave cycles go: SQ counters of PropagateStep and
Propagate on a search's next node (rows_bench.stable_next_node, 1M), shipped
kernels and the tuning build's LDS-prefetch forms (k_stable_dma, U = 1 / 2
LifeStables per wave), each launch alone on a fresh copy after a 768 MiB
scrub, 3 launches per workload.

  python tools/stable_stall_probe.py run
      the driver, run under rocprofv3 --pmc (tools/gpu_stall_probe.sh); prints
      its manifest (one JSON line per workload, dispatch order).
  python tools/stable_stall_probe.py summarize MANIFEST DIR...
      the counter CSVs of the passes -> one JSON line per workload: per
      LifeStable the VALU / SALU instructions, and the wave-cycle split
      (MI355X_MICROARCH.md: SQ_WAIT_ANY = parked on s_waitcnt, SQ_WAIT_INST_ANY
      = issue stall, SQ_ACTIVE_INST_ANY = issuing; quad-cycles, summed over
      waves), the VALU-active share, and the held clock (GRBM_GUI_ACTIVE / 8 /
      kernel time)."""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 1 << 20
REPS = 3


def run():
    import torch
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
    import bench
    import lifeapi_amd.hip as hip
    import tune_hip
    from rows_bench import stable_inputs, stable_next_node

    class RT:
        kind = "hip"
        device = torch.device("cuda", 0)
        stream = torch.cuda.current_stream()

    scrub = bench.Scrub(RT())
    src = stable_next_node(stable_inputs(N))
    w = torch.empty_like(src)
    torch.cuda.synchronize()
    for pname in ("step", "propagate"):
        p = hip.STABLE_PASSES.index(pname)
        forms = {"shipped": lambda x: hip.stable_pass(x, pname),
                 "dma_u1": lambda x: tune_hip.stable_pass(x, 16 + p, 0, upw=1),
                 "dma_u2": lambda x: tune_hip.stable_pass(x, 16 + p, 0, upw=2),
                 "plain": lambda x: tune_hip.stable_pass(x, p, 0)}
        for fname, fn in forms.items():
            for _ in range(REPS):
                w.copy_(src)
                scrub()
                fn(w)
            print(json.dumps({"workload": f"{pname} (next) {fname}", "dispatches": REPS, "objects": N}), flush=True)
    torch.cuda.synchronize()


def summarize(manifest, dirs):
    disp = {}
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for r in csv.DictReader(f):
                    if "k_stable" not in r["Kernel_Name"]:
                        continue
                    key = (d, int(r["Dispatch_Id"]))
                    e = disp.setdefault(key, {"ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), "c": {}})
                    e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    per_dir = {}
    for (d, k), e in sorted(disp.items()):
        per_dir.setdefault(d, []).append(e)
    work = [json.loads(line) for line in open(manifest) if line.strip()]
    out = []
    pos = {d: 0 for d in per_dir}
    for wl in work:
        ctr, ns = {}, []
        for d, lst in per_dir.items():
            seg = lst[pos[d]:pos[d] + wl["dispatches"]]
            pos[d] += wl["dispatches"]
            for e in seg:
                ns.append(e["ns"])
                for c, v in e["c"].items():
                    ctr.setdefault(c, []).append(v)
        med = {c: statistics.median(v) for c, v in ctr.items()}
        n = wl["objects"]
        row = {"workload": wl["workload"], "kernel_ms_median": statistics.median(ns) / 1e6}
        if "SQ_INSTS_VALU" in med:
            row["valu_per_object"] = med["SQ_INSTS_VALU"] / n
        if "SQ_INSTS_SALU" in med:
            row["salu_per_object"] = med["SQ_INSTS_SALU"] / n
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in med:
                    row[c.lower() + "_share"] = med[c] / wc
        if "GRBM_GUI_ACTIVE" in med:
            row["clock_GHz"] = med["GRBM_GUI_ACTIVE"] / 8 / (statistics.median(ns))
        row["counters_median"] = med
        out.append(row)
        print(json.dumps(row))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2], sys.argv[3:])
