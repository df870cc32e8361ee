"""The iterated search filter (first hits only, 3-15 generations) on 1M
universes, priced on both of its bounds.

  python tools/filter_iter_probe.py time [FORMS=a,b] [TARGETS=..] [GENS=..]
      per target x generations x form: the call back to back (K launches
      between two events, median of 5) and alone after a 768 MiB scrub
      (median of 9); every form's answers checked against the shipped path's.
      One JSON line per row.
  python tools/filter_iter_probe.py pmc
      the kernel driver for rocprofv3 --pmc (tools/gpu_r06_filter.sh): per
      row a delimiter launch (k_pop on one universe), then REPS calls each
      after a scrub; prints its manifest (one JSON line per row).
  python tools/filter_iter_probe.py summarize MANIFEST DIR [DIR ...]
      the counter CSVs of the pmc passes -> per row the counters per call and
      per universe, and the VALU bound (SQ_INSTS_VALU / 1.2288e12 per s).

Targets (1M config-2 universes, seed 2; but full_height none is ever contained): `full` -- a random universe as both planes (care
cells in every row and column: no window of any kind), `full_height` --
bench.py's full-height target (16 cells that must be dead, one in every
fourth row: no window either, 2-10 % of universes hit), `one_row` -- bench.py's
whole-board target (row 10 of every third column must be dead), `block` --
bench.py's 2x2 block + ring (4 columns x 4 rows), `five_rows` -- rows 0, 12,
29, 46, 63 of every third column (no row window)."""
import csv
import glob
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "tune"))
import bench  # noqa: E402
import lifeapi_amd.hip as hip  # noqa: E402

VALU_PEAK = 1024 * 2.4e9 / 2  # wave64 VALU issue slots per second (MI355X_MICROARCH.md)
PEAK_GBPS = 8000.0
K = 10
REPS = 3


class RT:
    kind = "hip"

    def __init__(self):
        self.device = torch.device("cuda", 0)
        self.stream = torch.cuda.current_stream()

    @staticmethod
    def event():
        return torch.cuda.Event(enable_timing=True)


def _t(v):
    return torch.from_numpy(np.asarray(v, np.uint64).view(np.int64)[None].copy()).cuda()


def targets(x):
    out = {"full": (x[:1].clone(), x[:1].clone())}
    for name, rowmask in (("one_row", 1 << 10), ("five_rows", 0x8000400020001001)):
        u = np.zeros(64, np.uint64)
        u[0::3] = np.uint64(rowmask)
        out[name] = (_t(np.zeros(64, np.uint64)), _t(u))
    bw, bu = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    bw[10] = bw[11] = np.uint64(3 << 40)
    bu[9:13] = np.uint64(15 << 39)
    bu &= ~bw
    out["block"] = (_t(bw), _t(bu))
    fu = np.zeros(64, np.uint64)  # tests/golden/make_golden.py full_height_target
    for y in range(0, 64, 4):
        fu[(3 * y) % 64] |= np.uint64(1 << y)
    out["full_height"] = (_t(np.zeros(64, np.uint64)), _t(fu))
    return out


def cone_lines(tname, gens):
    """128-byte lines of a universe the filter must read: the block's cone
    columns; every other target needs the whole board"""
    if tname != "block":
        return 4
    xs = (9 - gens) % 64
    return len({((xs + c) % 64) // 16 for c in range(min(64, 4 + 2 * gens))})


_Y = {}


def forms(x, tw, tu, gens):
    fs = {"shipped": lambda: hip.step_contains(x, tw, tu, gens)[0]}
    y = _Y.setdefault(x.data_ptr(), torch.empty_like(x))
    # the plain Stepped(gens) of the same batch (final states stored, no test): not an answer
    fs["step_only"] = lambda: hip.step(x, out=y, generations=gens)
    try:
        import tune_hip as tune
    except Exception:  # noqa: BLE001 (the tuning build is optional here)
        return fs
    if gens > 2:
        fs["pair"] = lambda: tune.step_contains_pair(x, tw, tu, gens, 32, 32)
        fs["pair_uncapped"] = lambda: tune.step_contains_pair(x, tw, tu, gens, 0, 0)
        fs["hi_only"] = lambda: tune.step_contains(x, tw, tu, gens, 8)
    # k_cone_adapt's capped form (16 / 32 blocks per CU): the packed row-window
    # passes (cone_wave_rows) against the window split layout (cone_split.hpp)
    # the 1-2 generation filter's LDS form on the capped grid (no report needed)
    fs["dma_capped16"] = lambda: tune.cone(x, tw, tu, gens, 16003, 8, first=True)
    fs["dma_capped16_late"] = lambda: tune.cone(x, tw, tu, gens, 16010, 8, first=True)  # (no early fetch)
    fs["dma_capped8"] = lambda: tune.cone(x, tw, tu, gens, 8003, 8, first=True)
    fs["rows_capped"] = lambda: tune.cone(x, tw, tu, gens, 16000, 8, first=True)
    fs["win_capped"] = lambda: tune.cone(x, tw, tu, gens, 16008, 8, first=True)
    fs["win_capped32"] = lambda: tune.cone(x, tw, tu, gens, 32008, 8, first=True)
    for name, var in getattr(tune, "FILTER_ITER_FORMS", {}).items():
        fs[name] = (lambda v=var: tune.filter_iter(x, tw, tu, gens, v))
    return fs


def selected(env, default):
    v = os.environ.get(env)
    return v.split(",") if v else default


def time_mode():
    rt = RT()
    n = int(os.environ.get("N", str(1 << 20)))
    x = hip.fill_random(n, seed=2)
    scrub = bench.Scrub(rt)
    tg = targets(x)
    gens_list = [int(g) for g in selected("GENS", ["3", "5", "8", "13"])]
    want_forms = os.environ.get("FORMS")
    for tname in selected("TARGETS", list(tg)):
        tw, tu = tg[tname]
        for gens in gens_list:
            fs = forms(x, tw, tu, gens)
            ref = fs["shipped"]().clone()
            ref = fs["shipped"]().clone()  # (the second call runs the reported form)
            torch.cuda.synchronize()
            for fname, fn in fs.items():
                if want_forms and fname not in want_forms.split(","):
                    continue
                got = fn()
                torch.cuda.synchronize()
                ok = None if fname == "step_only" else bool(torch.equal(got.to(torch.int32), ref.to(torch.int32)))
                b2b = []
                for _ in range(5):
                    a, b = rt.event(), rt.event()
                    a.record()
                    for _ in range(K):
                        fn()
                    b.record()
                    b.synchronize()
                    b2b.append(a.elapsed_time(b) / K)
                alone = []
                for k in range(12):
                    scrub()
                    a, b = rt.event(), rt.event()
                    a.record()
                    fn()
                    b.record()
                    b.synchronize()
                    if k >= 3:
                        alone.append(a.elapsed_time(b))
                ms = statistics.median(b2b)
                row = {"target": tname, "gens": gens, "form": fname, "n": n, "ms": ms,
                       "ms_alone": statistics.median(alone), "matches_shipped": ok,
                       "hits": int((ref > 0).sum()),
                       "bytes_bound_ms": n * (cone_lines(tname, gens) * 128 + 4) / PEAK_GBPS / 1e6,
                       "split16_valu_bound_ms": n * gens * 16 / VALU_PEAK * 1e3}
                print(json.dumps(row), flush=True)


def pmc_mode():
    rt = RT()
    n = 1 << 20
    x = hip.fill_random(n, seed=2)
    scrub = bench.Scrub(rt)
    tg = targets(x)
    marker = x[:1]
    gens_list = [int(g) for g in selected("GENS", ["3", "5", "8", "13"])]
    want_forms = os.environ.get("FORMS", "shipped")
    for tname in selected("TARGETS", list(tg)):
        tw, tu = tg[tname]
        for gens in gens_list:
            fs = forms(x, tw, tu, gens)
            for fname in want_forms.split(","):
                if fname not in fs:
                    continue
                fn = fs[fname]
                fn()
                fn()  # (reported form)
                hip.pop(marker)
                for _ in range(REPS):
                    scrub()
                    fn()
                hip.pop(marker)
                torch.cuda.synchronize()
                print(json.dumps({"target": tname, "gens": gens, "form": fname, "n": n, "calls": REPS,
                                  "match": r"k_step_contains|k_cone|k_filter"}), flush=True)


def _dispatches(d):
    paths = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not paths:
        raise SystemExit(f"no counter_collection.csv under {d}")
    by = {}
    with open(paths[0]) as f:
        for r in csv.DictReader(f):
            e = by.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "ctr": {}})
            e["ctr"][r["Counter_Name"]] = e["ctr"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [by[k] for k in sorted(by)]


def summarize(manifest, *dirs):
    import re
    with open(manifest) as f:
        rows = [json.loads(ln) for ln in f if ln.startswith("{")]
    per_row = [dict() for _ in rows]
    for d in dirs:
        disp = _dispatches(d)
        # segments between consecutive markers: row i is segment 2 i + 1
        marks = [i for i, e in enumerate(disp) if re.search(r"k_pop", e["name"])]
        if len(marks) != 2 * len(rows):
            raise SystemExit(f"{d}: {len(marks)} markers for {len(rows)} rows")
        for i, m in enumerate(rows):
            seg = disp[marks[2 * i] + 1:marks[2 * i + 1]]
            kern = [e for e in seg if re.search(m["match"], e["name"])]
            names = sorted({e["name"].split("(")[0][:60] for e in kern})
            tot = {}
            for e in kern:
                for c, v in e["ctr"].items():
                    tot[c] = tot.get(c, 0.0) + v
            per_row[i].update({c: v / m["calls"] for c, v in tot.items()})
            per_row[i].setdefault("kernels", names)
            per_row[i]["dispatches_per_call"] = len(kern) / m["calls"]
    keyed = {}
    for m, c in zip(rows, per_row):
        out = dict(m)
        out.update(c)
        n = m["n"]
        if "SQ_INSTS_VALU" in c:
            out["valu_per_universe"] = c["SQ_INSTS_VALU"] / n
            out["valu_bound_ms"] = c["SQ_INSTS_VALU"] / VALU_PEAK * 1e3
        if "SQ_INSTS_SALU" in c:
            out["salu_per_universe"] = c["SQ_INSTS_SALU"] / n
        if "FETCH_SIZE" in c:
            out["fetch_bytes_per_universe"] = c["FETCH_SIZE"] * 1024 * 2.0 / n  # (x 2: MI355X_MICROARCH.md HBM)
        if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum") is not None:
            tot = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
            out["tcc_hit_rate"] = c["TCC_HIT_sum"] / tot if tot else None
        if "SQ_WAVE_CYCLES" in c and "SQ_WAVES" in c and c["SQ_WAVES"]:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if k in c:
                    out[k.lower() + "_frac"] = c[k] / c["SQ_WAVE_CYCLES"]
        print(json.dumps(out))
        if m["form"] == "shipped":
            keyed[f"{m['target']} {m['gens']}"] = out
    if os.environ.get("PMC_JSON"):  # the table tools/rows_bench.py prices the filter rows on
        with open(os.environ["PMC_JSON"], "w") as f:
            json.dump({"source": "tools/filter_iter_probe.py pmc + summarize (rocprofv3 --pmc, one counter "
                                 "group per run; each call after a 768 MiB scrub, 3 calls per row, per-call "
                                 "counters over every dispatch of the call)",
                       "corrections": {"FETCH_SIZE": 2.0, "why": "MI355X_MICROARCH.md HBM: FETCH_SIZE reads "
                                                                 "half the bytes of wide streaming reads"},
                       "rows": keyed}, f, indent=1)


if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "time"
    if mode == "time":
        time_mode()
    elif mode == "pmc":
        pmc_mode()
    else:
        summarize(*sys.argv[2:])
