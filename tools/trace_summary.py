"""Per-(kernel, grid) summary of a rocprofv3 --kernel-trace CSV: calls,
average / median duration, and, for the step kernels, the algorithmic
GB/s (1024 B per universe-generation).  rocprofv3's own
--stats lumps every launch of one kernel together; the bench launches the
config-2 step (1M universes) and config 4 on one GPU (16M) with the same
kernel, so this splits them by grid size.

usage: python tools/trace_summary.py <..._kernel_trace.csv> [> summary.txt]
"""
import csv
import statistics
import sys
from collections import defaultdict

rows = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    short = name.replace("(anonymous namespace)::", "").replace("lifeapi_impl::", "").replace("void ", "")
    short = short.split("(")[0]
    rows[(short, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

print(f"{'kernel':58s} {'grid threads':>12s} {'calls':>5s} {'avg us':>10s} {'median us':>10s} {'universes':>10s} {'GB/s (1 gen)':>12s}")
for (k, grid), t in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
    waves = grid // 64
    uni = waves * 4 if k.startswith(("k_step<", "k_step_split")) else None
    gbs = f"{uni * 1024 / (statistics.mean(t) * 1e3):12.1f}" if uni and k.startswith("k_step<") else ""
    print(f"{k[:58]:58s} {grid:12d} {len(t):5d} {statistics.mean(t):10.2f} {statistics.median(t):10.2f} "
          f"{uni if uni else '':>10} {gbs}")
