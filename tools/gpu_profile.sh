#!/bin/bash
# Profiling pass: rocprofv3 kernel trace + stats of the full bench (config 2
# headline + config 3 / config 5 secondaries), then FETCH_SIZE and WRITE_SIZE
# in separate --pmc passes (gfx950 slot limits) on the step and refined
# kernels, plus the same counters on a copy kernel of the identical access
# shape (build/membw calib) to calibrate the byte counters.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/prof"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o bench --output-format csv -- $B --steps 50 --warmup 10 > "$O/trace_bench.json" 2> "$O/trace.err" || { tail -20 "$O/trace.err"; exit 2; }
echo trace ok
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "k_step|k_refined" -d "$O/pmc_$C" -o bench --output-format csv -- $B --no-verify --steps 10 --warmup 2 > "$O/pmc_$C.json" 2> "$O/pmc_$C.err" || { tail -20 "$O/pmc_$C.err"; exit 3; }
  timeout -k 10 200 rocprofv3 --pmc $C --kernel-include-regex "k_copy" -d "$O/calib_$C" -o calib --output-format csv -- "$R/build/membw" calib > "$O/calib_$C.json" 2> "$O/calib_$C.err" || { tail -20 "$O/calib_$C.err"; exit 4; }
  echo "$C ok"
done
