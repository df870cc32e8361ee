#!/bin/bash
# round 4 profiling pass: kernel trace + stats of the full bench, then PMC
# passes (one counter group per run, gfx950 slot limits) on single cold
# launches (tools/pmc_r04.py): address translation at 1M and 16M universes,
# and the light-cone kernels' fetched bytes and request sizes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${PROF_TAG:-r04/prof}"
mkdir -p "$O"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace" -o bench --output-format csv -- python3 "$R/bench.py" --steps 50 --warmup 10 > "$O/trace_bench.json" 2> "$O/trace.err" || { tail -20 "$O/trace.err"; exit 2; }
echo trace ok
P="python3 $R/tools/pmc_r04.py"
run() {  # name counters args...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "k_step|k_cone|k_fill|k_stable" -d "$O/$name" -o pmc --output-format csv -- $P "$@" > "$O/$name.out" 2> "$O/$name.err" || { tail -20 "$O/$name.err"; exit 3; }
  echo "$name ok"
}
run tlb_1m "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum" step 1048576
run tlb_16m "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum" step 16777216
run fetch_cone FETCH_SIZE cone
run rdreq_cone "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum" cone
run write_cone WRITE_SIZE cone
run fetch_step_1m FETCH_SIZE step 1048576
run write_stable WRITE_SIZE stable
run fetch_stable FETCH_SIZE stable
