#!/bin/bash
# round 4: fetched and written bytes of the 16M step (config 4 on one GPU),
# each launch alone after a scrub (tools/pmc_r04.py step 16777216)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${PROF_TAG:-r04/pmc16m}"
mkdir -p "$O"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
P="python3 $R/tools/pmc_r04.py"
run() {  # name counters args...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-include-regex "k_step" -d "$O/$name" -o pmc --output-format csv -- $P "$@" > "$O/$name.out" 2> "$O/$name.err" || { tail -20 "$O/$name.err"; exit 3; }
  echo "$name ok"
}
run fetch_step_16m FETCH_SIZE step 16777216
run write_step_16m WRITE_SIZE step 16777216
run write_step_1m WRITE_SIZE step 1048576
