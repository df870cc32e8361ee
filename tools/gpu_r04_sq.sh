#!/bin/bash
# round 4: SQ instruction counts and the busy clock (GRBM_GUI_ACTIVE) of the
# step, the light-cone filter / Contains and Propagate, each launch alone
# after a scrub (tools/pmc_r04.py): how much of each kernel's time its VALU
# work takes at 2 clocks per wave64 instruction
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${PROF_TAG:-r04/sq}"
mkdir -p "$O"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
P="python3 $R/tools/pmc_r04.py"
run() {  # name counters args...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "k_step|k_cone|k_stable" -d "$O/$name" -o pmc --output-format csv -- $P "$@" > "$O/$name.out" 2> "$O/$name.err" || { tail -20 "$O/$name.err"; exit 3; }
  echo "$name ok"
}
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
run sq_step "$C" step 1048576
run sq_cone "$C" cone
run sq_stable "$C" stable
