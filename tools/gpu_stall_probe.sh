#!/bin/bash
# SQ counters of the LifeStable PropagateStep / Propagate forms
# (tools/stable_stall_probe.py), one counter group per run, each under its own
# limit; the summary into $O/stall.jsonl.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${PROF_TAG:-r05stall}"
mkdir -p "$O"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
run() {  # name counters
  local name=$1 ctr=$2
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "k_stable" -d "$O/$name" -o pmc \
    --output-format csv -- python3 "$R/tools/stable_stall_probe.py" run > "$O/$name.manifest" 2> "$O/$name.err" \
    || { tail -20 "$O/$name.err"; exit 3; }
  echo "$name ok"
}
run a "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
python3 "$R/tools/stable_stall_probe.py" summarize "$O/a.manifest" "$O/a" > "$O/stall.jsonl" || exit 4
echo summary ok
