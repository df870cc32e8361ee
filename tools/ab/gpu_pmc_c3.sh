#!/bin/bash
# SQ / LDS counters on the config-3 kernel (default cfg), one counter group
# per pass, kernel trace only; each pass under its own hard time limit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/pmc_c3"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
i=0
for G in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --kernel-include-regex "k_step" -d "$O/p$i" -o p --output-format csv -- python3 "$R/tools/c3_once.py" 3 > "$O/p$i.log" 2>&1 || { tail -5 "$O/p$i.log"; echo "pass $i failed"; exit 1; }
done
echo done
