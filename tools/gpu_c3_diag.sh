#!/bin/bash
# Config-3 diagnostics of the SHIPPED kernel: held clock (in-kernel stamps),
# then SQ / LDS / GRBM counters in two --pmc passes (kernel trace only).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r02/pmc_c3"
mkdir -p "$O"
cd "$R"
timeout -k 10 120 python tools/c3_clock.py > "$O/clock.json" 2> "$O/clock.err" || { tail -20 "$O/clock.err"; exit 1; }
cat "$O/clock.json"
export TMPDIR=/tmp
cd /tmp
i=0
for G in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --kernel-include-regex "k_step" -d "$O/p$i" -o p --output-format csv -- python3 "$R/tools/c3_once.py" 5 > "$O/p$i.log" 2>&1 || { tail -5 "$O/p$i.log"; echo "pass $i failed"; exit 2; }
done
echo pmc ok
