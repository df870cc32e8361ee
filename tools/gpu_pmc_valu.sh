#!/bin/bash
# SQ counters on the config-3 generation loop (valu_probe), one counter group
# per pass, kernel-trace only (no sys/runtime trace with --pmc on this pool).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/pmc_valu"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
i=0
for G in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES" "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" "SQ_WAIT_ANY SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G --kernel-include-regex "k_iter" -d "$O/p$i" -o p --output-format csv -- "$R/build/valu_probe" > "$O/p$i.log" 2>&1 || { tail -5 "$O/p$i.log"; echo "pass $i failed"; }
done
echo done
