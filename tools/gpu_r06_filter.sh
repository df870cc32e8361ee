#!/bin/bash
# Round 6: the iterated search filter priced on both bounds
# (tools/filter_iter_probe.py): timings, a kernel trace, and SQ / FETCH
# counter passes (one counter group per run, each under its own limit).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${PROF_TAG:-r06filter}"
mkdir -p "$O"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
P="$R/tools/filter_iter_probe.py"
timeout -k 10 300 python3 "$P" time > "$O/time.jsonl" 2> "$O/time.err" || { tail -20 "$O/time.err"; exit 2; }
echo "time ok"
FORMS=${TRACE_FORMS:-shipped} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o trace \
  --output-format csv -- python3 "$P" time > "$O/trace_time.jsonl" 2> "$O/trace.err" || { tail -20 "$O/trace.err"; exit 3; }
echo "trace ok"
pmc() {  # name counters
  FORMS=${PMC_FORMS:-shipped} timeout -s KILL 200 rocprofv3 --pmc $2 -d "$O/$1" -o pmc --output-format csv \
    -- python3 "$P" pmc > "$O/$1.manifest" 2> "$O/$1.err" || { tail -20 "$O/$1.err"; exit 4; }
  echo "$1 ok"
}
pmc sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
pmc sq2 "SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS"
pmc fetch "FETCH_SIZE"
pmc tcc "TCC_HIT_sum TCC_MISS_sum"
PMC_JSON="$O/pmc_filter.json" python3 "$P" summarize "$O/sq.manifest" "$O/sq" "$O/sq2" "$O/fetch" "$O/tcc" \
  > "$O/pmc.jsonl" || exit 5
echo "summary ok"
