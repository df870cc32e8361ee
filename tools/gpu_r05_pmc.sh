#!/bin/bash
# Round 5: the LifeStable rows' PMC (tools/pmc_rows.py): FETCH_SIZE, WRITE_SIZE
# and SQ VALU counts, one counter group per run, each under its own limit;
# the summary into $O/pmc_rows.json.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${PROF_TAG:-r05pmc}"
mkdir -p "$O"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
run() {  # name counters
  local name=$1 ctr=$2
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "k_stable" -d "$O/$name" -o pmc \
    --output-format csv -- python3 "$R/tools/pmc_rows.py" run > "$O/$name.manifest" 2> "$O/$name.err" \
    || { tail -20 "$O/$name.err"; exit 3; }
  echo "$name ok"
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq "SQ_INSTS_VALU SQ_WAVES"
python3 "$R/tools/pmc_rows.py" summarize "$O/fetch" "$O/write" "$O/sq" "$O/fetch.manifest" > "$O/pmc_rows.json" \
  || exit 4
echo summary ok
