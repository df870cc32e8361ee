#!/bin/bash
# Round 6: parity of the new filter routing (targeted GPU tests), then the
# shipped path's timings and the report-loop probe.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${TAG:-r06d}"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd "$R"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "${TESTK:-iterated or filter or cone or contains or step_contains}" tests/test_ref_gpu.py tests/test_gpu_parity.py \
  > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 2; }
tail -3 "$O/pytest.log"
FORMS=shipped GENS=${GENS:-1,2,3,5,8,13} timeout -k 10 300 python3 tools/filter_iter_probe.py time > "$O/time.jsonl" 2> "$O/time.err" \
  || { tail -20 "$O/time.err"; exit 3; }
echo "time ok"
timeout -k 10 300 python3 tools/report_loop_probe.py > "$O/report_loop.jsonl" 2> "$O/report_loop.err" \
  || { tail -20 "$O/report_loop.err"; exit 4; }
echo "report loop ok"
