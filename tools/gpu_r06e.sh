#!/bin/bash
# Round 6: parity of the unified iterated filter and the windowed Propagate
# (targeted GPU tests), then timings (filter forms, Propagate A/B, report loop).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${TAG:-r06e}"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd "$R"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "${TESTK:-iterated or filter or cone or contains or stable or propagate}" tests/test_ref_gpu.py tests/test_gpu_parity.py \
  tests/test_tune_parity.py > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 2; }
tail -3 "$O/pytest.log"
FORMS=shipped GENS=3,5,8,13 timeout -k 10 300 python3 tools/filter_iter_probe.py time > "$O/time.jsonl" 2> "$O/time.err" \
  || { tail -20 "$O/time.err"; exit 3; }
FORMS=shipped,dma_capped16,dma_capped8 GENS=1,2 timeout -k 10 300 python3 tools/filter_iter_probe.py time > "$O/time12.jsonl" \
  2> "$O/time12.err" || { tail -20 "$O/time12.err"; exit 3; }
echo "time ok"
timeout -k 10 300 python3 tools/propagate_window_ab.py > "$O/propagate.jsonl" 2> "$O/propagate.err" \
  || { tail -20 "$O/propagate.err"; exit 4; }
echo "propagate ok"
timeout -k 10 300 python3 tools/report_loop_probe.py > "$O/report_loop.jsonl" 2> "$O/report_loop.err" \
  || { tail -20 "$O/report_loop.err"; exit 5; }
echo "report loop ok"
