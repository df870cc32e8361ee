#!/bin/bash
# Round-4 validation and profiles on one MI355X: GPU tests, smoke, the
# default bench line, every 8(f) kernel's roofline with its scrubbed (HBM-only)
# figure (rows_bench), the footprint sweep, a 4-rank gloo rehearsal of bench.py
# sharing the GPU, rocprofv3 kernel-trace summaries and the PMC passes of
# tools/gpu_r04_prof.sh.  Each step under its own time limit; stop at the
# first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/${OUT_TAG:-r04final}"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --maxfail=20 \
  -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.log"
if [ $rc -ne 0 ]; then grep -E "(FAILED|ERROR)" "$O/pytest_gpu.log" | head -30; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 3; }
echo smoke ok
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 4; }
echo bench ok
timeout -k 10 300 python tools/rows_bench.py > "$O/rows_bench.jsonl" 2> "$O/rows_bench.err" || { tail -20 "$O/rows_bench.err"; exit 5; }
echo rows ok
timeout -k 10 300 python tools/footprint_sweep.py > "$O/footprint.jsonl" 2> "$O/footprint.err" || { tail -20 "$O/footprint.err"; exit 6; }
echo sweep ok
LIFEAPI_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 4 --steps 10 --warmup 3 \
  > "$O/dist_rehearsal.json" 2> "$O/dist_rehearsal.err" || { tail -30 "$O/dist_rehearsal.err"; exit 7; }
echo rehearsal ok
if [ -z "$SKIP_PROF" ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_c2" -o bench --output-format csv -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-secondary --steps 50 --warmup 10 > "$O/trace_c2_bench.json" 2> "$O/trace_c2.err" \
    || { tail -20 "$O/trace_c2.err"; exit 8; }
  echo trace ok
  cd "$R"
  PROF_TAG="${OUT_TAG:-r04final}/prof" bash tools/gpu_r04_prof.sh || exit 9
fi
