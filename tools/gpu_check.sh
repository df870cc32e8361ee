#!/bin/bash
# First-pass GPU check: parity tests, smoke, bench, kernel-trace profile.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== rocminfo"; (rocm-smi --showproductname 2>&1 | head -20) > gpurun_out/smi.txt
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=30 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 3; }
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 4; }
cat gpurun_out/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$GRAFT_REPO_ROOT/gpurun_out/prof_trace" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/prof_trace.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_trace.log"; exit 5; }
find "$GRAFT_REPO_ROOT/gpurun_out/prof_trace" -name "*stats*" | head
