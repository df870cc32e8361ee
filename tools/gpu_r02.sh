#!/bin/bash
# Round-2 validation on one MI355X: GPU tests, smoke, the N=1 bench line, a
# 2-rank rehearsal of `bench.py --gpus 2` (bench spawns the ranks itself; both
# share the one GPU over gloo), and a rocprofv3 kernel-trace summary of the
# bench.  Each step time-limited; the script stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/r02
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --maxfail=20 \
  -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"
if [ $rc -ne 0 ]; then grep -E "(FAILED|ERROR)" "$O/pytest_gpu.log" | head -30; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 3; }
echo smoke ok
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 4; }
cat "$O/bench.json"
LIFEAPI_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 \
  > "$O/dist_rehearsal.json" 2> "$O/dist_rehearsal.err" || { tail -30 "$O/dist_rehearsal.err"; exit 5; }
cat "$O/dist_rehearsal.json"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/trace" -o bench --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --steps 50 --warmup 10 > "$R/$O/trace_bench.json" 2> "$R/$O/trace.err" \
  || { tail -20 "$R/$O/trace.err"; exit 6; }
echo trace ok
