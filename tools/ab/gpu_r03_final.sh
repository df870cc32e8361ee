#!/bin/bash
# Round-3 validation and profiles on one MI355X: GPU tests, smoke, the
# default bench line, every 8(f) kernel's roofline (rows_bench), the 2-rank
# rehearsal of bench.py --gpus 2, rocprofv3 kernel-trace summaries (the
# default command, and config 2 alone so the k_step average is one launch
# shape), calibrated FETCH/WRITE passes (config 2 via the bench, config 3
# via tools/c3_once.py, the copy-kernel calibration) and two SQ counter
# passes on the config-3 loop.  Each step under its own time limit; stop at
# the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/${OUT_TAG:-r03final}"
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --maxfail=20 \
  -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.log"
if [ $rc -ne 0 ]; then grep -E "(FAILED|ERROR)" "$O/pytest_gpu.log" | head -30; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 3; }
echo smoke ok
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 4; }
echo bench ok
timeout -k 10 200 python tools/rows_bench.py > "$O/rows_bench.jsonl" 2> "$O/rows_bench.err" || { tail -20 "$O/rows_bench.err"; exit 5; }
echo rows ok
LIFEAPI_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 \
  > "$O/dist_rehearsal.json" 2> "$O/dist_rehearsal.err" || { tail -30 "$O/dist_rehearsal.err"; exit 6; }
echo rehearsal ok
timeout -k 10 200 python tools/c3_clock.py > "$O/c3_clock.json" 2> "$O/c3_clock.err" || { tail -20 "$O/c3_clock.err"; exit 12; }
echo clock ok
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace" -o bench --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --steps 50 --warmup 10 > "$O/trace_bench.json" 2> "$O/trace.err" \
  || { tail -20 "$O/trace.err"; exit 7; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_c2" -o bench --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-secondary --steps 50 --warmup 10 > "$O/trace_c2_bench.json" 2> "$O/trace_c2.err" \
  || { tail -20 "$O/trace_c2.err"; exit 8; }
echo traces ok
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_step" -d "$O/prof/pmc_$C" -o bench --output-format csv -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-secondary --no-verify --steps 10 --warmup 2 > "$O/pmc_$C.json" 2> "$O/pmc_$C.err" \
    || { tail -20 "$O/pmc_$C.err"; exit 9; }
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_step" -d "$O/prof/c3_$C" -o c3 --output-format csv -- \
    python3 "$R/tools/c3_once.py" 3 > "$O/c3_$C.log" 2>&1 || { tail -20 "$O/c3_$C.log"; exit 10; }
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_copy" -d "$O/prof/calib_$C" -o calib --output-format csv -- \
    "$R/build/membw" calib > "$O/calib_$C.json" 2> "$O/calib_$C.err" || { tail -20 "$O/calib_$C.err"; exit 11; }
done
echo pmc ok
i=0
for G in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --kernel-include-regex "k_step_split" -d "$O/prof/sq$i" -o sq --output-format csv -- \
    python3 "$R/tools/c3_once.py" 3 > "$O/sq$i.log" 2>&1 || { tail -5 "$O/sq$i.log"; exit 13; }
done
echo sq ok
