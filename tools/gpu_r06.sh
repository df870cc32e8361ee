#!/bin/bash
# Round-6 validation on one MI355X.  Steps chosen by STEPS (space-separated,
# default "test smoke bench"):
#   test      pytest -m gpu
#   smoke     __graft_entry__.smoke()
#   bench     the default bench line (+ its side file)
#   rccl      bench.py under torch.distributed.run with one rank and the nccl
#             (RCCL) backend: the collective code path of the N > 1 lines
#   rehearse8 8 gloo ranks sharing the GPU on the full 16M config 4 (2M each)
#   rows      tools/rows_bench.py
#   trace     rocprofv3 kernel trace of the default bench
#   filterpmc tools/gpu_r06_filter.sh: the iterated filter's timings, trace
#             and PMC (-> pmc_filter.json, the table rows_bench prices on)
#   reportloop tools/report_loop_probe.py
#   filtertime tools/filter_iter_probe.py time, the shipped path only
#   propagate tools/propagate_window_ab.py (Propagate and StabiliseOptions)
# Each step under its own time limit; stop at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/${OUT_TAG:-r06}"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
for s in ${STEPS:-test smoke bench}; do
  case $s in
  test)
    timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --maxfail=20 \
      -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > "$O/pytest_gpu.log" 2>&1
    rc=$?; tail -2 "$O/pytest_gpu.log"
    if [ $rc -ne 0 ]; then grep -E "(FAILED|ERROR)" "$O/pytest_gpu.log" | head -30; exit $rc; fi ;;
  smoke)
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
      || { cat "$O/smoke.log"; exit 3; } ;;
  bench)
    LIFEAPI_BENCH_DETAIL="$O/bench_detail.json" timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" \
      || { tail -20 "$O/bench.err"; exit 4; }
    wc -c "$O/bench.json" ;;
  rccl)
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 \
      --master-port=29533 bench.py --gpus 1 --config 4 --steps 10 --warmup 3 --no-secondary --no-cpu-baseline \
      > "$O/rccl_world1.json" 2> "$O/rccl_world1.err" || { tail -30 "$O/rccl_world1.err"; exit 5; } ;;
  rehearse8)
    LIFEAPI_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 8 --steps 10 --warmup 3 \
      > "$O/dist_rehearsal8.json" 2> "$O/dist_rehearsal8.err" || { tail -30 "$O/dist_rehearsal8.err"; exit 6; } ;;
  rows)  # (priced on this call's filter PMC table when the filterpmc step ran before it)
    [ -f "$O/filterpmc/pmc_filter.json" ] && export LIFEAPI_PMC_FILTER="$O/filterpmc/pmc_filter.json"
    timeout -k 10 300 python tools/rows_bench.py > "$O/rows_bench.jsonl" 2> "$O/rows_bench.err" \
      || { tail -20 "$O/rows_bench.err"; exit 7; } ;;
  trace)
    export TMPDIR=/tmp
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_c2" -o bench --output-format csv -- \
      python3 "$R/bench.py" --no-cpu-baseline --no-secondary --steps 50 --warmup 10 > "$O/trace_c2_bench.json" \
      2> "$O/trace_c2.err") || { tail -20 "$O/trace_c2.err"; exit 8; } ;;
  filterpmc)
    FORMS=shipped GENS=${FILTER_GENS:-1,2,3,5,8,13} PROF_TAG="${OUT_TAG:-r06}/filterpmc" \
      bash "$R/tools/gpu_r06_filter.sh" || exit 10 ;;
  reportloop)
    timeout -k 10 300 python tools/report_loop_probe.py > "$O/report_loop.jsonl" 2> "$O/report_loop.err" \
      || { tail -20 "$O/report_loop.err"; exit 11; } ;;
  filtertime)
    FORMS=shipped GENS=1,2,3,5,8,13 timeout -k 10 300 python3 tools/filter_iter_probe.py time > "$O/filter_time.jsonl" \
      2> "$O/filter_time.err" || { tail -20 "$O/filter_time.err"; exit 12; } ;;
  propagate)
    timeout -k 10 300 python tools/propagate_window_ab.py > "$O/propagate.jsonl" 2> "$O/propagate.err" \
      && PASS=stabilise timeout -k 10 300 python tools/propagate_window_ab.py >> "$O/propagate.jsonl" 2>> "$O/propagate.err" \
      || { tail -20 "$O/propagate.err"; exit 13; } ;;
  *) echo "unknown step $s"; exit 9 ;;
  esac
  echo "$s ok"
done
