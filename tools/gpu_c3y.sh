#!/bin/bash
# Config-3 split-layout sweep + probe (parity of the split variants first).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "all_cfgs" > gpurun_out/c3x_pytest.log 2>&1 || { tail -30 gpurun_out/c3x_pytest.log; exit 2; }
tail -1 gpurun_out/c3x_pytest.log
timeout -k 10 300 python tools/tune.py --workload c3 --rounds 4 --reps 5 > gpurun_out/tune_c3y.jsonl 2> gpurun_out/tune_c3y.err || { tail gpurun_out/tune_c3y.err; exit 3; }
cat gpurun_out/tune_c3y.jsonl
timeout -k 10 120 ./build/split_probe > gpurun_out/split_probe.jsonl || exit 4
cat gpurun_out/split_probe.jsonl
