#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -k "refined" -p no:cacheprovider > gpurun_out/pytest_refined.log 2>&1 || { tail -30 gpurun_out/pytest_refined.log; exit 2; }
tail -1 gpurun_out/pytest_refined.log
timeout -k 10 600 python tools/tune.py --workload c5 --rounds 3 --reps 5 > gpurun_out/tune_c5.jsonl 2> gpurun_out/tune_c5.err || { tail gpurun_out/tune_c5.err; exit 3; }
echo tuned
