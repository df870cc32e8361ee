#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head; exit $rc; fi
timeout -k 10 600 python tools/tune.py --workload all --rounds 3 --reps 5 > gpurun_out/tune_all.jsonl 2> gpurun_out/tune_all.err || { tail gpurun_out/tune_all.err; exit 3; }
echo tuned
