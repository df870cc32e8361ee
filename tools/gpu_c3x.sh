#!/bin/bash
# Config-3 exchange/layout variants: parity of every launch variant, then the sweeps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "all_cfgs" > gpurun_out/c3x_pytest.log 2>&1 || { tail -30 gpurun_out/c3x_pytest.log; exit 2; }
tail -2 gpurun_out/c3x_pytest.log
timeout -k 10 300 python tools/tune.py --workload c3 --rounds 4 --reps 5 > gpurun_out/tune_c3x.jsonl 2> gpurun_out/tune_c3x.err || { tail gpurun_out/tune_c3x.err; exit 3; }
cat gpurun_out/tune_c3x.jsonl
timeout -k 10 300 python tools/tune.py --workload gsweep --rounds 3 --reps 5 > gpurun_out/tune_gsweep.jsonl 2> gpurun_out/tune_gsweep.err || { tail gpurun_out/tune_gsweep.err; exit 3; }
cat gpurun_out/tune_gsweep.jsonl
