#!/bin/bash
# 6-LUT tail (rules 10-13): parity of every launch variant and the fused
# contains kernel, then the config-3 A/B against the 7-LUT tail.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "all_cfgs or contains or config3" > gpurun_out/net6_pytest.log 2>&1 || { tail -30 gpurun_out/net6_pytest.log; exit 2; }
tail -2 gpurun_out/net6_pytest.log
timeout -k 10 400 python -u tools/tune.py --workload ${TUNE:-c3net} --rounds 5 > gpurun_out/tune_${TUNE:-c3net}.jsonl 2> gpurun_out/tune.err || { tail -20 gpurun_out/tune.err; exit 3; }
cat gpurun_out/tune_${TUNE:-c3net}.jsonl
