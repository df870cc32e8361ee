#!/bin/bash
# Tile layouts (rules 8, 9): parity of the new launch variants, then the config-3 sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "all_cfgs and (-8] or -9])" > gpurun_out/tile_pytest.log 2>&1 || { tail -30 gpurun_out/tile_pytest.log; exit 2; }
tail -2 gpurun_out/tile_pytest.log
timeout -k 10 300 python tools/tune.py --workload c3 --rounds 4 --reps 5 > gpurun_out/tune_tile.jsonl 2> gpurun_out/tune_tile.err || { tail gpurun_out/tune_tile.err; exit 3; }
cat gpurun_out/tune_tile.jsonl
