#!/bin/bash
# Tuning pass: HBM copy ceilings + step-kernel launch-config sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 ./build/membw > gpurun_out/membw.jsonl 2> gpurun_out/membw.err || { cat gpurun_out/membw.err; exit 2; }
echo "membw done"
timeout -k 10 600 python tools/tune.py --rounds 3 --reps 4 > gpurun_out/tune.jsonl 2> gpurun_out/tune.err || { tail gpurun_out/tune.err; exit 3; }
echo "tune done"
