#!/bin/bash
# Generation-count sweep: which layout to default to for small `gens`.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune.py --workload gsweep --rounds 3 --reps 5 > gpurun_out/tune_gsweep.jsonl 2> gpurun_out/tune_gsweep.err || { tail gpurun_out/tune_gsweep.err; exit 3; }
cat gpurun_out/tune_gsweep.jsonl
