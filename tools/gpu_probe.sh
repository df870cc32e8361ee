#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 ./build/membw > gpurun_out/membw2.jsonl 2> gpurun_out/membw2.err || { cat gpurun_out/membw2.err; exit 2; }
timeout -k 10 300 ./build/valu_probe > gpurun_out/valu_probe2.jsonl 2>&1 || exit 3
echo probes done
