#!/bin/bash
# Tile-loop issue-rate probe (tools/ab/tile_probe.hip); build happens on CPU beforehand.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./build/tile_probe > gpurun_out/tile_probe.jsonl 2>&1 || { cat gpurun_out/tile_probe.jsonl; exit 2; }
cat gpurun_out/tile_probe.jsonl
