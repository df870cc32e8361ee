#!/bin/bash
# Rehearse bench.py's multi-rank path on a 1-GPU box: 2 ranks share cuda:0 and
# talk over gloo (RCCL does not allow two ranks on one GPU).  The real N>1
# runs use RCCL, one rank per GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIFEAPI_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 \
  > gpurun_out/dist_rehearsal.json 2> gpurun_out/dist_rehearsal.err || { tail -30 gpurun_out/dist_rehearsal.err; exit 2; }
cat gpurun_out/dist_rehearsal.json
