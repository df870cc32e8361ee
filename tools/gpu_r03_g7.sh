set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/c3_overhead.py > gpurun_out/c3_overhead.jsonl 2> gpurun_out/c3_overhead.err
