set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py > gpurun_out/bench_g8.json 2> gpurun_out/bench_g8.err
