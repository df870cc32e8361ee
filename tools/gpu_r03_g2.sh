set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/rows_bench.py > gpurun_out/rows_bench_b2b.jsonl 2> gpurun_out/rows_bench_b2b.err
