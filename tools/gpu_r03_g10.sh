set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/bench_gap_probe.py > gpurun_out/bench_gap_probe.jsonl 2> gpurun_out/bench_gap_probe.err
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/bench_g10.json 2> gpurun_out/bench_g10.err
