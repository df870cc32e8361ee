set -o pipefail
cd $GRAFT_REPO_ROOT
(rocm-smi --showcomputepartition --showmemorypartition 2>&1 || true) > gpurun_out/partition.txt
timeout -k 10 300 python -u tools/order_policy_ab.py --rounds 5 > gpurun_out/order_policy_ab2.jsonl 2> gpurun_out/order_policy_ab2.err && \
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_g9.json 2> gpurun_out/bench_g9.err
