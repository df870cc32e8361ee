set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/order_policy_ab.py > gpurun_out/order_policy_ab.jsonl 2> gpurun_out/order_policy_ab.err
