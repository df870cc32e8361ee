set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 180 ./build/c3_sched 65536 9 > gpurun_out/c3_sched.jsonl 2>&1 && \
timeout -k 10 400 python -u tools/filter_rule_ab.py --rounds 7 > gpurun_out/filter_rule_ab.jsonl 2>&1
