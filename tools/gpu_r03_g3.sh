set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/stable_pf_ab.py > gpurun_out/stable_pf_ab.jsonl 2> gpurun_out/stable_pf_ab.err && \
timeout -k 10 400 python -u tools/filter_rule_ab.py --rounds 5 > gpurun_out/filter_pf_ab.jsonl 2> gpurun_out/filter_pf_ab.err
