set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/filter_more_ab.py > gpurun_out/filter_more_ab.jsonl 2> gpurun_out/filter_more_ab.err
