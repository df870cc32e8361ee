set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/c3_wpb_ab.py > gpurun_out/c3_wpb_ab.jsonl 2> gpurun_out/c3_wpb_ab.err
