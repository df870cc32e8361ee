set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/pairnat_ab.py > gpurun_out/pairnat_ab.jsonl 2> gpurun_out/pairnat_ab.err
