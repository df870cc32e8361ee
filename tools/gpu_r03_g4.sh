set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/stable_xcd_ab.py > gpurun_out/stable_xcd_ab.jsonl 2> gpurun_out/stable_xcd_ab.err && \
timeout -k 10 400 python -u tools/step_xcd_ab.py > gpurun_out/step_xcd_ab.jsonl 2> gpurun_out/step_xcd_ab.err
