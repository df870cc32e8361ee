set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/pair_rounds_ab.py > gpurun_out/pair_rounds_ab.jsonl 2> gpurun_out/pair_rounds_ab.err && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "stable" > gpurun_out/pytest_g6.log 2>&1
