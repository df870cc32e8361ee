set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "config4 or large_batch or stable or weld or counts or refined" > gpurun_out/pytest_g5.log 2>&1 && \
timeout -k 10 400 python -u tools/stencil_xcd_ab.py > gpurun_out/stencil_xcd_ab.jsonl 2> gpurun_out/stencil_xcd_ab.err
