#!/bin/bash
# Round 6: the window-offset test on the in-tree build (must pass), then the
# LifeStable tests on build/abs/liblifeapi_hip_mW.so, a build whose write-back
# merge takes the unmasked band at the seam (place_rows<WRAP>(band, sh) for bw;
# must fail).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${TAG:-r06w}"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  -k "every_row_offset" tests/test_ref_gpu.py > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 2; }
tail -2 "$O/pytest.log"
set +e
LIFEAPI_HIP_LIB="$R/build/abs/liblifeapi_hip_mW.so" timeout -k 10 400 python3 -u -m pytest -q --timeout 200 \
  --timeout-method thread -m gpu -k "stable or propagate or stabilise" tests/test_ref_gpu.py tests/test_gpu_parity.py \
  > "$O/pytest_mW.log" 2>&1
rc=$?
echo "mutant W: pytest exit $rc"
grep -E "^(FAILED|[0-9]+ (passed|failed))" "$O/pytest_mW.log" | head -8
[ $rc -le 1 ]
