#!/bin/bash
# Round 6: mutation check of the filter's GPU tests.  Each build/abs/liblifeapi_hip_m?.so is
# the shipped step.hip with one deliberate fault (tools/filter_mutants.py writes and builds them):
#   mA  the window test ORs 7 of the 8 difference registers
#   mB  the whole-board LDS-DMA chunk read takes the neighbouring universe's word
#   mC  the packed row window starts one row late
#   mD  the column light cone one column narrower on each side
# Every mutant must FAIL the filter tests; a mutant that passes is a coverage gap.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${TAG:-r06m}"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd "$R"
K="${TESTK:-iterated or filter or cone or contains or step_contains}"
for m in ${MUTANTS:-A B C D}; do
  set +e
  LIFEAPI_HIP_LIB="$R/build/abs/liblifeapi_hip_m$m.so" timeout -k 10 400 python3 -u -m pytest -q --maxfail=3 \
    --timeout 120 --timeout-method thread -m gpu -k "$K" tests/test_ref_gpu.py tests/test_gpu_parity.py \
    > "$O/pytest_m$m.log" 2>&1
  rc=$?
  set -e
  echo "mutant $m: pytest exit $rc; $(grep -E '^(FAILED|[0-9]+ (passed|failed))' "$O/pytest_m$m.log" | head -4 | tr '\n' ' ')"
  # 1 = tests failed (the expected outcome); anything but 0/1 is a crash or a time limit: stop.
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
  set +e
done
