#!/bin/bash
# Round 6: Propagate's window step with the seam side as a compile-time branch
# (stable_kernels.hpp stable_iter_window_at) -- the LifeStable GPU tests on the
# in-tree build, then tools/propagate_lib_ab.py on the build before it
# (build/abs/liblifeapi_hip_oldwin.so: HEAD's stencils.hip, the other objects
# in-tree; or ALT_LIB) and the in-tree build, alternating old / new / old / new
# (NOTEST=1: the A/B only).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${TAG:-r06p}"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd "$R"
[ -n "$NOTEST" ] || timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "${TESTK:-stable or propagate or stabilise or Stable}" tests/ > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 2; }
[ -n "$NOTEST" ] || tail -3 "$O/pytest.log"
for k in 1 2; do
  LIFEAPI_HIP_LIB="$R/${ALT_LIB:-build/abs/liblifeapi_hip_oldwin.so}" timeout -k 10 300 python3 tools/propagate_lib_ab.py \
    >> "$O/ab.jsonl" 2> "$O/ab_old$k.err" || { tail -20 "$O/ab_old$k.err"; exit 3; }
  timeout -k 10 300 python3 tools/propagate_lib_ab.py >> "$O/ab.jsonl" 2> "$O/ab_new$k.err" \
    || { tail -20 "$O/ab_new$k.err"; exit 4; }
  echo "round $k ok"
done
