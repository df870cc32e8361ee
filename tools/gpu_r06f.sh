#!/bin/bash
# Round 6: the column-shrinking window split pass -- parity (targeted GPU
# tests), then the shipped filter against the same build without it
# (build/abs/liblifeapi_hip_noshrink.so, LIFE_SHRINK_MASK=0), built on the CPU:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -DLIFE_SHRINK_MASK=0 \
#     -c lifeapi_amd/csrc/step.hip -o build/abs/step_noshrink.o
#   hipcc --offload-arch=gfx950 -shared -fPIC -o build/abs/liblifeapi_hip_noshrink.so \
#     build/abs/step_noshrink.o <build/obj/*.o but step.o>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${TAG:-r06f}"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd "$R"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "${TESTK:-iterated or filter or cone or contains or step_contains}" tests/test_ref_gpu.py tests/test_gpu_parity.py \
  > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 2; }
tail -3 "$O/pytest.log"
FORMS=shipped GENS=${GENS:-3,5,8,13} timeout -k 10 300 python3 tools/filter_iter_probe.py time > "$O/time_shrink.jsonl" 2> "$O/time_shrink.err" \
  || { tail -20 "$O/time_shrink.err"; exit 3; }
echo "shrink ok"
LIFEAPI_HIP_LIB="$R/build/abs/liblifeapi_hip_noshrink.so" FORMS=shipped GENS=${GENS:-3,5,8,13} timeout -k 10 300 \
  python3 tools/filter_iter_probe.py time > "$O/time_noshrink.jsonl" 2> "$O/time_noshrink.err" \
  || { tail -20 "$O/time_noshrink.err"; exit 4; }
echo "noshrink ok"
