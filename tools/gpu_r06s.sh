#!/bin/bash
# Round 6: the batched test for targets with no row window
# (split_contains_asm_batch_h8) -- parity (targeted GPU tests), then the
# shipped filter against the same build with the per-generation lean test
# (build/abs/liblifeapi_hip_nob8.so, LIFE_BATCH_H8=0), built on the CPU:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -DLIFE_BATCH_H8=0 \
#     -c lifeapi_amd/csrc/step.hip -o build/abs/step_nob8.o
#   hipcc --offload-arch=gfx950 -shared -fPIC -o build/abs/liblifeapi_hip_nob8.so \
#     build/abs/step_nob8.o <build/obj/*.o but step.o>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${TAG:-r06s}"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd "$R"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "${TESTK:-iterated or filter or contains or step_contains or config3}" tests/test_ref_gpu.py tests/test_gpu_parity.py \
  > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 2; }
tail -2 "$O/pytest.log"
T="TARGETS=full,full_height,five_rows,block,one_row"
env $T FORMS=shipped GENS=${GENS:-3,5,8,13} timeout -k 10 300 python3 tools/filter_iter_probe.py time > "$O/time_b8.jsonl" 2> "$O/time_b8.err" \
  || { tail -20 "$O/time_b8.err"; exit 3; }
echo "b8 ok"
env $T LIFEAPI_HIP_LIB="$R/build/abs/liblifeapi_hip_nob8.so" FORMS=shipped GENS=${GENS:-3,5,8,13} timeout -k 10 300 \
  python3 tools/filter_iter_probe.py time > "$O/time_nob8.jsonl" 2> "$O/time_nob8.err" \
  || { tail -20 "$O/time_nob8.err"; exit 4; }
echo "nob8 ok"
env $T FORMS=shipped GENS=${GENS:-3,5,8,13} timeout -k 10 300 python3 tools/filter_iter_probe.py time > "$O/time_b8_again.jsonl" 2> "$O/time_b8_again.err" \
  || { tail -20 "$O/time_b8_again.err"; exit 5; }
echo "b8 again ok"
