#!/bin/bash
# Round 6: the whole-board window split pass with its chunks fetched by
# LDS-DMA (cone_split.hpp DMA) -- parity (targeted GPU tests), then the
# shipped filter against the same build without it
# (build/abs/liblifeapi_hip_nodma.so, LIFE_WIN_DMA=0), built on the CPU:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -DLIFE_WIN_DMA=0 \
#     -c lifeapi_amd/csrc/step.hip -o build/abs/step_nodma.o
#   hipcc --offload-arch=gfx950 -shared -fPIC -o build/abs/liblifeapi_hip_nodma.so \
#     build/abs/step_nodma.o <build/obj/*.o but step.o>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${TAG:-r06h}"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd "$R"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "${TESTK:-iterated or filter or cone or contains or step_contains}" tests/test_ref_gpu.py tests/test_gpu_parity.py \
  > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 2; }
tail -3 "$O/pytest.log"
FORMS=shipped GENS=${GENS:-5,8,13} timeout -k 10 300 python3 tools/filter_iter_probe.py time > "$O/time_dma.jsonl" 2> "$O/time_dma.err" \
  || { tail -20 "$O/time_dma.err"; exit 3; }
echo "dma ok"
LIFEAPI_HIP_LIB="$R/build/abs/liblifeapi_hip_nodma.so" FORMS=shipped GENS=${GENS:-5,8,13} timeout -k 10 300 \
  python3 tools/filter_iter_probe.py time > "$O/time_nodma.jsonl" 2> "$O/time_nodma.err" \
  || { tail -20 "$O/time_nodma.err"; exit 4; }
echo "nodma ok"
