#!/bin/bash
# round 4, first GPU pass: light-cone parity + A/B
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_ref_gpu.py -k "cone or contains" tests/test_tune_parity.py::test_cone_shapes \
  > gpurun_out/r04/cone_tests.log 2>&1 || { tail -40 gpurun_out/r04/cone_tests.log; exit 1; }
tail -3 gpurun_out/r04/cone_tests.log
timeout -k 10 300 python -u tools/cone_ab.py > gpurun_out/r04/cone_ab.jsonl 2> gpurun_out/r04/cone_ab.err || { tail -20 gpurun_out/r04/cone_ab.err; exit 1; }
cat gpurun_out/r04/cone_ab.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['target'],d['op'],d['kernel'],'%.4f ms'%d['ms'],'%.3g obj/s'%d['objects_per_s'])"
