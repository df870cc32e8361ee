#!/bin/bash
# round 4: the cone kernels' coalesced result stores -- parity of every cone /
# filter / search path, the iterated-loop A/B, the cone rows, and bench
set -o pipefail
O=gpurun_out/${OUT_TAG:-r04n}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  -k "contains or cone or search or filter or tune" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/ab/search_iter_caps_ab.py > $O/caps.jsonl 2> $O/caps.err || { tail -20 $O/caps.err; exit 2; }
echo caps ok
