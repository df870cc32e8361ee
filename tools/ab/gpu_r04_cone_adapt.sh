#!/bin/bash
# round 4: k_cone_adapt shipped for Contains and the 1-2 generation filter --
# parity of every cone / filter / contains path, the cone A/B, bench
set -o pipefail
O=gpurun_out/${OUT_TAG:-r04y}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  -k "contains or cone or search or filter or tune or Contains or disjoint or Disjoint" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/cone_ab.py > $O/cone_ab.jsonl 2> $O/cone_ab.err || { tail -20 $O/cone_ab.err; exit 3; }
echo cone_ab ok
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 5; }
echo bench ok
