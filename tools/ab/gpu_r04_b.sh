#!/bin/bash
# round 4, second measurement pass: the read-only scrub (footprint sweep with
# both scrub forms, rows, bench) and the k_weld welds-per-wave A/B
set -o pipefail
O=gpurun_out/${OUT_TAG:-r04b}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "weld or cone or filter" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/ab/weld_u_ab.py > $O/weld_u_ab.jsonl 2> $O/weld.err || { tail -20 $O/weld.err; exit 2; }
echo weld ok
timeout -k 10 300 python -u tools/footprint_sweep.py > $O/footprint.jsonl 2> $O/footprint.err || { tail -20 $O/footprint.err; exit 3; }
echo sweep ok
timeout -k 10 300 python -u tools/rows_bench.py > $O/rows_bench.jsonl 2> $O/rows_bench.err || { tail -20 $O/rows_bench.err; exit 4; }
echo rows ok
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 5; }
echo bench ok
