#!/bin/bash
# round 4: parity of the stable passes (changed-line stores), the cone
# kernels (quick whole-board test) and the iterated search loop; the stable
# store A/B and the cone A/B
set -o pipefail
O=gpurun_out/${OUT_TAG:-r04s}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  -k "stable or Stable or iterated or cone or contains or filter" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/ab/stable_dirty_ab.py > $O/stable_dirty_ab.jsonl 2> $O/stable.err || { tail -20 $O/stable.err; exit 2; }
echo stable ok
timeout -k 10 300 python -u tools/cone_ab.py > $O/cone_ab.jsonl 2> $O/cone_ab.err || { tail -20 $O/cone_ab.err; exit 3; }
echo cone_ab ok
