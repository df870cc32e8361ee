#!/bin/bash
# round 4, first GPU pass: light-cone parity + A/B, footprint sweep, short bench
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
O=gpurun_out/r04
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_ref_gpu.py -k "cone or contains" tests/test_tune_parity.py::test_cone_shapes tests/test_abi.py \
  tests/test_cpp_facade.py > $O/cone_tests.log 2>&1 || { tail -60 $O/cone_tests.log; exit 1; }
tail -3 $O/cone_tests.log
timeout -k 10 300 python -u tools/cone_ab.py > $O/cone_ab.jsonl 2> $O/cone_ab.err || { tail -20 $O/cone_ab.err; exit 1; }
python -c "
import json,sys
for l in open('$O/cone_ab.jsonl'):
    d=json.loads(l); print(d['target'],d['op'],d['kernel'],'%.4f ms'%d['ms'],'%.3g obj/s'%d['objects_per_s'])"
timeout -k 10 300 python -u tools/footprint_sweep.py > $O/footprint.jsonl 2> $O/footprint.err || { tail -20 $O/footprint.err; exit 1; }
python -c "
import json
for l in open('$O/footprint.jsonl'):
    d=json.loads(l); print(d['universes'], *['%s %.0f'%(k,d[k+'_GBps']) for k in ('b2b','scrubbed','fixed_b2b','fixed_scrubbed')])"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('value %.3e frac %.3f neutral %s fixed %s'%(d['value'], r['frac'], r['cache_neutral'], r['fixed_order_nt_back_to_back']))
s=d['secondary']; print('c4', s['config4']['roofline']); print(json.dumps(s['filter'])[:3000])"
rocprofv3 -L > $O/counters.txt 2>&1 || true
