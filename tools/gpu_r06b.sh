#!/bin/bash
# Round 6 A/B of the iterated filter forms (tools/filter_iter_probe.py time)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/${TAG:-r06b} && export PYTHONUNBUFFERED=1 && \
FORMS=${FORMS:-shipped,pair32,all32,all32_pf,all7_pf,all14_pf,rows_capped,win_capped,win_capped32} \
TARGETS=${TARGETS:-full,full_height,block,one_row} GENS=${GENS:-3,5,8,13} \
timeout -k 10 400 python3 tools/filter_iter_probe.py time > gpurun_out/${TAG:-r06b}/time.jsonl 2> gpurun_out/${TAG:-r06b}/time.err
echo rc=$?
