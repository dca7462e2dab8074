#!/bin/bash
# GPU box, round 3: K2g v6 -- group length x gathers in flight x LDS floor (workgroups per CU)
# on cfg3, kernel trace split per setting.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g7
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/probe|rocprofv3 --kernel-trace -d gpurun_out/$o/tr -o run --output-format csv -- python3 -u tools/probe_k2g.py --groups 12,14,16,18,21,24 --chunks 8,11 --tbits 4 --lds 0 --reps 10" \
  "400|$o/probe_lds|rocprofv3 --kernel-trace -d gpurun_out/$o/trl -o run --output-format csv -- python3 -u tools/probe_k2g.py --groups 21 --chunks 0 --tbits 4,5 --lds 0,45000,54000,80000 --reps 10"
