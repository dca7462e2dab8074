#!/bin/bash
# GPU box, round 3: K2g v6 -- waves per SIMD the evaluation is built for (register cap, with
# spills) x gathers in flight, cfg3 at G = 21, kernel trace split per setting.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g8
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/probe|rocprofv3 --kernel-trace -d gpurun_out/$o/tr -o run --output-format csv -- python3 -u tools/probe_k2g.py --groups 21 --chunks 8,11 --minw 0,5,6,8 --tbits 4 --lds 0 --reps 10"
