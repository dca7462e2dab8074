#!/bin/bash
# GPU box, round 3: K2g evaluation time by sort-tile bits and LDS floor (pass 1 in the output
# launch, so the evaluation runs alone), kernel trace split per setting.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g_order
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/probe|rocprofv3 --kernel-trace -d gpurun_out/$o/tr -o run --output-format csv -- python3 -u tools/probe_k2g.py --groups 16,21 --tbits 3,4,5,6 --lds 0,24576,40960 --pass1 2 --reps 10"
