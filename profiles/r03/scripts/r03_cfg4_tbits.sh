#!/bin/bash
# GPU box, round 3: K2g at cfg4's size (8192^2, 200k pairs): tile bits 4-6, both curves.
cd "$GRAFT_REPO_ROOT"
o=r03/cfg4_tbits
mkdir -p gpurun_out/$o
tools/gpu_session.sh \
  "300|$o/sweep|python -u tools/probe_k2g.py --R 8192 --pairs 200000 --groups 16,21 --tbits 4,5,6 --chunks 8 --curves 0,1 --reps 10"
