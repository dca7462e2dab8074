#!/bin/bash
# GPU box, round 3: K2g group length at cfg4's size (8192^2, 200k pairs, tile bits auto).
cd "$GRAFT_REPO_ROOT"
o=r03/cfg4_groups
mkdir -p gpurun_out/$o
tools/gpu_session.sh \
  "300|$o/sweep|python -u tools/probe_k2g.py --R 8192 --pairs 200000 --groups 18,21,24,28,32 --tbits 0 --chunks 8 --reps 10"
