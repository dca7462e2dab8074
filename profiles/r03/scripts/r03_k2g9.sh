#!/bin/bash
# GPU box, round 3: K2g v7 (one unconditional 16-B load per waypoint, branch-free consume):
# K2g parity tests, then the cfg3 step over chunk lengths and group lengths.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g9
mkdir -p gpurun_out/$o
tools/gpu_session.sh \
  "300|$o/k2g_tests|python -u -m pytest tests/test_gpu_k2g.py -x -q --timeout 120 --timeout-method thread" \
  "240|$o/chunks|python -u tools/probe_k2g.py --groups 21 --tbits 4 --chunks 6,8,10,11 --reps 20" \
  "240|$o/groups|python -u tools/probe_k2g.py --groups 12,16,18,24,28,32 --tbits 4 --chunks 8,11 --reps 20" \
  "240|$o/tbits|python -u tools/probe_k2g.py --groups 21 --tbits 4,5,6 --chunks 0 --reps 20"
