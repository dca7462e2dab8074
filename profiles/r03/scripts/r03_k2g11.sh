#!/bin/bash
# GPU box, round 3: K2g v8 (straight-line chunks, sqrt_mid, pinned sums, last-group bins):
# K2g tests, sweeps over chunk / group lengths, bench line.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g11
mkdir -p gpurun_out/$o
tools/gpu_session.sh \
  "300|$o/k2g_tests|python -u -m pytest tests/test_gpu_k2g.py -x -q --timeout 120 --timeout-method thread" \
  "240|$o/sweep|python -u tools/probe_k2g.py --groups 16,21,24,26,28,32 --tbits 4 --chunks 6,8,11 --reps 20" \
  "200|$o/bench|python -u bench.py"
