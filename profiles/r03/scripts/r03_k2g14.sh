#!/bin/bash
# GPU box, round 3: K2g chunk 16 at two waves per SIMD against 8 at four; LDS floors.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g14
mkdir -p gpurun_out/$o
tools/gpu_session.sh \
  "300|$o/k2g_tests|python -u -m pytest tests/test_gpu_k2g.py -x -q --timeout 120 --timeout-method thread" \
  "300|$o/sweep|python -u tools/probe_k2g.py --groups 16,21,24 --tbits 4,5 --chunks 8,11,16 --lds 0,40960 --reps 10" \
  "200|$o/bench|python -u bench.py"
