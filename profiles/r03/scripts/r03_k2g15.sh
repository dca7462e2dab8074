#!/bin/bash
# GPU box, round 3: K2g with one-round-trip LDS staging: tests, sweep, bench, trace.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g15
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/k2g_tests|python -u -m pytest tests/test_gpu_k2g.py -x -q --timeout 120 --timeout-method thread" \
  "300|$o/sweep|python -u tools/probe_k2g.py --groups 18,21,24 --tbits 4 --chunks 8,16 --reps 20" \
  "200|$o/bench|python -u bench.py" \
  "120|$o/trace|rocprofv3 --kernel-trace --stats -d gpurun_out/$o/trace -o run --output-format csv -- python3 tools/probe_k2g.py --tbits 4 --chunks 8 --reps 5 --groups 21"
