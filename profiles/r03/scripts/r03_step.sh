#!/bin/bash
# GPU box, round 3: step overhead probe (measurement events, scratch wait) + K2g / K2s / parity
# tests that share a context between streams.
cd "$GRAFT_REPO_ROOT"
o=r03/step
mkdir -p gpurun_out/$o
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k2g.py tests/test_gpu_k2s.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread" \
  "200|$o/overhead|python -u tools/probe_step_overhead.py" \
  "150|$o/bench|python -u bench.py"
