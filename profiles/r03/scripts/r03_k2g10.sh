#!/bin/bash
# GPU box, round 3: K2g v7 defaults (G = 24, 8 gathers in flight): K2g tests, bench line,
# trace + PMC passes of the bench step.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g10
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/k2g_tests|python -u -m pytest tests/test_gpu_k2g.py -x -q --timeout 120 --timeout-method thread" \
  "200|$o/bench|python -u bench.py" \
  "600|$o/prof|PASSES=\"trace fetch write tcc sq\" bash tools/profile_bench.sh gpurun_out/$o/raster --steps 5 --warmup 1"
