#!/bin/bash
# GPU box, round 3: the K2g v6 default -- full GPU suite, smoke, trace + PMC passes of the
# default bench step (tools/profile_bench.sh), the bench line.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g_final
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "900|$o/gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "200|$o/smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "600|$o/prof|PASSES=\"trace fetch write tcc sq\" bash tools/profile_bench.sh gpurun_out/$o/raster --steps 5 --warmup 1" \
  "200|$o/bench|python -u bench.py"
