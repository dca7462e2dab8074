#!/bin/bash
# GPU box, round 3 final tree: full GPU suite, smoke, cfg3 bench line.
cd "$GRAFT_REPO_ROOT"
o=${OUT:-r03/final}
mkdir -p gpurun_out/$o
tools/gpu_session.sh \
  "600|$o/gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "120|$o/smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "150|$o/bench|python -u bench.py"
