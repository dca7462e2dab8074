#!/bin/bash
# GPU box, round 3: full GPU suite, smoke, and the cfg3 / cfg4 / cfg5 bench lines.
cd "$GRAFT_REPO_ROOT"
o=${OUT:-r03/suite}
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "600|$o/gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "120|$o/smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "150|$o/bench|python -u bench.py" \
  "200|$o/bench_cfg4|python -u bench.py --workload cfg4" \
  "150|$o/bench_cfg5|python -u bench.py --workload cfg5"
