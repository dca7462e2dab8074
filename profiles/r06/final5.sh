#!/bin/bash
# Round 6 closing check on the committed tree (c28's setup kernels): the whole GPU suite,
# smoke, the default and cfg4 bench lines
cd "$GRAFT_REPO_ROOT"
o=r06/final5
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "700|$o/suite|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "300|$o/smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "300|$o/bench|python -u bench.py" \
  "400|$o/bench_cfg4|python -u bench.py --workload cfg4" \
  "300|$o/bench_cfg5|python -u bench.py --workload cfg5"
