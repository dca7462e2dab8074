#!/bin/bash
# Round 6 closing check on the committed tree: the whole GPU suite (with the randomized parity
# tests), smoke, and the default bench line.  usage: final3.sh
cd "$GRAFT_REPO_ROOT"
o=r06/final3
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "700|$o/suite|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "300|$o/smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "300|$o/bench|python -u bench.py"
