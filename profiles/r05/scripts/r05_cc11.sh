#!/bin/bash
# GPU box, round 5: the whole GPU suite and smoke on the cells-on-the-side-stream build; the
# default bench, cfg3 with cells and cfg5 with the CPU baseline / parity; the cells PMC set.
cd "$GRAFT_REPO_ROOT"
o=r05/cc11
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "600|$o/suite|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300|$o/smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "300|$o/bench|python -u bench.py" \
  "300|$o/cells|python -u bench.py --cells" \
  "300|$o/cfg5|python -u bench.py --workload cfg5" \
  "400|$o/prof_cells|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cellsp --cells --steps 5 --warmup 1"
