#!/bin/bash
# round 6 call 27: randomized parity with the form draw (sorted / the library's choice /
# sequential order) and waypoint cells: the suite's seeds, then seeds 48-2999
cd "$GRAFT_REPO_ROOT"
o=r06/c27
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_fuzz.py -rf"
tools/gpu_session.sh \
  "300|$o/default|$T -x" \
  "900|$o/sweep1|UAM_FUZZ_SEEDS=48:1500 $T" \
  "900|$o/sweep2|UAM_FUZZ_SEEDS=1500:3000 $T"
