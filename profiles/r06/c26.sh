#!/bin/bash
# round 6 call 26: randomized parity, a long sweep (seeds 300-2999) after c25's 0-299
cd "$GRAFT_REPO_ROOT"
o=r06/c26
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_fuzz.py -rf"
tools/gpu_session.sh \
  "300|$o/default|$T -x" \
  "900|$o/sweep1|UAM_FUZZ_SEEDS=300:1600 $T" \
  "900|$o/sweep2|UAM_FUZZ_SEEDS=1600:3000 $T"
