#!/bin/bash
# round 6 call 25: randomized parity (tests/test_gpu_fuzz.py) -- the default seeds 0-11, then
# a sweep of seeds 12-299 (K1, K2h / K2g, K4h, analytic; every output against the oracle)
cd "$GRAFT_REPO_ROOT"
o=r06/c25
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_fuzz.py"
tools/gpu_session.sh \
  "600|$o/default|$T -x" \
  "900|$o/sweep|UAM_FUZZ_SEEDS=12:300 $T -rf"
