#!/bin/bash
# GPU box, round 3: K6 restarts -- refinement tests, then cfg3-map refinement (20k pairs x 5,
# default settings) with 0, 1 and 2 restarts: throughput and the share of feasible-endpoint
# candidates / pairs reaching sum g^2 <= 1e-3.
cd "$GRAFT_REPO_ROOT"
o=r03/k6
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/refine_tests|python -u -m pytest tests/test_gpu_refine.py -x -q --timeout 300 --timeout-method thread" \
  "200|$o/r0|python3 -u tools/time_refine.py --pairs 20000 --nfz 64 --outer 15 --inner 50 --set n_restart=0" \
  "300|$o/r1|python3 -u tools/time_refine.py --pairs 20000 --nfz 64 --outer 15 --inner 50 --set n_restart=1" \
  "300|$o/r2|python3 -u tools/time_refine.py --pairs 20000 --nfz 64 --outer 15 --inner 50 --set n_restart=2"
