#!/bin/bash
# round 6 call 12: K4h seeds from the groups' middle waypoints, formed with the sort keys in
# k_v_hist (one terrain load + one atomicMin per item) instead of a per-path sampling loop --
# the K4h tests (bit-exact vs the oracle), then cfg5 bench + trace
cd "$GRAFT_REPO_ROOT"
o=r06/c12
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "600|$o/tests|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_k4h.py tests/test_gpu_fullsize.py" \
  "300|$o/probe|python -u tools/probe_opts.py --tag cfg5 --volume --reps 20 --settings 'k2h_lb_stride=16;k2h_lb_stride=0;k2h_lb_stride=16'" \
  "300|$o/bench_cfg5|python -u bench.py --workload cfg5" \
  "300|$o/trace|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
