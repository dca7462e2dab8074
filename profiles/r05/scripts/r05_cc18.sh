#!/bin/bash
# GPU box, round 5: K4h's clearance seeds on the side stream (default) vs inside the histogram
# launch (build variant); the K4h tests; a trace of the default.
cd "$GRAFT_REPO_ROOT"
o=r05/cc18
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
b="python -u bench.py --no-cpu-baseline --workload cfg5"
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k4h.py -x -q --timeout 120 --timeout-method thread" \
  "120|$o/side|$b" "120|$o/hist|UAM_LIB_PATH=$V/libuampath_seedh.so $b" \
  "120|$o/side2|$b" "120|$o/hist2|UAM_LIB_PATH=$V/libuampath_seedh.so $b" \
  "120|$o/side_s16|$b --opt k2h_lb_stride=16" \
  "300|$o/prof|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/c5 --workload cfg5 --steps 5 --warmup 1"
