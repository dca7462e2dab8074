#!/bin/bash
# GPU box, round 5: K2h branch-free issue loop (e8 at the p4/t4 index): GPU tests of the sorted
# forms, cfg3 bench + stride sweep, SQ and TCC passes.
cd "$GRAFT_REPO_ROOT"
o=r05/k2h3
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
tools/gpu_session.sh \
  "600|$o/tests|python -u -m pytest tests/test_gpu_k2h.py tests/test_gpu_k4h.py tests/test_gpu_k2s.py tests/test_gpu_k2g.py -x -q --timeout 300 --timeout-method thread" \
  "90|$o/def|$b" \
  "90|$o/lbs16|$b --opt k2h_lb_stride=16" \
  "90|$o/lbs32|$b --opt k2h_lb_stride=32" \
  "90|$o/cfg5|$b --workload cfg5" \
  "300|$o/prof|PASSES='sq tcc' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1"
