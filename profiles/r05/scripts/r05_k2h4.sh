#!/bin/bash
# GPU box, round 5: K2h / K4h in three phases (cells / header reads / decisions + loads), 32-bit
# offsets from the packed base (r16 / v16 planes at the p4 index), per-path bounds from the
# histogram launch: the whole GPU suite, cfg3 + cfg5 bench + stride sweep, cfg3 / cfg5 trace +
# SQ + TCC passes.
cd "$GRAFT_REPO_ROOT"
o=r05/k2h4
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
tools/gpu_session.sh \
  "900|$o/tests|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "90|$o/def|$b" \
  "90|$o/lbs4|$b --opt k2h_lb_stride=4" \
  "90|$o/lbs2|$b --opt k2h_lb_stride=2" \
  "90|$o/cfg5|$b --workload cfg5" \
  "90|$o/cfg5l4|$b --workload cfg5 --opt k2h_lb_stride=4" \
  "300|$o/prof|PASSES='trace sq tcc' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1" \
  "300|$o/prof5|PASSES='trace sq tcc' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
