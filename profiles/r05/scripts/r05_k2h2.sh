#!/bin/bash
# GPU box, round 5: K2h v2 sweeps (sample stride of the terrain lower bound, chunk, workgroups per
# CU) on cfg3 and the SQ wave-cycle pass of the default.
cd "$GRAFT_REPO_ROOT"
o=r05/k2h2
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
tools/gpu_session.sh \
  "90|$o/def|$b" \
  "90|$o/lbs1024|$b --opt k2h_lb_stride=1024" \
  "90|$o/lbs16|$b --opt k2h_lb_stride=16" \
  "90|$o/lbs4|$b --opt k2h_lb_stride=4" \
  "90|$o/ch6|$b --opt k2g_chunk=6" \
  "90|$o/ch8|$b --opt k2g_chunk=8" \
  "90|$o/ch11|$b --opt k2g_chunk=11" \
  "90|$o/floor90k|$b --opt k2g_lds_floor=90000" \
  "300|$o/prof_sq|PASSES='sq' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1"
