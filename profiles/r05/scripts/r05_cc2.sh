#!/bin/bash
# GPU box, round 5: K4h bound-form combinations; the cells output (k_cells beside K2h); cfg4 at
# the 8-GPU per-rank share (25 000 pairs) and whole (200 000 pairs); traces + PMC passes.
cd "$GRAFT_REPO_ROOT"
o=r05/cc
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
b5="$b --workload cfg5"
tools/gpu_session.sh \
  "90|$o/k4_ch7_s0|$b5 --opt k2g_chunk=7 --opt k2h_lb_stride=0" \
  "90|$o/k4_ch7_f40|$b5 --opt k2g_chunk=7 --opt k2g_lds_floor=40000" \
  "90|$o/k4_ch7_f40_s0|$b5 --opt k2g_chunk=7 --opt k2g_lds_floor=40000 --opt k2h_lb_stride=0" \
  "90|$o/k4_ch6|$b5 --opt k2g_chunk=6" \
  "90|$o/k4_ch6_s0|$b5 --opt k2g_chunk=6 --opt k2h_lb_stride=0" \
  "90|$o/k4_ch7_f28|$b5 --opt k2g_chunk=7 --opt k2g_lds_floor=28000" \
  "120|$o/cells|$b --cells" \
  "300|$o/q25k|$b --workload cfg4 --pairs 25000" \
  "300|$o/q200k|$b --workload cfg4" \
  "400|$o/prof_cells|PASSES='trace fetch write tcc' bash tools/profile_bench.sh gpurun_out/$o/cells --cells --steps 5 --warmup 1" \
  "600|$o/prof_q25k|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/q25k --workload cfg4 --pairs 25000 --steps 5 --warmup 1" \
  "600|$o/prof_q200k|PASSES='trace fetch write tcc' bash tools/profile_bench.sh gpurun_out/$o/q200k --workload cfg4 --steps 5 --warmup 1"
