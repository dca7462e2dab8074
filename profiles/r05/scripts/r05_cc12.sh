#!/bin/bash
# GPU box, round 5: K4h's seed stride (k2h_lb_stride 0 / 4 / 16 / 32 vs the default 8) on
# cfg5; cfg4 rank 3's share with fewer sort bins (tile bits 4 / 3 vs 5) -- traces for the
# sort launches' split.
cd "$GRAFT_REPO_ROOT"
o=r05/cc12
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
tools/gpu_session.sh \
  "120|$o/c5_s8|$b --workload cfg5" \
  "120|$o/c5_s0|$b --workload cfg5 --opt k2h_lb_stride=0" \
  "120|$o/c5_s4|$b --workload cfg5 --opt k2h_lb_stride=4" \
  "120|$o/c5_s16|$b --workload cfg5 --opt k2h_lb_stride=16" \
  "120|$o/c5_s32|$b --workload cfg5 --opt k2h_lb_stride=32" \
  "120|$o/s3_t5|$b --workload cfg4 --share 3/8" \
  "120|$o/s3_t4|$b --workload cfg4 --share 3/8 --opt k2g_tile_bits=4" \
  "120|$o/s3_t3|$b --workload cfg4 --share 3/8 --opt k2g_tile_bits=3" \
  "120|$o/c3_t3|$b --opt k2g_tile_bits=3" \
  "300|$o/p_s3t4|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/s3t4 --workload cfg4 --share 3/8 --opt k2g_tile_bits=4 --steps 5 --warmup 1" \
  "300|$o/p_c5s16|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/c5s16 --workload cfg5 --opt k2h_lb_stride=16 --steps 5 --warmup 1"
