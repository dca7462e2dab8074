#!/bin/bash
# GPU box, round 4: the histogram with 8 items per thread per round (one round at cfg3) against
# 4 (two rounds): cfg3 traces of bench.py with each build.
cd "$GRAFT_REPO_ROOT"
o=r04/hist2
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "200|$o/prof_base|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/base --steps 5 --warmup 1" \
  "200|$o/prof_u8|UAM_LIB_PATH=build/variants/libuampath_histu8.so PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/u8 --steps 5 --warmup 1"
