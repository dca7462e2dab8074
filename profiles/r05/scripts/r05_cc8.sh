#!/bin/bash
# GPU box, round 5: the store floor of the cells output (tools/write_bw.hip) and k_cells alone
# (inline build, kernel trace).
cd "$GRAFT_REPO_ROOT"
o=r05/cc8
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "60|$o/write_bw|build/probes/write_bw" \
  "300|$o/prof_inl|UAM_LIB_PATH=build/variants/libuampath_cinl.so PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cinlp --cells --steps 5 --warmup 1"
