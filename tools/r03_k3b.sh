#!/bin/bash
# GPU box, round 3: K3b with the two shape walks interleaved (one inequality of each shape per
# step; lib/libuampath_fused.so, -DUAM_K3B_FUSED_WALKS) against the default sequential walks:
# the analytic cfg3 bench line of each, twice.
cd "$GRAFT_REPO_ROOT"
o=r03/k3b
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
F=$GRAFT_REPO_ROOT/uam_path_planning_amd/lib/libuampath_fused.so
tools/gpu_session.sh \
  "200|$o/bench_seq|python -u bench.py --mode analytic --no-cpu-baseline" \
  "200|$o/bench_fused1|env UAM_LIB_PATH=$F python -u bench.py --mode analytic --no-cpu-baseline" \
  "200|$o/bench_seq2|python -u bench.py --mode analytic --no-cpu-baseline" \
  "200|$o/bench_fused1b|env UAM_LIB_PATH=$F python -u bench.py --mode analytic --no-cpu-baseline"
