#!/bin/bash
# GPU box, round 5: the waypoint cells on a lowest-priority side stream (grid 512 / uncapped /
# 2048, 256 / 384 / 1024, forked after the scatter; build variants) against the default.
cd "$GRAFT_REPO_ROOT"
o=r05/cc21
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
b="python -u bench.py --no-cpu-baseline --cells"
steps=()
for v in clo clo256 clo384 clo1024 clos2 clo; do steps+=("120|$o/$v|UAM_LIB_PATH=$V/libuampath_$v.so $b"); done
tools/gpu_session.sh "120|$o/def|$b" "${steps[@]}" \
  "120|$o/nocells|python -u bench.py --no-cpu-baseline"
