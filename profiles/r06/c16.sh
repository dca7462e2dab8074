#!/bin/bash
# round 6 call 16: K1 -- a shape's inequality loop ended once no needed cell can change
# (measurement build) against the product build
cd "$GRAFT_REPO_ROOT"
o=r06/c16
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
P="python -u tools/probe_k1.py --cases cfg3,cfg3-obstacles,regions,empty --reps 20"
tools/gpu_session.sh \
  "200|$o/col|$P" \
  "200|$o/exit|env UAM_LIB_PATH=$V/libuampath_exit.so $P" \
  "200|$o/exit_cpl4|env UAM_LIB_PATH=$V/libuampath_exit.so $P --cpl 4" \
  "200|$o/col2|$P"
