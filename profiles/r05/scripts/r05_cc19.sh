#!/bin/bash
# GPU box, round 5: K1 rows per lane (k1_rows 2 default / 4 / 8) with the column strip order
# and the capped grid.
cd "$GRAFT_REPO_ROOT"
o=r05/cc19
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
k1="tools/probe_k1.py --cases cfg3,empty,cfg3"
tools/gpu_session.sh "120|$o/cpl2|python -u $k1" "120|$o/cpl4|python -u $k1 --cpl 4" \
  "120|$o/cpl8|python -u $k1 --cpl 8" "120|$o/cpl2b|python -u $k1"
