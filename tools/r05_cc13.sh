#!/bin/bash
# GPU box, round 5: the GPU suite on the column-order K1 default (128 rows); K1 alone by strip
# order -- the default, row-major, columns of 256 / 512 / 4096 rows (build variants).
cd "$GRAFT_REPO_ROOT"
o=r05/cc14
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
k1="tools/probe_k1.py --cases cfg3,empty,cfg3"
steps=("120|$o/k1_def|python -u $k1")
for v in k1row k1t256 k1t512 k1t4096; do
  steps+=("120|$o/$v|UAM_LIB_PATH=$V/libuampath_$v.so python -u $k1")
done
steps+=("120|$o/k1_def2|python -u $k1")
tools/gpu_session.sh "600|$o/suite|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" "${steps[@]}"
