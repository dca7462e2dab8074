#!/bin/bash
# GPU box, round 5: K1 alone with the next strip's DEM prefetched, uncapped (default) vs
# capped grids of 1024-8192 workgroups looping over strips (build variants); raster parity.
cd "$GRAFT_REPO_ROOT"
o=r05/cc16
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
k1="tools/probe_k1.py --cases cfg3,empty,cfg3"
steps=("120|$o/k1_def|python -u $k1")
for v in k1c6144 k1c8192 k1c12288 k1c16384; do
  steps+=("120|$o/$v|UAM_LIB_PATH=$V/libuampath_$v.so python -u $k1")
done
steps+=("120|$o/k1_def2|python -u $k1")
tools/gpu_session.sh "${steps[@]}"
