#!/bin/bash
# GPU box, round 3: K2g time decomposition -- the default build against measurement builds
# without memory (-DUAM_K2G_PROBE=1: synthetic records from the addresses), without pass 1
# (=2) and without either (=3); cfg3 (4096^2) and an L2-resident 512^2 raster.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g_decomp
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
L=uam_path_planning_amd/lib
steps=()
for v in libuampath probe1 probe2 probe3; do
  for R in 4096 512; do
    steps+=("240|$o/${v}_R$R|UAM_LIB_PATH=$L/$v.so python -u tools/probe_k2g.py --groups 21 --tbits 4 --R $R --reps 20")
  done
done
tools/gpu_session.sh "${steps[@]}"
