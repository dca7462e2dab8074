#!/bin/bash
# GPU box, round 3: K2g evaluation time vs raster size (512^2 .. 8192^2: table in L2 ... beyond
# the Infinity Cache), same cfg3 pairs, G = 21 and 8, kernel trace split per setting.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g_rsweep
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
steps=()
for R in 512 1024 2048 4096 8192; do
  steps+=("300|$o/R$R|rocprofv3 --kernel-trace -d gpurun_out/$o/tr$R -o run --output-format csv -- python3 -u tools/probe_k2g.py --groups 8,21 --tbits 4 --lds 0,40960 --reps 10 --R $R")
done
tools/gpu_session.sh "${steps[@]}"
