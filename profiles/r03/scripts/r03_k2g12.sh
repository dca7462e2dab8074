#!/bin/bash
# GPU box, round 3: K2g v8 counters (sq pass) and the last-group bins on / off.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g12
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
L=uam_path_planning_amd/lib
tools/gpu_session.sh \
  "240|$o/lastbin_on|python -u tools/probe_k2g.py --groups 21,24 --tbits 4 --chunks 8 --reps 20" \
  "240|$o/lastbin_off|UAM_LIB_PATH=$L/nolastbin.so python -u tools/probe_k2g.py --groups 21,24 --tbits 4 --chunks 8 --reps 20" \
  "600|$o/prof|PASSES=\"trace sq\" bash tools/profile_bench.sh gpurun_out/$o/raster --steps 5 --warmup 1"
tools/gpu_session.sh \
  "300|$o/grid|python -u tools/probe_k2g.py --groups 8,12,16,21 --tbits 4,5,6 --lds 0,40960,54000 --chunks 8 --reps 10"
