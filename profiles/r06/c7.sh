#!/bin/bash
# round 6 call 7: cfg5 (K4h) seed stride sweep -- the histogram launch's per-path clearance
# seeds (every n-th waypoint sampled) against the evaluation's terrain fetches
cd "$GRAFT_REPO_ROOT"
o=r06/c7
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/lbs|python -u tools/probe_opts.py --tag lbs --volume --reps 20 --settings 'k2h_lb_stride=8;k2h_lb_stride=16;k2h_lb_stride=32;k2h_lb_stride=81;k2h_lb_stride=0;k2h_lb_stride=4;k2h_lb_stride=8'" \
  "300|$o/trace16|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cfg5_16 --workload cfg5 --steps 5 --warmup 1 --opt k2h_lb_stride=16"
