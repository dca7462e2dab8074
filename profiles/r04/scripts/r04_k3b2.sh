#!/bin/bash
# GPU box, round 4: K3b at 1 workgroup per CU (measurement build, LDS floor 90 000 B) against
# the product build (2 per CU).
cd "$GRAFT_REPO_ROOT"
o=r04/k3b2
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
S="k3b_segment=8,k3b_points_per_lane=1;k3b_segment=8,k3b_points_per_lane=2;k3b_segment=16,k3b_points_per_lane=1;k3b_segment=8,k3b_points_per_lane=1"
tools/gpu_session.sh \
  "300|$o/base|python -u tools/probe_opts.py --analytic --reps 10 --tag base --settings '$S'" \
  "300|$o/f1|UAM_LIB_PATH=build/variants/libuampath_k3bf1.so python -u tools/probe_opts.py --analytic --reps 10 --tag f1 --settings '$S'"
