#!/bin/bash
# GPU box, round 4: K3b with every psi term in the segment's term list (52.9 KiB of LDS per
# workgroup instead of 70.8: 3 per CU instead of 2) against the previous build; K3b tests.
cd "$GRAFT_REPO_ROOT"
o=r04/k3b1
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
S="k3b_segment=8,k3b_points_per_lane=1;k3b_segment=6,k3b_points_per_lane=1;k3b_segment=8,k3b_points_per_lane=2;k3b_segment=4,k3b_points_per_lane=1;k3b_segment=8,k3b_points_per_lane=1"
tools/gpu_session.sh \
  "600|$o/tests|python -u -m pytest tests/test_gpu_k3b.py -x -q --timeout 300 --timeout-method thread" \
  "300|$o/new|python -u tools/probe_opts.py --analytic --reps 10 --tag new --settings '$S'" \
  "300|$o/old|UAM_LIB_PATH=build/variants/libuampath_k3bold.so python -u tools/probe_opts.py --analytic --reps 10 --tag old --settings '$S'"
