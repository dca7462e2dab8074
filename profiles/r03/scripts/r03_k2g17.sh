#!/bin/bash
# GPU box, round 3: batched-load k_g_hist / k_g_scatter against the previous commit's library
# (lib/prev.so), same box, alternating; kernel trace of the new sort.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g17
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
L=uam_path_planning_amd/lib
P3="python -u tools/probe_k2g.py --groups 21 --chunks 8 --tbits 0 --reps 20"
tools/gpu_session.sh \
  "300|$o/k2g_tests|python -u -m pytest tests/test_gpu_k2g.py -x -q --timeout 120 --timeout-method thread" \
  "120|$o/new_a|$P3" "120|$o/prev_a|UAM_LIB_PATH=$L/prev.so $P3" \
  "120|$o/new_b|$P3" "120|$o/prev_b|UAM_LIB_PATH=$L/prev.so $P3" \
  "120|$o/trace|rocprofv3 --kernel-trace --stats -d gpurun_out/$o/trace -o run --output-format csv -- python3 tools/probe_k2g.py --groups 21 --chunks 8 --tbits 0 --reps 5"
