#!/bin/bash
# GPU box, round 3: persistent K2g evaluation (one-item-ahead order / pair loads) against the
# previous commit's library (lib/prev.so), same box, alternating; cfg3 and cfg4 sizes.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g16
mkdir -p gpurun_out/$o
L=uam_path_planning_amd/lib
P3="python -u tools/probe_k2g.py --groups 21 --tbits 4 --chunks 8 --reps 20"
P4="python -u tools/probe_k2g.py --R 8192 --pairs 200000 --groups 21 --tbits 5 --chunks 8 --reps 10"
tools/gpu_session.sh \
  "300|$o/k2g_tests|python -u -m pytest tests/test_gpu_k2g.py -x -q --timeout 120 --timeout-method thread" \
  "120|$o/new_a|$P3" "120|$o/prev_a|UAM_LIB_PATH=$L/prev.so $P3" \
  "120|$o/new_b|$P3" "120|$o/prev_b|UAM_LIB_PATH=$L/prev.so $P3" \
  "200|$o/new4|$P4" "200|$o/prev4|UAM_LIB_PATH=$L/prev.so $P4"
