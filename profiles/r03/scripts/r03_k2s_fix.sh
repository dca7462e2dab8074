#!/bin/bash
# GPU box, round 3: K2s+pack (sequential sums, UAM_OPT_GROUP = 0) with one unconditional gather
# per waypoint against the previous build (lib/prev.so), same box.
cd "$GRAFT_REPO_ROOT"
o=r03/k2s_fix
mkdir -p gpurun_out/$o
L=uam_path_planning_amd/lib
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k2s.py tests/test_gpu_k2g.py -x -q --timeout 120 --timeout-method thread" \
  "150|$o/new|python -u bench.py --group 0 --no-cpu-baseline" \
  "150|$o/prev|UAM_LIB_PATH=$L/prev.so python -u bench.py --group 0 --no-cpu-baseline" \
  "150|$o/new2|python -u bench.py --group 0 --no-cpu-baseline"
