#!/bin/bash
# GPU box, round 3: K2g v5 (pass 1 in the items, division-free kinematic rows) -- its tests,
# the group-length sweep on cfg3 under a kernel trace split per setting, the bench line.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g5
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/k2g_tests|python -u -m pytest tests/test_gpu_k2g.py tests/test_gpu_k2s.py -x -q --timeout 200 --timeout-method thread" \
  "400|$o/probe|rocprofv3 --kernel-trace -d gpurun_out/$o/tr -o run --output-format csv -- python3 -u tools/probe_k2g.py --groups 16,21,28,32,41 --tbits 4 --lds 0 --reps 10" \
  "200|$o/bench|python -u bench.py"
