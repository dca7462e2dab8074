#!/bin/bash
# GPU box, round 3: K2g v6 (each point generated once, pass 1 folded into the gather loop,
# Phi / N by one fma residual step) -- its tests, the group sweep on cfg3 and at 512^2 (table
# in L2: the compute floor), kernel trace split per setting.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g6
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/k2g_tests|python -u -m pytest tests/test_gpu_k2g.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread" \
  "400|$o/probe|rocprofv3 --kernel-trace -d gpurun_out/$o/tr -o run --output-format csv -- python3 -u tools/probe_k2g.py --groups 16,21,28,32 --tbits 4 --lds 0 --reps 10" \
  "300|$o/probe512|rocprofv3 --kernel-trace -d gpurun_out/$o/tr512 -o run --output-format csv -- python3 -u tools/probe_k2g.py --groups 21,28 --tbits 4 --lds 0 --reps 10 --R 512"
