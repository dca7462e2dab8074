#!/bin/bash
# GPU box, round 4: K4h (packed volume, sorted grouped evaluation) tests + cfg5 bench; K2h
# tests after the unit-sum block change; cfg3 trace + bench.
cd "$GRAFT_REPO_ROOT"
o=r04/k4h1
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/tests|python -u -m pytest tests/test_gpu_k4h.py tests/test_gpu_k2h.py -x -q --timeout 200 --timeout-method thread" \
  "200|$o/bench_cfg5|python -u bench.py --workload cfg5" \
  "200|$o/trace|rocprofv3 --kernel-trace --stats -d gpurun_out/$o/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10" \
  "150|$o/bench|python -u bench.py"
