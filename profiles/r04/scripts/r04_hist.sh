#!/bin/bash
# GPU box, round 4: the unit sums of the histogram's extra block computed term-parallel
# (k_g_hist was 29.9 us in suite1's trace, the other blocks ~11 us): K2h / K4h tests, cfg3 + cfg5
# traces, bench lines.
cd "$GRAFT_REPO_ROOT"
o=r04/hist
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k4h.py tests/test_gpu_k2h.py -x -q --timeout 200 --timeout-method thread" \
  "200|$o/prof_cfg3|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1" \
  "200|$o/prof_cfg5|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1" \
  "150|$o/bench|python -u bench.py" \
  "200|$o/bench_cfg5|python -u bench.py --workload cfg5"
