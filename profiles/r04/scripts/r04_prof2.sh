#!/bin/bash
# GPU box, round 4: K4h at 2 workgroups per CU with 11 gathers in flight, K2h at 3 per CU with 11
# on rasters over 2^25 cells; unit sums beside the scatter.  Tests, bench lines for cfg3 / cfg4 /
# cfg5, cfg4 + cfg5 traces and PMC passes.
cd "$GRAFT_REPO_ROOT"
o=r04/prof2
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "600|$o/tests|python -u -m pytest tests/test_gpu_k4h.py tests/test_gpu_k2h.py tests/test_gpu_fullsize.py -x -v --timeout 500 --timeout-method thread" \
  "150|$o/bench|python -u bench.py" \
  "300|$o/bench_cfg4|python -u bench.py --workload cfg4" \
  "200|$o/bench_cfg5|python -u bench.py --workload cfg5" \
  "500|$o/prof_cfg4|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg4 --workload cfg4 --steps 5 --warmup 1" \
  "400|$o/prof_cfg5|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
