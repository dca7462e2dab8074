#!/bin/bash
# GPU box, round 4: the block-total scan folded into the scatter (no k_scan_totals launch for
# up to 1024 scan blocks): grouped tests, cfg3 / cfg5 traces, bench lines.
cd "$GRAFT_REPO_ROOT"
o=r04/scan
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "600|$o/tests|python -u -m pytest tests/test_gpu_k4h.py tests/test_gpu_k2h.py tests/test_gpu_k2g.py tests/test_gpu_fullsize.py -x -q --timeout 500 --timeout-method thread" \
  "200|$o/prof_cfg3|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1" \
  "200|$o/prof_cfg5|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1" \
  "150|$o/bench|python -u bench.py" \
  "200|$o/bench_cfg5|python -u bench.py --workload cfg5"
