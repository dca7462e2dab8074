#!/bin/bash
# GPU box, round 3: the split volume (8-B voxels + column plane) -- its tests, the cfg5 bench
# line and its trace + PMC passes (tools/profile_bench.sh).  cfg4: tools/r03_cfg4.sh.
cd "$GRAFT_REPO_ROOT"
o=r03/vol
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/vol_tests|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k 'volume or cfg5' -x -q --timeout 300 --timeout-method thread" \
  "200|$o/bench_cfg5|python -u bench.py --workload cfg5" \
  "500|$o/prof5|PASSES=\"trace fetch write tcc sq\" bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
