#!/bin/bash
# GPU box, round 3: K2g v8 (unconditional gathers, straight-line chunks, Hilbert tiles, G = 21):
# full GPU suite, smoke, cfg3 / cfg4 / cfg5 bench lines, trace + PMC passes for cfg3 and cfg4.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g_v8
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "600|$o/gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "120|$o/smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "150|$o/bench|python -u bench.py" \
  "200|$o/bench_cfg4|python -u bench.py --workload cfg4" \
  "150|$o/bench_cfg5|python -u bench.py --workload cfg5" \
  "600|$o/prof3|PASSES=\"trace fetch write tcc sq\" bash tools/profile_bench.sh gpurun_out/$o/raster --steps 5 --warmup 1" \
  "600|$o/prof4|PASSES=\"trace fetch write tcc\" bash tools/profile_bench.sh gpurun_out/$o/cfg4 --workload cfg4 --steps 5 --warmup 1"
