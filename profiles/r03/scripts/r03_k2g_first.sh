#!/bin/bash
# GPU box, round 3: first K2g run -- its tests, the K2s / kernel-identity tests, the cfg3
# bench at several group lengths (and K2s for A/B), a kernel trace of the default step.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g1
mkdir -p gpurun_out/$o
tools/gpu_session.sh \
  "400|$o/k2g_tests|python -u -m pytest tests/test_gpu_k2g.py -x -v --timeout 200 --timeout-method thread" \
  "200|$o/bench_g8|python -u bench.py --group 8" \
  "150|$o/bench_g4|python -u bench.py --group 4 --no-cpu-baseline" \
  "150|$o/bench_g12|python -u bench.py --group 12 --no-cpu-baseline" \
  "150|$o/bench_g16|python -u bench.py --group 16 --no-cpu-baseline" \
  "150|$o/bench_g0|python -u bench.py --group 0 --no-cpu-baseline" \
  "240|$o/prof|PASSES=\"trace\" bash tools/profile_bench.sh gpurun_out/$o/raster --steps 5 --warmup 1" \
  "500|$o/k2s_parity|python -u -m pytest tests/test_gpu_k2s.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 'k2s or bit_identical or full_size or raster'"
