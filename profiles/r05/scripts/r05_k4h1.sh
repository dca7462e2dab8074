#!/bin/bash
# GPU box, round 5: K4h terrain-in-entry with 16-B voxels in 4 x 2-column blocks (round 4's
# layout): K4h tests, cfg5 chunk / LDS-floor / chunk-ahead sweep, trace + TCC.
cd "$GRAFT_REPO_ROOT"
o=r05/k4h1
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline --workload cfg5"
ah="env UAM_LIB_PATH=build/variants/libuampath_ah.so"
tools/gpu_session.sh \
  "600|$o/tests|python -u -m pytest tests/test_gpu_k4h.py -x -q --timeout 300 --timeout-method thread" \
  "90|$o/def|$b" \
  "90|$o/ch7|$b --opt k2g_chunk=7" \
  "90|$o/ch7_f40|$b --opt k2g_chunk=7 --opt k2g_lds_floor=40000" \
  "90|$o/ch7_f28|$b --opt k2g_chunk=7 --opt k2g_lds_floor=28000" \
  "90|$o/ch8_f40|$b --opt k2g_chunk=8 --opt k2g_lds_floor=40000" \
  "90|$o/ch6_f28|$b --opt k2g_chunk=6 --opt k2g_lds_floor=28000" \
  "90|$o/ah|$ah $b" \
  "90|$o/ah_ch7|$ah $b --opt k2g_chunk=7" \
  "90|$o/bd|$b --opt k2h_terrain=0" \
  "300|$o/prof|PASSES='trace tcc' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
