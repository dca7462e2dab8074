#!/bin/bash
# GPU box, round 5: K4h bound form (default) sweep: chunk, seed stride, LDS floor, chunk-ahead;
# trace + TCC + SQ of the default.
cd "$GRAFT_REPO_ROOT"
o=r05/k4h2
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline --workload cfg5"
ah="env UAM_LIB_PATH=build/variants/libuampath_ah.so"
tools/gpu_session.sh \
  "600|$o/tests|python -u -m pytest tests/test_gpu_k4h.py -x -q --timeout 300 --timeout-method thread" \
  "90|$o/def|$b" \
  "90|$o/ch7|$b --opt k2g_chunk=7" \
  "90|$o/ch8|$b --opt k2g_chunk=8" \
  "90|$o/ch16|$b --opt k2g_chunk=16" \
  "90|$o/s0|$b --opt k2h_lb_stride=0" \
  "90|$o/s4|$b --opt k2h_lb_stride=4" \
  "90|$o/s2|$b --opt k2h_lb_stride=2" \
  "90|$o/f40|$b --opt k2g_lds_floor=40000" \
  "90|$o/f80|$b --opt k2g_lds_floor=80000" \
  "90|$o/ah|$ah $b" \
  "300|$o/prof|PASSES='trace tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
