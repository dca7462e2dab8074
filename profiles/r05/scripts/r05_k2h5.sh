#!/bin/bash
# GPU box, round 5: K2h / K4h one chunk ahead (chunk c + 1's loads in flight while chunk c is
# consumed), per-path bounds sampled four at a time: GPU tests of the sorted forms + parity,
# cfg3 chunk / waves sweep (w3: the 3-waves-per-SIMD build), cfg5, trace + SQ + TCC.
cd "$GRAFT_REPO_ROOT"
o=r05/k2h5
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
w3="env UAM_LIB_PATH=build/variants/libuampath_w3.so"
tools/gpu_session.sh \
  "900|$o/tests|python -u -m pytest tests/test_gpu_k2h.py tests/test_gpu_k4h.py tests/test_gpu_parity.py tests/test_gpu_k2g.py tests/test_gpu_k2s.py -x -q --timeout 300 --timeout-method thread" \
  "90|$o/def|$b" \
  "90|$o/ch6|$b --opt k2g_chunk=6" \
  "90|$o/w3ch7|$w3 $b" \
  "90|$o/w3ch8|$w3 $b --opt k2g_chunk=8" \
  "90|$o/w3ch11|$w3 $b --opt k2g_chunk=11" \
  "90|$o/cfg5|$b --workload cfg5" \
  "90|$o/cfg5ch16|$b --workload cfg5 --opt k2g_chunk=16" \
  "300|$o/prof|PASSES='trace sq tcc' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1" \
  "300|$o/prof5|PASSES='trace sq tcc' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
