#!/bin/bash
# GPU box, round 5: K2h terrain in the entry with p8 in 4 x 4-cell blocks and only the code map
# in LDS; one ahead vs not (na build); LDS floors (workgroups per CU); trace + SQ + TCC.
cd "$GRAFT_REPO_ROOT"
o=r05/k2h9
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
na="env UAM_LIB_PATH=build/variants/libuampath_na.so"
tools/gpu_session.sh \
  "900|$o/tests|python -u -m pytest tests/test_gpu_k2h.py -x -q --timeout 300 --timeout-method thread" \
  "90|$o/te|$b --opt k2h_terrain=1" \
  "90|$o/te_f40|$b --opt k2h_terrain=1 --opt k2g_lds_floor=40000" \
  "90|$o/te_f27|$b --opt k2h_terrain=1 --opt k2g_lds_floor=27000" \
  "90|$o/te_na|$na $b --opt k2h_terrain=1" \
  "90|$o/te_na_ch8|$na $b --opt k2h_terrain=1 --opt k2g_chunk=8" \
  "90|$o/bd|$b" \
  "90|$o/bd_na|$na $b" \
  "300|$o/prof|PASSES='trace sq tcc' bash tools/profile_bench.sh gpurun_out/$o/te --opt k2h_terrain=1 --steps 5 --warmup 1"
