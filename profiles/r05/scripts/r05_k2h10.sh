#!/bin/bash
# GPU box, round 5: K2h mixed terrain form (UAM_OPT_K2H_TERRAIN 1: code 1 the 8-B {phi, terrain}
# entry, codes 2/3 the record, code 0 by the bound rule): tests, seeds on / off, chunks, bounds
# form beside it, trace + SQ + TCC of the mixed form.
cd "$GRAFT_REPO_ROOT"
o=r05/k2h10
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
tools/gpu_session.sh \
  "900|$o/tests|python -u -m pytest tests/test_gpu_k2h.py tests/test_gpu_k4h.py -x -q --timeout 300 --timeout-method thread" \
  "90|$o/te|$b --opt k2h_terrain=1" \
  "90|$o/te_s0|$b --opt k2h_terrain=1 --opt k2h_lb_stride=0" \
  "90|$o/te_s4|$b --opt k2h_terrain=1 --opt k2h_lb_stride=4" \
  "90|$o/te_ch6|$b --opt k2h_terrain=1 --opt k2g_chunk=6" \
  "90|$o/te_ch8|$b --opt k2h_terrain=1 --opt k2g_chunk=8" \
  "90|$o/bd|$b" \
  "90|$o/bd_s0|$b --opt k2h_lb_stride=0" \
  "300|$o/prof|PASSES='trace sq tcc' bash tools/profile_bench.sh gpurun_out/$o/te --opt k2h_terrain=1 --steps 5 --warmup 1"
