#!/bin/bash
# GPU box, round 5: terrain-in-entry defaults for K2h and K4h (256-item K2h workgroups, no
# chunk-ahead): the whole GPU suite, cfg3 / cfg5 benches and chunk sweeps, traces + PMC.
cd "$GRAFT_REPO_ROOT"
o=r05/k2h13
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
tools/gpu_session.sh \
  "1000|$o/tests|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "90|$o/cfg3|$b" \
  "90|$o/cfg3_ch8|$b --opt k2g_chunk=8" \
  "90|$o/cfg3_ch6|$b --opt k2g_chunk=6" \
  "90|$o/cfg5|$b --workload cfg5" \
  "90|$o/cfg5_ch7|$b --workload cfg5 --opt k2g_chunk=7" \
  "90|$o/cfg5_ch8|$b --workload cfg5 --opt k2g_chunk=8" \
  "90|$o/cfg5_ch16|$b --workload cfg5 --opt k2g_chunk=16" \
  "90|$o/cfg5_bd|$b --workload cfg5 --opt k2h_terrain=0" \
  "300|$o/prof|PASSES='trace sq tcc fetch write' bash tools/profile_bench.sh gpurun_out/$o/cfg3p --steps 5 --warmup 1" \
  "300|$o/prof5|PASSES='trace sq tcc fetch write' bash tools/profile_bench.sh gpurun_out/$o/cfg5p --workload cfg5 --steps 5 --warmup 1"
