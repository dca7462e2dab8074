#!/bin/bash
# GPU box, round 5: K2h terrain in the entry (UAM_OPT_K2H_TERRAIN 1: 8-B {phi, terrain} / 16-B
# records, no bounds) against the bound form: tests, cfg3 benches, trace + SQ + TCC.
cd "$GRAFT_REPO_ROOT"
o=r05/k2h8
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
tools/gpu_session.sh \
  "900|$o/tests|python -u -m pytest tests/test_gpu_k2h.py -x -q --timeout 300 --timeout-method thread" \
  "90|$o/def|$b" \
  "90|$o/te|$b --opt k2h_terrain=1" \
  "90|$o/te6|$b --opt k2h_terrain=1 --opt k2g_chunk=6" \
  "90|$o/te8|$b --opt k2h_terrain=1 --opt k2g_chunk=8" \
  "90|$o/te11|$b --opt k2h_terrain=1 --opt k2g_chunk=11" \
  "300|$o/prof|PASSES='trace sq tcc' bash tools/profile_bench.sh gpurun_out/$o/te --opt k2h_terrain=1 --steps 5 --warmup 1"
