#!/bin/bash
# GPU box, round 5: code 0 = nothing at all (terrain +0.0 too); K2h terrain-in-entry form with
# round 4's semantics (code 1 the 8-B {phi, terrain}, 2/3 the record) beside the bound form.
cd "$GRAFT_REPO_ROOT"
o=r05/k2h11
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
tools/gpu_session.sh \
  "900|$o/tests|python -u -m pytest tests/test_gpu_k2h.py tests/test_gpu_k2g.py tests/test_gpu_k2s.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread" \
  "90|$o/te|$b --opt k2h_terrain=1" \
  "90|$o/te_ch6|$b --opt k2h_terrain=1 --opt k2g_chunk=6" \
  "90|$o/bd|$b" \
  "90|$o/bd_ch6|$b --opt k2g_chunk=6" \
  "300|$o/prof|PASSES='trace sq tcc' bash tools/profile_bench.sh gpurun_out/$o/te --opt k2h_terrain=1 --steps 5 --warmup 1" \
  "300|$o/profb|PASSES='trace tcc' bash tools/profile_bench.sh gpurun_out/$o/bd --steps 5 --warmup 1"
