#!/bin/bash
# GPU box, round 5: the cells output (k_cells beside K2h) and cfg4 at the 8-GPU per-rank share
# (25 000 pairs) beside the 1-GPU whole (200 000 pairs): benches, traces, FETCH / WRITE / TCC
# passes (profiles/r05/cells, profiles/r05/cfg4_q25k, profiles/r05/cfg4).
cd "$GRAFT_REPO_ROOT"
o=r05/cc
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
tools/gpu_session.sh \
  "120|$o/cells|$b --cells" \
  "300|$o/q25k|$b --workload cfg4 --pairs 25000" \
  "300|$o/q200k|$b --workload cfg4" \
  "400|$o/prof_cells|PASSES='trace fetch write tcc' bash tools/profile_bench.sh gpurun_out/$o/cells --cells --steps 5 --warmup 1" \
  "600|$o/prof_q25k|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/q25k --workload cfg4 --pairs 25000 --steps 5 --warmup 1" \
  "600|$o/prof_q200k|PASSES='trace fetch write tcc' bash tools/profile_bench.sh gpurun_out/$o/q200k --workload cfg4 --steps 5 --warmup 1"
