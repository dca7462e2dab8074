#!/bin/bash
# GPU box, round 5: cfg4 (8192^2) at the per-rank shares of the strong-scaling run on one GPU --
# 25k pairs (125k paths: rank 0 at 8 GPUs), 50k (4 GPUs), 100k (2 GPUs), 200k (1 GPU) -- and the
# trace + PMC passes of the 8-GPU share (the round-4 tree's K2h).
cd "$GRAFT_REPO_ROOT"
o=r05/cfg4share
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "240|$o/q25k|python -u bench.py --workload cfg4 --pairs 25000 --no-cpu-baseline" \
  "240|$o/q50k|python -u bench.py --workload cfg4 --pairs 50000 --no-cpu-baseline" \
  "240|$o/q100k|python -u bench.py --workload cfg4 --pairs 100000 --no-cpu-baseline" \
  "300|$o/q200k|python -u bench.py --workload cfg4 --no-cpu-baseline" \
  "500|$o/prof_q25k|PASSES='trace fetch write tcc' bash tools/profile_bench.sh gpurun_out/$o/q25k_prof --workload cfg4 --pairs 25000 --steps 5 --warmup 1"
