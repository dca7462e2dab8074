#!/bin/bash
# GPU box, round 5: the round-4 tree (build/r4, commit e64183f, its own library and bench) beside
# this tree on the same box: cfg3 and cfg5.
cd "$GRAFT_REPO_ROOT"
o=r05/r4cmp
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "120|$o/r4_cfg3|cd build/r4 && python -u bench.py --no-cpu-baseline" \
  "120|$o/r5_te|python -u bench.py --no-cpu-baseline --opt k2h_terrain=1" \
  "120|$o/r4_cfg3b|cd build/r4 && python -u bench.py --no-cpu-baseline" \
  "120|$o/r4_cfg5|cd build/r4 && python -u bench.py --no-cpu-baseline --workload cfg5" \
  "120|$o/r5_cfg5|python -u bench.py --no-cpu-baseline --workload cfg5" \
  "300|$o/r4prof|cd build/r4 && PASSES='trace sq tcc' bash ../../tools/profile_bench.sh ../../gpurun_out/$o/r4 --steps 5 --warmup 1"
