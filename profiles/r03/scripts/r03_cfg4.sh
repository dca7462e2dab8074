#!/bin/bash
# GPU box, round 3: the cfg4 bench line (8192^2 from GeoTIFF tiles) and its trace + PMC passes.
cd "$GRAFT_REPO_ROOT"
o=r03/cfg4
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/bench_cfg4|python -u bench.py --workload cfg4" \
  "850|$o/prof4|PASSES=\"trace fetch write tcc sq\" bash tools/profile_bench.sh gpurun_out/$o/cfg4 --workload cfg4 --steps 5 --warmup 1"
