#!/bin/bash
# GPU box, round 5: K4h altitude bands on the round-5 layout, repeated -- k4h_band 4 (the
# default at 64 layers) / 2 / 1 (cc22: tiles 3 best; bands 2 0.390 vs 0.394-0.396 ms).
cd "$GRAFT_REPO_ROOT"
o=r05/cc23
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline --workload cfg5"
tools/gpu_session.sh "120|$o/def|$b" "120|$o/b2|$b --opt k4h_band=2" "120|$o/b1|$b --opt k4h_band=1" \
  "120|$o/def2|$b" "120|$o/b2_2|$b --opt k4h_band=2" "120|$o/b1_2|$b --opt k4h_band=1"
