#!/bin/bash
# GPU box, round 5: K4h's sort key on the round-5 layout -- tiles (k2g_tile_bits 3 default / 4 /
# 2) and altitude bands (k4h_band 4 default at 64 layers / 2 / 8 / 16).
cd "$GRAFT_REPO_ROOT"
o=r05/cc22
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline --workload cfg5"
tools/gpu_session.sh "120|$o/def|$b" "120|$o/t4|$b --opt k2g_tile_bits=4" \
  "120|$o/t2|$b --opt k2g_tile_bits=2" "120|$o/b2|$b --opt k4h_band=2" "120|$o/b8|$b --opt k4h_band=8" \
  "120|$o/b16|$b --opt k4h_band=16" "120|$o/t4b8|$b --opt k2g_tile_bits=4 --opt k4h_band=8" "120|$o/def2|$b"
