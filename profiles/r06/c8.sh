#!/bin/bash
# round 6 call 8: cfg3 K2h group length x tile bits (a group's reach around its sort tile sets
# the lines an XCD's window touches; round 4 swept G with K2g's per-waypoint geometry only)
cd "$GRAFT_REPO_ROOT"
o=r06/c8
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
S=""
for g in 21 7 10 12 14 17 18 28; do for tb in 0 5 3; do S="$S;group=$g,k2g_tile_bits=$tb"; done; done
S="${S#;};group=21,k2g_tile_bits=0"
tools/gpu_session.sh \
  "600|$o/tests|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_k2s.py tests/test_gpu_k2g.py tests/test_gpu_k2h.py tests/test_gpu_k4h.py tests/test_gpu_parity.py" \
  "500|$o/gsweep|python -u tools/probe_opts.py --tag gsweep --reps 20 --settings '$S'"
