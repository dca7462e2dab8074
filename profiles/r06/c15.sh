#!/bin/bash
# round 6 call 15: K1 with the inequality kind branch taken once per column (ineq_h_col) and
# nontemporal record stores -- raster parity tests, then K1 against the previous NT build
cd "$GRAFT_REPO_ROOT"
o=r06/c15
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
P="python -u tools/probe_k1.py --cases cfg3,cfg3-obstacles,regions,empty --reps 20"
tools/gpu_session.sh \
  "400|$o/tests|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k 'raster_build or raster_eval or snapped or raster_kernels'" \
  "200|$o/col|$P" \
  "200|$o/nt|env UAM_LIB_PATH=$V/libuampath_nt.so $P" \
  "200|$o/col_8k|python -u tools/probe_k1.py --R 8192 --cases cfg3 --reps 20" \
  "200|$o/col_cpl4|$P --cpl 4"
