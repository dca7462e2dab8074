#!/bin/bash
# round 6 call 29: K1 after the round-6 changes -- grid caps, 256-row strip columns and rows per
# lane, at 4096^2 and 8192^2 (measurement builds; the product is cap 8192, 128 rows, 2 per lane)
cd "$GRAFT_REPO_ROOT"
o=r06/c29
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
P="python -u tools/probe_k1.py --cases cfg3 --reps 20"
tools/gpu_session.sh \
  "200|$o/base|$P && $P --R 8192 && $P --cpl 4 && $P --R 8192 --cpl 4" \
  "200|$o/cap4k|env UAM_LIB_PATH=$V/libuampath_cap4k.so $P && env UAM_LIB_PATH=$V/libuampath_cap4k.so $P --R 8192" \
  "200|$o/cap16k|env UAM_LIB_PATH=$V/libuampath_cap16k.so $P && env UAM_LIB_PATH=$V/libuampath_cap16k.so $P --R 8192" \
  "200|$o/cap32k|env UAM_LIB_PATH=$V/libuampath_cap32k.so $P && env UAM_LIB_PATH=$V/libuampath_cap32k.so $P --R 8192" \
  "200|$o/rows256|env UAM_LIB_PATH=$V/libuampath_rows256.so $P && env UAM_LIB_PATH=$V/libuampath_rows256.so $P --R 8192" \
  "200|$o/base2|$P && $P --R 8192"
