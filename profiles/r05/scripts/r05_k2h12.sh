#!/bin/bash
# GPU box, round 5: the terrain-in-entry K2h (code map alone in LDS): workgroups of 512 / 256,
# one chunk ahead or not (measurement builds).
cd "$GRAFT_REPO_ROOT"
o=r05/k2h12
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline --opt k2h_terrain=1"
v="env UAM_LIB_PATH=build/variants/libuampath"
tools/gpu_session.sh \
  "90|$o/te|$b" \
  "90|$o/te_na|${v}_na.so $b" \
  "90|$o/te_b256|${v}_b256.so $b" \
  "90|$o/te_b256na|${v}_b256na.so $b" \
  "90|$o/te_b256_f40|${v}_b256.so $b --opt k2g_lds_floor=40000" \
  "90|$o/te2|$b" \
  "90|$o/r4|cd build/r4 && python -u bench.py --no-cpu-baseline"
