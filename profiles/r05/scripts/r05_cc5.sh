#!/bin/bash
# GPU box, round 5: K1 alone (no summary / pack) by shape-grid resolution (64 default, 128,
# 256 build variants) and rows per lane (2, 4); K3 (cfg2, analytic: the same grid lists per
# waypoint) by grid resolution; the round's final PMC sets (cfg5 K4h bounds form, cells,
# cfg4, cfg3 with the K2h bounds form) for profiles/traffic.json.
cd "$GRAFT_REPO_ROOT"
o=r05/cc5
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
k1="tools/probe_k1.py --cases cfg3,empty"
tools/gpu_session.sh \
  "120|$o/k1_g64|python -u $k1 && python -u $k1 --cpl 4" \
  "120|$o/k1_g128|UAM_LIB_PATH=$V/libuampath_g128.so python -u $k1 && UAM_LIB_PATH=$V/libuampath_g128.so python -u $k1 --cpl 4" \
  "120|$o/k1_g256|UAM_LIB_PATH=$V/libuampath_g256.so python -u $k1 && UAM_LIB_PATH=$V/libuampath_g256.so python -u $k1 --cpl 4" \
  "180|$o/cfg2_g64|python -u bench.py --no-cpu-baseline --workload cfg2" \
  "180|$o/cfg2_g128|UAM_LIB_PATH=$V/libuampath_g128.so python -u bench.py --no-cpu-baseline --workload cfg2" \
  "180|$o/cfg2_g256|UAM_LIB_PATH=$V/libuampath_g256.so python -u bench.py --no-cpu-baseline --workload cfg2" \
  "300|$o/par_g256|UAM_LIB_PATH=$V/libuampath_g256.so python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread" \
  "300|$o/prof5|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg5p --workload cfg5 --steps 5 --warmup 1" \
  "300|$o/profc|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cellsp --cells --steps 5 --warmup 1" \
  "400|$o/prof4|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg4p --workload cfg4 --steps 5 --warmup 1" \
  "300|$o/prof3b|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg3bp --opt k2h_terrain=0 --steps 5 --warmup 1"
