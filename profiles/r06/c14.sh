#!/bin/bash
# round 6 call 14: K1 with nontemporal record stores -- DEM loads nontemporal, strip order
# (row-major / 256-row columns), grid cap 12288, 4 rows per lane; the bench's setup lines
cd "$GRAFT_REPO_ROOT"
o=r06/c14
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
P="python -u tools/probe_k1.py --cases cfg3,empty --reps 20"
tools/gpu_session.sh \
  "200|$o/nt|env UAM_LIB_PATH=$V/libuampath_nt.so $P" \
  "200|$o/ntl|env UAM_LIB_PATH=$V/libuampath_ntl.so $P" \
  "200|$o/ntrm|env UAM_LIB_PATH=$V/libuampath_ntrm.so $P" \
  "200|$o/nt256|env UAM_LIB_PATH=$V/libuampath_nt256.so $P" \
  "200|$o/nt12k|env UAM_LIB_PATH=$V/libuampath_nt12k.so $P" \
  "200|$o/nt_cpl4|env UAM_LIB_PATH=$V/libuampath_nt.so $P --cpl 4" \
  "200|$o/base|$P" \
  "300|$o/bench_nt|env UAM_LIB_PATH=$V/libuampath_nt.so python -u bench.py --no-cpu-baseline" \
  "300|$o/bench_base|python -u bench.py --no-cpu-baseline"
