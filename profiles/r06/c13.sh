#!/bin/bash
# round 6 call 13: K1 raster build -- nontemporal record stores and grid caps (measurement
# builds from tools/build_variant.sh), against torch's fill of the same records (store floor)
cd "$GRAFT_REPO_ROOT"
o=r06/c13
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
tools/gpu_session.sh \
  "200|$o/base|python -u tools/probe_k1.py --cases cfg3,empty --reps 20" \
  "200|$o/nt|env UAM_LIB_PATH=$V/libuampath_nt.so python -u tools/probe_k1.py --cases cfg3,empty --reps 20" \
  "200|$o/nt16k|env UAM_LIB_PATH=$V/libuampath_nt16k.so python -u tools/probe_k1.py --cases cfg3,empty --reps 20" \
  "200|$o/nt4k|env UAM_LIB_PATH=$V/libuampath_nt4k.so python -u tools/probe_k1.py --cases cfg3,empty --reps 20" \
  "200|$o/base2|python -u tools/probe_k1.py --cases cfg3,empty --reps 20" \
  "200|$o/nt_8k|env UAM_LIB_PATH=$V/libuampath_nt.so python -u tools/probe_k1.py --R 8192 --cases cfg3,empty --reps 20" \
  "200|$o/base_8k|python -u tools/probe_k1.py --R 8192 --cases cfg3,empty --reps 20"
