#!/bin/bash
# round 6 call 17: K1's store floor -- a diagnostic build with the shape walks removed (records
# still written, phi = psi = 0) against the product, and plain vs nontemporal 16-B stores of
# the same 268 MB (tools/write_bw.hip)
cd "$GRAFT_REPO_ROOT"
o=r06/c17
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
P="python -u tools/probe_k1.py --cases cfg3,empty --reps 20"
tools/gpu_session.sh \
  "120|$o/write_bw|$V/write_bw 268435456" \
  "200|$o/stream|env UAM_LIB_PATH=$V/libuampath_stream.so $P" \
  "200|$o/stream_cpl4|env UAM_LIB_PATH=$V/libuampath_stream.so $P --cpl 4" \
  "200|$o/col|$P"
