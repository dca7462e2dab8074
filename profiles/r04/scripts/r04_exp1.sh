#!/bin/bash
# GPU box, round 4: K2g measurement builds (slot stores, no-gather / no-slot decomposition, CH 7)
# beside the product build, cfg3, plus the default bench line.
cd "$GRAFT_REPO_ROOT"
o=r04/exp1
mkdir -p gpurun_out/$o
V=build/variants
tools/gpu_session.sh \
  "200|$o/default|python -u tools/probe_opts.py --tag default --settings 'k2g_chunk=0;k2g_chunk=6;k2g_chunk=16;group=0;group=21,k2g_chunk=0'" \
  "120|$o/ch7|UAM_LIB_PATH=$V/libuampath_ch7.so python -u tools/probe_opts.py --tag ch7 --settings 'k2g_chunk=6;k2g_chunk=0'" \
  "120|$o/nt|UAM_LIB_PATH=$V/libuampath_nt.so python -u tools/probe_opts.py --tag nt" \
  "120|$o/noslot|UAM_LIB_PATH=$V/libuampath_noslot.so python -u tools/probe_opts.py --tag noslot" \
  "120|$o/nogather|UAM_LIB_PATH=$V/libuampath_nogather.so python -u tools/probe_opts.py --tag nogather" \
  "120|$o/nogns|UAM_LIB_PATH=$V/libuampath_nogns.so python -u tools/probe_opts.py --tag nogns" \
  "150|$o/bench|python -u bench.py"
