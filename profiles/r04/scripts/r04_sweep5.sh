#!/bin/bash
# GPU box, round 4: group length / tile / band sweeps for K2h (cfg3, cfg4's size) and K4h (cfg5)
# now that an item's geometry is the similarity form (shorter groups cost less than under K2g);
# hist trace with and without the unit-sum block (k2g_sim 0 / 1).
cd "$GRAFT_REPO_ROOT"
o=r04/sweep5
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "200|$o/cfg3|python -u tools/probe_opts.py --tag cfg3 --settings 'group=21;group=16;group=14;group=11;group=28;group=21'" \
  "300|$o/cfg5|python -u tools/probe_opts.py --volume --tag cfg5 --settings 'group=21,k4h_band=4;group=16,k4h_band=4;group=11,k4h_band=4;group=21,k4h_band=2;group=21,k4h_band=8;group=16,k4h_band=2;group=16,k4h_band=8;group=21,k4h_band=4'" \
  "300|$o/cfg4|python -u tools/probe_opts.py --R 8192 --pairs 200000 --reps 10 --tag cfg4 --settings 'group=21,k2g_tile_bits=0;group=21,k2g_tile_bits=6;group=16,k2g_tile_bits=0;group=16,k2g_tile_bits=6;group=11,k2g_tile_bits=6;group=21,k2g_tile_bits=4;group=21,k2g_tile_bits=0'" \
  "200|$o/histtrace|rocprofv3 --kernel-trace --stats -d gpurun_out/$o/histtrace -o run -- python -u tools/probe_opts.py --reps 5 --tag hist --settings 'k2g_sim=0;k2g_sim=1'"
