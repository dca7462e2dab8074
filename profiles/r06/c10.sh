#!/bin/bash
# round 6 call 10: cfg4 (8192^2) tile bits 4 vs 5 (the default: ~256^2-cell tiles) for the
# whole 1M-path job and rank 3's share of 8, K2h, library events per call
cd "$GRAFT_REPO_ROOT"
o=r06/c10
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/full|python -u tools/probe_opts.py --tag full --R 8192 --pairs 200000 --reps 10 --settings 'k2g_tile_bits=0;k2g_tile_bits=4;k2g_tile_bits=0;k2g_tile_bits=4'" \
  "400|$o/share3|python -u tools/probe_opts.py --tag share3 --R 8192 --pairs 200000 --share 3/8 --reps 20 --settings 'k2g_tile_bits=0;k2g_tile_bits=4;k2g_tile_bits=0;k2g_tile_bits=4'" \
  "400|$o/share0|python -u tools/probe_opts.py --tag share0 --R 8192 --pairs 200000 --share 0/8 --reps 20 --settings 'k2g_tile_bits=0;k2g_tile_bits=4'"
