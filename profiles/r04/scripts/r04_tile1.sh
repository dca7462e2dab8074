#!/bin/bash
# GPU box, round 4: the K2h tile form (one workgroup per 128^2 / 64^2 tile, its packed plane
# staged in LDS once; the round-3 verdict's item 1) -- parity tests, then a sweep of tile side x
# group length at cfg3 and cfg4's size, against the default K2h.
cd "$GRAFT_REPO_ROOT"
o=r04/tile1
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
S="k2g_tile_owner=0,group=21;k2g_tile_owner=128,group=21;k2g_tile_owner=128,group=14;k2g_tile_owner=128,group=11;k2g_tile_owner=128,group=7;k2g_tile_owner=64,group=21;k2g_tile_owner=64,group=11;k2g_tile_owner=64,group=7;k2g_tile_owner=0,group=21"
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k2h.py -x -q --timeout 200 --timeout-method thread -k 'tile_form or lds_floor or partial'" \
  "300|$o/cfg3|python -u tools/probe_opts.py --tag cfg3 --settings '$S'" \
  "400|$o/cfg4|python -u tools/probe_opts.py --R 8192 --pairs 200000 --reps 10 --tag cfg4 --settings '$S'"
