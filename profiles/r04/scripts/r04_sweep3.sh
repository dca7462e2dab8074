#!/bin/bash
# GPU box, round 4: four-launch sort back; K2h / K4h tests; K4h group / band / tile sweep;
# the LDS-window experiment; K2h with cells.
cd "$GRAFT_REPO_ROOT"
o=r04/sweep3
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k4h.py tests/test_gpu_k2h.py -x -q --timeout 200 --timeout-method thread" \
  "300|$o/vol|python -u tools/probe_opts.py --volume --tag k4h --settings 'group=21;group=14;group=11;group=7;group=28;group=21,k4h_band=1;k4h_band=2;k4h_band=8;k4h_band=0,k2g_tile_bits=3;k2g_tile_bits=5;k2g_tile_bits=0,k2g_chunk=7;k2g_chunk=0,group=0'" \
  "200|$o/lwin|python -u tools/probe_opts.py --tag lwin --settings 'k2g_lds_window=0;k2g_lds_window=96;k2g_lds_window=128;k2g_lds_window=0,k2g_chunk=7'" \
  "120|$o/cells|python -u tools/probe_opts.py --tag cells --cells" \
  "150|$o/bench|python -u bench.py"
