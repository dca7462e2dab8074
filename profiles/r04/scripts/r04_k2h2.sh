#!/bin/bash
# GPU box, round 4: K2h with the two-launch sort (atomic bin totals, scan in the scatter):
# tests, option sweep, kernel trace.
cd "$GRAFT_REPO_ROOT"
o=r04/k2h2
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/k2h_tests|python -u -m pytest tests/test_gpu_k2h.py tests/test_gpu_k2g.py -x -q --timeout 200 --timeout-method thread" \
  "240|$o/sweep|python -u tools/probe_opts.py --tag k2h2 --settings 'group=21;k2g_chunk=6;k2g_chunk=7;k2g_chunk=0,k2g_tile_bits=5;k2g_tile_bits=0,k2g_lds_floor=32768;k2g_lds_floor=40960;k2g_lds_floor=0,group=14;group=24;group=21,k2g_sim=0'" \
  "200|$o/trace|rocprofv3 --kernel-trace --stats -d gpurun_out/$o/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10" \
  "150|$o/bench|python -u bench.py"
