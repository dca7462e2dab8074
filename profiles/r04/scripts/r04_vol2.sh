#!/bin/bash
# GPU box, round 4: K4h with the two-table packed volume (8-B {risk, terrain} voxels in 4x4
# blocks, 16-B voxels in no-fly column blocks): tests, sweep, cfg5 bench.
cd "$GRAFT_REPO_ROOT"
o=r04/vol2
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k4h.py -x -q --timeout 200 --timeout-method thread" \
  "300|$o/vol|python -u tools/probe_opts.py --volume --tag k4h2 --settings 'group=21;k2g_tile_bits=3;k2g_tile_bits=3,k4h_band=8;k4h_band=16;k4h_band=0,group=14;group=21,k2g_chunk=7;k2g_chunk=0,k2g_tile_bits=0'" \
  "200|$o/bench_cfg5|python -u bench.py --workload cfg5"
