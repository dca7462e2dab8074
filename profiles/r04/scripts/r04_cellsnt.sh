#!/bin/bash
# GPU box, round 4: K2h's waypoint cells as streaming (non-temporal) stores (measurement build)
# against the product build, cfg3 --cells.
cd "$GRAFT_REPO_ROOT"
o=r04/cellsnt
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "200|$o/base|python -u tools/probe_opts.py --cells --tag base --settings 'group=21;group=21'" \
  "200|$o/nt|UAM_LIB_PATH=build/variants/libuampath_cellsnt.so python -u tools/probe_opts.py --cells --tag nt --settings 'group=21;group=21'" \
  "200|$o/base2|python -u tools/probe_opts.py --cells --tag base --settings 'group=21'"
