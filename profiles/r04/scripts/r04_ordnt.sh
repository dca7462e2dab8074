#!/bin/bash
# GPU box, round 4: K2h's order entries as streaming loads (measurement build) against the
# product build, cfg3.
cd "$GRAFT_REPO_ROOT"
o=r04/ordnt
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "200|$o/base|python -u tools/probe_opts.py --tag base --settings 'group=21;group=21'" \
  "200|$o/nt|UAM_LIB_PATH=build/variants/libuampath_ordnt.so python -u tools/probe_opts.py --tag nt --settings 'group=21;group=21'" \
  "200|$o/base2|python -u tools/probe_opts.py --tag base --settings 'group=21'"
