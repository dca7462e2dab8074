#!/bin/bash
# round 6 call 23: cfg5 (K4h) group length on the final tree (library events)
cd "$GRAFT_REPO_ROOT"
o=r06/c23
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
S="group=21;group=14;group=17;group=24;group=28;group=11;group=21"
tools/gpu_session.sh \
  "400|$o/cfg5|python -u tools/probe_opts.py --volume --tag cfg5 --reps 20 --settings '$S'"
