#!/bin/bash
# round 6 call 24: the whole cfg4 job (8192^2, 1M paths, HBM-line bound) -- K2h's bound form
# (4-B / 8-B entries, terrain by the bound rule) against the terrain-in-entry default
cd "$GRAFT_REPO_ROOT"
o=r06/c24
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
S="k2h_terrain=1;k2h_terrain=0;k2h_terrain=0,k2h_lb_stride=8;k2h_terrain=0,k2h_lb_stride=4;k2h_terrain=1"
tools/gpu_session.sh \
  "500|$o/cfg4|python -u tools/probe_opts.py --R 8192 --pairs 200000 --tag cfg4 --reps 20 --settings '$S'"
