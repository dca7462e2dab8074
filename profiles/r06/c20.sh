#!/bin/bash
# round 6 call 20: cfg4 rank shares (8192^2, 25k pairs each) -- K2h's bound form (4-B / 8-B
# entries, the terrain plane read by the bound rule) against the terrain-in-entry default,
# with group lengths 14 / 17 / 21 / 28; library events (probe_opts seq_ms)
cd "$GRAFT_REPO_ROOT"
o=r06/c20
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
S="k2h_terrain=1,group=21;k2h_terrain=0,group=21;k2h_terrain=0,group=14;k2h_terrain=1,group=14;k2h_terrain=0,group=17;k2h_terrain=1,group=17;k2h_terrain=0,group=28;k2h_terrain=1,group=21;k2h_terrain=0,group=21"
P="python -u tools/probe_opts.py --R 8192 --pairs 200000 --reps 20"
tools/gpu_session.sh \
  "300|$o/s3|$P --tag s3 --share 3/8 --settings '$S'" \
  "300|$o/s0|$P --tag s0 --share 0/8 --settings '$S'" \
  "300|$o/s7|$P --tag s7 --share 7/8 --settings '$S'" \
  "300|$o/cfg3|python -u tools/probe_opts.py --tag cfg3 --reps 20 --settings '$S'"
