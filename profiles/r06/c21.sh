#!/bin/bash
# round 6 call 21: K2h group length on 8192^2 -- the whole cfg4 job (1M paths) and the rank
# shares 3 / 0 / 7 of 8 (125k paths each), G = 10..21; library events (probe_opts seq_ms)
cd "$GRAFT_REPO_ROOT"
o=r06/c21
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
S="group=21;group=14;group=12;group=11;group=10;group=16;group=17;group=21;group=14"
P="python -u tools/probe_opts.py --R 8192 --pairs 200000 --reps 20"
tools/gpu_session.sh \
  "400|$o/cfg4|$P --tag cfg4 --settings '$S'" \
  "300|$o/s3|$P --tag s3 --share 3/8 --settings '$S'" \
  "300|$o/s0|$P --tag s0 --share 0/8 --settings '$S'" \
  "300|$o/s7|$P --tag s7 --share 7/8 --settings '$S'"
