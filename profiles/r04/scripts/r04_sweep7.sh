#!/bin/bash
# GPU box, round 4: workgroups per CU (LDS floor) x gathers in flight, K4h (cfg5; CH 8 / 11 now
# built for 3 waves per SIMD) and K2h (cfg3, cfg4's size).
cd "$GRAFT_REPO_ROOT"
o=r04/sweep7
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/cfg5|python -u tools/probe_opts.py --volume --tag cfg5 --settings 'k2g_lds_floor=0,k2g_chunk=6;k2g_lds_floor=54000,k2g_chunk=6;k2g_lds_floor=54000,k2g_chunk=7;k2g_lds_floor=54000,k2g_chunk=8;k2g_lds_floor=54000,k2g_chunk=11;k2g_lds_floor=0,k2g_chunk=8;k2g_lds_floor=0,k2g_chunk=11;k2g_lds_floor=60000,k2g_chunk=8;k2g_lds_floor=60000,k2g_chunk=11;k2g_lds_floor=60000,k2g_chunk=6'" \
  "300|$o/cfg3|python -u tools/probe_opts.py --tag cfg3 --settings 'k2g_lds_floor=0,k2g_chunk=7;k2g_lds_floor=41000,k2g_chunk=7;k2g_lds_floor=54000,k2g_chunk=7;k2g_lds_floor=54000,k2g_chunk=11;k2g_lds_floor=41000,k2g_chunk=11;k2g_lds_floor=0,k2g_chunk=11;k2g_lds_floor=0,k2g_chunk=7'" \
  "400|$o/cfg4|python -u tools/probe_opts.py --R 8192 --pairs 200000 --reps 10 --tag cfg4 --settings 'k2g_lds_floor=0,k2g_chunk=7;k2g_lds_floor=41000,k2g_chunk=7;k2g_lds_floor=54000,k2g_chunk=7;k2g_lds_floor=54000,k2g_chunk=11;k2g_lds_floor=80000,k2g_chunk=11;k2g_lds_floor=0,k2g_chunk=11'"
