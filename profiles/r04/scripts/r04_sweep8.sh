#!/bin/bash
# GPU box, round 4: a whole group's gathers in flight (CH 16 / 21, built for 2 waves per SIMD)
# with 1-2 workgroups per CU: fewer resident items per XCD without fewer loads in flight.
cd "$GRAFT_REPO_ROOT"
o=r04/sweep8
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
S="k2g_chunk=7,k2g_lds_floor=0;k2g_chunk=16,k2g_lds_floor=0;k2g_chunk=21,k2g_lds_floor=0;k2g_chunk=21,k2g_lds_floor=90000;k2g_chunk=16,k2g_lds_floor=60000;k2g_chunk=16,k2g_lds_floor=90000;k2g_chunk=11,k2g_lds_floor=54000;k2g_chunk=7,k2g_lds_floor=0"
V="k2g_chunk=11,k2g_lds_floor=60000;k2g_chunk=16,k2g_lds_floor=0;k2g_chunk=16,k2g_lds_floor=90000;k2g_chunk=21,k2g_lds_floor=0;k2g_chunk=21,k2g_lds_floor=90000;k2g_chunk=11,k2g_lds_floor=60000"
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k4h.py tests/test_gpu_k2h.py tests/test_gpu_k2g.py -x -q --timeout 200 --timeout-method thread" \
  "300|$o/cfg3|python -u tools/probe_opts.py --tag cfg3 --settings '$S'" \
  "300|$o/cfg5|python -u tools/probe_opts.py --volume --tag cfg5 --settings '$V'" \
  "400|$o/cfg4|python -u tools/probe_opts.py --R 8192 --pairs 200000 --reps 10 --tag cfg4 --settings '$S'"
