#!/bin/bash
# GPU box, round 4: the K2h persistent form (a few workgroups per CU looping over the sorted
# chunks, LDS tables staged once) against the per-chunk launch: tests, cfg3 / cfg4 probes.
cd "$GRAFT_REPO_ROOT"
o=r04/persist
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
S="k2h_persist=0;k2h_persist=5;k2h_persist=4;k2h_persist=6;k2h_persist=8;k2h_persist=5,k2g_chunk=11;k2h_persist=0,k2g_chunk=0"
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k2h.py -x -q --timeout 200 --timeout-method thread -k 'persistent or lds_floor'" \
  "300|$o/cfg3|python -u tools/probe_opts.py --tag cfg3 --settings '$S'" \
  "400|$o/cfg4|python -u tools/probe_opts.py --R 8192 --pairs 200000 --reps 10 --tag cfg4 --settings 'k2h_persist=0;k2h_persist=3;k2h_persist=2;k2h_persist=0'"
