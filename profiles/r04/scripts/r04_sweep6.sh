#!/bin/bash
# GPU box, round 4: unit sums moved to the scatter's extra block (hist back to its own time);
# K4h workgroups per CU (LDS floor) and gathers in flight; K2h / K4h tests; cfg3 + cfg5 traces.
cd "$GRAFT_REPO_ROOT"
o=r04/sweep6
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k4h.py tests/test_gpu_k2h.py tests/test_gpu_k2g.py -x -q --timeout 200 --timeout-method thread" \
  "300|$o/cfg5|python -u tools/probe_opts.py --volume --tag cfg5 --settings 'k2g_lds_floor=0;k2g_lds_floor=28000;k2g_lds_floor=33000;k2g_lds_floor=41000;k2g_lds_floor=54000;k2g_lds_floor=0,k2g_chunk=7;k2g_chunk=8;k2g_chunk=6'" \
  "200|$o/prof_cfg3|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1" \
  "200|$o/prof_cfg5|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
