#!/bin/bash
# GPU box, round 4: K4h with the column table (code 2: the 8-B voxel plus the column's
# {psi, flags}; the 16-B voxels only where psi varies by layer): tests, probe, bench, PMC.
cd "$GRAFT_REPO_ROOT"
o=r04/vol4
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/tests|python -u -m pytest tests/test_gpu_k4h.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k 'k4h or cfg5'" \
  "200|$o/cfg5|python -u tools/probe_opts.py --volume --tag cfg5 --settings 'k2g_chunk=11;k2g_chunk=8;k2g_chunk=7;k2g_chunk=11,k2g_lds_floor=54000;k2g_chunk=0,k2g_lds_floor=0'" \
  "200|$o/bench_cfg5|python -u bench.py --workload cfg5" \
  "400|$o/prof_cfg5|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
