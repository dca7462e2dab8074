#!/bin/bash
# GPU box, round 4: the scatter's partitions sorted by bin in LDS before their stores (runs
# instead of one scattered 4-B store per item): grouped tests, probe on / off, cfg3 / cfg5 traces.
cd "$GRAFT_REPO_ROOT"
o=r04/sc
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/tests|python -u -m pytest tests/test_gpu_k4h.py tests/test_gpu_k2h.py tests/test_gpu_k2g.py -x -q --timeout 200 --timeout-method thread" \
  "200|$o/cfg3|python -u tools/probe_opts.py --tag cfg3 --settings 'k2g_scatter_lds=1;k2g_scatter_lds=0;k2g_scatter_lds=1;k2g_scatter_lds=0'" \
  "200|$o/cfg5|python -u tools/probe_opts.py --volume --tag cfg5 --settings 'k2g_scatter_lds=1;k2g_scatter_lds=0;k2g_scatter_lds=1'" \
  "200|$o/prof_cfg3|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1"
