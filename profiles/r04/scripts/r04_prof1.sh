#!/bin/bash
# GPU box, round 4: K2h / K4h after the histogram-LDS fix: quick tests, cfg3 + cfg5 traces and
# PMC passes (profile_bench.sh), the LDS-window experiment, bench lines.
cd "$GRAFT_REPO_ROOT"
o=r04/prof1
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k4h.py tests/test_gpu_k2h.py -x -q --timeout 200 --timeout-method thread" \
  "200|$o/lwin|python -u tools/probe_opts.py --tag lwin --settings 'k2g_lds_window=0;k2g_lds_window=96;k2g_lds_window=128;k2g_lds_window=0'" \
  "400|$o/prof_cfg3|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1" \
  "400|$o/prof_cfg5|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1" \
  "150|$o/bench|python -u bench.py" \
  "200|$o/bench_cfg5|python -u bench.py --workload cfg5"
