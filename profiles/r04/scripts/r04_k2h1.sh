#!/bin/bash
# GPU box, round 4: K2h (similarity-form geometry) tests, group / chunk sweep, bench line.
cd "$GRAFT_REPO_ROOT"
o=r04/k2h1
mkdir -p gpurun_out/$o
tools/gpu_session.sh \
  "400|$o/k2h_tests|python -u -m pytest tests/test_gpu_k2h.py tests/test_gpu_k2g.py -x -q --timeout 200 --timeout-method thread" \
  "200|$o/sweep|python -u tools/probe_opts.py --tag k2h --settings 'group=21;group=21,k2g_chunk=7;group=17;group=14;group=12;group=11;group=9;group=7,k2g_chunk=7;group=21,k2g_sim=0;group=21,k2g_chunk=11'" \
  "150|$o/bench|python -u bench.py"
