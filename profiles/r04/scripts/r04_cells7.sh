#!/bin/bash
# GPU box, round 4: K2h cells at 7 gathers in flight (the non-cells default) against 8.
cd "$GRAFT_REPO_ROOT"
o=r04/cells7
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k2h.py tests/test_gpu_k2g.py -x -q --timeout 200 --timeout-method thread -k cells" \
  "200|$o/cfg3|python -u tools/probe_opts.py --cells --tag cells --settings 'k2g_chunk=0;k2g_chunk=8;k2g_chunk=7;k2g_chunk=8'"
