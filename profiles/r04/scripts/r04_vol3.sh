#!/bin/bash
# GPU box, round 4: K4h histogram with a reciprocal for the key's altitude; bands of 4 / 8
# layers at the 2-workgroup default; cfg5 trace.
cd "$GRAFT_REPO_ROOT"
o=r04/vol3
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k4h.py -x -q --timeout 200 --timeout-method thread" \
  "200|$o/cfg5|python -u tools/probe_opts.py --volume --tag cfg5 --settings 'k4h_band=0;k4h_band=8;k4h_band=2;k4h_band=0'" \
  "200|$o/prof_cfg5|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
