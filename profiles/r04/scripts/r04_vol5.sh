#!/bin/bash
# GPU box, round 4: the K4h code map from every layer's psi (a voxel's own psi, not layer 0's):
# K4h tests incl. a layer-varying-psi volume, the cfg5 full-size test, cfg5 probe.
cd "$GRAFT_REPO_ROOT"
o=r04/vol5
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "400|$o/tests|python -u -m pytest tests/test_gpu_k4h.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k 'k4h or cfg5'" \
  "200|$o/cfg5|python -u tools/probe_opts.py --volume --tag cfg5 --settings 'k2g_chunk=0;k2g_chunk=0'"
