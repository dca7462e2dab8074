#!/bin/bash
# GPU box, round 4: K2g without its geometry work (measurement builds) and the cell-writing
# K2g form's tests.
cd "$GRAFT_REPO_ROOT"
o=r04/exp2
mkdir -p gpurun_out/$o
V=build/variants
tools/gpu_session.sh \
  "300|$o/k2g_tests|python -u -m pytest tests/test_gpu_k2g.py -x -q --timeout 200 --timeout-method thread" \
  "120|$o/nogeo|UAM_LIB_PATH=$V/libuampath_nogeo.so python -u tools/probe_opts.py --tag nogeo" \
  "120|$o/nogeo_nogather|UAM_LIB_PATH=$V/libuampath_nogeo_nogather.so python -u tools/probe_opts.py --tag nogeo_nogather" \
  "120|$o/nogeo_noslot|UAM_LIB_PATH=$V/libuampath_nogeo_noslot.so python -u tools/probe_opts.py --tag nogeo_noslot" \
  "120|$o/cells|python -u tools/probe_opts.py --tag cells --cells"
