#!/bin/bash
# GPU box, round 4: cells as streaming stores (now the product build): cells tests, bench
# --cells + PMC; K2h's slots as streaming stores (measurement build) against the product build.
cd "$GRAFT_REPO_ROOT"
o=r04/nt
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k2h.py tests/test_gpu_k2g.py -x -q --timeout 200 --timeout-method thread -k cells" \
  "200|$o/base|python -u tools/probe_opts.py --tag base --settings 'group=21;group=21'" \
  "200|$o/slotnt|UAM_LIB_PATH=build/variants/libuampath_slotnt.so python -u tools/probe_opts.py --tag slotnt --settings 'group=21;group=21'" \
  "200|$o/base_cells|python -u tools/probe_opts.py --cells --tag base --settings 'group=21;group=21'" \
  "150|$o/bench_cells|python -u bench.py --cells" \
  "400|$o/prof_cells|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cells --cells --steps 5 --warmup 1"
