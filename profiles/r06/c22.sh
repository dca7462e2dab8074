#!/bin/bash
# round 6 call 22: the inequality records pipelined (for_ineqs_pipe: the next record's scalar
# load issued after the current one arrived, overlapping its arithmetic) in K1 and K3b --
# parity with the measurement build, then K1 and analytic cfg3 against the product build
cd "$GRAFT_REPO_ROOT"
o=r06/c22
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants/libuampath_pipe.so
tools/gpu_session.sh \
  "500|$o/tests|env UAM_LIB_PATH=$V python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_k3b.py tests/test_gpu_parity.py -k 'k3b or analytic or raster_build or golden or random'" \
  "200|$o/k1_pipe|env UAM_LIB_PATH=$V python -u tools/probe_k1.py --cases cfg3,regions,cfg3-obstacles --reps 20" \
  "200|$o/k1_base|python -u tools/probe_k1.py --cases cfg3,regions,cfg3-obstacles --reps 20" \
  "300|$o/k3b_pipe|env UAM_LIB_PATH=$V python -u tools/probe_opts.py --analytic --tag pipe --reps 5" \
  "300|$o/k3b_base|python -u tools/probe_opts.py --analytic --tag base --reps 5"
