#!/bin/bash
# GPU box, round 5: the waypoint-cells launch placed (inline after the evaluation / on the side
# stream from the start / beside the evaluation only) and sized (one workgroup per 64 paths or
# a capped grid looping over them); cfg3 with cells; a trace of the default; K2h cells tests.
cd "$GRAFT_REPO_ROOT"
o=r05/cc10
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
b="python -u bench.py --no-cpu-baseline --cells"
steps=()
for v in cs1g256u cs1g512u cs1u cs1g256 cinlu cs2u; do
  steps+=("120|$o/$v|UAM_LIB_PATH=$V/libuampath_$v.so $b")
done
tools/gpu_session.sh \
  "120|$o/default|$b" \
  "${steps[@]}" \
  "120|$o/default2|$b" \
  "120|$o/nocells|python -u bench.py --no-cpu-baseline" \
  "300|$o/prof|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cellsp --cells --steps 5 --warmup 1" \
  "300|$o/prof_inl|UAM_LIB_PATH=$V/libuampath_cinlu.so PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cinlp --cells --steps 5 --warmup 1" \
  "300|$o/tests|python -u -m pytest tests/test_gpu_k2h.py -x -q -k cells --timeout 120 --timeout-method thread"
