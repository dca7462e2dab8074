#!/bin/bash
# GPU box, round 5: path seeds (the exact terrain / clearance of the best sampled waypoint starts
# every item's running bound; header and unit arcs staged in the histogram launch's LDS): GPU
# tests of the sorted forms, fetch counts by sample stride, cfg3 / cfg5 benches, traces.
cd "$GRAFT_REPO_ROOT"
o=r05/k2h7
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
c="env UAM_LIB_PATH=build/variants/libuampath_cnt.so python -u tools/k2h_counts.py"
tools/gpu_session.sh \
  "900|$o/tests|python -u -m pytest tests/test_gpu_k2h.py tests/test_gpu_k4h.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread" \
  "120|$o/cnt8|$c" \
  "120|$o/cnt4|$c --opt=k2h_lb_stride=4" \
  "120|$o/cnt2|$c --opt=k2h_lb_stride=2" \
  "120|$o/cnt1|$c --opt=k2h_lb_stride=1" \
  "90|$o/def|$b" \
  "90|$o/lbs4|$b --opt k2h_lb_stride=4" \
  "90|$o/lbs2|$b --opt k2h_lb_stride=2" \
  "90|$o/lbs1|$b --opt k2h_lb_stride=1" \
  "90|$o/cfg5|$b --workload cfg5" \
  "90|$o/cfg5l4|$b --workload cfg5 --opt k2h_lb_stride=4" \
  "90|$o/cfg5l2|$b --workload cfg5 --opt k2h_lb_stride=2" \
  "300|$o/prof|PASSES='trace sq tcc' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1" \
  "300|$o/prof5|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
