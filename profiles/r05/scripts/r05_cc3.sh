#!/bin/bash
# GPU box, round 5: cfg4 by spatial shards (the 8-GPU rank shares rehearsed one at a time) vs
# index shards; k_cells (plain vs streaming stores); K4h defaults; cfg3 default; K2h / K4h
# tests; traces + PMC of the per-rank share and cells.
cd "$GRAFT_REPO_ROOT"
o=r05/cc3
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
tools/gpu_session.sh \
  "900|$o/tests|python -u -m pytest tests/test_gpu_k2h.py tests/test_gpu_k4h.py -x -q --timeout 300 --timeout-method thread" \
  "90|$o/cfg3|$b" \
  "90|$o/cfg5|$b --workload cfg5" \
  "120|$o/cells|$b --cells" \
  "120|$o/cells_nt|env UAM_LIB_PATH=build/variants/libuampath_cells_nt.so $b --cells" \
  "300|$o/s0|$b --workload cfg4 --share 0/8" \
  "300|$o/s3|$b --workload cfg4 --share 3/8" \
  "300|$o/s7|$b --workload cfg4 --share 7/8" \
  "300|$o/i3|$b --workload cfg4 --share 3/8 --shard index" \
  "300|$o/full|$b --workload cfg4" \
  "400|$o/prof_cells|PASSES='trace fetch write' bash tools/profile_bench.sh gpurun_out/$o/cellsp --cells --steps 5 --warmup 1" \
  "600|$o/prof_s3|PASSES='trace fetch write tcc' bash tools/profile_bench.sh gpurun_out/$o/s3p --workload cfg4 --share 3/8 --steps 5 --warmup 1"
