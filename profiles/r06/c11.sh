#!/bin/bash
# round 6 call 11: the batch-size-adaptive default tile bits -- sorted-form tests, then the
# cfg3, cfg4 and cfg4 rank-share bench lines (bit-identical outputs; only the item order moves)
cd "$GRAFT_REPO_ROOT"
o=r06/c11
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "600|$o/tests|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_k2s.py tests/test_gpu_k2g.py tests/test_gpu_k2h.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py" \
  "300|$o/bench|python -u bench.py --no-cpu-baseline" \
  "300|$o/bench_cfg4_s3|python -u bench.py --workload cfg4 --share 3/8" \
  "300|$o/bench_cfg4_s0|python -u bench.py --workload cfg4 --share 0/8 --no-cpu-baseline" \
  "300|$o/bench_cfg4_s7|python -u bench.py --workload cfg4 --share 7/8 --no-cpu-baseline" \
  "400|$o/bench_cfg4|python -u bench.py --workload cfg4 --no-cpu-baseline"
