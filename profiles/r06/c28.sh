#!/bin/bash
# round 6 call 28: the summary bitmap and the pack code map with one wave per block (coalesced
# record rows) -- their parity tests and the sorted forms' suites, the randomized parity, then
# the setup times in the bench lines and a kernel trace of the cfg3 / cfg4 setup
cd "$GRAFT_REPO_ROOT"
o=r06/c28
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "600|$o/tests|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_k2h.py tests/test_gpu_k2g.py tests/test_gpu_k2s.py tests/test_gpu_fuzz.py" \
  "300|$o/bench|python -u bench.py --no-cpu-baseline" \
  "400|$o/bench_cfg4|python -u bench.py --workload cfg4 --no-cpu-baseline" \
  "300|$o/trace3|rocprofv3 --kernel-trace --stats -d gpurun_out/$o/trace3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1" \
  "400|$o/trace4|rocprofv3 --kernel-trace --stats -d gpurun_out/$o/trace4 -o run --output-format csv -- python3 bench.py --workload cfg4 --no-cpu-baseline --steps 3 --warmup 1"
