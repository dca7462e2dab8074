#!/bin/bash
# Round 6 closing check after the setup kernels' batched loads: the whole GPU suite, smoke, the
# default and cfg4 bench lines, kernel traces of both (setup kernels included)
cd "$GRAFT_REPO_ROOT"
o=r06/final4
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "700|$o/suite|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "300|$o/smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "300|$o/bench|python -u bench.py" \
  "400|$o/bench_cfg4|python -u bench.py --workload cfg4" \
  "300|$o/trace3|rocprofv3 --kernel-trace --stats -d gpurun_out/$o/trace3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1" \
  "400|$o/trace4|rocprofv3 --kernel-trace --stats -d gpurun_out/$o/trace4 -o run --output-format csv -- python3 bench.py --workload cfg4 --no-cpu-baseline --steps 3 --warmup 1"
