#!/bin/bash
# round 6 call 2: the new tests (device checks, create_x_init cells, batches API), then the
# cfg3 bench with 1 / 2 / 4 / 8 steps per call (uam_eval_generated_batches) and a kernel trace
# of the batched form
cd "$GRAFT_REPO_ROOT"
o=r06/c2
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "600|$o/tests|python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_k2h.py tests/test_gpu_k4h.py tests/test_gpu_k2g.py" \
  "240|$o/b1|python -u bench.py --no-cpu-baseline" \
  "240|$o/b2|python -u bench.py --no-cpu-baseline --batches 2" \
  "240|$o/b4|python -u bench.py --no-cpu-baseline --batches 4" \
  "240|$o/b8|python -u bench.py --no-cpu-baseline --batches 8" \
  "240|$o/b20|python -u bench.py --no-cpu-baseline --batches 20" \
  "300|$o/prof|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/trace4 --steps 8 --warmup 4 --batches 4"
