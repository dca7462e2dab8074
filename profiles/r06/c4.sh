#!/bin/bash
# round 6 call 4: the K2h / K4h / K2g tests (batches API, device checks, create_x_init cells),
# the pipelined form's three stream layouts against one call per step (probe_opts.py), then the
# TA / TD / TCP / SQ counters of the cfg3 step (verdict r5 item 2), entry and bound forms
cd "$GRAFT_REPO_ROOT"
o=r06/c4
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "600|$o/tests|python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_k2h.py tests/test_gpu_k4h.py tests/test_gpu_k2g.py" \
  "300|$o/one|python -u tools/probe_opts.py --tag one --reps 20 --settings 'group=21'" \
  "300|$o/b4|python -u tools/probe_opts.py --tag b4 --batches 4 --reps 5 --settings 'batch_form=0;batch_form=1;batch_form=2;batch_form=0'" \
  "300|$o/b2|python -u tools/probe_opts.py --tag b2 --batches 2 --reps 10 --settings 'batch_form=0;batch_form=1'" \
  "300|$o/prof|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/trace4 --steps 8 --warmup 4 --batches 4" \
  "900|$o/cnt_entry|bash profiles/r06/counters.sh gpurun_out/$o/entry" \
  "900|$o/cnt_bound|bash profiles/r06/counters.sh gpurun_out/$o/bound --opt k2h_terrain=0"
