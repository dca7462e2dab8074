#!/bin/bash
# GPU box, round 4 (final tree; final2 = after the K4h code-map fix): full GPU suite + smoke, bench lines (cfg3, cfg3 --cells, cfg4,
# cfg5), cfg3 and cfg3 --cells traces + PMC passes.
cd "$GRAFT_REPO_ROOT"
o=r04/final2
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "900|$o/gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "120|$o/smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "150|$o/bench|python -u bench.py" \
  "150|$o/bench_cells|python -u bench.py --cells" \
  "300|$o/bench_cfg4|python -u bench.py --workload cfg4" \
  "200|$o/bench_cfg5|python -u bench.py --workload cfg5" \
  "400|$o/prof_cfg3|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1" \
  "400|$o/prof_cells|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cells --cells --steps 5 --warmup 1"
