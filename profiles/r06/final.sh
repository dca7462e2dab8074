#!/bin/bash
# Round 6 final: the whole GPU suite, smoke, the default bench and the other configs' bench
# lines (CPU baseline, parity), kernel trace + PMC passes of cfg3, cfg3 --cells and cfg5
# (tools/pmc_traffic.py turns them into profiles/traffic.json's keys).  usage: final.sh <tag>
cd "$GRAFT_REPO_ROOT"
o=r06/${1:-final}
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "600|$o/suite|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "300|$o/smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "300|$o/bench|python -u bench.py" \
  "300|$o/bench_cells|python -u bench.py --cells" \
  "300|$o/bench_cfg5|python -u bench.py --workload cfg5" \
  "400|$o/bench_cfg4|python -u bench.py --workload cfg4" \
  "300|$o/bench_cfg4_s3|python -u bench.py --workload cfg4 --share 3/8" \
  "300|$o/bench_cfg2|python -u bench.py --workload cfg2" \
  "400|$o/prof|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1" \
  "400|$o/prof_cells|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cells --cells --steps 5 --warmup 1" \
  "400|$o/prof_cfg5|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
