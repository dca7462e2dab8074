#!/bin/bash
# GPU box, round 5: the packed raster v2 (4-B phi / 8-B phi+psi|nfz / 4-B terrain planes, terrain
# bounds), K2h with the exact terrain-bound rule and K4h on the packed volume v2 -- the sorted-
# form GPU tests, bench lines (cfg3, cfg4 at the 8-GPU per-rank share and whole, cfg5), the cfg3
# trace + PMC passes, and the waypoint-cell store-pattern probe (tools/write_runs.hip).
cd "$GRAFT_REPO_ROOT"
o=r05/k2h1
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "900|$o/tests|python -u -m pytest tests/test_gpu_k2h.py tests/test_gpu_k4h.py tests/test_gpu_k2s.py tests/test_gpu_k2g.py -x -q --timeout 300 --timeout-method thread" \
  "150|$o/bench|python -u bench.py" \
  "240|$o/bench_cfg4_q25k|python -u bench.py --workload cfg4 --pairs 25000 --no-cpu-baseline" \
  "300|$o/bench_cfg4|python -u bench.py --workload cfg4 --no-cpu-baseline" \
  "240|$o/bench_cfg5|python -u bench.py --workload cfg5 --no-cpu-baseline" \
  "400|$o/prof_cfg3|PASSES='trace fetch write tcc' bash tools/profile_bench.sh gpurun_out/$o/cfg3 --steps 5 --warmup 1"
st=$?
[ "$st" -le 1 ] || exit "$st"   # a fault / abort / timeout above: nothing more on this GPU
tools/gpu_session.sh \
  "120|$o/write_runs|./tools/write_runs" \
  "120|$o/write_runs_pmc|rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$o/wr_pmc -o run --output-format csv -- ./tools/write_runs"
