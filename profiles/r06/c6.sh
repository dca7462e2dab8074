#!/bin/bash
# round 6 call 6 (verdict r5 item 5): cfg5 (K4h) with k_v_eval<7> at 3 waves per SIMD (no
# scratch spill), its trace and its TA / TCP / SQ counters
cd "$GRAFT_REPO_ROOT"
o=r06/c6
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "900|$o/suite|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "300|$o/bench_cfg5|python -u bench.py --workload cfg5 --no-cpu-baseline" \
  "300|$o/probe_cfg5|python -u tools/probe_opts.py --tag cfg5 --volume --reps 20 --settings 'k2g_chunk=0;k2g_chunk=8;k2g_chunk=6;k2g_chunk=0'" \
  "300|$o/trace|PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1" \
  "600|$o/cnt|bash profiles/r06/counters.sh gpurun_out/$o/cnt5 --workload cfg5"
