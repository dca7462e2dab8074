#!/bin/bash
# GPU box, round 3: L2 counters of K2g at 8 gathers in flight (4 waves / SIMD) against 16 (2
# waves / SIMD): the same loads in flight per SIMD, half the resident items.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g21
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
for c in 8 16; do
  P="python3 tools/probe_k2g.py --groups 21 --tbits 0 --chunks $c --reps 5"
  tools/gpu_session.sh \
    "120|$o/tcc$c|rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_128B_sum -d gpurun_out/$o/tcc$c -o run --output-format csv -- $P" \
    "120|$o/trace$c|rocprofv3 --kernel-trace --stats -d gpurun_out/$o/trace$c -o run --output-format csv -- $P" || exit $?
done
