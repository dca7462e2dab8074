#!/bin/bash
# GPU box, round 3: K2g with the Hilbert tile order: tests, sweep over group / tile bits /
# curve, L2 counters and kernel trace for G = 16 and G = 21 (tile bits 5, Hilbert).
cd "$GRAFT_REPO_ROOT"
o=r03/k2g13
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
P="python3 tools/probe_k2g.py --tbits 5 --chunks 8 --curves 1 --reps 5"
tools/gpu_session.sh \
  "300|$o/k2g_tests|python -u -m pytest tests/test_gpu_k2g.py -x -q --timeout 120 --timeout-method thread" \
  "300|$o/sweep|python -u tools/probe_k2g.py --groups 12,14,16,18,21,24 --tbits 4,5,6 --chunks 8 --curves 0,1 --reps 10" \
  "120|$o/tcc16|rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_128B_sum -d gpurun_out/$o/tcc16 -o run --output-format csv -- $P --groups 16" \
  "120|$o/tcc21|rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_128B_sum -d gpurun_out/$o/tcc21 -o run --output-format csv -- $P --groups 21" \
  "120|$o/trace|rocprofv3 --kernel-trace --stats -d gpurun_out/$o/trace -o run --output-format csv -- python3 tools/probe_k2g.py --tbits 5 --chunks 8 --curves 1 --reps 5 --groups 16,21"
