#!/bin/bash
# round 6 call 9: k_h_eval alone at finer sort tiles (tile bits 5 / 6: the Hilbert order's
# major key unchanged, items reordered by 128^2 / 64^2 sub-tiles inside each 256^2 tile) --
# kernel traces, so the evaluation's time separates from the bigger sort's
cd "$GRAFT_REPO_ROOT"
o=r06/c9
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
for tb in 4 5 6; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$o/tb$tb -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 --opt k2g_tile_bits=$tb > gpurun_out/$o/tb$tb.log 2>&1 || exit $?
done
