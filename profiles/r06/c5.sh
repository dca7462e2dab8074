#!/bin/bash
# round 6 call 5: cfg3 K2h occupancy sweep (LDS floor = workgroups per CU) x gathers in flight,
# one call per step and 4 batches per call (the side stream then has room beside the
# evaluation), with the library's HIP events (probe_opts.py seq_ms); then call 3's cfg4-share
# sweep and counters
cd "$GRAFT_REPO_ROOT"
o=r06/c5
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
S="k2g_lds_floor=0,k2g_chunk=0"
for f in 28000 33000 40000 54000; do for c in 0 8 11; do S="$S;k2g_lds_floor=$f,k2g_chunk=$c"; done; done
S="$S;k2g_lds_floor=0,k2g_chunk=8;k2g_lds_floor=0,k2g_chunk=0"
B="batch_form=0,k2g_lds_floor=0;batch_form=0,k2g_lds_floor=40000;batch_form=1,k2g_lds_floor=40000;batch_form=0,k2g_lds_floor=54000;batch_form=1,k2g_lds_floor=54000"
tools/gpu_session.sh \
  "400|$o/occ|python -u tools/probe_opts.py --tag occ --reps 20 --settings '$S'" \
  "300|$o/b4occ|python -u tools/probe_opts.py --tag b4occ --batches 4 --reps 5 --settings '$B'" &&
bash profiles/r06/c3.sh
