#!/bin/bash
# round 6 call 19: traces + PMC (FETCH/WRITE/TCC) of cfg4 -- the whole job on one GPU and rank
# 3's spatial share of the 8-GPU run -- on the final tree, for profiles/traffic.json's
# cfg4 keys (round 5's were from before the batch-sized tile bits)
cd "$GRAFT_REPO_ROOT"
o=r06/c19
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "500|$o/prof_s3|PASSES='trace fetch write tcc' bash tools/profile_bench.sh gpurun_out/$o/s3 --workload cfg4 --share 3/8 --steps 5 --warmup 1" \
  "600|$o/prof_cfg4|PASSES='trace fetch write tcc' bash tools/profile_bench.sh gpurun_out/$o/cfg4 --workload cfg4 --steps 5 --warmup 1"
