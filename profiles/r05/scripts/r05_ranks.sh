#!/bin/bash
# GPU box, round 5: bench.py's N-rank path rehearsed on one GPU (ranks sharing it, gloo for
# the host collectives): cfg3 at 2 ranks, cfg5 at 2, cfg4 at 8 ranks over spatial shards.
cd "$GRAFT_REPO_ROOT"
o=r05/ranks
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
r="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
tools/gpu_session.sh \
  "300|$o/ranks2_cfg3|UAM_BENCH_RANKS_PER_GPU=2 UAM_DIST_BACKEND=gloo $r --nproc-per-node 2 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2" \
  "300|$o/ranks2_cfg5|UAM_BENCH_RANKS_PER_GPU=2 UAM_DIST_BACKEND=gloo $r --nproc-per-node 2 --master-port 29535 bench.py --gpus 2 --workload cfg5 --steps 5 --warmup 2" \
  "400|$o/ranks8_cfg4|UAM_BENCH_RANKS_PER_GPU=8 UAM_DIST_BACKEND=gloo $r --nproc-per-node 8 --master-port 29534 bench.py --gpus 8 --workload cfg4 --steps 3 --warmup 1"
