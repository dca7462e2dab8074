#!/bin/bash
# GPU box, round 4: multi-rank rehearsal of bench.py on one GPU (gloo, several ranks per GPU):
# cfg3 at 2 ranks, cfg5 at 2 ranks, cfg4 (strong scaling, tiles on rank 0) at 4 ranks.
cd "$GRAFT_REPO_ROOT"
o=r04/ranks
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/ranks2_cfg3|UAM_BENCH_RANKS_PER_GPU=2 UAM_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2" \
  "300|$o/ranks2_cfg5|UAM_BENCH_RANKS_PER_GPU=2 UAM_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --workload cfg5 --steps 5 --warmup 2" \
  "300|$o/ranks4_cfg4|UAM_BENCH_RANKS_PER_GPU=4 UAM_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --workload cfg4 --steps 3 --warmup 1"
