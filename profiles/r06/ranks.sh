#!/bin/bash
# Round 6: bench.py's N-rank path rehearsed on one GPU after the round's library changes (ranks
# sharing the GPU, gloo for the host collectives): cfg3 at 2 ranks, cfg4 at 8 ranks over
# spatial shards (the driver's 8-GPU cfg4 layout); per-rank parity in each line.
cd "$GRAFT_REPO_ROOT"
o=r06/${1:-ranks}
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
r="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
tools/gpu_session.sh \
  "300|$o/ranks2_cfg3|UAM_BENCH_RANKS_PER_GPU=2 UAM_DIST_BACKEND=gloo $r --nproc-per-node 2 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2" \
  "400|$o/ranks8_cfg4|UAM_BENCH_RANKS_PER_GPU=8 UAM_DIST_BACKEND=gloo $r --nproc-per-node 8 --master-port 29534 bench.py --gpus 8 --workload cfg4 --steps 3 --warmup 1"
