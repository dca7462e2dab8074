#!/bin/bash
# GPU box, round 3 final K2g state (batched sort loads, batched output launch): full GPU suite,
# smoke, cfg3 / cfg4 / cfg5 / analytic bench lines, trace + PMC passes for cfg3 and cfg4.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g_v9
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "600|$o/gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "120|$o/smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "150|$o/bench|python -u bench.py" \
  "200|$o/bench_cfg4|python -u bench.py --workload cfg4" \
  "150|$o/bench_cfg5|python -u bench.py --workload cfg5" \
  "600|$o/prof3|PASSES=\"trace fetch write tcc sq\" bash tools/profile_bench.sh gpurun_out/$o/raster --steps 5 --warmup 1" \
  "600|$o/prof4|PASSES=\"trace fetch write tcc sq\" bash tools/profile_bench.sh gpurun_out/$o/cfg4 --workload cfg4 --steps 5 --warmup 1"
# N-rank rehearsal on the one-GPU box (gloo, ranks share the GPU): rendezvous, rank-0 raster
# build + broadcast, pair shards, max over ranks, per-rank parity (the driver runs N = 8 on RCCL)
tools/gpu_session.sh \
  "300|$o/ranks2_cfg3|UAM_BENCH_RANKS_PER_GPU=2 UAM_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2" \
  "300|$o/ranks4_cfg4|UAM_BENCH_RANKS_PER_GPU=4 UAM_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --workload cfg4 --steps 3 --warmup 1"
