bash tools/gpu_session.sh \
 "240|bench_n2|UAM_DIST_BACKEND=gloo UAM_BENCH_RANKS_PER_GPU=2 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2" \
 "240|bench_n4|UAM_DIST_BACKEND=gloo UAM_BENCH_RANKS_PER_GPU=4 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 5 --warmup 2 --pairs 20000"
bash tools/gpu_session.sh \
 "240|bench_n8|UAM_DIST_BACKEND=gloo UAM_BENCH_RANKS_PER_GPU=8 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 8 --steps 5 --warmup 2 --pairs 10000"
