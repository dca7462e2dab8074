#!/bin/bash
# GPU box, round 4: 6-workgroup K2h build A/B, cfg4 / cfg5 bench lines, 2-rank cfg3 and 4-rank
# cfg4 rehearsals on one GPU (gloo), cfg5 PMC.
cd "$GRAFT_REPO_ROOT"
o=r04/run6
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
tools/gpu_session.sh \
  "200|$o/minw6|UAM_LIB_PATH=$V/libuampath_minw6.so python -u tools/probe_opts.py --tag minw6 --settings 'k2g_chunk=6;k2g_chunk=7;k2g_chunk=8'" \
  "200|$o/minw4|python -u tools/probe_opts.py --tag minw4 --settings 'k2g_chunk=6;k2g_chunk=7;k2g_chunk=8'" \
  "300|$o/bench_cfg4|python -u bench.py --workload cfg4" \
  "200|$o/bench_cfg5|python -u bench.py --workload cfg5" \
  "300|$o/ranks2_cfg3|UAM_BENCH_RANKS_PER_GPU=2 UAM_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2" \
  "400|$o/prof_cfg5|PASSES='trace fetch write tcc sq' bash tools/profile_bench.sh gpurun_out/$o/cfg5 --workload cfg5 --steps 5 --warmup 1"
