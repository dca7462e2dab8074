#!/bin/bash
# GPU box, round 4: the grouped sort with 512 / 1024 partitions (measurement builds) against
# 256: cfg3 and cfg4-size probes, cfg3 traces.
cd "$GRAFT_REPO_ROOT"
o=r04/nbk
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
tools/gpu_session.sh \
  "200|$o/c3_256|python -u tools/probe_opts.py --tag 256 --settings 'group=21;group=21'" \
  "200|$o/c3_512|UAM_LIB_PATH=$V/libuampath_nbk512.so python -u tools/probe_opts.py --tag 512 --settings 'group=21;group=21'" \
  "200|$o/c3_1024|UAM_LIB_PATH=$V/libuampath_nbk1024.so python -u tools/probe_opts.py --tag 1024 --settings 'group=21;group=21'" \
  "300|$o/c4_256|python -u tools/probe_opts.py --R 8192 --pairs 200000 --reps 10 --tag 256 --settings 'group=21'" \
  "300|$o/c4_512|UAM_LIB_PATH=$V/libuampath_nbk512.so python -u tools/probe_opts.py --R 8192 --pairs 200000 --reps 10 --tag 512 --settings 'group=21'" \
  "200|$o/c5_256|python -u tools/probe_opts.py --volume --tag 256 --settings 'group=21'" \
  "200|$o/c5_512|UAM_LIB_PATH=$V/libuampath_nbk512.so python -u tools/probe_opts.py --volume --tag 512 --settings 'group=21'" \
  "200|$o/prof_512|UAM_LIB_PATH=$V/libuampath_nbk512.so PASSES='trace' bash tools/profile_bench.sh gpurun_out/$o/t512 --steps 5 --warmup 1"
