cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k2s
for rep in 1 2; do
for v in def t5; do
  if [ $v = t5 ]; then export UAM_LIB_PATH=$PWD/build/var/libuampath_t5.so; else unset UAM_LIB_PATH; fi
  timeout -k 10 240 python -u bench.py --steps 30 --warmup 3 > gpurun_out/k2s/tb_$v.log 2>&1 || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/k2s/tb_$v.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/k2s/tb_$v.log)"
done; done
