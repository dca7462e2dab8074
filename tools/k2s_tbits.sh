# bench.py with tuning builds of libuampath (build/var/libuampath_<v>.so, e.g. -DUAM_SEG_TBITS=5
# as t5) beside the default build, twice each: VARS="def t5 t4" bash tools/k2s_tbits.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k2s
for rep in 1 2; do
for v in ${VARS:-def t5}; do
  if [ $v != def ]; then export UAM_LIB_PATH=$PWD/build/var/libuampath_$v.so; else unset UAM_LIB_PATH; fi
  timeout -k 10 240 python -u bench.py --steps 30 --warmup 3 > gpurun_out/k2s/tb_$v.log 2>&1 || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/k2s/tb_$v.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/k2s/tb_$v.log)"
done; done
