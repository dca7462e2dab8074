# K2s (segment-sorted raster evaluation) on the GPU box: its parity tests, then bench.py
# under "segments lds-floor split fuse lds0-floor first order0" settings (CFGS, one per line; segments 0 =
# K2; missing columns take the library defaults).
#   bash tools/k2s_run.sh            (NOTEST=1 skips the tests)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k2s
if [ -z "$NOTEST" ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_k2s.py "tests/test_gpu_parity.py::test_full_size_cfg3_properties" \
    "tests/test_gpu_parity.py::test_raster_summary_table" \
    "tests/test_gpu_parity.py::test_raster_pair_order_and_gather_skip" \
    > gpurun_out/k2s/pytest.log 2>&1 || { tail -30 gpurun_out/k2s/pytest.log; exit 1; }
  tail -3 gpurun_out/k2s/pytest.log
fi
CFGS=${CFGS:-"0 0 1 1 0
4 81920 1 1 0
4 81920 1 1 40960
4 81920 1 1 81920
3 81920 1 1 0
2 81920 1 1 0
4 81920 1 0 0"}
while read -r sg ld sp fu l0 fi o0; do
  [ -z "$sg" ] && continue
  log=gpurun_out/k2s/b_s${sg}_l${ld}_h${sp}_f${fu}_z${l0}_F${fi:-0}_o${o0:-1}.log
  UAM_K2S_SEGS=$sg UAM_K2S_LDS=$ld UAM_K2S_SPLIT=$sp UAM_K2S_FUSE=${fu:-1} UAM_K2S_LDS0=${l0:-0} UAM_K2S_FIRST=${fi:-0} UAM_K2S_ORDER0=${o0:-1} \
    timeout -k 10 240 python -u bench.py --steps 30 --warmup 3 > $log 2>&1 || exit 1
  echo "segs=$sg lds=$ld split=$sp fuse=$fu lds0=$l0 first=${fi:-0} order0=${o0:-1} $(grep -o '"ms_per_step": [0-9.]*' $log) $(grep -o '"kernel_ms": [0-9.]*' $log)"
done <<< "$CFGS"
