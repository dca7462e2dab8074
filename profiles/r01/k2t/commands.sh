P="python tools/probe_raster.py --variants 12 --sizes '' --analytic-pairs 0 --rounds 1"
bash tools/gpu_session.sh \
 "300|t_tiled|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 'tiled'" \
 "100|pv|python tools/probe_raster.py --variants 2,12 --sizes '' --analytic-pairs 0 --rounds 2" \
 "100|p0|rocprofv3 --kernel-trace -d gpurun_out/pr0 -o run -- $P" \
 "100|p1|UAM_TB_DBG=1 rocprofv3 --kernel-trace -d gpurun_out/pr1 -o run -- $P" \
 "100|p2|UAM_TB_DBG=2 rocprofv3 --kernel-trace -d gpurun_out/pr2 -o run -- $P" \
 "100|p4|UAM_TB_DBG=4 rocprofv3 --kernel-trace -d gpurun_out/pr4 -o run -- $P" \
 "100|p16|UAM_TB_PB=16 rocprofv3 --kernel-trace -d gpurun_out/pr16 -o run -- $P"
