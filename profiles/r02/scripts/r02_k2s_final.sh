# GPU box: full GPU suite, the default bench line, and the profile passes of the K2s build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k2s_final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/k2s_final/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/k2s_final/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/k2s_final/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/k2s_final/bench.log 2>&1 || { tail -20 gpurun_out/k2s_final/bench.log; exit 1; }
tail -1 gpurun_out/k2s_final/bench.log | cut -c1-300
PASSES="trace fetch write tcc sq" bash tools/profile_bench.sh gpurun_out/k2s_final/raster --steps 5 --warmup 1
