# GPU box: the packed-K2s build's bench lines (cfg3 default, cfg4, cfg5, analytic), the profile
# passes of the default raster step, smoke and the full GPU suite (tools/gpu_session.sh steps)
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/pack_final
mkdir -p $o
tools/gpu_session.sh \
  "240|pack_final/bench|python -u bench.py" \
  "300|pack_final/prof|PASSES=\"trace fetch write tcc sq\" bash tools/profile_bench.sh $o/raster --steps 5 --warmup 1" \
  "240|pack_final/bench_cfg4|python -u bench.py --workload cfg4 --no-cpu-baseline" \
  "240|pack_final/bench_cfg5|python -u bench.py --workload cfg5 --no-cpu-baseline" \
  "240|pack_final/bench_analytic|python -u bench.py --mode analytic --no-cpu-baseline" \
  "120|pack_final/smoke|python -u -c \"import __graft_entry__ as g; g.smoke()\"" \
  "700|pack_final/pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
