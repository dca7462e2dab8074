#!/bin/bash
# GPU box, round 5: the counting sort's partitions (G_NBK 128 / 256 default / 512 / 1024 build
# variants) on cfg3, cfg4 rank 3's share and cfg5; K2h parity on the 512 build.
cd "$GRAFT_REPO_ROOT"
o=r05/cc17
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
V=build/variants
b="python -u bench.py --no-cpu-baseline"
steps=()
for v in def nbk128 nbk512 nbk1024 def; do
  if [ $v = def ]; then e=""; else e="UAM_LIB_PATH=$V/libuampath_$v.so"; fi
  steps+=("120|$o/${v}_c3|$e $b" "120|$o/${v}_s3|$e $b --workload cfg4 --share 3/8" "120|$o/${v}_c5|$e $b --workload cfg5")
done
tools/gpu_session.sh "${steps[@]}" \
  "300|$o/par512|UAM_LIB_PATH=$V/libuampath_nbk512.so python -u -m pytest tests/test_gpu_k2h.py tests/test_gpu_k4h.py -x -q -k 'vs_oracle' --timeout 120 --timeout-method thread"
