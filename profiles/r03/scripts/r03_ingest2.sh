#!/bin/bash
# GPU box, round 3: uam_load_tiles (chunked page-locked streaming) -- its tests, the ingest
# probe and the cfg4 bench line.
cd "$GRAFT_REPO_ROOT"
o=r03/ingest2
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/tests|python -u -m pytest tests/test_gpu_parity.py -k 'load_tiles or vrt_ingest' -x -q --timeout 200 --timeout-method thread" \
  "300|$o/ingest|python3 -u tools/probe_ingest.py --threads 8,16" \
  "200|$o/bench_cfg4|python -u bench.py --workload cfg4"
