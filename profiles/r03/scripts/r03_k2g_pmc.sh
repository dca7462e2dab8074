#!/bin/bash
# GPU box, round 3: trace + PMC passes (fetch / write / tcc / sq) of the default K2g step.
cd "$GRAFT_REPO_ROOT"
o=r03/k2g_pmc2
mkdir -p gpurun_out/$o
tools/gpu_session.sh \
  "500|$o/prof|PASSES=\"trace fetch write tcc sq\" bash tools/profile_bench.sh gpurun_out/$o/raster --steps 5 --warmup 1" \
  "200|$o/bench|python -u bench.py"
