#!/bin/bash
# GPU box, round 3: cfg4's DEM ingest by phase (tools/probe_ingest.py) and the K2g group /
# tile-bit sweep at 8192^2 (200k pairs x 5), kernel trace split per setting.
cd "$GRAFT_REPO_ROOT"
o=r03/ingest
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
tools/gpu_session.sh \
  "300|$o/ingest|python3 -u tools/probe_ingest.py --threads 1,4,8,16" \
  "600|$o/k2g8192|rocprofv3 --kernel-trace -d gpurun_out/$o/tr -o run --output-format csv -- python3 -u tools/probe_k2g.py --R 8192 --pairs 200000 --groups 11,14,16,21 --tbits 4,5,6 --lds 0 --reps 5"
