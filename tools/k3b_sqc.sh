#!/bin/bash
# K3b scalar-cache and issue counters (one rocprofv3 pass each; kernel trace only beside --pmc)
set -e
export TMPDIR=/tmp
out=${1:-gpurun_out/k3b_sqc}
mkdir -p "$out"
B="python3 bench.py --no-cpu-baseline --mode analytic --steps 2 --warmup 1"
timeout -k 10 120 rocprofv3 --pmc SQC_DCACHE_BUSY_CYCLES SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES -d "$out/p1" -o run --output-format csv -- $B > "$out/p1.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY -d "$out/p2" -o run --output-format csv -- $B > "$out/p2.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_ANY -d "$out/p3" -o run --output-format csv -- $B > "$out/p3.log" 2>&1
