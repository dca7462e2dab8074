#!/bin/bash
# K6 (k_refine) counter collection: kernel trace, SQ wait/issue counters, f64 instruction mix
# (separate --pmc passes, kernel trace only; DESIGN.md §5 "Refinement").  Run on the GPU box:
#   bash tools/k6_counters.sh <out_dir>
set -e
out=${1:-gpurun_out/k6}
mkdir -p "$out"
cmd="python3 tools/time_refine.py --pairs 2048 --outer 15 --inner 50"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- $cmd > "$out/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$out/pmc1" -o run --output-format csv -- $cmd > "$out/pmc1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d "$out/pmc2" -o run --output-format csv -- $cmd > "$out/pmc2.log" 2>&1
