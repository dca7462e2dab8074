#!/bin/bash
# Kernel trace + PMC passes of one bench.py configuration (run on the GPU box), one rocprofv3
# run per pass (kernel trace only beside --pmc; MI355X_MICROARCH.md rocprofv3 rules):
#   bash tools/profile_bench.sh <out_dir> <bench args...>
# Passes: trace (--kernel-trace --stats), fetch (FETCH_SIZE), write (WRITE_SIZE),
# tcc (TCC_HIT/MISS/EA0_RDREQ_128B), sq (SQ wave-cycle shares), f64 (f64 VALU instruction mix).
# Summarise afterwards with tools/pmc_traffic.py (key = bench.py's roofline.profile_key).
# PASSES="trace fetch" limits the run to those passes.
set -eu
out=$1
shift
mkdir -p "$out"
export TMPDIR=/tmp
bench="python3 bench.py --no-cpu-baseline $*"
passes=${PASSES:-"trace fetch write tcc sq f64"}
for p in $passes; do
    case $p in
        trace) args="--kernel-trace --stats" ;;
        fetch) args="--pmc FETCH_SIZE" ;;
        write) args="--pmc WRITE_SIZE" ;;
        tcc)   args="--pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_128B_sum" ;;
        sq)    args="--pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" ;;
        f64)   args="--pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" ;;
        *) echo "unknown pass $p"; exit 2 ;;
    esac
    echo "=== pass $p: rocprofv3 $args -- $bench"
    timeout -k 10 240 rocprofv3 $args -d "$out/$p" -o run --output-format csv -- $bench \
        > "$out/$p.log" 2>&1
    tail -n 1 "$out/$p.log"
done
