#!/bin/bash
# round 6 call 18: K1 (cfg3 map, 4096^2) wave-cycle split and instruction counts after the
# nontemporal stores and ineq_h_col (SQ counters, two passes; compare profiles/r05 k1sq)
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06/c18
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$o/list.txt" 2>&1 || true
have() { grep -qw -- "${1%_sum}" "$o/list.txt"; }
prog="python3 tools/probe_k1.py --cases cfg3 --reps 5"
run_pass() {
    local name=$1; shift
    local keep=()
    for c in "$@"; do if have "$c"; then keep+=("$c"); else echo "$name $c" >> "$o/missing.txt"; fi; done
    [ ${#keep[@]} -eq 0 ] && return 0
    echo "=== pass $name: ${keep[*]}"
    timeout -s KILL 120 rocprofv3 --pmc "${keep[@]}" -d "$o/$name" -o run --output-format csv -- $prog \
        > "$o/$name.log" 2>&1
}
run_pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU &&
run_pass sq2 SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 &&
python3 tools/pmc_kernel_sum.py $o k_raster_build_cells > $o/summary.txt && cat $o/summary.txt
