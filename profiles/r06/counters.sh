#!/bin/bash
# Round 6, verdict item 2: what the 60% SQ_WAIT_INST_ANY of k_h_eval is.  TA / TD / TCP / SQ
# VMEM counters of the cfg3 bench step, entry form (default) and bound form (K2H_TERRAIN=0),
# one rocprofv3 run per pass; counters absent from `rocprofv3 -L` on this box are dropped (and
# listed in <out>/missing.txt).  usage: bash profiles/r06/counters.sh <out_dir> [bench args]
set -u
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$out/list.txt" 2>&1 || true
bench="python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 $*"
have() { grep -qw -- "${1%_sum}" "$out/list.txt"; }
run_pass() {  # name counters...
    local name=$1; shift
    local keep=()
    for c in "$@"; do if have "$c"; then keep+=("$c"); else echo "$name $c" >> "$out/missing.txt"; fi; done
    [ ${#keep[@]} -eq 0 ] && return 0
    echo "=== pass $name: ${keep[*]}"
    timeout -s KILL 200 rocprofv3 --pmc "${keep[@]}" -d "$out/$name" -o run --output-format csv -- $bench \
        > "$out/$name.log" 2>&1
    local st=$?
    tail -n 1 "$out/$name.log"
    return $st
}
run_pass ta  TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum &&
run_pass ta2 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum &&
run_pass td  TD_TD_BUSY_sum TD_TC_STALL_sum &&
run_pass tcp TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum &&
run_pass tcp2 TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum &&
run_pass tcp3 TCP_GATE_EN1_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_PERMISSION_MISS_sum &&
run_pass sqv SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD &&
run_pass sqb SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INST_LEVEL_VMEM &&
run_pass tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_128B_sum TCC_TAG_STALL_sum
