#!/bin/bash
# round 6 call 3 (verdict r5 item 4): cfg4's rank-3-of-8 spatial share (25k pairs x 5 on the
# 8192^2 raster) re-tuned -- tile bits, group length, LDS floor (workgroups per CU), gathers in
# flight -- with the library's HIP events around each call (probe_opts.py: seq_ms), then the
# pipelined form (4 batches per call) at the defaults.
cd "$GRAFT_REPO_ROOT"
o=r06/c5/c3
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
d="k2g_tile_bits=0,group=21,k2g_lds_floor=0,k2g_chunk=0"
S="$d"
for tb in 4 6; do S="$S;k2g_tile_bits=$tb,group=21,k2g_lds_floor=0,k2g_chunk=0"; done
for g in 14 16 18 24 28; do S="$S;k2g_tile_bits=0,group=$g,k2g_lds_floor=0,k2g_chunk=0"; done
for f in 24000 40000 70000; do S="$S;k2g_tile_bits=0,group=21,k2g_lds_floor=$f,k2g_chunk=0"; done
for c in 7 8; do for f in 0 40000 54000; do S="$S;k2g_tile_bits=0,group=21,k2g_lds_floor=$f,k2g_chunk=$c"; done; done
S="$S;$d"
tools/gpu_session.sh \
  "600|$o/share3|python -u tools/probe_opts.py --tag share3 --R 8192 --pairs 200000 --share 3/8 --reps 20 --settings '$S'" \
  "300|$o/share3_b4|python -u tools/probe_opts.py --tag share3_b4 --R 8192 --pairs 200000 --share 3/8 --reps 8 --batches 4 --settings '$d'" \
  "300|$o/share0|python -u tools/probe_opts.py --tag share0 --R 8192 --pairs 200000 --share 0/8 --reps 20 --settings '$d'"
# the share's counters: L2 hits / misses, UTCL1 translation misses (the 2.5 GiB packed copy's
# pages), TA / TD busy, wave-cycle split
P="python3 tools/probe_opts.py --tag pmc --R 8192 --pairs 200000 --share 3/8 --reps 5 --settings $d"
for pass in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_128B_sum" \
            "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
            "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"; do
  n=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -s KILL 200 rocprofv3 --pmc $pass -d gpurun_out/$o/pmc_$n -o run --output-format csv -- $P \
      > gpurun_out/$o/pmc_$n.log 2>&1 || { echo "pmc pass $n failed: $?"; break; }
done
