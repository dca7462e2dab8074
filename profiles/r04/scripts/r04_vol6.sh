#!/bin/bash
# GPU box, round 4: K4h L2 misses per setting (one rocprofv3 --pmc pass per probe run):
# bands of 2 / 4 layers, 8 x 8 / 16 x 16 tiles, CH 8 / 11.
cd "$GRAFT_REPO_ROOT"
o=r04/vol6
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
run() {  # name settings
    echo "=== $1: $2"
    timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/$o/$1 -o run --output-format csv -- python3 tools/probe_opts.py --volume --reps 5 --tag $1 --settings "$2" > gpurun_out/$o/$1.log 2>&1 || exit $?
    grep '^{' gpurun_out/$o/$1.log
}
run base "k4h_band=0" && run band2 "k4h_band=2" && run tb4 "k2g_tile_bits=4" && run ch8 "k2g_chunk=8" && run base2 "k4h_band=0"
