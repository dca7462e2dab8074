#!/bin/bash
# round 6 call 1: the new device-check and waypoint-cell tests, then the counters of the cfg3
# step (entry form, then bound form)
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06/c1
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_k2h.py tests/test_gpu_k4h.py -k "device_check or cells_vs_create" > $o/tests.log 2>&1
echo "tests exit $?"; tail -5 $o/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 &&
bash profiles/r06/counters.sh $o/entry &&
bash profiles/r06/counters.sh $o/bound --opt k2h_terrain=0
