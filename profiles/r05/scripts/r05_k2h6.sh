#!/bin/bash
# GPU box, round 5: K2h slot-class counts (counting builds, one ahead vs consumed at once) and
# the cfg3 step one ahead vs not.
cd "$GRAFT_REPO_ROOT"
o=r05/k2h6
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
b="python -u bench.py --no-cpu-baseline"
tools/gpu_session.sh \
  "120|$o/cnt|env UAM_LIB_PATH=build/variants/libuampath_cnt.so python -u tools/k2h_counts.py" \
  "120|$o/cnt0|env UAM_LIB_PATH=build/variants/libuampath_cnt0.so python -u tools/k2h_counts.py" \
  "120|$o/cnt_l2|env UAM_LIB_PATH=build/variants/libuampath_cnt.so python -u tools/k2h_counts.py --opt=k2h_lb_stride=2" \
  "90|$o/def|$b" \
  "90|$o/na|env UAM_LIB_PATH=build/variants/libuampath_na.so $b" \
  "90|$o/na_ch8|env UAM_LIB_PATH=build/variants/libuampath_na.so $b --opt k2g_chunk=8"
