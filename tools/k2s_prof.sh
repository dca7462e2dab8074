# kernel traces of bench.py with the K2s launches, one per segment count in SEGS_LIST
# (default "2 4"); prints each run's per-kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
for sg in ${SEGS_LIST:-2 4}; do
  UAM_K2S_SEGS=$sg PASSES=trace bash tools/profile_bench.sh gpurun_out/k2s_prof/s$sg --steps 10 --warmup 2 || exit 1
  f=gpurun_out/k2s_prof/s$sg/trace/run_kernel_stats.csv
  echo "== segments $sg"
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print(f\"{r['Name'][:90]:90s} {int(r['Calls']):4d} {float(r['AverageNs'])/1e3:9.1f} us\")
"
done
