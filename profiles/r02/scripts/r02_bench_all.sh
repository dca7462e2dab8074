# GPU box: the bench lines of this build (cfg3 raster default, cfg3 analytic, cfg4, cfg5)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/bench_all
mkdir -p $out
for w in "cfg3" "cfg3 --mode analytic" "cfg4" "cfg5"; do
  set -- $w
  tag=$(echo "$w" | tr ' ' '_' | tr -d '-')
  timeout -k 10 400 python -u bench.py --workload $w > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$out/$tag.log').read().strip().splitlines()[-1])
r=d['roofline']
print('$tag', d['value'], d['ms_per_step'], r.get('kernel_ms'), r.get('frac'), r.get('library_kernel'), r.get('traffic'), r.get('l2_hit_rate'))
"
done
