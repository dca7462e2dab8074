"""Per-call wall time of uam_dem_polygons (the per-phase stamps of a -DUAM_K8_PROF build were removed in round 6).
usage: python tools/k8_call_timing.py [size=8192] [calls=4]"""
import sys, time, os
sys.path.insert(0, os.getcwd())
import torch
from uam_path_planning_amd.engine import Engine
from uam_path_planning_amd.scenario import raster_geo
from uam_path_planning_amd.synthetic import synthetic_dem
eng = Engine(0)
R = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
geo = raster_geo(R)
dem = torch.tensor(synthetic_dem(R, seed=3), device="cuda")
for i in range(K):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = eng.dem_polygons(dem, geo, 0.0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"call {i}: {1e3*(t1-t0):.3f} ms in call, {1e3*(t2-t0):.3f} ms incl sync", file=sys.stderr, flush=True)
