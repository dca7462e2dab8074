import sys, time, os
sys.path.insert(0, os.getcwd())
import torch
from uam_path_planning_amd.engine import Engine
from uam_path_planning_amd.scenario import raster_geo
from uam_path_planning_amd.synthetic import synthetic_dem
eng = Engine(0)
geo = raster_geo(8192)
dem = torch.tensor(synthetic_dem(8192, seed=3), device="cuda")
for i in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = eng.dem_polygons(dem, geo, 0.0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"call {i}: {1e3*(t1-t0):.3f} ms in call, {1e3*(t2-t0):.3f} ms incl sync", file=sys.stderr, flush=True)
