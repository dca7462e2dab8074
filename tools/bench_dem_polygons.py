"""Land polygons from the DEM (K8) at scale: end-to-end uam_dem_polygons
(mask + GPU union-find labelling + component stats + row extents + box-piece relabelling +
host rectangles) on synthetic plane DEMs; cells/s; the 1-core oracle on the 2048^2 case.
usage: python tools/bench_dem_polygons.py [--sizes 2048,8192,12288] [--reps 5]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="2048,8192,12288")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.scenario import raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    eng = Engine(0)
    for R in [int(x) for x in a.sizes.split(",")]:
        geo = raster_geo(R)
        dem = torch.tensor(synthetic_dem(R, seed=3), device="cuda")
        for _ in range(3):                               # warm-up (the arenas grow here)
            rects = eng.dem_polygons(dem, geo, 0.0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            rects = eng.dem_polygons(dem, geo, 0.0)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        row = {"op": "uam_dem_polygons", "dem": f"{R}x{R}", "pixel_m": 60000.0 / R,
               "ms": round(ms, 3), "cells_per_s": R * R / (ms / 1e3), "rectangles": len(rects)}
        if not a.no_cpu and R <= 2048:
            from oracle import oracle as O

            rd = O.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy)
            d = dem.cpu().numpy()
            t0 = time.perf_counter()
            ref = O.dem_polygons(d, rd, 0.0, 1000.0)
            row["cpu_oracle_ms_1core"] = round((time.perf_counter() - t0) * 1e3, 1)
            row["parity"] = bool(np.array_equal(np.asarray(rects).reshape(-1, 4, 2), ref))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
