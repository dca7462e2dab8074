"""Full-scale DEM reprojection (K7): a lat/lon mosaic the size of
mergeLL.vrt (18225 x 14250 Float32, 0.2" pixels, mergeLL.vrt:1-3) onto the cfg4 plane grid
(8192^2 over x 0..60 km, y -40..20 km).  Source synthesized on the device (smooth field with
nodata sea).  Reports ms, output cells/s, algorithmic bytes (4 B store + 4 B (nearest) /
16 B (bilinear) source reads per cell) and the 1-core oracle on a 512^2 sample.
usage: python tools/bench_reproject.py [--R 8192] [--reps 10] [--no-cpu]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch
    from uam_path_planning_amd._lib import GeoGridDesc
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.scenario import raster_geo

    eng = Engine(0)
    nx, ny = 18225, 14250
    lon0, lat_top, d = 129.325, 33.333333333, 5.5555555555554013e-05
    gg = GeoGridDesc(nx, ny, lon0, lat_top, d, d, -9999.0, 0)
    u = torch.arange(nx, device="cuda", dtype=torch.float32)
    v = torch.arange(ny, device="cuda", dtype=torch.float32)[:, None]
    src = 150.0 + 120.0 * torch.sin(u * 0.0011) * torch.cos(v * 0.0013)
    src = torch.where(torch.sin(u * 0.0002 + v * 0.0003) > 0.3, torch.tensor(-9999.0,
                      device="cuda"), src).contiguous()
    geo = raster_geo(a.R)
    for resample in (0, 1):
        out = eng.reproject_dem(src, gg, geo, 1000.0, resample)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            eng.reproject_dem(src, gg, geo, 1000.0, resample)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        cells = a.R * a.R
        byts = cells * (4 + (4 if resample == 0 else 16))
        row = {"kernel": "k_reproject", "resample": ["nearest", "bilinear"][resample],
               "src": f"{nx}x{ny}", "dst": f"{a.R}x{a.R}", "ms": round(ms, 4),
               "cells_per_s": cells / (ms / 1e3), "algorithmic_GBps": byts / (ms / 1e3) / 1e9,
               "valid_frac": float((out != -9999.0).double().mean())}
        if not a.no_cpu and resample == 0:
            sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
            from oracle import oracle as O

            # CPU baseline on a 512^2 sample grid (same extent) from a 2048^2 source window
            s_np = src[:2048, :2048].cpu().numpy()
            sg = raster_geo(512)
            rd = O.Oracle.raster_desc(sg.nx, sg.ny, sg.x0, sg.y_top, sg.dx, sg.dy)
            t0 = time.perf_counter()
            O.reproject(s_np, O.geo_grid(2048, 2048, lon0, lat_top, d * 8, d * 8), rd)
            dt = time.perf_counter() - t0
            row["cpu_oracle_cells_per_s_1core"] = 512 * 512 / dt
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
