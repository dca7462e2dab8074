#!/usr/bin/env python3
"""CPU probe (no GPU): how many of K2g's gathers could a block-level bound remove on the cfg3
map?  A waypoint's gather feeds three things: Phi/N, the no-fly psi / hit count (code-3 blocks
only) and the terrain maximum.  In a block where Phi is +-0 everywhere and no cell is on no-fly
support, the only thing the gather can change is the maximum -- and it cannot change it when
an upper bound of the block's terrain is <= the item's running maximum (max is order-free, so
skipping such a read is exact).  This counts, per (path, group) item in waypoint order, the
gathers the current rule issues (code 1 and 3 blocks) and the ones left with the bound rule,
for block sizes 16 / 32 / 64 and the bound quantised to 8 bits (rounded up).

usage: python tools/probe_terrain_skip.py [--R 2048] [--pairs 20000] [--group 24]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=2048)
    ap.add_argument("--pairs", type=int, default=20000)
    ap.add_argument("--group", type=int, default=24)
    a = ap.parse_args()
    from oracle import oracle as O
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec, displacements, raster_geo
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    O.build()
    spec = canonical_spec(nfz_polygons=64)
    N, D = 80, 5
    orc = O.Oracle(O.compile_spec(spec), N, spec["options"], spec["maxratio"], spec["maxalpha"],
                   spec["enlargement"], spec["weights"], altitude=320.0)
    geo = raster_geo(a.R)
    rd = O.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy, geo.nodata,
                              geo.dem_threshold)
    t0 = time.time()
    rec = orc.raster_build(rd, synthetic_dem(a.R))
    print(f"raster {a.R}^2 built in {time.time() - t0:.1f} s", flush=True)
    phi, psi, ter = rec[..., 0], rec[..., 1], rec[..., 2].copy()
    flags = rec[..., 3].view(np.uint32)
    ter[(flags & 4) != 0] = 0.0
    nfz = (flags & 1) != 0
    wp = O.gen_paths(random_pairs(a.pairs, seed=0), arc_table(N, displacements(D)))
    wp = wp.reshape(-1, N + 2, 2)
    ix = np.floor((wp[..., 0] - geo.x0) / geo.dx)
    iy = np.floor((geo.y_top - wp[..., 1]) / geo.dy)
    inr = (ix >= 0) & (ix < geo.nx) & (iy >= 0) & (iy < geo.ny)
    ix = np.where(inr, ix, 0).astype(np.int64)
    iy = np.where(inr, iy, 0).astype(np.int64)
    P, W = ix.shape
    G = a.group
    print(f"{P} paths x {W} waypoints, groups of {G}; "
          f"{100 * (1 - inr.mean()):.2f}% off the raster", flush=True)
    lo, hi = float(np.nanmin(ter)), float(np.nanmax(ter))
    for B in (16, 32, 64):
        nb = a.R // B
        blk = lambda v: v.reshape(nb, B, nb, B)
        phi_any = (blk(phi) != 0).any(axis=(1, 3))
        need_full = (blk(np.abs(psi)) != 0).any(axis=(1, 3)) | blk(nfz).any(axis=(1, 3))
        tmax = blk(ter).max(axis=(1, 3))
        # 8-bit upper bound of the block maximum (rounded up), as a table would hold it
        step = (hi - lo) / 255.0
        q = np.ceil((tmax - lo) / step).clip(0, 255)
        tbound = lo + q * step
        tbound = np.maximum(tbound, tmax)
        skip0 = ~phi_any & ~need_full & (tmax == 0)  # the current code-0 rule (+0.0 terrain)
        by, bx = iy // B, ix // B
        code0 = skip0[by, bx] | ~inr
        full = need_full[by, bx] & inr
        phiz = ~phi_any[by, bx] & ~need_full[by, bx] & inr & ~code0
        bound = tbound[by, bx]
        t_exact = ter[iy, ix]
        now = (~code0).sum()
        left = 0
        for s0 in range(0, W, G):
            run = np.full(P, -np.inf)
            for j in range(s0, min(s0 + G, W)):
                rd_ = ~code0[:, j] & ~(phiz[:, j] & (bound[:, j] <= run))
                left += int(rd_.sum())
                run = np.where(rd_, np.maximum(run, t_exact[:, j]), run)
        tot = P * W
        print(f"B={B:3d}: gathers now {now / tot:.3f} of waypoints (full {full.sum() / tot:.3f}, "
              f"phi-zero blocks {phiz.sum() / tot:.3f}); with the terrain bound {left / tot:.3f} "
              f"({100 * (1 - left / now):.1f}% fewer)", flush=True)


if __name__ == "__main__":
    main()
