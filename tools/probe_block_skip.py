"""How many of K2's record gathers a block summary table could skip, bit-exactly, on the bench
workload (cfg3).  A waypoint's gather is needed unless its 8x8 cell block has Φ = Σψ = 0 in
every cell (adding +0.0 is exact), one flags value, and a block-maximum DEM that cannot raise
the path's maximum DEM (the min-clearance input): blockmax(w) <= LB, where LB = max over the
path's waypoints of blockmin(w) <= the true maximum.  Measurement for DESIGN.md §9.
usage: python tools/probe_block_skip.py [--pairs 20000] [--B 8]"""
import argparse
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=20000)
    ap.add_argument("--B", type=int, nargs="+", default=[4, 8, 16])
    a = ap.parse_args()
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (CONFIGS, build_region_map, canonical_params,
                                                canonical_spec, displacements, raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    cfg = CONFIGS["cfg3"]
    R, N, D = cfg["R"], cfg["N"], cfg["D"]
    spec = canonical_spec(nfz_polygons=cfg["nfz_polygons"])
    eng = Engine(0)
    eng.set_geometry(compile_map(build_region_map(spec)))
    eng.set_params(canonical_params(spec, N=N, altitude=320.0))
    geo = raster_geo(R)
    raster = eng.raster_build(geo, eng.tensor(synthetic_dem(R), torch.float32))
    rec = raster.rec
    f = rec.view(torch.float32)
    phi, psi, dem, flags = f[..., 0], f[..., 1], f[..., 2], rec[..., 3]
    zero = (phi == 0) & (psi == 0)
    print(f"cells with phi = psi = 0: {zero.float().mean().item():.3f}")
    ut = eng.tensor(arc_table(N, displacements(D)), torch.float64)
    pairs = eng.tensor(random_pairs(a.pairs, seed=0), torch.float64)
    g = eng.eval_generated(pairs, ut, raster=raster, want_cells=True)
    cells = g["cells"].long()  # [P, W] linear cell index, < 0 outside the raster
    inside = cells >= 0
    print(f"waypoints inside the raster: {inside.float().mean().item():.3f}")
    cy, cx = cells.clamp(min=0) // R, cells.clamp(min=0) % R
    for B in a.B:
        nb = R // B

        def blk(t):
            return t.view(nb, B, nb, B).permute(0, 2, 1, 3).reshape(nb, nb, B * B)

        bzero = blk(zero).all(-1)
        fl = blk(flags)
        bunif = fl.min(-1).values == fl.max(-1).values
        dm = blk(dem)
        bmax, bmin = dm.max(-1).values, dm.min(-1).values
        bi = (cy // B, cx // B)
        ok = (bzero & bunif)[bi] & inside
        lb = torch.where(inside, bmin[bi], torch.full_like(bmin[bi], -3e38)).max(1, True).values
        skip = ok & (bmax[bi] <= lb)
        need = inside & ~skip
        print(f"B={B:2d}: blocks zero+uniform {(bzero & bunif).float().mean().item():.3f}; "
              f"waypoints in such blocks {ok.float().sum().item() / inside.sum().item():.3f}; "
              f"gathers still needed {need.float().sum().item() / inside.sum().item():.3f}; "
              f"summary table {nb * nb * 8 / 2**20:.1f} MiB")


if __name__ == "__main__":
    main()
