#!/usr/bin/env python3
"""Packed-raster probe (GPU box): on cfg3's map and pairs, the share of waypoints in each
block code of uam_raster_pack (0 = nothing gathered, 1 = the 8-B plane-A entry, 3 = the full
16-B record, off = off the raster), i.e. the requests and bytes a packed K2s issues per waypoint.
usage: python tools/probe_pack.py [--pairs 100000]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100000)
    a = ap.parse_args()
    import numpy as np
    import torch
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (CONFIGS, build_region_map, canonical_params,
                                                canonical_spec, displacements, raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    spec = canonical_spec(nfz_polygons=CONFIGS["cfg3"]["nfz_polygons"])
    e = Engine(0)
    e.set_geometry(compile_map(build_region_map(spec)))
    e.set_params(canonical_params(spec, N=80, altitude=320.0))
    R = 4096
    raster = e.raster_build(raster_geo(R), synthetic_dem(R), packed=True)
    pairs = e.tensor(random_pairs(a.pairs, seed=0), torch.float64)
    g = e.eval_generated(pairs, arc_table(80, displacements(5)), raster=raster, want_cells=True)
    cells = g["cells"].reshape(-1).long()
    B = raster.block
    nbx = -(-R // B)
    nb = nbx * nbx
    words = -(-2 * nb // 32)
    pk = raster.packed.reshape(-1)[:4 * words].view(torch.int32)
    bits = torch.stack([(pk >> (2 * i)) & 3 for i in range(16)], 1).reshape(-1)[:nb]
    ok = cells >= 0
    c = cells.clamp(min=0)
    blk = (c // R // B) * nbx + (c % R) // B
    code = torch.where(ok, bits[blk], torch.full_like(blk, -1))
    n = code.numel()
    h = {k: float((code == v).sum()) / n for k, v in (("off", -1), ("0", 0), ("1", 1), ("3", 3))}
    print(f"cfg3 waypoints {n}: shares by block code {h}")
    print(f"blocks by code: " + ", ".join(f"{v}: {float((bits == v).sum()) / nb:.3f}"
                                         for v in (0, 1, 3)))
    print(f"gathers per waypoint {h['1'] + h['3']:.3f}; bytes per waypoint packed "
          f"{8 * h['1'] + 16 * h['3']:.2f}, 16-B form {16 * (h['1'] + h['3']):.2f}")
    # a finer "needs the full record" map: the share of gathered waypoints that would still
    # read 16 B if the psi / no-fly test were made per F x F cells (F = 1: per cell)
    rec = raster.rec.reshape(R, R, 4)
    need = ((rec[..., 1] & 0x7fffffff) != 0) | ((rec[..., 3] & 1) != 0)
    gathered = code > 0
    for F in (16, 8, 4, 1):
        nf = need.reshape(R // F, F, R // F, F).any(3).any(1)
        cf = nf[(c // R) // F, (c % R) // F] & gathered
        print(f"need-full map at {F:2d}x{F:<2d} cells: {float(cf.sum()) / n:.3f} of waypoints "
              f"read 16 B ({(R // F) ** 2 // 8 // 1024} KiB as a bitmap)")


if __name__ == "__main__":
    main()
