#!/usr/bin/env python3
"""K2g sweep (GPU box): cfg3 (4096^2 DEM + 70 no-fly shapes, 100k pairs x 5, W = 82) built once,
then the segment-grouped evaluation timed (uam_kernel_timing: HIP events around the whole
launch sequence, mean over --reps) for every combination of group length, sort-tile bits and
evaluation LDS floor given (gathers-in-flight and register-cap settings of
profiles/r03/k2g7-8 were measured with a build that had those knobs).  Runs with the same group length must give
identical bits (the other knobs only change which lane does the work); every run is checked
against the first run of its group length.  One JSON line per setting.
usage: python tools/probe_k2g.py --groups 8,16 --tbits 4,6 --lds 0,32768 --chunks 0,8"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ints(s):
    return [int(x) for x in s.split(",") if x != ""]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", default="8,12,16,21")
    ap.add_argument("--tbits", default="6")
    ap.add_argument("--lds", default="0")
    ap.add_argument("--chunks", default="0")
    ap.add_argument("--curves", default="1")
    ap.add_argument("--pairs", type=int, default=100000)
    ap.add_argument("--R", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (build_region_map, canonical_params,
                                                canonical_spec, displacements, raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    spec = canonical_spec(nfz_polygons=64)
    e = Engine(0)
    e.set_geometry(compile_map(build_region_map(spec)))
    e.set_params(canonical_params(spec, N=80, altitude=320.0))
    raster = e.raster_build(raster_geo(a.R), synthetic_dem(a.R))
    D = 5
    pairs = e.tensor(random_pairs(a.pairs, seed=0), torch.float64)
    ut = e.tensor(arc_table(80, displacements(D)), torch.float64)
    outs = e.outputs(a.pairs * D, 82, n_pairs=a.pairs)
    o = outs[0]
    first = {}
    for g in ints(a.groups):
        for tb in ints(a.tbits):
            for lds in ints(a.lds):
                for chk, cv in [(c, v) for c in ints(a.chunks) for v in ints(a.curves)]:
                    e.set_option("k2g_chunk", chk)
                    e.set_option("k2g_curve", cv)
                    e.set_option("group", g)
                    e.set_option("k2g_tile_bits", tb)
                    e.set_option("k2g_lds_floor", lds)
                    for _ in range(3):
                        e.eval_generated(pairs, ut, raster=raster, outputs=outs)
                    torch.cuda.synchronize()
                    e.kernel_timing(True)
                    for _ in range(a.reps):
                        e.eval_generated(pairs, ut, raster=raster, outputs=outs)
                    ms, n = e.kernel_time()
                    e.kernel_timing(False)
                    cost = o["cost"].clone()
                    row = {"group": g, "tbits": tb, "lds": lds, "chunk": chk, "curve": cv,
                           "kernel": e.last_kernel(), "ms": round(ms / n, 4),
                           "paths_per_s": round(a.pairs * D / (ms / n * 1e-3), 1)}
                    if g in first:
                        row["identical"] = bool(torch.equal(cost, first[g]))
                    else:
                        first[g] = cost
                        if 8 in first and g != 8:
                            rel = ((cost - first[8]).abs() / first[8].abs()).max().item()
                            row["max_rel_vs_g8"] = rel
                    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
