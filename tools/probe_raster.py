#!/usr/bin/env python3
"""Diagnostic: kernel time of the fused raster path kernel vs raster size (same paths, same
geometry).  R=64 keeps the record table in L2 (compute/issue floor); 2048^2 = 64 MiB fits the
256 MiB Infinity Cache; 4096^2 = 256 MiB is at its size; 8192^2 = 1 GiB streams from HBM.
Also times the analytic kernel (K3) and the raster build (K1).  Prints JSON lines."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def timed(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100_000)
    ap.add_argument("--sizes", default="64,512,1024,2048,4096,8192")
    ap.add_argument("--analytic-pairs", type=int, default=20_000)
    ap.add_argument("--variants", default="", help="comma list: interleaved A/B at R=4096")
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (build_region_map, canonical_params,
                                                canonical_spec, displacements, raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    spec = canonical_spec(nfz_polygons=64)
    eng = Engine(0)
    eng.set_geometry(compile_map(build_region_map(spec)))
    eng.set_params(canonical_params(spec, N=80, altitude=320.0))
    ut = eng.tensor(arc_table(80, displacements(5)), torch.float64)
    pairs = eng.tensor(random_pairs(args.pairs, seed=0), torch.float64)
    P = args.pairs * 5
    outs = eng.outputs(P, 82, n_pairs=args.pairs)
    if args.variants:
        geo = raster_geo(4096)
        raster = eng.raster_build(geo, eng.tensor(synthetic_dem(4096), torch.float32))
        vs = [int(x) for x in args.variants.split(",")]
        res = {v: [] for v in vs}
        ref = None
        for _ in range(args.rounds):
            for v in vs:
                eng.set_tuning(v)
                med, best = timed(lambda: eng.eval_generated(pairs, ut, raster=raster,
                                                             outputs=outs), reps=10)
                res[v].append(med)
                cur = (outs[0]["cost"].clone(), outs[0]["best_fval_idx"].clone())
                if ref is None:
                    ref = cur
                assert torch.equal(cur[0], ref[0]) and torch.equal(cur[1], ref[1]), v
        for v in vs:
            ts = sorted(res[v])
            print(json.dumps({"probe": "variant", "variant": v, "R": 4096, "paths": P,
                              "kernel_ms_median": round(ts[len(ts) // 2], 4),
                              "kernel_ms_min": round(ts[0], 4),
                              "paths_per_s": round(P / (ts[len(ts) // 2] * 1e-3), 1)}),
                  flush=True)
        eng.set_tuning(0)
        del raster
        torch.cuda.empty_cache()
    for R in [int(x) for x in args.sizes.split(",") if x]:
        geo = raster_geo(R)
        dem = eng.tensor(synthetic_dem(R), torch.float32)
        t_build, _ = timed(lambda: eng.raster_build(geo, dem), reps=3, warm=1)
        raster = eng.raster_build(geo, dem)
        med, best = timed(lambda: eng.eval_generated(pairs, ut, raster=raster, outputs=outs))
        print(json.dumps({"probe": "raster_eval", "R": R, "table_MiB": R * R * 16 / 2**20,
                          "paths": P, "kernel_ms_med": round(med, 4),
                          "kernel_ms_best": round(best, 4),
                          "paths_per_s": round(P / (med * 1e-3), 1),
                          "gathers_per_s": round(P * 82 / (med * 1e-3), 1),
                          "raster_build_ms": round(t_build, 3),
                          "cells_per_s_build": round(R * R / (t_build * 1e-3), 1)}), flush=True)
        del raster, dem
        torch.cuda.empty_cache()
    Qa = args.analytic_pairs
    if not Qa:
        return
    pa = pairs[:Qa]
    oa = eng.outputs(Qa * 5, 82)
    med, best = timed(lambda: eng.eval_generated(pa, ut, raster=None, outputs=oa), reps=5)
    print(json.dumps({"probe": "analytic_eval", "paths": Qa * 5, "kernel_ms_med": round(med, 4),
                      "paths_per_s": round(Qa * 5 / (med * 1e-3), 1),
                      "shapes": int(eng.geometry.shape_first.shape[0]),
                      "inequalities": int(eng.geometry.ineq_kind.shape[0])}), flush=True)


if __name__ == "__main__":
    main()
