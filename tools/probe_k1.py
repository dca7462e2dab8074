#!/usr/bin/env python3
"""Diagnostic: K1 raster build (k_raster_build) time on the cfg3 map at R^2, against the same
build with fewer shapes, to split its time into the memory floor (no shapes) and the shape
tables.  Prints JSON lines.  Run on the GPU box (optionally under rocprofv3 --pmc)."""
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
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=4096)
    ap.add_argument("--cases", default="cfg3,cfg3-obstacles,canonical,regions,obstacles,empty")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpl", type=int, default=0, help="k1_rows option (0: the default)")
    args = ap.parse_args()
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (build_region_map, canonical_params,
                                                canonical_spec, raster_geo)
    from uam_path_planning_amd.synthetic import synthetic_dem

    geo = raster_geo(args.R)
    eng = Engine(0)
    if args.cpl:
        eng.set_option("k1_rows", args.cpl)
    dem = eng.tensor(synthetic_dem(args.R), torch.float32)
    out = eng.empty((geo.ny, geo.nx, 4), torch.int32)
    # the store floor: torch's fill of the same 16 B-per-cell records
    ms = timed(lambda: out.fill_(0), reps=args.reps)
    print(json.dumps({"probe": "k1", "case": "fill_records", "R": args.R, "ms": round(ms, 4),
                      "GBps": round(out.numel() * 4 / (ms * 1e-3) / 1e9, 1)}), flush=True)
    for case in args.cases.split(","):
        spec = canonical_spec(nfz_polygons=64 if case.startswith("cfg3") else 0)
        if case == "regions":       # region shapes only (Φ table)
            spec["obstacles"] = spec["obstacles"][:0]
        elif case.endswith("obstacles"):   # no-fly shapes only (ψ and hit tables)
            spec["regions"], spec["weights"] = [], []
        elif case == "empty":
            spec["obstacles"] = spec["obstacles"][:0]
            spec["regions"], spec["weights"] = [], []
        try:
            eng.set_geometry(compile_map(build_region_map(spec)))
        except Exception as e:  # noqa: BLE001 -- a spec the map builder refuses
            print(json.dumps({"probe": "k1", "case": case, "error": repr(e)}), flush=True)
            continue
        eng.set_params(canonical_params(spec, N=80, altitude=320.0))
        # K1 alone (no gather-skip summary, no packed copy)
        ms = timed(lambda: eng.raster_build(geo, dem, out=out, summary=False), reps=args.reps)
        cells = geo.nx * geo.ny
        print(json.dumps({"probe": "k1", "case": case, "R": args.R, "cpl": args.cpl,
                          "ms": round(ms, 4),
                          "cells_per_s": round(cells / (ms * 1e-3), 1),
                          "GBps_algorithmic": round(cells * 20 / (ms * 1e-3) / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
