"""Lane-per-path (tuning 2) vs wave-per-path (tuning 9) raster evaluation across batch sizes,
to place the automatic crossover (UAM_OPT_WAVE_MAX_PATHS, default 16384).
usage: python tools/probe_wave.py [--R 4096] [--N 80]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=4096)
    ap.add_argument("--N", type=int, default=80)
    ap.add_argument("--pairs", default="20,200,1000,4000,13107,40000,100000")
    a = ap.parse_args()
    import torch
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (build_region_map, canonical_params,
                                                canonical_spec, displacements, raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    spec = canonical_spec(nfz_polygons=64)
    eng = Engine(0)
    eng.set_geometry(compile_map(build_region_map(spec)))
    eng.set_params(canonical_params(spec, N=a.N))
    raster = eng.raster_build(raster_geo(a.R), synthetic_dem(a.R))
    ut = arc_table(a.N, displacements(5))
    for Q in [int(x) for x in a.pairs.split(",")]:
        pairs = torch.tensor(random_pairs(Q, seed=0), device="cuda")
        out = eng.outputs(Q * 5, a.N + 2, n_pairs=Q)
        outd = out[0]
        row = {"pairs": Q, "paths": Q * 5, "N": a.N, "R": a.R}
        res = {}
        for v, wmax in ((2, 0), (9, 1 << 40)):   # 2 = lane per path, 9 = wave per path
            eng.set_option("wave_max_paths", wmax)
            for _ in range(3):
                eng.eval_generated(pairs, ut, raster=raster, outputs=out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record()
            for _ in range(reps):
                eng.eval_generated(pairs, ut, raster=raster, outputs=out)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            row[f"ms_v{v}"] = ms
            row[f"paths_per_s_v{v}"] = Q * 5 / (ms / 1e3)
            res[v] = {k: t.clone() for k, t in outd.items()}
        row["identical"] = all(torch.equal(res[2][k], res[9][k]) for k in res[2])
        eng.set_option("wave_max_paths", 16384)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
