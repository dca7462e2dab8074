#!/usr/bin/env python3
"""GPU probe: wall time per cfg3 step (back-to-back uam_eval_generated_p calls, one sync at the
end) with and without the measurement events bench.py records (uam_kernel_timing pairs,
torch.cuda.Event pairs), against the K2g sequence's own HIP-event time.
usage: python tools/probe_step_overhead.py [--steps 50]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
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
    raster = e.raster_build(raster_geo(4096), synthetic_dem(4096))
    pairs = e.tensor(random_pairs(100000, seed=0), torch.float64)
    ut = e.tensor(arc_table(80, displacements(5)), torch.float64)
    outs = e.outputs(500000, 82, n_pairs=100000)
    for _ in range(5):
        e.eval_generated(pairs, ut, raster=raster, outputs=outs)
    torch.cuda.synchronize()

    def run(ktime, tev):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(a.steps)] if tev else None
        e.kernel_timing(ktime)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            if tev:
                evs[i][0].record()
            e.eval_generated(pairs, ut, raster=raster, outputs=outs)
            if tev:
                evs[i][1].record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.steps * 1e3
        row = {"ktime": ktime, "torch_events": tev, "wall_ms_per_step": round(wall, 4)}
        if ktime:
            ms, n = e.kernel_time()
            row["sequence_ms"] = round(ms / n, 4)
        e.kernel_timing(False)
        print(json.dumps(row), flush=True)

    for ktime, tev in ((False, False), (True, False), (False, True), (True, True), (False, False)):
        run(ktime, tev)
    # host cost of one call, GPU kept busy by a long queue
    t0 = time.perf_counter()
    for _ in range(a.steps):
        e.eval_generated(pairs, ut, raster=raster, outputs=outs)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(json.dumps({"host_ms_per_call_enqueue": round((t1 - t0) / a.steps * 1e3, 4)}))


if __name__ == "__main__":
    main()
