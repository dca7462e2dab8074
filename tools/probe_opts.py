#!/usr/bin/env python3
"""GPU probe: the cfg3 step (4096^2 DEM + 70 no-fly shapes, 100k pairs x 5, W = 82) timed with
HIP events around the library's launch sequence (uam_kernel_timing, mean over --reps) and by
wall clock over back-to-back calls, for one library build (UAM_LIB_PATH selects a measurement
build) and a list of option settings.  Prints one JSON line per setting with a checksum of the
costs (bits) so runs that must agree can be compared.
usage: UAM_LIB_PATH=build/variants/libuampath_x.so python tools/probe_opts.py --tag x \
           --settings "k2g_chunk=8;k2g_chunk=6" [--cells]"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="default")
    ap.add_argument("--settings", default="")
    ap.add_argument("--pairs", type=int, default=100000)
    ap.add_argument("--R", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cells", action="store_true")
    ap.add_argument("--share", default=None,
                    help="R/N: rank R's spatial shard (distributed.spatial_shard) of the --pairs "
                         "pairs over N ranks (cfg4: --R 8192 --pairs 200000 --share 3/8)")
    ap.add_argument("--volume", action="store_true",
                    help="cfg5: 1024^2 x 64 volume, packed copy, 100k pairs x 5 (K4h / K4)")
    ap.add_argument("--analytic", action="store_true",
                    help="cfg3 in analytic mode (K3b): the reference formulas, no raster")
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
    D = 5
    ut = e.tensor(arc_table(80, displacements(D)), torch.float64)
    if a.volume:
        from uam_path_planning_amd.scenario import layer_weights
        from uam_path_planning_amd.synthetic import random_pairs3d
        r2 = e.raster_build(raster_geo(1024), synthetic_dem(1024))
        vol = e.volume_build(r2, 64, 0.0, 10.0, layer_weights(64))
        e.volume_pack(vol)
        pairs = e.tensor(random_pairs3d(a.pairs, seed=0), torch.float64)

        def run():
            e.eval_generated3d(pairs, ut, vol, outputs=outs)
    elif a.analytic:
        pairs = e.tensor(random_pairs(a.pairs, seed=0), torch.float64)

        def run():
            e.eval_generated(pairs, ut, raster=None, outputs=outs)
    else:
        raster = e.raster_build(raster_geo(a.R), synthetic_dem(a.R))
        ph = random_pairs(a.pairs, seed=0)
        if a.share:
            from uam_path_planning_amd.distributed import spatial_shard
            r, n = (int(v) for v in a.share.split("/"))
            ph, _ = spatial_shard(ph, r, n)
            a.pairs = len(ph)
        pairs = e.tensor(ph, torch.float64)

        def run():
            e.eval_generated(pairs, ut, raster=raster, outputs=outs)
    outs = e.outputs(a.pairs * D, 82, n_pairs=a.pairs, want_cells=a.cells)
    o = outs[0]
    settings = [s for s in a.settings.split(";") if s.strip()] or [""]
    for st in settings:
        kv = [x.split("=") for x in st.split(",") if x.strip()]
        for k, v in kv:
            e.set_option(k.strip(), int(v))
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e.kernel_timing(True)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            run()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.reps * 1e3
        ms, n = e.kernel_time()
        e.kernel_timing(False)
        h = hashlib.sha1()
        for k in ("cost", "length", "kin_sum", "nfz_sum", "min_clearance", "best_fval_idx"):
            h.update(o[k].cpu().numpy().tobytes())
        row = {"tag": a.tag, "settings": st, "kernel": e.last_kernel(),
               "group": e.last_group(), "seq_ms": round(ms / n, 4),
               "wall_ms": round(wall, 4), "paths_per_s": round(a.pairs * D / (wall * 1e-3), 1),
               "sha1": h.hexdigest()[:16]}
        if a.cells:
            row["cells_sha1"] = hashlib.sha1(o["cells"].cpu().numpy().tobytes()).hexdigest()[:16]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
