"""Measurement tool (not product code): K2h's slot classes per cfg3 step from the counting
build (tools/build_variant.sh cnt "-DUAM_K2H_COUNT"): valid slots, in-raster, terrain fetches,
codes 1 / 2 / 3, items whose path bound is -inf.
  UAM_LIB_PATH=build/variants/libuampath_cnt.so python tools/k2h_counts.py [--opt NAME=VALUE]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from uam_path_planning_amd import _lib
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (CONFIGS, build_region_map, canonical_params,
                                                canonical_spec, displacements, raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    cfg = CONFIGS["cfg3"]
    spec = canonical_spec(nfz_polygons=cfg["nfz_polygons"])
    eng = Engine(0)
    eng.set_geometry(compile_map(build_region_map(spec)))
    eng.set_params(canonical_params(spec, N=80, altitude=320.0))
    for kv in sys.argv[1:]:
        if kv.startswith("--opt="):
            k, v = kv[6:].split("=")
            eng.set_option(k, int(v))
    R = 4096
    geo = raster_geo(R)
    raster = eng.raster_build(geo, eng.tensor(synthetic_dem(R), torch.float32), summary=False)
    eng.raster_summary(raster, 0, packed=True)
    pairs = eng.tensor(random_pairs(cfg["pairs"], seed=0), torch.float64)
    ut = eng.tensor(arc_table(80, displacements(5)), torch.float64)
    lib = eng.lib
    fn = lib.uam_debug_k2h_counts
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 8)()
    eng.eval_generated(pairs, ut, raster=raster)
    torch.cuda.synchronize()
    fn(buf, 1)
    eng.eval_generated(pairs, ut, raster=raster)
    torch.cuda.synchronize()
    fn(buf, 1)
    names = ["valid", "in_raster", "fetched", "code1", "code2", "code3", "items_Lb_-inf"]
    v = list(buf)[:7]
    print({n: x for n, x in zip(names, v)}, "fetch per valid slot %.4f" % (v[2] / max(v[0], 1)),
          "kernel", eng.last_kernel())


if __name__ == "__main__":
    main()
