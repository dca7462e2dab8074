"""Phase timing of the wave-per-path kernel (K2w) on configs[1] (1k paths x 256 waypoints,
2048^2 DEM): needs a library built with -DUAM_EW_PROF (s_memtime stamps at the phase
boundaries).  Prints the median shader-clock cycles per phase over the first 1000 paths.
usage: UAM_HIPCC_EXTRA=-DUAM_EW_PROF python tools/probe_ew_prof.py"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["points", "segments+kinematics", "gathers", "reductions", "chains", "cost chain"]


def main():
    import numpy as np
    import torch
    from uam_path_planning_amd import build
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (build_region_map, canonical_params,
                                                canonical_spec, displacements, raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    build.build_library(force=True)
    spec = canonical_spec()
    eng = Engine(0)
    if not hasattr(eng.lib, "uam_debug_ew_prof"):
        raise SystemExit("library built without -DUAM_EW_PROF")
    eng.set_geometry(compile_map(build_region_map(spec)))
    eng.set_params(canonical_params(spec, N=254))
    raster = eng.raster_build(raster_geo(2048), synthetic_dem(2048))
    pairs = torch.tensor(random_pairs(200, seed=0), device="cuda")
    ut = arc_table(254, displacements(5))
    eng.set_option("wave_max_paths", 1 << 40)
    for _ in range(5):
        eng.eval_generated(pairs, ut, raster=raster)
    torch.cuda.synchronize()
    buf = np.zeros(1024 * 8, np.uint64)
    eng.lib.uam_debug_ew_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert eng.lib.uam_debug_ew_prof(buf.ctypes.data, buf.size) == 0
    st = buf.reshape(1024, 8)[:1000].astype(np.int64)
    d = np.diff(st[:, :7], axis=1)
    row = {ph: int(np.median(d[:, i])) for i, ph in enumerate(PHASES)}
    row["total_cycles_median"] = int(np.median(st[:, 6] - st[:, 0]))
    row["span_cycles"] = int(st[:, 6].max() - st[:, 0].min())
    print(json.dumps(row))


if __name__ == "__main__":
    main()
