"""Canonical Nagasaki scenario (reference path_generation/main.py:21-61, 122-160) and the
BASELINE.json configs, as JSON-style map specs that both the product and the test oracle
can build from."""
import json
import os

import numpy as np

from .arcs import REFERENCE_DISPLACEMENTS
from .engine import PathParams, RasterGeo
from .synthetic import EXTENT, EXTENT_X0, EXTENT_Y_TOP, random_convex_polygons

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "canonical_map.json")


def canonical_spec(nfz_polygons=0, seed=2):
    """Map spec of main.py's scenario.  nfz_polygons > 0 adds the reference's
    no_fly_area.txt polygon plus that many random convex polygons (config 3)."""
    with open(DATA) as f:
        spec = json.load(f)
    if nfz_polygons:
        spec["obstacles"] = spec["obstacles"] + spec["no_fly_polygons"] + [
            {"kind": "polygon", "vertices": v}
            for v in random_convex_polygons(nfz_polygons, seed=seed)]
    return spec


def build_region_map(spec):
    """Product RegionMap (GPU-backed drop-in classes) from a spec."""
    from .path_generation import RegionMap, ball, polygon, square

    def mk(s):
        if s["kind"] == "polygon":
            return polygon(*s["vertices"])
        if s["kind"] == "ball":
            return ball(s["center"], s.get("r1"), s.get("r2"))
        if s["kind"] == "square":
            return square(s["center"], s["r1"], s.get("r2"))
        raise ValueError(s["kind"])

    m = RegionMap()
    m.add_obstacles(*[mk(s) for s in spec["obstacles"]])
    for reg in spec["regions"]:
        m.new_region(reg["name"], reg["color"])
        m.add_shapes_to_region(reg["name"], *[mk(s) for s in reg["shapes"]])
    m.x_start = list(spec["x_start"])
    m.x_goal = list(spec["x_goal"])
    return m


def canonical_params(spec, N=None, anchor=None, altitude=150.0):
    return PathParams(N=int(N or spec["N"]), **spec["options"], maxratio=spec["maxratio"],
                      maxalpha=spec["maxalpha"], enlargement=spec["enlargement"],
                      weights=tuple(spec["weights"]), quirk_length=True, anchor=anchor,
                      altitude=altitude)


def canonical_problem(N=None):
    from .path_generation import Problem

    spec = canonical_spec()
    m = build_region_map(spec)
    prob = Problem(m, int(N or spec["N"]), spec["options"])
    prob.params.update({"maxratio": spec["maxratio"], "maxalpha": spec["maxalpha"],
                        "enlargement": spec["enlargement"]})
    for name, w in zip(m.region_names(), spec["weights"]):
        prob.set_weight(name, w)
    return prob


def raster_geo(R, dem_threshold=0.0):
    """R x R raster over x in [0, 60] km, y in [-40, 20] km; 60/R is exact for R = 2^k."""
    return RasterGeo(nx=R, ny=R, x0=EXTENT_X0, y_top=EXTENT_Y_TOP, dx=EXTENT / R, dy=EXTENT / R,
                     nodata=-9999.0, dem_threshold=dem_threshold)


# BASELINE.json configs.  pairs x D displacements = paths, W = N + 2.
CONFIGS = {
    "cfg1": dict(name="single start->goal, 256^2 DEM (CPU plumbing / goldens)", R=256, pairs=1,
                 D=5, N=80, nfz_polygons=0, mode="raster"),
    "cfg2": dict(name="1k candidate paths x 256 waypoints, 2048^2 DEM, 1 GPU", R=2048,
                 pairs=200, D=5, N=254, nfz_polygons=0, mode="raster"),
    "cfg3": dict(name="100k start/goal pairs x 5 displacements, 4096^2 DEM + polygon NFZ, 1 GPU",
                 R=4096, pairs=100_000, D=5, N=80, nfz_polygons=64, mode="raster"),
    # strong scaling: 200k pairs x 5 = 1M paths IN TOTAL, sharded over the GPUs (shard_range)
    "cfg4": dict(name="8192^2 DEM from synthetic GeoTIFF tiles + polygon NFZ, RCCL raster "
                      "broadcast, 8 GPUs",
                 R=8192, pairs=200_000, D=5, N=80, nfz_polygons=64, mode="raster"),
    "cfg5": dict(name="3-D 1024x1024x64 (x,y,alt) altitude-dependent risk volume",
                 R=1024, nz=64, z0=0.0, dz=10.0, pairs=100_000, D=5, N=80, nfz_polygons=64,
                 mode="volume"),
}


def layer_weights(nz):
    """Altitude weight of the ground risk per layer (config 5, build-defined): 1 / (1 + k)."""
    return 1.0 / (1.0 + np.arange(nz, dtype=np.float64))


def displacements(D):
    if D == 5:
        return list(REFERENCE_DISPLACEMENTS)
    return np.linspace(-0.9, 0.9, D).tolist()
