"""DataProcessor -- map_generation/data_processor.py:8-75 of the reference: polygons (plane
metres) -> union -> area filter -> min-area rectangles (large polygons split into a
divisions x divisions grid first) -> area filter.  The computation is the library's host code
(uam_process_polygons, csrc/polyproc.cpp); for DEM rasters the polygonisation runs on the GPU
(DataManager.load_dem_polygons_from_geotiff + process_dem, uam_dem_polygons).
Pinned: the reference's populated_area pipeline, 29/29 rectangles (tests/golden/polygons.npz).
select_polygons / _approximate_douglas_peucker (interactive UI / unused) are out of scope."""
import ctypes

import numpy as np

from .. import _lib


def _as_polygon(p):
    """ring [n, 2] | (shell, [holes]) | {"shell": .., "holes": [..]} -> (shell, holes)."""
    if isinstance(p, dict):
        return np.asarray(p["shell"], np.float64), [np.asarray(h, np.float64)
                                                     for h in p.get("holes", [])]
    if isinstance(p, tuple) and len(p) == 2 and np.ndim(p[0]) == 2:
        return np.asarray(p[0], np.float64), [np.asarray(h, np.float64) for h in p[1]]
    return np.asarray(p, np.float64).reshape(-1, 2), []


class DataProcessor:
    def __init__(self, min_area=750000, large_area=32000000, divisions=5,
                 min_approx_polygon_area=780000):
        self.min_area = min_area
        self.large_area = large_area
        self.divisions = divisions
        self.min_approx_polygon_area = min_approx_polygon_area

    def params(self):
        return _lib.PolyprocParams(float(self.min_area), float(self.large_area),
                                   float(self.min_approx_polygon_area), int(self.divisions), 0)

    def process_polygons(self, polygons):
        """-> list of int64 [4, 2] rectangles (cv2.boxPoints order, metres).  ``polygons``:
        vector polygons (plane metres), or the DemRegions that
        DataManager.load_dem_polygons_from_geotiff returns (GPU route, uam_dem_polygons)."""
        from .data_manager import DemRegions

        if isinstance(polygons, DemRegions):
            return polygons.engine.dem_polygons(polygons.dem, polygons.geo, polygons.threshold,
                                                polygons.unit_m, self.params())
        rings, holes = [], []
        for p in polygons:
            shell, hs = _as_polygon(p)
            rings.append(shell)
            holes.append(0)
            for h in hs:
                rings.append(h)
                holes.append(1)
        xy = np.ascontiguousarray(np.vstack(rings) if rings else np.zeros((0, 2)), np.float64)
        start = np.zeros(len(rings) + 1, np.int64)
        start[1:] = np.cumsum([len(r) for r in rings])
        hole = np.asarray(holes, np.int32)
        lib = _lib.load()
        n = ctypes.c_int32(0)
        cap = 64
        while True:
            out = np.zeros((cap, 4, 2), np.int64)
            st = lib.uam_process_polygons(xy.ctypes.data, start.ctypes.data, len(rings),
                                          hole.ctypes.data, ctypes.byref(self.params()),
                                          out.ctypes.data, cap, ctypes.byref(n))
            if st == 0:
                return [out[i] for i in range(n.value)]
            if n.value > cap:
                cap = n.value
                continue
            _lib.check(st, "uam_process_polygons")
