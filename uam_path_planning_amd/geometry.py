"""Geometry compiler: RegionMap / shapes -> the flat device tables of include/uampath.h.

Layout (what the kernels walk, in the reference's summation order):
  * shapes [0, n_obstacles): ``map.obstacles`` in ``add`` order (map.py:13-17) -- the no-fly
    zones behind get_nonlincon's obstacle rows (problem.py:109-112) and Map.collides;
  * then every region's shapes, regions in insertion order (region_map.py:59-61), shapes in
    ``add_shape_to_region`` order -- the Φ sum of get_total_penalty_function (problem.py:49-56).
  * one inequality record (kind, p[6]) per h_i, in the shape's inequality order (the order of
    the product in quadratic_obstacle.py:33-38).
"""
import ctypes

import numpy as np

from . import _lib


class FlatGeometry:
    def __init__(self, obstacles, regions):
        kinds, pars, first, count, centers = [], [], [], [], []

        def add(obs):
            first.append(len(kinds))
            count.append(len(obs.inequalities))
            if len(obs.inequalities) == 0:
                raise ValueError("shape has no inequalities")
            c = np.asarray(obs.center, dtype=np.float64).reshape(-1)
            centers.append((float(c[0]), float(c[1])) if c.size >= 2 else (np.nan, np.nan))
            for h in obs.inequalities:
                spec = getattr(h, "spec", None)
                if spec is None:
                    raise ValueError("only polygon/ball/square inequalities run on the device "
                                     "(this Function has no device spec)")
                kinds.append(int(spec[0]))
                pars.append([float(v) for v in spec[1]])

        for o in obstacles:
            add(o)
        region_first = [len(first)]
        for shapes in regions:
            for o in shapes:
                add(o)
            region_first.append(len(first))
        if len(regions) > _lib.MAX_REGIONS:
            raise ValueError(f"at most {_lib.MAX_REGIONS} regions are supported")
        self.n_obstacles = len(obstacles)
        self.n_regions = len(regions)
        self.ineq_kind = np.ascontiguousarray(kinds, dtype=np.int32).reshape(-1)
        self.ineq_par = np.ascontiguousarray(pars, dtype=np.float64).reshape(-1, 6)
        self.shape_first = np.ascontiguousarray(first, dtype=np.int32)
        self.shape_count = np.ascontiguousarray(count, dtype=np.int32)
        self.shape_center = np.ascontiguousarray(centers, dtype=np.float64).reshape(-1, 2)
        self.region_first = np.ascontiguousarray(region_first, dtype=np.int32)

    def as_struct(self):
        i32 = ctypes.POINTER(ctypes.c_int32)
        f64 = ctypes.POINTER(ctypes.c_double)
        return _lib.Geometry(_lib.ABI_VERSION, len(self.ineq_kind),
                             self.ineq_kind.ctypes.data_as(i32),
                             self.ineq_par.ctypes.data_as(f64), len(self.shape_first),
                             self.shape_first.ctypes.data_as(i32),
                             self.shape_count.ctypes.data_as(i32),
                             self.shape_center.ctypes.data_as(f64), self.n_obstacles,
                             self.n_regions, self.region_first.ctypes.data_as(i32))

    def signature(self):
        return (self.ineq_kind.tobytes(), self.ineq_par.tobytes(), self.shape_first.tobytes(),
                self.shape_count.tobytes(), self.shape_center.tobytes(),
                self.region_first.tobytes(), self.n_obstacles)


def compile_map(m):
    regions = getattr(m, "regions", {})
    return FlatGeometry(list(m.obstacles), [list(r["shapes"]) for r in regions.values()])


def compile_shapes(obstacles=(), regions=()):
    return FlatGeometry(list(obstacles), [list(r) for r in regions])
