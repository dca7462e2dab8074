"""ctypes front-end of the CPU oracle (oracle/uam_oracle.c).  TEST INFRASTRUCTURE, NOT PRODUCT.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, as the
checker / the timed CPU baseline.  The product path never does.  See uam_oracle.c's header for
the reference file:line each routine restates, and tests/test_oracle_golden.py for the golden
vectors (recorded from the reference itself) that pin it.
"""
import ctypes
import os
import subprocess

import numpy as np

from .geometry import MAX_REGIONS, FlatGeometry, compile_spec  # noqa: F401

HERE = os.path.dirname(os.path.abspath(__file__))
# UAM_ORACLE_LIB: another build of the same source (tools/sanitize_host.sh: ASan + UBSan)
LIB_PATH = os.environ.get("UAM_ORACLE_LIB") or os.path.join(HERE, "build", "liboracle.so")

_i32p = ctypes.POINTER(ctypes.c_int32)
_f64p = ctypes.POINTER(ctypes.c_double)
_f32p = ctypes.POINTER(ctypes.c_float)


class _Geom(ctypes.Structure):
    _fields_ = [("n_ineq", ctypes.c_int32), ("ineq_kind", _i32p), ("ineq_par", _f64p),
                ("n_shapes", ctypes.c_int32), ("shape_first", _i32p), ("shape_count", _i32p),
                ("shape_center", _f64p), ("n_obstacles", ctypes.c_int32),
                ("n_regions", ctypes.c_int32), ("region_first", _i32p)]


class _Params(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int32), ("length_smooth", ctypes.c_int32),
                ("penalty_smooth", ctypes.c_int32), ("obstacle_smooth", ctypes.c_int32),
                ("maxratio_smooth", ctypes.c_int32), ("quirk_length", ctypes.c_int32),
                ("anchor_mode", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("anchor_x", ctypes.c_double), ("anchor_y", ctypes.c_double),
                ("maxratio", ctypes.c_double), ("maxalpha", ctypes.c_double),
                ("enlargement", ctypes.c_double), ("altitude", ctypes.c_double),
                ("weights", ctypes.c_double * MAX_REGIONS)]


class _Raster(ctypes.Structure):
    _fields_ = [("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("x0", ctypes.c_double),
                ("y_top", ctypes.c_double), ("dx", ctypes.c_double), ("dy", ctypes.c_double),
                ("nodata", ctypes.c_float), ("dem_threshold", ctypes.c_float)]


class _Volume(ctypes.Structure):
    _fields_ = [("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("nz", ctypes.c_int32),
                ("x0", ctypes.c_double), ("y_top", ctypes.c_double), ("dx", ctypes.c_double),
                ("dy", ctypes.c_double), ("z0", ctypes.c_double), ("dz", ctypes.c_double)]


class _RefineParams(ctypes.Structure):
    _fields_ = [("n_outer", ctypes.c_int32), ("n_inner", ctypes.c_int32),
                ("max_backtrack", ctypes.c_int32), ("memory", ctypes.c_int32),
                ("c0", ctypes.c_double), ("rho", ctypes.c_double), ("c_max", ctypes.c_double),
                ("alpha0", ctypes.c_double), ("armijo", ctypes.c_double),
                ("theta", ctypes.c_double), ("max_step", ctypes.c_double),
                ("inner_tol", ctypes.c_double), ("delta", ctypes.c_double),
                ("n_restart", ctypes.c_int32), ("restart_margin", ctypes.c_double)]


def refine_params(n_outer=15, n_inner=50, max_backtrack=30, c0=10.0, rho=5.0, c_max=1e8,
                  alpha0=1e-4, armijo=1e-4, theta=0.25, max_step=0.5, memory=8, inner_tol=1e-3,
                  delta=1e-4, n_restart=0, restart_margin=0.05):
    return _RefineParams(n_outer, n_inner, max_backtrack, memory, c0, rho, c_max, alpha0,
                         armijo, theta, max_step, inner_tol, delta, n_restart, restart_margin)


class _TM(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in ("a", "f", "k0", "lat0_deg", "lon0_deg", "fe",
                                                "fn")]


class _GeoGrid(ctypes.Structure):
    _fields_ = [("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("lon0", ctypes.c_double),
                ("lat_top", ctypes.c_double), ("dlon", ctypes.c_double),
                ("dlat", ctypes.c_double), ("nodata", ctypes.c_float), ("pad", ctypes.c_int32)]


# Japan Plane Rectangular CS origins (lat0, lon0) in degrees, zones I..XIX (EPSG:2443..2461)
JPRCS_ORIGINS = [(33.0, 129.5), (33.0, 131.0), (36.0, 132.0 + 10 / 60), (33.0, 133.5),
                 (36.0, 134.0 + 20 / 60), (36.0, 136.0), (36.0, 137.0 + 10 / 60),
                 (36.0, 138.5), (36.0, 139.0 + 50 / 60), (40.0, 140.0 + 50 / 60),
                 (44.0, 140.25), (44.0, 142.25), (44.0, 144.25), (26.0, 142.0), (26.0, 127.5),
                 (26.0, 124.0), (26.0, 131.0), (20.0, 136.0), (26.0, 154.0)]


def tm_zone(zone=1):
    """GRS80, k0 = 0.9999, no false origin: JGD2000 / Japan Plane Rectangular CS zone."""
    lat0, lon0 = JPRCS_ORIGINS[zone - 1]
    return _TM(6378137.0, 1 / 298.257222101, 0.9999, lat0, lon0, 0.0, 0.0)


def tm_fwd(lonlat, tm=None):
    tm = tm or tm_zone(1)
    ll = np.ascontiguousarray(lonlat, dtype=np.float64).reshape(-1, 2)
    out = np.zeros_like(ll)
    lib().orc_tm_fwd(ctypes.byref(tm), _ptr(ll, _f64p), ctypes.c_int64(ll.shape[0]),
                     _ptr(out, _f64p))
    return out


def tm_inv(xy, tm=None):
    tm = tm or tm_zone(1)
    p = np.ascontiguousarray(xy, dtype=np.float64).reshape(-1, 2)
    out = np.zeros_like(p)
    lib().orc_tm_inv(ctypes.byref(tm), _ptr(p, _f64p), ctypes.c_int64(p.shape[0]),
                     _ptr(out, _f64p))
    return out


def geo_grid(nx, ny, lon0, lat_top, dlon, dlat, nodata=-9999.0):
    return _GeoGrid(int(nx), int(ny), float(lon0), float(lat_top), float(dlon), float(dlat),
                    float(nodata), 0)


def reproject(src, ggrid, rdesc, unit=1000.0, resample=0, tm=None):
    tm = tm or tm_zone(1)
    s = np.ascontiguousarray(src, dtype=np.float32)
    out = np.zeros((rdesc.ny, rdesc.nx), dtype=np.float32)
    lib().orc_reproject(ctypes.byref(tm), _ptr(s, _f32p), ctypes.byref(ggrid),
                        ctypes.byref(rdesc), ctypes.c_double(unit), ctypes.c_int(resample),
                        _ptr(out, _f32p))
    return out


class _Polyproc(ctypes.Structure):
    _fields_ = [("min_area", ctypes.c_double), ("large_area", ctypes.c_double),
                ("min_approx_area", ctypes.c_double), ("divisions", ctypes.c_int32),
                ("pad", ctypes.c_int32)]


def polyproc(min_area=750000, large_area=32000000, divisions=5, min_approx_polygon_area=780000):
    return _Polyproc(float(min_area), float(large_area), float(min_approx_polygon_area),
                     int(divisions), 0)


def min_area_rect(points):
    """cv2.boxPoints(cv2.minAreaRect(float32 points)) -> np.intp  (restatement)."""
    p = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 2)
    box = np.zeros(8, np.int64)
    lib().orc_min_area_rect(_ptr(p, _f64p), ctypes.c_int64(len(p)),
                            box.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    return box.reshape(4, 2)


def dem_polygons(dem, rdesc, threshold=0.0, unit=1000.0, pp=None):
    """load_dem_polygons_from_geotiff + process_polygons -> [n, 4, 2] int64 rectangles."""
    d = np.ascontiguousarray(dem, dtype=np.float32)
    pp = pp or polyproc()
    cap = 4096
    out = np.zeros((cap, 4, 2), np.int64)
    n = lib().orc_dem_polygons(_ptr(d, _f32p), ctypes.byref(rdesc), ctypes.c_float(threshold),
                               ctypes.c_double(unit), ctypes.byref(pp),
                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                               ctypes.c_int64(cap))
    assert n <= cap
    return out[:n]


def build():
    """Compile liboracle.so (gcc) if it is missing or older than its source."""
    src = os.path.join(HERE, "uam_oracle.c")
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        for name in ("orc_eval_points", "orc_gen_paths", "orc_raster_build", "orc_eval_paths",
                     "orc_eval_paths_g", "orc_argmin", "orc_volume_build", "orc_gen_paths3d", "orc_eval_paths3d",
                     "orc_refine"):
            getattr(_lib, name).restype = ctypes.c_int
        _lib.orc_dem_polygons.restype = ctypes.c_int64
    return _lib


def _ptr(a, t):
    return None if a is None else a.ctypes.data_as(t)


class Oracle:
    """Bundle of flat geometry + params in the oracle's own C structs."""

    def __init__(self, geom, N, options=None, maxratio=1.0, maxalpha=0.0, enlargement=0.0,
                 weights=(), quirk_length=True, anchor=None, altitude=0.0):
        opts = {"length_smooth": False, "penalty_smooth": True, "obstacle_smooth": False,
                "maxratio_smooth": False}
        if options:
            opts.update(options)
        self.geom = geom
        self.N = int(N)
        self._keep = [geom.ineq_kind, geom.ineq_par, geom.shape_first, geom.shape_count,
                      geom.shape_center, geom.region_first]
        self.g = _Geom(len(geom.ineq_kind), _ptr(geom.ineq_kind, _i32p),
                       _ptr(geom.ineq_par, _f64p), len(geom.shape_first),
                       _ptr(geom.shape_first, _i32p), _ptr(geom.shape_count, _i32p),
                       _ptr(geom.shape_center, _f64p), geom.n_obstacles, geom.n_regions,
                       _ptr(geom.region_first, _i32p))
        w = (ctypes.c_double * MAX_REGIONS)(*([float(x) for x in weights] +
                                              [1.0] * (MAX_REGIONS - len(weights))))
        self.p = _Params(self.N, int(bool(opts["length_smooth"])),
                         int(bool(opts["penalty_smooth"])), int(bool(opts["obstacle_smooth"])),
                         int(bool(opts["maxratio_smooth"])), int(bool(quirk_length)),
                         0 if anchor is None else 1, 0,
                         0.0 if anchor is None else float(anchor[0]),
                         0.0 if anchor is None else float(anchor[1]),
                         float(maxratio), float(maxalpha), float(enlargement), float(altitude), w)

    # -- refinement (§8(f) rank 1) ---------------------------------------------------------
    def refine(self, wp, rp):
        W = self.N + 2
        wp = np.array(wp, dtype=np.float64, copy=True).reshape(-1, W, 2)
        P = wp.shape[0]
        out = {"cost": np.zeros(P), "infeas": np.zeros(P), "iters": np.zeros(P, np.int32)}
        st = lib().orc_refine(ctypes.byref(self.g), ctypes.byref(self.p), ctypes.byref(rp),
                              _ptr(wp, _f64p), ctypes.c_int64(P), _ptr(out["cost"], _f64p),
                              _ptr(out["infeas"], _f64p), _ptr(out["iters"], _i32p))
        if st != 0:
            raise ValueError("refinement needs penalty_smooth and obstacle_smooth")
        out["wp"] = wp
        return out

    # -- volume (config 5) -----------------------------------------------------------------
    def eval_paths3d(self, wp3, vdesc, vol, want_cells=False):
        """vol = (voxels [ny, nx, nz, 2], columns [ny, nx, 2]) as volume_build returns them."""
        W = self.N + 2
        wp3 = np.ascontiguousarray(wp3, dtype=np.float64).reshape(-1, W, 3)
        P = wp3.shape[0]
        vox = np.ascontiguousarray(vol[0], dtype=np.float32)
        cols = np.ascontiguousarray(vol[1], dtype=np.float32)
        out = {k: np.zeros(P) for k in ("cost", "lq", "length", "kin", "nfz", "min_clearance")}
        for k in ("nfz_hits", "offmap", "below"):
            out[k] = np.zeros(P, np.int32)
        cells = np.zeros((P, W), np.int32) if want_cells else None
        lib().orc_eval_paths3d(ctypes.byref(self.g), ctypes.byref(self.p), ctypes.byref(vdesc),
                               _ptr(vox, _f32p), _ptr(cols, _f32p), _ptr(wp3, _f64p),
                               ctypes.c_int64(P),
                               _ptr(out["cost"], _f64p), _ptr(out["lq"], _f64p),
                               _ptr(out["length"], _f64p), _ptr(out["kin"], _f64p),
                               _ptr(out["nfz"], _f64p), _ptr(out["nfz_hits"], _i32p),
                               _ptr(out["min_clearance"], _f64p), _ptr(out["offmap"], _i32p),
                               _ptr(out["below"], _i32p), _ptr(cells, _i32p))
        if want_cells:
            out["cells"] = cells
        return out

    # -- generated candidates, similarity form (K2h / K4h) ---------------------------------
    def eval_generated_h(self, pairs, utab, mode="raster", rdesc=None, rec=None, vdesc=None,
                         vol=None, group=0, want_cells=False):
        """Candidates of pairs ([Q, 4], or [Q, 6] with altitudes in volume mode) x the rows of
        utab [D, N, 2], path q*D + d: the geometry terms in the similarity form (the unit
        polyline's sums scaled by h = |x0 - xf| / 2), the raster / volume terms per generated
        waypoint with their sums grouped by `group` (0: sequential) -- uam_oracle.c
        orc_eval_generated_h, the definition K2h / K4h reproduce."""
        W = self.N + 2
        ut = np.ascontiguousarray(utab, dtype=np.float64)
        D = ut.shape[0]
        m = 1 if mode == "raster" else 2
        pr = np.ascontiguousarray(pairs, dtype=np.float64).reshape(-1, 4 if m == 1 else 6)
        Q = pr.shape[0]
        P = Q * D
        out = {k: np.zeros(P) for k in ("cost", "lq", "length", "kin", "nfz", "min_clearance")}
        for k in ("nfz_hits", "offmap", "below"):
            out[k] = np.zeros(P, np.int32)
        cells = np.zeros((P, W), np.int32) if want_cells else None
        vox = cols = None
        if m == 1:
            rec = np.ascontiguousarray(rec, dtype=np.float32)
        else:
            vox = np.ascontiguousarray(vol[0], dtype=np.float32)
            cols = np.ascontiguousarray(vol[1], dtype=np.float32)
        st = lib().orc_eval_generated_h(
            ctypes.byref(self.g), ctypes.byref(self.p), ctypes.c_int32(m),
            None if rdesc is None else ctypes.byref(rdesc), _ptr(rec if m == 1 else None, _f32p),
            None if vdesc is None else ctypes.byref(vdesc), _ptr(vox, _f32p),
            _ptr(cols, _f32p), _ptr(pr, _f64p), ctypes.c_int64(Q), _ptr(ut, _f64p),
            ctypes.c_int32(D), ctypes.c_int32(int(group)), _ptr(out["cost"], _f64p),
            _ptr(out["lq"], _f64p), _ptr(out["length"], _f64p), _ptr(out["kin"], _f64p),
            _ptr(out["nfz"], _f64p), _ptr(out["nfz_hits"], _i32p),
            _ptr(out["min_clearance"], _f64p), _ptr(out["offmap"], _i32p),
            _ptr(out["below"], _i32p), _ptr(cells, _i32p))
        if st != 0:
            raise ValueError("the similarity form needs maxratio_smooth = False")
        if want_cells:
            out["cells"] = cells
        return out

    # -- points ----------------------------------------------------------------------------
    def eval_points(self, pts):
        pts = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 2)
        n = pts.shape[0]
        R = self.geom.n_regions
        out = {"phi": np.zeros(n), "phi_regions": np.zeros((n, R)), "obs_norm": np.zeros(n),
               "psi_raw": np.zeros(n), "collide": np.zeros(n, np.int32)}
        lib().orc_eval_points(ctypes.byref(self.g), ctypes.byref(self.p), _ptr(pts, _f64p),
                              ctypes.c_int64(n), _ptr(out["phi"], _f64p),
                              _ptr(out["phi_regions"], _f64p), _ptr(out["obs_norm"], _f64p),
                              _ptr(out["psi_raw"], _f64p), _ptr(out["collide"], _i32p))
        return out

    # -- raster ----------------------------------------------------------------------------
    @staticmethod
    def raster_desc(nx, ny, x0, y_top, dx, dy, nodata=-9999.0, dem_threshold=0.0):
        return _Raster(int(nx), int(ny), float(x0), float(y_top), float(dx), float(dy),
                       float(nodata), float(dem_threshold))

    def raster_build(self, rdesc, dem=None):
        rec = np.zeros((rdesc.ny, rdesc.nx, 4), dtype=np.float32)
        dem_a = None if dem is None else np.ascontiguousarray(dem, dtype=np.float32)
        lib().orc_raster_build(ctypes.byref(self.g), ctypes.byref(self.p), ctypes.byref(rdesc),
                               _ptr(dem_a, _f32p), _ptr(rec, _f32p))
        return rec

    # -- paths -----------------------------------------------------------------------------
    def eval_paths(self, wp, mode="analytic", rdesc=None, rec=None, want_cells=False,
                   want_g=False, group=0):
        """group > 0 (raster mode): the segment-grouped summation order of K2g (partial sums
        over waypoint groups of `group`, added in group order; uam_oracle.c orc_eval_paths_g);
        0 = the reference's sequential order."""
        W = self.N + 2
        wp = np.ascontiguousarray(wp, dtype=np.float64).reshape(-1, W, 2)
        P = wp.shape[0]
        out = {k: np.zeros(P) for k in ("cost", "lq", "length", "kin", "nfz", "min_clearance")}
        out["nfz_hits"] = np.zeros(P, np.int32)
        out["offmap"] = np.zeros(P, np.int32)
        cells = np.zeros((P, W), np.int32) if want_cells else None
        n_rows = 3 * self.N + self.geom.n_obstacles * W
        g = np.zeros((P, n_rows)) if want_g else None
        m = 0 if mode == "analytic" else 1
        if m == 1:
            rec = np.ascontiguousarray(rec, dtype=np.float32)
        lib().orc_eval_paths_g(ctypes.byref(self.g), ctypes.byref(self.p), ctypes.c_int32(m),
                               None if rdesc is None else ctypes.byref(rdesc),
                               _ptr(rec if m == 1 else None, _f32p), _ptr(wp, _f64p),
                               ctypes.c_int64(P), _ptr(out["cost"], _f64p),
                               _ptr(out["lq"], _f64p), _ptr(out["length"], _f64p),
                               _ptr(out["kin"], _f64p), _ptr(out["nfz"], _f64p),
                               _ptr(out["nfz_hits"], _i32p), _ptr(out["min_clearance"], _f64p),
                               _ptr(out["offmap"], _i32p), _ptr(cells, _i32p), _ptr(g, _f64p),
                               ctypes.c_int32(int(group)))
        if want_cells:
            out["cells"] = cells
        if want_g:
            out["g"] = g
        return out


def volume_desc(nx, ny, nz, x0, y_top, dx, dy, z0, dz):
    return _Volume(int(nx), int(ny), int(nz), float(x0), float(y_top), float(dx), float(dy),
                   float(z0), float(dz))


def volume_build(vdesc, rec2, layer_w):
    """(voxels [ny, nx, nz, 2] {risk, psi_nfz}, columns [ny, nx, 2] {terrain, flags bits})"""
    rec2 = np.ascontiguousarray(rec2, dtype=np.float32)
    lw = np.ascontiguousarray(layer_w, dtype=np.float64)
    vox = np.zeros((vdesc.ny, vdesc.nx, vdesc.nz, 2), dtype=np.float32)
    cols = np.zeros((vdesc.ny, vdesc.nx, 2), dtype=np.float32)
    lib().orc_volume_build(ctypes.byref(vdesc), _ptr(rec2, _f32p), _ptr(lw, _f64p),
                           _ptr(vox, _f32p), _ptr(cols, _f32p))
    return vox, cols


def gen_paths3d(pairs6, utab):
    pairs6 = np.ascontiguousarray(pairs6, dtype=np.float64).reshape(-1, 6)
    utab = np.ascontiguousarray(utab, dtype=np.float64)
    D, N = utab.shape[0], utab.shape[1]
    out = np.zeros((pairs6.shape[0] * D, N + 2, 3))
    lib().orc_gen_paths3d(_ptr(pairs6, _f64p), ctypes.c_int64(pairs6.shape[0]),
                          _ptr(utab, _f64p), ctypes.c_int32(D), ctypes.c_int32(N),
                          _ptr(out, _f64p))
    return out


def gen_paths(pairs, utab):
    pairs = np.ascontiguousarray(pairs, dtype=np.float64).reshape(-1, 4)
    utab = np.ascontiguousarray(utab, dtype=np.float64)
    D, N = utab.shape[0], utab.shape[1]
    out = np.zeros((pairs.shape[0] * D, N + 2, 2))
    lib().orc_gen_paths(_ptr(pairs, _f64p), ctypes.c_int64(pairs.shape[0]), _ptr(utab, _f64p),
                        ctypes.c_int32(D), ctypes.c_int32(N), _ptr(out, _f64p))
    return out


def argmin(values, G, take_sqrt):
    v = np.ascontiguousarray(values, dtype=np.float64).reshape(-1)
    groups = v.shape[0] // G
    best = np.zeros(groups, np.int32)
    lib().orc_argmin(_ptr(v, _f64p), ctypes.c_int64(groups), ctypes.c_int32(G),
                     ctypes.c_int32(1 if take_sqrt else 0), _ptr(best, _i32p))
    return best


def arc_table(N, displacements):
    """Oracle copy of the unit-arc table (solver.py:103-136 normalised by a = |x0-xf|/2):
    u_k(d) such that p_k = C + 0.5*[[vx,-vy],[vy,vx]] u_k, k = 1..N."""
    ds = np.asarray(displacements, dtype=np.float64).reshape(-1)
    out = np.zeros((ds.shape[0], N, 2))
    for i, d in enumerate(ds):
        if abs(d) > 1:
            raise ValueError(f"abs(displacement) = {abs(d)} must be smaller than 1")
        if d == 0:
            s = np.arange(1, N + 1, dtype=np.float64) / (N + 1)
            out[i, :, 0] = 1.0 - 2.0 * s
            continue
        with np.errstate(divide="ignore"):
            beta = 2 * np.arctan(2 * d / (1 - d * d))
        rho = (1 + d * d) / (2 * d)
        off = (d * d - 1) / (2 * d)
        t = np.linspace((np.pi - beta) / 2, (np.pi + beta) / 2, N + 2)[1:-1]
        out[i, :, 0] = rho * np.cos(t)
        out[i, :, 1] = off + rho * np.sin(t)
    return out
