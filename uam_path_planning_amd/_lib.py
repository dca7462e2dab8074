"""ctypes binding of libuampath.so (include/uampath.h).

The library is built in-tree (uam_path_planning_amd/lib/libuampath.so) by
``uam_path_planning_amd.build.build_library()`` / ``__graft_entry__.build()``.  There is no
CPU fallback: if the library is missing or no GPU is visible, every entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# UAM_LIB_PATH: load another build of the same ABI (tuning experiments, e.g. tools/ builds
# with different compile-time knobs); the default is the in-tree build
LIB_PATH = os.environ.get("UAM_LIB_PATH") or os.path.join(HERE, "lib", "libuampath.so")

ABI_VERSION = 2  # include/uampath.h UAM_ABI_VERSION
MAX_REGIONS = 16
RECORD_BYTES = 16
COMM_ID_BYTES = 128

UAM_OK, UAM_E_INVALID, UAM_E_HIP, UAM_E_NOMEM, UAM_E_STATE, UAM_E_VERSION = 0, -1, -2, -3, -4, -5
UAM_E_DEVICE = -6  # a device-side check of an earlier call failed (uam_device_status)
# uam_set_option keys (include/uampath.h)
OPTIONS = {"group": 1, "sorted_min_paths": 2, "k2s_segments": 3, "wave_max_paths": 4,
           "pair_order": 5, "k1_rows": 6, "k3b_segment": 7, "k3b_points_per_lane": 8,
           "k8_tiled": 9, "k8_streams": 10, "k2g_tile_bits": 11, "k2g_lds_floor": 12,
           "k2g_chunk": 13, "k2g_curve": 14, "k2g_sim": 15, "k4h_band": 17,
           "k2h_lb_stride": 19, "k2h_terrain": 20, "k4h_terrain": 21,
           "test_sort_fault": 22}
INEQ_HALFPLANE, INEQ_ELLIPSE, INEQ_AXIS = 0, 1, 2
MODE_ANALYTIC, MODE_RASTER, MODE_VOLUME = 0, 1, 2
FLAG_NFZ, FLAG_MASK, FLAG_NODATA = 1, 2, 4

_i32p = ctypes.POINTER(ctypes.c_int32)
_f64p = ctypes.POINTER(ctypes.c_double)
_vp = ctypes.c_void_p


class Geometry(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("n_ineq", ctypes.c_int32),
                ("ineq_kind", _i32p), ("ineq_par", _f64p), ("n_shapes", ctypes.c_int32),
                ("shape_first", _i32p), ("shape_count", _i32p), ("shape_center", _f64p),
                ("n_obstacles", ctypes.c_int32), ("n_regions", ctypes.c_int32),
                ("region_first", _i32p)]


class Params(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("N", ctypes.c_int32),
                ("length_smooth", ctypes.c_int32), ("penalty_smooth", ctypes.c_int32),
                ("obstacle_smooth", ctypes.c_int32), ("maxratio_smooth", ctypes.c_int32),
                ("quirk_length", ctypes.c_int32), ("anchor_mode", ctypes.c_int32),
                ("anchor_x", ctypes.c_double), ("anchor_y", ctypes.c_double),
                ("maxratio", ctypes.c_double), ("maxalpha", ctypes.c_double),
                ("enlargement", ctypes.c_double), ("altitude", ctypes.c_double),
                ("weights", ctypes.c_double * MAX_REGIONS)]


class RasterDesc(ctypes.Structure):
    _fields_ = [("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("x0", ctypes.c_double),
                ("y_top", ctypes.c_double), ("dx", ctypes.c_double), ("dy", ctypes.c_double),
                ("nodata", ctypes.c_float), ("dem_threshold", ctypes.c_float)]


class VolumeDesc(ctypes.Structure):
    _fields_ = [("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("nz", ctypes.c_int32),
                ("x0", ctypes.c_double), ("y_top", ctypes.c_double), ("dx", ctypes.c_double),
                ("dy", ctypes.c_double), ("z0", ctypes.c_double), ("dz", ctypes.c_double)]


class PathOutputs(ctypes.Structure):
    _fields_ = [(name, _vp) for name in ("cost", "length_q", "length", "kin_sum", "nfz_sum",
                                         "nfz_hits", "min_clearance", "offmap", "cells",
                                         "g_rows", "best_fval_idx", "best_length_idx",
                                         "below_terrain")]


class RefineParams(ctypes.Structure):
    _fields_ = [("n_outer", ctypes.c_int32), ("n_inner", ctypes.c_int32),
                ("max_backtrack", ctypes.c_int32), ("memory", ctypes.c_int32),
                ("c0", ctypes.c_double), ("rho", ctypes.c_double), ("c_max", ctypes.c_double),
                ("alpha0", ctypes.c_double), ("armijo", ctypes.c_double),
                ("theta", ctypes.c_double), ("max_step", ctypes.c_double),
                ("inner_tol", ctypes.c_double), ("delta", ctypes.c_double),
                ("n_restart", ctypes.c_int32), ("restart_margin", ctypes.c_double)]


class TmParams(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in ("a", "f", "k0", "lat0_deg", "lon0_deg",
                                                "false_easting", "false_northing")]


class GeoGridDesc(ctypes.Structure):
    _fields_ = [("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("lon0", ctypes.c_double),
                ("lat_top", ctypes.c_double), ("dlon", ctypes.c_double),
                ("dlat", ctypes.c_double), ("nodata", ctypes.c_float), ("pad", ctypes.c_int32)]


class PolyprocParams(ctypes.Structure):
    _fields_ = [("min_area", ctypes.c_double), ("large_area", ctypes.c_double),
                ("min_approx_area", ctypes.c_double), ("divisions", ctypes.c_int32),
                ("pad", ctypes.c_int32)]


# name -> (restype, argtypes); the full exported surface of include/uampath.h
SIGNATURES = {
    "uam_abi_version": (ctypes.c_int, []),
    "uam_last_error": (ctypes.c_char_p, []),
    "uam_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "uam_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "uam_ctx_destroy": (None, [_vp]),
    "uam_set_geometry": (ctypes.c_int, [_vp, ctypes.POINTER(Geometry)]),
    "uam_set_params": (ctypes.c_int, [_vp, ctypes.POINTER(Params), _vp]),
    "uam_eval_points": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "uam_raster_build": (ctypes.c_int, [_vp, ctypes.POINTER(RasterDesc), _vp, _vp, _vp]),
    "uam_dem_mosaic": (ctypes.c_int, [_vp, _vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                      _vp, _vp, _vp, ctypes.c_int32, ctypes.c_int32, _vp]),
    "uam_gen_paths": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, ctypes.c_int32, _vp, _vp]),
    "uam_eval_waypoints": (ctypes.c_int, [_vp, ctypes.c_int32, ctypes.POINTER(RasterDesc), _vp,
                                          _vp, ctypes.c_int64, ctypes.POINTER(PathOutputs), _vp]),
    "uam_eval_generated": (ctypes.c_int, [_vp, ctypes.c_int32, ctypes.POINTER(RasterDesc), _vp,
                                          _vp, ctypes.c_int32, _vp, _vp, ctypes.c_int64, _vp,
                                          ctypes.c_int32, ctypes.POINTER(PathOutputs), _vp]),
    "uam_raster_summary_shape": (ctypes.c_int, [ctypes.POINTER(RasterDesc), ctypes.c_int32,
                                                _i32p, _i32p, _i32p]),
    "uam_raster_summary": (ctypes.c_int, [_vp, ctypes.POINTER(RasterDesc), _vp, ctypes.c_int32,
                                          _vp, _vp]),
    "uam_raster_pack_shape": (ctypes.c_int, [ctypes.POINTER(RasterDesc), ctypes.c_int32,
                                             _i32p, ctypes.POINTER(ctypes.c_int64)]),
    "uam_raster_pack": (ctypes.c_int, [_vp, ctypes.POINTER(RasterDesc), _vp, ctypes.c_int32,
                                       _vp, _vp]),
    "uam_argmin": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, _vp,
                                  _vp]),
    "uam_path_length": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, _vp, _vp]),
    "uam_synchronize": (ctypes.c_int, [_vp, _vp]),
    "uam_device_status": (ctypes.c_int, [_vp]),
    "uam_kernel_timing": (ctypes.c_int, [_vp, ctypes.c_int32]),
    "uam_kernel_time": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_int64)]),
    "uam_last_kernel": (ctypes.c_char_p, [_vp]),
    "uam_last_group": (ctypes.c_int32, [_vp]),
    "uam_set_option": (ctypes.c_int, [_vp, ctypes.c_int32, ctypes.c_int64]),
    "uam_get_option": (ctypes.c_int, [_vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]),
    "uam_read_tiles": (ctypes.c_int, [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_int32, _vp, ctypes.c_int32]),
    "uam_load_tiles": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_int32, _vp, ctypes.c_int32, _vp]),
    "uam_volume_shape": (ctypes.c_int, [ctypes.POINTER(VolumeDesc), ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_int64)]),
    "uam_volume_build": (ctypes.c_int, [_vp, ctypes.POINTER(VolumeDesc), _vp, _vp, _vp, _vp]),
    "uam_eval_generated3d": (ctypes.c_int, [_vp, ctypes.POINTER(VolumeDesc), _vp, _vp, _vp,
                                            ctypes.c_int64, _vp, ctypes.c_int32,
                                            ctypes.POINTER(PathOutputs), _vp]),
    "uam_volume_packed_bytes": (ctypes.c_int, [ctypes.POINTER(VolumeDesc),
                                               ctypes.POINTER(ctypes.c_int64)]),
    "uam_volume_pack": (ctypes.c_int, [_vp, ctypes.POINTER(VolumeDesc), _vp, _vp, _vp]),
    "uam_comm_unique_id": (ctypes.c_int, [_vp]),
    "uam_comm_init": (ctypes.c_int, [_vp, _vp, ctypes.c_int32, ctypes.c_int32]),
    "uam_comm_destroy": (ctypes.c_int, [_vp]),
    "uam_bcast_raster": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int32, _vp]),
    "uam_bcast_raster_group": (ctypes.c_int, [_vp, _vp, ctypes.c_int32, ctypes.c_int64,
                                              ctypes.c_int32, _vp]),
    "uam_tm_jprcs": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(TmParams)]),
    "uam_geo_to_plane": (ctypes.c_int, [_vp, ctypes.POINTER(TmParams), _vp, ctypes.c_int64, _vp,
                                        _vp]),
    "uam_plane_to_geo": (ctypes.c_int, [_vp, ctypes.POINTER(TmParams), _vp, ctypes.c_int64, _vp,
                                        _vp]),
    "uam_reproject_dem": (ctypes.c_int, [_vp, ctypes.POINTER(TmParams), _vp,
                                         ctypes.POINTER(GeoGridDesc), ctypes.POINTER(RasterDesc),
                                         ctypes.c_double, ctypes.c_int32, _vp, _vp]),
    "uam_process_polygons": (ctypes.c_int, [_vp, _vp, ctypes.c_int32, _vp,
                                            ctypes.POINTER(PolyprocParams), _vp, ctypes.c_int32,
                                            ctypes.POINTER(ctypes.c_int32)]),
    "uam_dem_polygons": (ctypes.c_int, [_vp, _vp, ctypes.POINTER(RasterDesc), ctypes.c_float,
                                        ctypes.c_double, ctypes.POINTER(PolyprocParams), _vp,
                                        ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), _vp]),
    "uam_refine_workspace_bytes": (ctypes.c_int64, [_vp, ctypes.c_int64,
                                                    ctypes.POINTER(RefineParams)]),
    "uam_refine": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.POINTER(RefineParams), _vp,
                                  ctypes.c_int64, _vp, _vp, _vp, _vp]),
}

_lib = None


class UamError(RuntimeError):
    pass


class DeviceCheckError(UamError):
    """UAM_E_DEVICE: a device-side consistency check of an earlier call failed; that call's
    outputs hold NaN / -1 (include/uampath.h uam_device_status)."""


def load():
    """Load libuampath.so (no fallback: raises if it was not built).

    torch is imported first on purpose: torch ships its own libamdhip64 (soname
    libamdhip64.so.7) and libtorch_hip links it unversioned.  Loaded after torch, libuampath's
    libamdhip64.so.7 dependency resolves to torch's already-loaded runtime, so device buffers
    and streams are shared by ONE HIP runtime.  Loaded before torch, the system runtime would
    come in first and torch would then load a second one that sees no device."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (see docstring: one HIP runtime per process)
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build the HIP library first "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.uam_abi_version() != ABI_VERSION:
        raise RuntimeError(f"libuampath ABI {lib.uam_abi_version()} != {ABI_VERSION}")
    _lib = lib
    return lib


def last_error():
    msg = load().uam_last_error()
    return msg.decode() if msg else ""


def check(status, what=""):
    if status == UAM_OK:
        return
    msg = last_error()
    text = f"{what}: {msg}" if what else msg
    if status == UAM_E_INVALID:
        raise ValueError(text)
    if status == UAM_E_DEVICE:
        raise DeviceCheckError(f"[status {status}] {text}")
    raise UamError(f"[status {status}] {text}")
