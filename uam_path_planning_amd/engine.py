"""Device engine: one libuampath context per GPU, torch tensors as device buffers.

PyTorch is plumbing here (allocation, streams, H2D/D2H); every arithmetic step of the hot path
runs in the hand-written HIP kernels of csrc/uampath.hip.  There is no CPU fallback: without a
visible GPU or without libuampath.so, constructing an Engine raises.
"""
import collections
import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .geometry import FlatGeometry, compile_map, compile_shapes


def _torch():
    import torch

    return torch


@dataclass
class PathParams:
    """Problem options + the OpEn parameter vector p (solver.py:60-78, problem.py:12-22)."""
    N: int
    length_smooth: bool = False
    penalty_smooth: bool = True
    obstacle_smooth: bool = False
    maxratio_smooth: bool = False
    maxratio: float = 1.0
    maxalpha: float = 0.0
    enlargement: float = 0.0
    weights: tuple = ()
    quirk_length: bool = True
    anchor: tuple = None          # map.x_start baked into a reference build; None = p_0
    altitude: float = 150.0       # cruise altitude (m) for min-clearance in raster mode

    def as_struct(self):
        w = [float(x) for x in self.weights]
        if len(w) > _lib.MAX_REGIONS:
            raise ValueError(f"at most {_lib.MAX_REGIONS} region weights")
        arr = (ctypes.c_double * _lib.MAX_REGIONS)(*(w + [1.0] * (_lib.MAX_REGIONS - len(w))))
        a = self.anchor
        return _lib.Params(_lib.ABI_VERSION, int(self.N), int(bool(self.length_smooth)),
                           int(bool(self.penalty_smooth)), int(bool(self.obstacle_smooth)),
                           int(bool(self.maxratio_smooth)), int(bool(self.quirk_length)),
                           0 if a is None else 1, 0.0 if a is None else float(a[0]),
                           0.0 if a is None else float(a[1]), float(self.maxratio),
                           float(self.maxalpha), float(self.enlargement), float(self.altitude),
                           arr)


@dataclass
class RasterGeo:
    """GeoTIFF-convention geotransform of the cost raster (row 0 = north edge)."""
    nx: int
    ny: int
    x0: float
    y_top: float
    dx: float
    dy: float
    nodata: float = -9999.0
    dem_threshold: float = 0.0

    def as_struct(self):
        return _lib.RasterDesc(int(self.nx), int(self.ny), float(self.x0), float(self.y_top),
                               float(self.dx), float(self.dy), float(self.nodata),
                               float(self.dem_threshold))

    def cell_centres(self):
        ix = np.arange(self.nx, dtype=np.float64)
        iy = np.arange(self.ny, dtype=np.float64)
        return self.x0 + (ix + 0.5) * self.dx, self.y_top - (iy + 0.5) * self.dy


@dataclass
class CostRaster:
    """Device record raster: rec [ny, nx, 4] int32 view of {phi f32, psi f32, dem f32, flags};
    summary: the K2 gather-skip bitmap of rec (uam_raster_summary, one bit per block x block
    cells; None = K2 gathers every waypoint); packed: the K2s packed copy of rec
    (uam_raster_pack, 8-B planes in 4 x 4-cell blocks; None = K2s gathers rec).  Rebuild both
    (Engine.raster_summary) after rec changes."""
    geo: RasterGeo
    rec: object = field(repr=False)
    summary: object = field(default=None, repr=False)
    block: int = 0
    packed: object = field(default=None, repr=False)  # uam_raster_pack copy for K2s (or None)

    @property
    def nbytes(self):
        return self.geo.nx * self.geo.ny * _lib.RECORD_BYTES


@dataclass
class VolumeGeo:
    """3-D risk volume grid (config 5): the raster's x/y grid x nz altitude layers (m)."""
    nx: int
    ny: int
    nz: int
    x0: float
    y_top: float
    dx: float
    dy: float
    z0: float
    dz: float

    def as_struct(self):
        return _lib.VolumeDesc(int(self.nx), int(self.ny), int(self.nz), float(self.x0),
                               float(self.y_top), float(self.dx), float(self.dy),
                               float(self.z0), float(self.dz))


@dataclass
class RiskVolume:
    geo: VolumeGeo
    buf: object = field(repr=False)     # the device buffer (uam_volume_shape bytes)
    vox: object = field(repr=False)     # [ny, nx, nz, 2] int32 view: 8-B voxels {risk, psi}
    cols: object = field(repr=False)    # [ny, nx, 2] int32 view: columns {terrain, flags}
    cbits: object = field(repr=False, default=None)  # int32 view: the column bitmap words
    # the packed copy K4h reads (Engine.volume_pack: 4-B / 8-B / 16-B voxel planes in 4 x 8-
    # column blocks per layer, codes, terrain bounds), or None; eval_generated3d rebuilds it
    # when buf (or a view of it: vox, cols) was written in place since (torch's version counter)
    packed: object = field(repr=False, default=None)
    packed_version: int = field(repr=False, default=-1)


def _ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _check_outputs(o, P, Q, W):
    """Caller-supplied outputs (Engine.outputs) must hold this batch: the kernels write P paths
    and Q best indices, so a smaller buffer set would be overrun."""
    for k, t in o.items():
        need = P * W if k == "cells" else (Q if k.startswith("best_") else P)
        if k == "g_rows":
            continue
        if t.numel() < need:
            raise ValueError(f"outputs[{k!r}] holds {t.numel()} entries, this batch needs {need}"
                             f" ({P} paths, {Q} pairs): allocate with Engine.outputs")


# refinement defaults (same as oracle.refine_params)
REFINE_DEFAULTS = dict(n_outer=15, n_inner=50, max_backtrack=30, c0=10.0, rho=5.0, c_max=1e8,
                       alpha0=1e-4, armijo=1e-4, theta=0.25, max_step=0.5, memory=8,
                       inner_tol=1e-3, delta=1e-4, n_restart=0, restart_margin=0.05)


class Engine:
    """libuampath context bound to one GPU."""

    def __init__(self, device=0):
        torch = _torch()
        if not torch.cuda.is_available():
            raise RuntimeError("no GPU visible: uam_path_planning_amd runs only on the HIP "
                               "kernels of libuampath.so (there is no CPU path)")
        self.lib = _lib.load()
        self.device = int(device)
        self.torch_device = torch.device("cuda", self.device)
        h = ctypes.c_void_p()
        _lib.check(self.lib.uam_ctx_create(self.device, ctypes.byref(h)), "uam_ctx_create")
        self._ctx = h
        self._geom_sig = None
        self.geometry = None
        self.params = None

    def __del__(self):
        try:
            if getattr(self, "_ctx", None):
                self.lib.uam_ctx_destroy(self._ctx)
                self._ctx = None
        except Exception:
            pass

    # -- helpers --------------------------------------------------------------------------
    @property
    def stream(self):
        return ctypes.c_void_p(_torch().cuda.current_stream(self.device).cuda_stream)

    def tensor(self, x, dtype):
        torch = _torch()
        if isinstance(x, torch.Tensor):
            t = x.to(device=self.torch_device, dtype=dtype)
        else:
            t = torch.as_tensor(np.asarray(x), dtype=dtype, device=self.torch_device)
        return t.contiguous()

    def empty(self, shape, dtype):
        return _torch().empty(shape, dtype=dtype, device=self.torch_device)

    # -- state ----------------------------------------------------------------------------
    def set_geometry(self, geom):
        if not isinstance(geom, FlatGeometry):
            geom = compile_map(geom)
        sig = geom.signature()
        if sig != self._geom_sig:
            _lib.check(self.lib.uam_set_geometry(self._ctx, ctypes.byref(geom.as_struct())),
                       "uam_set_geometry")
            self._geom_sig = sig
            self.params = None
        self.geometry = geom
        return geom

    def set_params(self, params):
        if params != self.params:
            _lib.check(self.lib.uam_set_params(self._ctx, ctypes.byref(params.as_struct()),
                                               self.stream), "uam_set_params")
            self.params = params
        return params

    # -- points ---------------------------------------------------------------------------
    def eval_points(self, pts, want=("phi", "phi_regions", "obs_norm", "psi_raw", "collide")):
        torch = _torch()
        p = self.tensor(pts, torch.float64).reshape(-1, 2)
        n = p.shape[0]
        R = self.geometry.n_regions
        out = {}
        if "phi" in want:
            out["phi"] = self.empty((n,), torch.float64)
        if "phi_regions" in want:
            out["phi_regions"] = self.empty((n, R), torch.float64)
        if "obs_norm" in want:
            out["obs_norm"] = self.empty((n,), torch.float64)
        if "psi_raw" in want:
            out["psi_raw"] = self.empty((n,), torch.float64)
        if "collide" in want:
            out["collide"] = self.empty((n,), torch.int32)
        _lib.check(self.lib.uam_eval_points(
            self._ctx, _ptr(p), n, _ptr(out.get("phi")), _ptr(out.get("phi_regions")),
            _ptr(out.get("obs_norm")), _ptr(out.get("psi_raw")), _ptr(out.get("collide")),
            self.stream), "uam_eval_points")
        return out

    # -- raster ---------------------------------------------------------------------------
    def raster_build(self, geo, dem=None, out=None, summary=True, packed=True):
        """K1 record raster (+ its K2 gather-skip summary and, with packed, the K2s packed copy,
        unless summary=False)."""
        torch = _torch()
        d = None if dem is None else self.tensor(dem, torch.float32).reshape(geo.ny, geo.nx)
        rec = out if out is not None else self.empty((geo.ny, geo.nx, 4), torch.int32)
        _lib.check(self.lib.uam_raster_build(self._ctx, ctypes.byref(geo.as_struct()), _ptr(d),
                                             _ptr(rec), self.stream), "uam_raster_build")
        r = CostRaster(geo, rec)
        return self.raster_summary(r, packed=packed) if summary else r

    def raster_summary(self, raster, block=0, packed=True):
        """(Re)build raster.summary (and raster.packed unless packed=False; else it is dropped)
        from raster.rec (block 0 = automatic); returns raster.  Both are derived copies that
        are not tracked: call this again after any write to raster.rec (raster_build into it,
        a broadcast, a raw-pointer writer) -- distributed.broadcast_raster does."""
        torch = _torch()
        g = raster.geo.as_struct()
        b, nbx, nby = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _lib.check(self.lib.uam_raster_summary_shape(ctypes.byref(g), int(block), ctypes.byref(b),
                                                     ctypes.byref(nbx), ctypes.byref(nby)),
                   "uam_raster_summary_shape")
        sm = self.empty(((nby.value * nbx.value + 31) // 32,), torch.int32)
        _lib.check(self.lib.uam_raster_summary(self._ctx, ctypes.byref(g), _ptr(raster.rec),
                                               b.value, _ptr(sm), self.stream),
                   "uam_raster_summary")
        raster.summary, raster.block, raster.packed = sm, b.value, None
        if packed:
            nbytes = ctypes.c_int64()
            _lib.check(self.lib.uam_raster_pack_shape(ctypes.byref(g), b.value, None,
                                                      ctypes.byref(nbytes)),
                       "uam_raster_pack_shape")
            pk = self.empty(((nbytes.value + 255) // 256, 256), torch.uint8)
            _lib.check(self.lib.uam_raster_pack(self._ctx, ctypes.byref(g), _ptr(raster.rec),
                                                b.value, _ptr(pk), self.stream),
                       "uam_raster_pack")
            raster.packed = pk
        return raster

    def read_tiles(self, paths, th, tw, n_threads=0, pinned=False):
        """GeoTIFF tiles -> host float32 [T, th, tw] (uam_read_tiles: parallel native reader;
        pinned=True reads into page-locked memory)."""
        torch = _torch()
        out = torch.empty((len(paths), th, tw), dtype=torch.float32, pin_memory=bool(pinned))
        arr = (ctypes.c_char_p * max(1, len(paths)))(*[os.fsencode(str(p)) for p in paths])
        _lib.check(self.lib.uam_read_tiles(arr, len(paths), int(th), int(tw),
                                           ctypes.c_void_p(out.data_ptr()), int(n_threads)),
                   "uam_read_tiles")
        return out

    def load_tiles(self, paths, th, tw, n_threads=0):
        """GeoTIFF tiles -> device float32 [T, th, tw] (uam_load_tiles: the parallel reader
        streaming ~32 MiB chunks through the context's page-locked buffers, each copied while
        the next is read)."""
        torch = _torch()
        out = self.empty((len(paths), th, tw), torch.float32)
        arr = (ctypes.c_char_p * max(1, len(paths)))(*[os.fsencode(str(p)) for p in paths])
        _lib.check(self.lib.uam_load_tiles(self._ctx, arr, len(paths), int(th), int(tw),
                                           _ptr(out), int(n_threads), self.stream),
                   "uam_load_tiles")
        return out

    def dem_mosaic(self, tiles, xoff, yoff, nx, ny, fill=-9999.0, dem=None):
        torch = _torch()
        t = self.tensor(tiles, torch.float32)
        nt, th, tw = t.shape
        xo = self.tensor(xoff, torch.int32)
        yo = self.tensor(yoff, torch.int32)
        if dem is None:
            dem = torch.full((ny, nx), float(fill), dtype=torch.float32, device=self.torch_device)
        _lib.check(self.lib.uam_dem_mosaic(self._ctx, _ptr(t), nt, th, tw, _ptr(xo), _ptr(yo),
                                           _ptr(dem), nx, ny, self.stream), "uam_dem_mosaic")
        return dem

    # -- paths ----------------------------------------------------------------------------
    def outputs(self, P, W, n_pairs=None, want_cells=False, want_g=False):
        """Preallocated per-path (and per-pair best-index) outputs, reusable across launches."""
        return self._outputs(P, W, None, want_cells, want_g, n_pairs)

    def kernel_timing(self, enable=True):
        """Start (and reset) or stop HIP-event timing of the path evaluation: the context records
        an event pair on the launch stream around every k_eval_pairs / k_eval_wave launch (not
        around K2's pair order or the selection kernels), and around the whole K2s sequence
        (its sorts, segment launches and output launch)."""
        _lib.check(self.lib.uam_kernel_timing(self._ctx, 1 if enable else 0),
                   "uam_kernel_timing")

    def kernel_time(self):
        """(total ms, launches) of the timed kernel launches since the last call / reset."""
        ms, n = ctypes.c_double(), ctypes.c_int64()
        _lib.check(self.lib.uam_kernel_time(self._ctx, ctypes.byref(ms), ctypes.byref(n)),
                   "uam_kernel_time")
        return ms.value, n.value

    def last_kernel(self):
        """Which path evaluation the last eval_generated / eval_generated3d ran (uam_last_kernel:
        "K2g+pack", "K2s+pack", "K2+skip", "K2w", "K3b", ...)."""
        return self.lib.uam_last_kernel(self._ctx).decode()

    def last_group(self):
        """Waypoint-group length of the last eval_generated's sums (uam_last_group): G > 0 when
        the segment-grouped K2g ran (the oracle's orc_eval_paths_g order), 0 = sequential."""
        return int(self.lib.uam_last_group(self._ctx))

    def set_option(self, name, value):
        """uam_set_option (include/uampath.h UAM_OPT_*): "group" (K2g waypoints per group,
        0 = K2s), "sorted_min_paths", "k2s_segments", "wave_max_paths", "pair_order",
        "k1_rows", "k3b_segment", "k3b_points_per_lane", "k8_tiled", "k8_streams"."""
        _lib.check(self.lib.uam_set_option(self._ctx, _lib.OPTIONS[name], int(value)),
                   "uam_set_option")

    def get_option(self, name):
        v = ctypes.c_int64()
        _lib.check(self.lib.uam_get_option(self._ctx, _lib.OPTIONS[name], ctypes.byref(v)),
                   "uam_get_option")
        return v.value

    def _outputs(self, P, W, mode, want_cells, want_g, n_pairs=None):
        torch = _torch()
        o = {k: self.empty((P,), torch.float64) for k in ("cost", "length_q", "length",
                                                           "kin_sum", "nfz_sum",
                                                           "min_clearance")}
        o["nfz_hits"] = self.empty((P,), torch.int32)
        o["offmap"] = self.empty((P,), torch.int32)
        o["below_terrain"] = self.empty((P,), torch.int32)
        if want_cells:
            o["cells"] = self.empty((P, W), torch.int32)
        if want_g:
            n_rows = 3 * (W - 2) + self.geometry.n_obstacles * W
            o["g_rows"] = self.empty((P, n_rows), torch.float64)
        if n_pairs is not None:
            o["best_fval_idx"] = self.empty((n_pairs,), torch.int32)
            o["best_length_idx"] = self.empty((n_pairs,), torch.int32)
        s = _lib.PathOutputs(*[ctypes.c_void_p(o[k].data_ptr()) if k in o else None
                               for k, _ in _lib.PathOutputs._fields_])
        return o, s

    def _mode(self, raster):
        return _lib.MODE_ANALYTIC if raster is None else _lib.MODE_RASTER

    def eval_waypoints(self, wp, raster=None, want_cells=False, want_g=False):
        """wp [P, N+2, 2] float64 (p_0 = start .. p_{N+1} = goal).  raster=None: analytic."""
        torch = _torch()
        N = self.params.N
        w = self.tensor(wp, torch.float64).reshape(-1, N + 2, 2)
        P = w.shape[0]
        o, s = self._outputs(P, N + 2, self._mode(raster), want_cells and raster is not None,
                             want_g and raster is None)
        geo = None if raster is None else ctypes.byref(raster.geo.as_struct())
        _lib.check(self.lib.uam_eval_waypoints(
            self._ctx, self._mode(raster), geo, _ptr(None if raster is None else raster.rec),
            _ptr(w), P, ctypes.byref(s), self.stream), "uam_eval_waypoints")
        return o

    def eval_generated(self, pairs, utab, raster=None, want_cells=False, outputs=None):
        """pairs [Q, 4] (x0, y0, xf, yf); utab [D, N, 2]; path p = q*D + d."""
        torch = _torch()
        pr = self.tensor(pairs, torch.float64).reshape(-1, 4)
        ut = self.tensor(utab, torch.float64)
        D = ut.shape[0]
        if ut.shape[1] != self.params.N:
            raise ValueError(f"arc table has N={ut.shape[1]}, params N={self.params.N}")
        Q = pr.shape[0]
        if outputs is None:
            o, s = self._outputs(Q * D, self.params.N + 2, self._mode(raster),
                                 want_cells and raster is not None, False, n_pairs=Q)
        else:
            o, s = outputs
            _check_outputs(o, Q * D, Q, self.params.N + 2)
        geo = None if raster is None else ctypes.byref(raster.geo.as_struct())
        rec = summary = packed = None
        block = 0
        if raster is not None:
            rec, summary, packed, block = raster.rec, raster.summary, raster.packed, raster.block
        _lib.check(self.lib.uam_eval_generated(
            self._ctx, self._mode(raster), geo, _ptr(rec), _ptr(summary), int(block or 0),
            _ptr(packed), _ptr(pr), Q, _ptr(ut), D, ctypes.byref(s), self.stream),
            "uam_eval_generated")
        return o

    # -- volume (config 5) -------------------------------------------------------------
    def volume_alloc(self, vg):
        """An uninitialised volume buffer of VolumeGeo vg (uam_volume_shape), e.g. for a rank
        that receives it by broadcast."""
        torch = _torch()
        nbytes, off = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self.lib.uam_volume_shape(ctypes.byref(vg.as_struct()), ctypes.byref(nbytes),
                                             ctypes.byref(off)), "uam_volume_shape")
        buf = self.empty((nbytes.value // 4,), torch.int32)   # caching allocator: 512-B aligned
        nv = vg.nx * vg.ny * vg.nz * 2
        vox = buf[:nv].view(vg.ny, vg.nx, vg.nz, 2)
        nc = vg.nx * vg.ny * 2
        cols = buf[off.value // 4: off.value // 4 + nc].view(vg.ny, vg.nx, 2)
        bits0 = off.value // 4 + (nc * 4 + 255) // 256 * 64
        return RiskVolume(vg, buf, vox, cols, buf[bits0:])

    def volume_build(self, raster, nz, z0, dz, layer_w):
        torch = _torch()
        g = raster.geo
        vg = VolumeGeo(g.nx, g.ny, int(nz), g.x0, g.y_top, g.dx, g.dy, float(z0), float(dz))
        lw = self.tensor(layer_w, torch.float64).reshape(-1)
        if lw.numel() != nz:
            raise ValueError(f"layer_w has {lw.numel()} entries, nz = {nz}")
        vol = self.volume_alloc(vg)
        _lib.check(self.lib.uam_volume_build(self._ctx, ctypes.byref(vg.as_struct()),
                                             _ptr(raster.rec), _ptr(lw), _ptr(vol.buf),
                                             self.stream), "uam_volume_build")
        return vol

    def volume_pack(self, volume):
        """Derive the packed copy K4h evaluates (uam_volume_pack) into volume.packed.
        eval_generated3d repacks by itself when torch's version counter of volume.buf moved;
        a write that bypasses torch (uam_volume_build into the same buffer, an RCCL broadcast
        through the C ABI, DLPack or ctypes writers) does not move it, so call this after
        one (distributed.broadcast_raster does)."""
        torch = _torch()
        nb = ctypes.c_int64()
        _lib.check(self.lib.uam_volume_packed_bytes(ctypes.byref(volume.geo.as_struct()),
                                                    ctypes.byref(nb)), "uam_volume_packed_bytes")
        packed = self.empty((nb.value // 4,), torch.int32)
        _lib.check(self.lib.uam_volume_pack(self._ctx, ctypes.byref(volume.geo.as_struct()),
                                            _ptr(volume.buf), _ptr(packed), self.stream),
                   "uam_volume_pack")
        volume.packed = packed
        volume.packed_version = volume.buf._version
        return packed

    def eval_generated3d(self, pairs6, utab, volume, outputs=None):
        """pairs6 [Q, 6] = (x0, y0, z0, xf, yf, zf) (km, km, m); path p = q*D + d."""
        torch = _torch()
        pr = self.tensor(pairs6, torch.float64).reshape(-1, 6)
        ut = self.tensor(utab, torch.float64)
        D = ut.shape[0]
        if ut.shape[1] != self.params.N:
            raise ValueError(f"arc table has N={ut.shape[1]}, params N={self.params.N}")
        Q = pr.shape[0]
        if outputs is not None:
            o, s = outputs
            _check_outputs(o, Q * D, Q, self.params.N + 2)
        else:
            o, s = self._outputs(Q * D, self.params.N + 2, _lib.MODE_VOLUME, False, False,
                                 n_pairs=Q)
        if volume.packed is not None and volume.buf._version != volume.packed_version:
            self.volume_pack(volume)   # the voxels changed since the copy: K4h reads only it
        _lib.check(self.lib.uam_eval_generated3d(
            self._ctx, ctypes.byref(volume.geo.as_struct()), _ptr(volume.buf),
            _ptr(volume.packed), _ptr(pr), Q, _ptr(ut), D, ctypes.byref(s), self.stream),
            "uam_eval_generated3d")
        return o

    def gen_paths(self, pairs, utab):
        torch = _torch()
        pr = self.tensor(pairs, torch.float64).reshape(-1, 4)
        ut = self.tensor(utab, torch.float64)
        D, N = ut.shape[0], ut.shape[1]
        if N != self.params.N:
            raise ValueError(f"arc table has N={N}, params N={self.params.N}")
        wp = self.empty((pr.shape[0] * D, N + 2, 2), torch.float64)
        _lib.check(self.lib.uam_gen_paths(self._ctx, _ptr(pr), pr.shape[0], _ptr(ut), D,
                                          _ptr(wp), self.stream), "uam_gen_paths")
        return wp

    def argmin(self, values, G, take_sqrt, out=None):
        torch = _torch()
        v = self.tensor(values, torch.float64).reshape(-1)
        groups = v.shape[0] // G
        best = out if out is not None else self.empty((groups,), torch.int32)
        _lib.check(self.lib.uam_argmin(self._ctx, _ptr(v), groups, int(G), int(bool(take_sqrt)),
                                       _ptr(best), self.stream), "uam_argmin")
        return best

    def path_length(self, pts, n_segments, smooth):
        torch = _torch()
        p = self.tensor(pts, torch.float64)
        if p.dim() == 2:
            p = p.unsqueeze(0)
        P, n_points = p.shape[0], p.shape[1]
        out = self.empty((P,), torch.float64)
        _lib.check(self.lib.uam_path_length(self._ctx, _ptr(p), P, n_points, int(n_segments),
                                            int(bool(smooth)), _ptr(out), self.stream),
                   "uam_path_length")
        return out

    def refine(self, wp, params=None, inplace=False):
        """Batched ALM refinement of waypoint paths (the reference's
        OpEn solve, solver.py:82-93).  wp: [P, N+2, 2] float64; endpoints stay fixed.
        Returns {"wp", "cost", "infeas", "iters"} (device tensors).  Definition and
        defaults: oracle/uam_oracle.c orc_refine, REFINE_DEFAULTS."""
        torch = _torch()
        W = self.params.N + 2
        z = self.tensor(wp, torch.float64)
        if z.dim() == 2:
            z = z.unsqueeze(0)
        if tuple(z.shape[1:]) != (W, 2):
            raise ValueError(f"wp must be [P, {W}, 2], got {tuple(z.shape)}")
        if not inplace:
            z = z.clone(memory_format=torch.contiguous_format)
        elif not z.is_contiguous():
            raise ValueError("inplace refinement needs a contiguous tensor")
        P = z.shape[0]
        rp = dict(REFINE_DEFAULTS)
        rp.update(params or {})
        unknown = set(rp) - set(REFINE_DEFAULTS)
        if unknown:
            raise ValueError(f"unknown refine settings {sorted(unknown)}")
        st = _lib.RefineParams(int(rp["n_outer"]), int(rp["n_inner"]), int(rp["max_backtrack"]),
                               int(rp["memory"]), float(rp["c0"]), float(rp["rho"]),
                               float(rp["c_max"]), float(rp["alpha0"]), float(rp["armijo"]),
                               float(rp["theta"]), float(rp["max_step"]),
                               float(rp["inner_tol"]), float(rp["delta"]),
                               int(rp["n_restart"]), float(rp["restart_margin"]))
        nbytes = self.lib.uam_refine_workspace_bytes(self._ctx, P, ctypes.byref(st))
        if nbytes < 0:
            raise _lib.UamError("uam_refine_workspace_bytes: set geometry and params first")
        ws = self.empty((max(nbytes, 8) // 8,), torch.float64)
        out = {"wp": z, "cost": self.empty((P,), torch.float64),
               "infeas": self.empty((P,), torch.float64), "iters": self.empty((P,), torch.int32)}
        _lib.check(self.lib.uam_refine(self._ctx, _ptr(z), P, ctypes.byref(st), _ptr(ws), nbytes,
                                       _ptr(out["cost"]), _ptr(out["infeas"]), _ptr(out["iters"]),
                                       self.stream), "uam_refine")
        return out

    # -- coordinate reference systems (K7) --------------------------
    def _tm(self, tm):
        if tm is None or isinstance(tm, int):
            out = _lib.TmParams()
            _lib.check(self.lib.uam_tm_jprcs(1 if tm is None else int(tm), ctypes.byref(out)),
                       "uam_tm_jprcs")
            return out
        return tm

    def _points(self, fn, name, pts, tm):
        torch = _torch()
        p = self.tensor(pts, torch.float64).reshape(-1, 2).contiguous()
        out = self.empty(tuple(p.shape), torch.float64)
        _lib.check(fn(self._ctx, ctypes.byref(self._tm(tm)), _ptr(p), p.shape[0], _ptr(out),
                      self.stream), name)
        return out

    def geo_to_plane(self, lonlat, tm=None):
        """[n, 2] lon, lat (deg) -> x (easting), y (northing) in metres; tm = JPRCS zone
        number (default 1 = EPSG:2443) or a TmParams."""
        return self._points(self.lib.uam_geo_to_plane, "uam_geo_to_plane", lonlat, tm)

    def plane_to_geo(self, xy, tm=None):
        """[n, 2] x, y metres -> lon, lat (deg)."""
        return self._points(self.lib.uam_plane_to_geo, "uam_plane_to_geo", xy, tm)

    def reproject_dem(self, src, src_grid, dst_geo, unit_m=1000.0, resample=0, tm=None):
        """Geographic DEM [ny, nx] float32 on src_grid (GeoGridDesc) -> plane DEM on the
        RasterGeo dst_geo (coordinates in units of unit_m metres)."""
        torch = _torch()
        s = self.tensor(src, torch.float32).contiguous()
        if tuple(s.shape) != (src_grid.ny, src_grid.nx):
            raise ValueError(f"src must be [{src_grid.ny}, {src_grid.nx}]")
        out = self.empty((dst_geo.ny, dst_geo.nx), torch.float32)
        _lib.check(self.lib.uam_reproject_dem(
            self._ctx, ctypes.byref(self._tm(tm)), _ptr(s), ctypes.byref(src_grid),
            ctypes.byref(dst_geo.as_struct()), float(unit_m), int(resample), _ptr(out),
            self.stream), "uam_reproject_dem")
        return out

    # -- land polygons from the DEM (K8) -------------------------------
    def dem_polygons(self, dem, geo, threshold=0.0, unit_m=1000.0, params=None):
        """DEM mask -> 4-connected regions (GPU labelling) -> DataProcessor approximation.
        dem [ny, nx] float32 on RasterGeo geo (units of unit_m metres).  -> list of int64
        [4, 2] rectangles in metres (cv2.boxPoints order)."""
        torch = _torch()
        d = self.tensor(dem, torch.float32).contiguous()
        if tuple(d.shape) != (geo.ny, geo.nx):
            raise ValueError(f"dem must be [{geo.ny}, {geo.nx}]")
        prm = params if params is not None else _lib.PolyprocParams(750000.0, 32000000.0,
                                                                    780000.0, 5, 0)
        n = ctypes.c_int32(0)
        cap = 256
        while True:
            out = np.zeros((cap, 4, 2), np.int64)
            st = self.lib.uam_dem_polygons(self._ctx, _ptr(d), ctypes.byref(geo.as_struct()),
                                           float(threshold), float(unit_m), ctypes.byref(prm),
                                           out.ctypes.data, cap, ctypes.byref(n), self.stream)
            if st == _lib.UAM_OK:
                return [out[i] for i in range(n.value)]
            if n.value > cap:
                cap = n.value
                continue
            _lib.check(st, "uam_dem_polygons")

    # -- raster broadcast over RCCL (uam_comm_* / uam_bcast_raster) ---------------------------
    def comm_unique_id(self):
        """128-byte RCCL unique id (rank 0 creates it, every rank passes it to comm_init)."""
        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
        _lib.check(self.lib.uam_comm_unique_id(buf), "uam_comm_unique_id")
        return bytes(buf)

    def comm_init(self, uid, nranks, rank):
        """Join the RCCL communicator of uid as rank of nranks (collective over the ranks)."""
        if len(uid) != _lib.COMM_ID_BYTES:
            raise ValueError(f"unique id must be {_lib.COMM_ID_BYTES} bytes")
        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(uid)
        _lib.check(self.lib.uam_comm_init(self._ctx, buf, int(nranks), int(rank)),
                   "uam_comm_init")

    def bcast_raster(self, t, root=0):
        """Broadcast device tensor t (in place) from root over the context's communicator, on
        this engine's current stream."""
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("bcast_raster needs a contiguous device tensor")
        _lib.check(self.lib.uam_bcast_raster(self._ctx, _ptr(t), t.numel() * t.element_size(),
                                             int(root), self.stream), "uam_bcast_raster")
        return t

    def synchronize(self):
        """Wait for this engine's stream; raises DeviceCheckError when a call's device-side
        check failed (its outputs then hold NaN / -1)."""
        _lib.check(self.lib.uam_synchronize(self._ctx, self.stream), "uam_synchronize")

    def device_status(self):
        """Raise DeviceCheckError if a completed call's device-side check failed (no wait)."""
        _lib.check(self.lib.uam_device_status(self._ctx), "uam_device_status")


_default = {}


def default_engine(device=None):
    torch = _torch()
    if device is None:
        device = torch.cuda.current_device() if torch.cuda.is_available() else 0
    if device not in _default:
        _default[device] = Engine(device)
    return _default[device]


# ---- single-shape helpers used by the drop-in classes (scratch contexts) ------------------
# The reference evaluates psi / contains / collides point by point (problem.py:72-80 calls
# psi(x) per shape per point).  Each distinct (geometry, options) pair gets one context with its
# geometry and parameters uploaded once, kept in a small LRU cache, so a per-point loop costs
# one copy in, one launch and one copy out per call -- no allocation, upload or k_prepare.
_SCRATCH_MAX = 64
_scratch_cache = collections.OrderedDict()


def _scratch(geom, params):
    dev = default_engine().device
    key = (dev, geom.signature(), repr(params))
    eng = _scratch_cache.get(key)
    if eng is not None:
        _scratch_cache.move_to_end(key)
        return eng
    eng = Engine(dev)
    eng.set_geometry(geom)
    eng.set_params(params)
    _scratch_cache[key] = eng
    if len(_scratch_cache) > _SCRATCH_MAX:
        _scratch_cache.popitem(last=False)
    return eng


def _as_points(x):
    a = np.asarray(x, dtype=np.float64)
    single = a.size == 2
    return a.reshape(-1, 2), single


def shape_psi(obs, x, smooth, enlargement):
    """psi(x) of one shape: a one-region geometry with no centre and weight 1 -> phi = psi."""
    pts, single = _as_points(x)
    shape = type(obs).__new__(type(obs))
    shape.__dict__.update(obs.__dict__)
    shape.center = float("nan")
    geom = compile_shapes((), [[shape]])
    eng = _scratch(geom, PathParams(N=1, penalty_smooth=smooth, enlargement=enlargement,
                                    weights=(1.0,)))
    v = eng.eval_points(pts, want=("phi",))["phi"].cpu().numpy()
    return float(v[0]) if single else v


def shape_contains(obs, x):
    pts, single = _as_points(x)
    eng = _scratch(compile_shapes([obs], []), PathParams(N=1))
    v = eng.eval_points(pts, want=("collide",))["collide"].cpu().numpy().astype(bool)
    return bool(v[0]) if single else v


def map_collides(m, x):
    pts, single = _as_points(x)
    eng = _scratch(compile_shapes(list(m.obstacles), []), PathParams(N=1))
    v = eng.eval_points(pts, want=("collide",))["collide"].cpu().numpy().astype(bool)
    return bool(v[0]) if single else v
