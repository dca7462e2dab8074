#!/usr/bin/env python3
"""Locality probe (GPU box): could a segment-sorted raster evaluation beat K2's direct gather?
cfg3's real cells (uam_eval_generated's `cells`), the real records; per path a float64 sum in
waypoint order.  Times (HIP events): the whole-path baseline in the pair order K2 uses, and the
segmented form -- paths split into segments of L waypoints, each segment index one launch over
the (path, segment) items sorted by the Morton tile of the segment's middle waypoint, the path's
running sum carried in HBM -- at several workgroup caps per CU (dynamic-LDS padding).  The
per-segment sorts are timed separately.  Both forms must give the same sums bit for bit.
usage: python tools/probe_seg_locality.py [--pairs 100000]"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (CONFIGS, build_region_map, canonical_params,
                                                canonical_spec, displacements, raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    so = os.path.join(ROOT, "build", "probe_seg", "libprobe_seg.so")
    if not os.path.exists(so):
        os.makedirs(os.path.dirname(so), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950",
                        "-o", so, os.path.join(ROOT, "tools", "probe_seg_locality.hip")],
                       check=True)
    lib = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    lib.probe_full.argtypes = [vp, vp, ctypes.c_int, vp, ctypes.c_int64, vp, vp]
    lib.probe_seg.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp,
                              ctypes.c_int64, vp, ctypes.c_int, vp]
    dd_ = ctypes.c_double
    lib.probe_gen.argtypes = [vp, vp, vp, ctypes.c_int, ctypes.c_int, dd_, dd_, dd_, dd_,
                              ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp,
                              ctypes.c_int64, vp, ctypes.c_int, vp]
    spec = canonical_spec(nfz_polygons=CONFIGS["cfg3"]["nfz_polygons"])
    e = Engine(0)
    e.set_geometry(compile_map(build_region_map(spec)))
    e.set_params(canonical_params(spec, N=80, altitude=320.0))
    R = 4096
    geo = raster_geo(R)
    raster = e.raster_build(geo, synthetic_dem(R))
    pairs_h = random_pairs(a.pairs, seed=0)
    pairs = e.tensor(pairs_h, torch.float64)
    D, W = 5, 82
    ut = arc_table(80, displacements(D))
    g = e.eval_generated(pairs, ut, raster=raster, want_cells=True)
    cells = g["cells"].contiguous()
    P = cells.shape[0]
    rec = raster.rec
    stream = vp(torch.cuda.current_stream().cuda_stream)

    def ptr(t):
        return vp(t.data_ptr())

    # K2's pair order: 2 bits of (yf, xf, y0, x0), Morton-interleaved (k_rorder), then d
    lo = torch.tensor([geo.x0, geo.y_top - R * geo.dy], device="cuda", dtype=torch.float64)
    ext = R * geo.dx
    q = ((pairs.view(-1, 2, 2) - lo) / ext * 4).clamp(0, 3).long()   # [Q][2 points][x, y]
    c = [q[:, 0, 0], q[:, 0, 1], q[:, 1, 0], q[:, 1, 1]]             # x0, y0, xf, yf
    key = torch.zeros(a.pairs, dtype=torch.long, device="cuda")
    for lvl in (1, 0):
        for dd in (3, 2, 1, 0):
            key = (key << 1) | ((c[dd] >> lvl) & 1)
    porder = torch.argsort(key, stable=True)
    order_full = (porder[:, None] * D + torch.arange(D, device="cuda")).reshape(-1).to(torch.int32)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.reps):
            fn()
        t1.record()
        torch.cuda.synchronize()
        return t0.elapsed_time(t1) / a.reps

    utd = e.tensor(ut, torch.float64)
    gargs = (D, 80, geo.x0, geo.y_top, 1.0 / geo.dx, 1.0 / geo.dy, R, R)

    def gen(j0, j1, o, acc, pad):
        return lib.probe_gen(ptr(rec), ptr(pairs), ptr(utd), *gargs, j0, j1, ptr(o), P, ptr(acc),
                             pad, stream)

    accg = torch.empty(P, dtype=torch.float64, device="cuda")
    for pad in (0, 40 * 1024, 80 * 1024):
        ms = timed(lambda: gen(0, W, order_full, accg, pad))
        print(f"generated, whole paths, pair order, lds_pad={pad // 1024:3d} KiB: {ms:.3f} ms",
              flush=True)
    acc0 = torch.empty(P, dtype=torch.float64, device="cuda")
    ms_full = timed(lambda: lib.probe_full(ptr(rec), ptr(cells), W, ptr(order_full), P,
                                           ptr(acc0), stream))
    ms_nord = timed(lambda: lib.probe_full(ptr(rec), ptr(cells), W, None, P, ptr(acc0), stream))
    print(f"baseline whole paths: {ms_full:.3f} ms (pair order), {ms_nord:.3f} ms (no order)",
          flush=True)
    T = 64  # tile of cells for the segment keys
    for L in (8, 16, 21, 41):
        segs = [(j0, min(W, j0 + L)) for j0 in range(0, W, L)]
        orders, t_sort = [], 0.0
        for j0, j1 in segs:
            mid = cells[:, (j0 + j1 - 1) // 2].long()
            ok = mid >= 0
            iy, ix = torch.div(mid, R, rounding_mode="floor"), mid % R
            ty, tx = (iy // T).clamp(min=0), (ix // T).clamp(min=0)
            k = torch.zeros_like(mid)
            for b in range(6, -1, -1):
                k = (k << 2) | (((ty >> b) & 1) << 1) | ((tx >> b) & 1)
            k = torch.where(ok, k, torch.full_like(k, 1 << 20))
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            o = torch.argsort(k).to(torch.int32)
            t1.record()
            torch.cuda.synchronize()
            t_sort += t0.elapsed_time(t1)
            orders.append(o)
        for pad in (0, 40 * 1024, 80 * 1024):
            acc = torch.empty(P, dtype=torch.float64, device="cuda")

            def run():
                for (j0, j1), o in zip(segs, orders):
                    gen(j0, j1, o, acc, pad)
            ms = timed(run)
            same = bool(torch.equal(acc, accg))
            print(f"generated L={L:2d} ({len(segs)} launches) lds_pad={pad // 1024:3d} KiB: "
                  f"{ms:.3f} ms; torch argsort of the keys {t_sort:.3f} ms; sums equal: {same}",
                  flush=True)


if __name__ == "__main__":
    main()
