#!/usr/bin/env python3
"""Record-layout probe (GPU box): does a blocked raster layout, or a smaller record, raise the
L2 reuse of K2s's segment-sorted gathers?  cfg3's real cells (uam_eval_generated's `cells`),
two segments of 41 waypoints each sorted on the 16x16-cell tile under the segment's middle
waypoint (K2s's key), an 80 KiB LDS floor (K2s's two workgroups per CU).  The cell index of
every waypoint is remapped on the device to the layout under test:

  rowmajor       the product layout, [ny][nx]
  blk{h}x{w}     h x w cells per contiguous block (h*w*rec bytes), blocks row-major
  tile{T}/{h}x{w} T x T cell tiles row-major, h x w blocks row-major inside a tile

and gathered from a 16-B or an 8-B record table, keeping a per-path f64 sum in waypoint
order (the sums must equal the row-major 16-B sums bit for bit: every layout gathers the
same records).  A measurement tool, not a product kernel.
usage: python tools/probe_layout.py [--pairs 100000]"""
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
    ap.add_argument("--reps", type=int, default=10)
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
    for f in (lib.probe_seg, lib.probe_seg8):
        f.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int64, vp,
                      ctypes.c_int, vp]
    spec = canonical_spec(nfz_polygons=CONFIGS["cfg3"]["nfz_polygons"])
    e = Engine(0)
    e.set_geometry(compile_map(build_region_map(spec)))
    e.set_params(canonical_params(spec, N=80, altitude=320.0))
    R = 4096
    geo = raster_geo(R)
    raster = e.raster_build(geo, synthetic_dem(R))
    pairs = e.tensor(random_pairs(a.pairs, seed=0), torch.float64)
    D, W = 5, 82
    ut = arc_table(80, displacements(D))
    g = e.eval_generated(pairs, ut, raster=raster, want_cells=True)
    cells = g["cells"].contiguous()
    P = cells.shape[0]
    rec16 = raster.rec.contiguous().view(torch.int32).view(-1, 4)     # [R*R][4]
    stream = vp(torch.cuda.current_stream().cuda_stream)

    def ptr(t):
        return vp(t.data_ptr())

    # K2s's segments and keys: 2 segments, 16x16 tile Morton key of the middle waypoint
    L = 41
    segs = [(j0, min(W, j0 + L)) for j0 in range(0, W, L)]
    orders = []
    for j0, j1 in segs:
        mid = cells[:, (j0 + j1 - 1) // 2].long()
        ok = mid >= 0
        iy, ix = torch.div(mid, R, rounding_mode="floor"), mid % R
        ty, tx = (iy // 16).clamp(min=0), (ix // 16).clamp(min=0)
        k = torch.zeros_like(mid)
        for b in range(7, -1, -1):
            k = (k << 2) | (((ty >> b) & 1) << 1) | ((tx >> b) & 1)
        k = torch.where(ok, k, torch.full_like(k, 1 << 20))
        orders.append(torch.argsort(k, stable=True).to(torch.int32))

    def remap(T, h, w):
        """cell index -> address in a layout of T x T tiles of h x w blocks (T = 0: no tiles)"""
        c = cells.long()
        ok = c >= 0
        iy, ix = torch.div(c, R, rounding_mode="floor"), c % R
        if T:
            tile = (iy // T) * (R // T) + ix // T
            ly, lx = iy % T, ix % T
            blk = (ly // h) * (T // w) + lx // w
            adr = tile * (T * T) + blk * (h * w) + (ly % h) * w + lx % w
        else:
            blk = (iy // h) * (R // w) + ix // w
            adr = blk * (h * w) + (iy % h) * w + ix % w
        return torch.where(ok, adr, c).to(torch.int32).contiguous()

    def table(T, h, w, words):
        """the record table in that layout, `words` 4-B words per record"""
        iy = torch.arange(R, device="cuda").view(R, 1).expand(R, R).reshape(-1)
        ix = torch.arange(R, device="cuda").view(1, R).expand(R, R).reshape(-1)
        lin = iy * R + ix
        c = lin
        if T:
            tile = (iy // T) * (R // T) + ix // T
            ly, lx = iy % T, ix % T
            adr = tile * (T * T) + ((ly // h) * (T // w) + lx // w) * (h * w) + (ly % h) * w + lx % w
        else:
            adr = ((iy // h) * (R // w) + ix // w) * (h * w) + (iy % h) * w + ix % w
        t = torch.empty(R * R, words, dtype=torch.int32, device="cuda")
        t[adr] = rec16[c, :words]
        return t.contiguous()

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

    ref = None
    layouts = [("rowmajor", 0, 1, 1)]
    for h, w in ((2, 4), (4, 2), (1, 8)):
        layouts.append((f"blk{h}x{w}", 0, h, w))
    for T, h, w in ((16, 2, 4), (32, 2, 4), (64, 2, 4), (16, 4, 4), (64, 4, 4)):
        layouts.append((f"tile{T}/{h}x{w}", T, h, w))
    for words in (4, 2):
        for name, T, h, w in layouts:
            if words == 4 and (h, w) == (4, 4):
                continue
            if words == 2 and (h, w) == (2, 4) and T == 0:
                pass
            adr = remap(T, h, w) if name != "rowmajor" else cells
            tab = table(T, h, w, words) if name != "rowmajor" or words == 2 else rec16
            fn_ = lib.probe_seg if words == 4 else lib.probe_seg8
            acc = torch.empty(P, dtype=torch.float64, device="cuda")

            def run():
                for (j0, j1), o in zip(segs, orders):
                    fn_(ptr(tab), ptr(adr), W, j0, j1, ptr(o), P, ptr(acc), 80 * 1024, stream)
            ms = timed(run)
            if ref is None:
                ref = acc.clone()
            same = bool(torch.equal(acc, ref))
            print(f"{4 * words:2d}-B records, {name:14s}: {ms:.3f} ms  sums equal: {same}",
                  flush=True)
            del tab
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
