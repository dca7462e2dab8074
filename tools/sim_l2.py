#!/usr/bin/env python3
"""CPU model of K2g's L2 traffic (a design probe; no GPU): cfg3's items (path, group) in the
sorted order a key gives, cut into 256-item workgroups, split over the 8 XCDs as xcd_chunk does,
each XCD running a window of `--window` items at once (waypoint t of every item in the window,
then t + 1, ...), and every gather's 128-B line through a 4 MiB 16-way LRU per XCD
(tools/sim_l2.c).  Lines: plane-A pairs (code-1 blocks, 16 cells per line in 4 x 4 blocks) and
16-B records (code-3 blocks, 8 cells per line); code-0 waypoints issue no request.  Prints the
modelled misses per step for each ordering, to be compared with the PMC's TCC_MISS.

usage: python tools/sim_l2.py [--R 4096] [--pairs 100000] [--groups 21,24] [--orders morton4,hilbert4]
"""
import argparse
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def hilbert_index(n_bits, x, y):
    """Hilbert curve index of (x, y) on a 2^n_bits grid (vectorised)."""
    x = x.astype(np.int64).copy()
    y = y.astype(np.int64).copy()
    d = np.zeros_like(x)
    s = 1 << (n_bits - 1)
    while s > 0:
        rx = ((x & s) > 0).astype(np.int64)
        ry = ((y & s) > 0).astype(np.int64)
        d += s * s * ((3 * rx) ^ ry)
        # rotate
        m = ry == 0
        flip = m & (rx == 1)
        x = np.where(flip, s - 1 - x, x)
        y = np.where(flip, s - 1 - y, y)
        x, y = np.where(m, y, x), np.where(m, x, y)
        s >>= 1
    return d


def morton_index(n_bits, x, y):
    k = np.zeros_like(x, dtype=np.int64)
    for b in range(n_bits - 1, -1, -1):
        k = (k << 2) | (((y >> b) & 1) << 1) | ((x >> b) & 1)
    return k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=4096)
    ap.add_argument("--pairs", type=int, default=100000)
    ap.add_argument("--groups", default="21,24")
    ap.add_argument("--orders", default="morton4,hilbert4,hilbert5,hilbert6")
    ap.add_argument("--window", type=int, default=32768)
    ap.add_argument("--rec-layouts", default="1x8",
                    help="16-B record lines: HxW cells per 128-B line (1x8 = row-major)")
    a = ap.parse_args()
    so = "/tmp/libsiml2.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so,
                    os.path.join(ROOT, "tools", "sim_l2.c")], check=True)
    lib = ctypes.CDLL(so)
    lib.sim_lru.restype = ctypes.c_int64
    lib.sim_lru.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]

    from oracle import oracle as O
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec, displacements, raster_geo
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    R, N, D = a.R, 80, 5
    W = N + 2
    geo = raster_geo(R)
    cache = f"/tmp/sim_l2_codes_{R}.npz"
    if os.path.exists(cache):
        z = np.load(cache)
        code = z["code"]
    else:
        O.build()
        spec = canonical_spec(nfz_polygons=64)
        orc = O.Oracle(O.compile_spec(spec), N, spec["options"], spec["maxratio"],
                       spec["maxalpha"], spec["enlargement"], spec["weights"], altitude=320.0)
        rd = O.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy, geo.nodata,
                                  geo.dem_threshold)
        t0 = time.time()
        rec = orc.raster_build(rd, synthetic_dem(R))
        print(f"raster built in {time.time() - t0:.0f} s", flush=True)
        bits = rec.view(np.uint32)
        ter = np.where((bits[..., 3] & 4) != 0, 0, bits[..., 2])
        B = 16 if R == 4096 else 8
        nb = R // B
        blk = lambda v: v.reshape(nb, B, nb, B)
        needb = (blk(bits[..., 1] & 0x7fffffff) != 0).any(axis=(1, 3)) | \
            (blk(bits[..., 3] & 1) != 0).any(axis=(1, 3))
        nz = (blk(bits[..., 0] & 0x7fffffff) != 0).any(axis=(1, 3)) | (blk(ter) != 0).any(axis=(1, 3))
        code = np.where(needb, 3, np.where(nz, 1, 0)).astype(np.uint8)
        np.savez(cache, code=code)
    B = R // code.shape[0]
    wp = O.gen_paths(random_pairs(a.pairs, seed=0), arc_table(N, displacements(D)))
    wp = wp.reshape(-1, W, 2)
    P = wp.shape[0]
    tx = (wp[..., 0] - geo.x0) / geo.dx
    ty = (geo.y_top - wp[..., 1]) / geo.dy
    inr = (tx >= 0) & (tx < R) & (ty >= 0) & (ty < R)
    ix = np.where(inr, tx, 0).astype(np.int64)
    iy = np.where(inr, ty, 0).astype(np.int64)
    del wp, tx, ty
    c = np.where(inr, code[iy // B, ix // B], 0)
    plane_line = (iy >> 2) * (R >> 2) + (ix >> 2)
    print(f"{P} paths; gathers {np.mean(c != 0):.3f} of waypoints, full {np.mean(c == 3):.3f}",
          flush=True)
    for lay in a.rec_layouts.split(","):
      bh, bw = (int(v) for v in lay.split("x"))
      rec_line = (1 << 22) + (iy // bh) * (R // bw) + ix // bw
      line = np.where(c == 3, rec_line, np.where(c == 1, plane_line, 0xFFFFFFFF)).astype(np.uint32)
      print(f"record lines {lay}", flush=True)
      for G in [int(g) for g in a.groups.split(",")]:
          nseg = (W + G - 1) // G
          items_p = np.repeat(np.arange(P), nseg)
          items_s = np.tile(np.arange(nseg), P)
          j0 = items_s * G
          j1 = np.minimum(j0 + G, W)
          mid = (j0 + j1 - 1) // 2
          mx, my, mi = ix[items_p, mid], iy[items_p, mid], inr[items_p, mid]
          last = (items_s == nseg - 1) & (W % G != 0)
          # the item's direction (its first to last waypoint) in 2^db bins, a minor key
          ex, ey = ix[items_p, j1 - 1] - ix[items_p, j0], iy[items_p, j1 - 1] - iy[items_p, j0]
          ang = (np.arctan2(ey, ex) + np.pi) / (2 * np.pi)
          for order in a.orders.split(","):
              db = 0
              if "d" in order:
                  order_t, db = order.split("d")
                  db = int(db)
              else:
                  order_t = order
              kind, tb = order_t[:-1], int(order_t[-1])
              sh = int(np.log2(R)) - tb
              tx_, ty_ = mx >> sh, my >> sh
              k = hilbert_index(tb, tx_, ty_) if kind == "hilbert" else morton_index(tb, tx_, ty_)
              k = np.where(mi, k + (last << (2 * tb)), 1 << (2 * tb + 1))
              if db:
                  dirb = np.minimum((ang * (1 << db)).astype(np.int64), (1 << db) - 1)
                  k = (k << db) | dirb
              perm = np.argsort(k, kind="stable")
              n = perm.size
              nb = (n + 255) // 256
              total = 0
              for x in range(8):
                  c0 = x * (nb >> 3) + min(x, nb & 7)
                  c1 = c0 + (nb >> 3) + (1 if x < (nb & 7) else 0)
                  its = perm[c0 * 256:min(c1 * 256, n)]
                  stream = []
                  for w0 in range(0, its.size, a.window):
                      win = its[w0:w0 + a.window]
                      p, s0 = items_p[win], j0[win]
                      L = j1[win] - s0
                      for t in range(G):
                          ok = t < L
                          stream.append(line[p[ok], s0[ok] + t])
                  st = np.ascontiguousarray(np.concatenate(stream))
                  total += lib.sim_lru(st.ctypes.data, st.size, 2048, 16)
              print(f"G={G:2d} {order:9s}: modelled L2 misses {total / 1e6:6.2f}M per step "
                    f"({total / max(1, (line != 0xFFFFFFFF).sum()):.3f} per gather)", flush=True)


if __name__ == "__main__":
    main()
