#!/usr/bin/env python3
"""CPU model for the Phi-only plane with exact terrain bounds (round-5 design probe; no GPU).

K2h gathers one 8-B {Phi, terrain} entry per waypoint (16 cells per 128-B line).  Terrain only
feeds the order-free path maximum, so it can leave the per-waypoint gather: a 4-B Phi plane
(32 cells per line) plus a per-block terrain bound table {ub, lb}; an item fetches the exact
terrain (from a 4-B terrain plane) only for a waypoint whose bound could still be the group's
maximum.  This script counts, on cfg3's real items and raster:

* the share of waypoints per block code (0 nothing / 1 Phi plane / 3 full record) under the
  old rule (terrain in the code) and the new one (terrain out of it);
* the exact-terrain fetches per waypoint for bound blocks of 8..64 cells, u8-quantised bounds,
  the ideal rule (group maximum of the lower bounds known up front) and the chunked rule the
  kernel can run (running bounds chunk by chunk, CH waypoints a chunk);
* the modelled L2 misses per step (tools/sim_l2.c, 4 MiB 16-way per XCD, 32k items resident per
  XCD, the hilbert5 sort) for the K2h layout and the new one.

usage: python tools/sim_terrain_bound.py [--R 4096] [--pairs 100000] [--bt 16,32,64] [--ch 7]
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
sys.path.insert(0, os.path.join(ROOT, "tools"))

from sim_l2 import hilbert_index  # noqa: E402

NONE = np.uint32(0xFFFFFFFF)


def build_raster(R):
    cache = f"/tmp/sim_rec_{R}.npy"
    if os.path.exists(cache):
        return np.load(cache)
    from oracle import oracle as O
    from uam_path_planning_amd.scenario import canonical_spec, raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem
    O.build()
    geo = raster_geo(R)
    spec = canonical_spec(nfz_polygons=64)
    orc = O.Oracle(O.compile_spec(spec), 80, spec["options"], spec["maxratio"],
                   spec["maxalpha"], spec["enlargement"], spec["weights"], altitude=320.0)
    rd = O.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy, geo.nodata,
                              geo.dem_threshold)
    t0 = time.time()
    rec = orc.raster_build(rd, synthetic_dem(R))
    print(f"raster built in {time.time() - t0:.0f} s", flush=True)
    np.save(cache, rec)
    return rec


def block_any(v, B):
    n = v.shape[0] // B
    return v.reshape(n, B, n, B).any(axis=(1, 3))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=4096)
    ap.add_argument("--pairs", type=int, default=100000)
    ap.add_argument("--G", type=int, default=21)
    ap.add_argument("--ch", type=int, default=7)
    ap.add_argument("--bt", default="8,16,32,64")
    ap.add_argument("--sb", type=int, default=16, help="code-map block (cells)")
    ap.add_argument("--window", type=int, default=32768)
    ap.add_argument("--tbits", type=int, default=5)
    ap.add_argument("--no-l2", action="store_true")
    ap.add_argument("--p8", action="store_true",
                    help="code-3 blocks read 8-B {phi, psi|flag} entries (4x4 cells per line) "
                         "instead of 16-B records; their terrain through the bounds too")
    ap.add_argument("--quant", default="exact,u8")
    ap.add_argument("--samples", default="", help="path lower-bound sample strides, e.g. 8,4,0")
    ap.add_argument("--lag", type=int, default=0,
                    help="chunks between a chunk's issue and its consume (1: the one-ahead "
                         "pipeline: chunk c's fetch rule sees E up to chunk c - 2)")
    ap.add_argument("--use-sampled", action="store_true",
                    help="the L2 model uses the last --samples rule's fetches")
    a = ap.parse_args()
    a.samples = [int(v) for v in a.samples.split(",") if v != ""]

    from oracle import oracle as O
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements, raster_geo
    from uam_path_planning_amd.synthetic import random_pairs

    R, N, D, G, CH = a.R, 80, 5, a.G, a.ch
    W = N + 2
    geo = raster_geo(R)
    rec = build_raster(R)
    bits = rec.view(np.uint32)
    nod = (bits[..., 3] & 4) != 0
    ter = np.where(nod, np.float32(0), rec[..., 2]).astype(np.float32)
    phi_nz = (bits[..., 0] & 0x7FFFFFFF) != 0
    need3 = ((bits[..., 1] & 0x7FFFFFFF) != 0) | ((bits[..., 3] & 1) != 0)
    SB = a.sb
    c3 = block_any(need3, SB)
    code_new = np.where(c3, 3, np.where(block_any(phi_nz, SB), 1, 0)).astype(np.uint8)
    code_old = np.where(c3, 3, np.where(block_any(phi_nz | (ter != 0), SB), 1, 0)).astype(np.uint8)
    tmin, tmax = float(ter.min()), float(ter.max())
    print(f"R={R}: terrain [{tmin:.2f}, {tmax:.2f}]; cells phi!=0 {phi_nz.mean():.3f}, "
          f"terrain!=0 {(ter != 0).mean():.3f}", flush=True)

    O.build()
    wp = O.gen_paths(random_pairs(a.pairs, seed=0), arc_table(N, displacements(D)))
    wp = wp.reshape(-1, W, 2)
    P = wp.shape[0]
    tx = (wp[..., 0] - geo.x0) / geo.dx
    ty = (geo.y_top - wp[..., 1]) / geo.dy
    inr = (tx >= 0) & (tx < R) & (ty >= 0) & (ty < R)
    ix = np.where(inr, tx, 0).astype(np.int64)
    iy = np.where(inr, ty, 0).astype(np.int64)
    del wp, tx, ty
    cn = np.where(inr, code_new[iy // SB, ix // SB], 0)
    co = np.where(inr, code_old[iy // SB, ix // SB], 0)
    T = np.where(inr, ter[iy, ix], np.float32(0))
    nwp = P * W
    print(f"{P} paths; old codes 0/1/3: {np.mean(co == 0):.3f} {np.mean(co == 1):.3f} "
          f"{np.mean(co == 3):.3f}; new codes: {np.mean(cn == 0):.3f} {np.mean(cn == 1):.3f} "
          f"{np.mean(cn == 3):.3f}", flush=True)

    nseg = (W + G - 1) // G
    Wp = nseg * G  # padded
    results = {}
    for BT in [int(b) for b in a.bt.split(",")]:
        nb = R // BT
        t4 = ter.reshape(nb, BT, nb, BT)
        ub = t4.max(axis=(1, 3)).astype(np.float64)
        lb = t4.min(axis=(1, 3)).astype(np.float64)
        step = (tmax - tmin) / 254.0
        for quant in a.quant.split(","):
            if quant == "f16":  # outward-rounded binary16
                u16 = ub.astype(np.float16)
                u16 = np.where(u16.astype(np.float64) < ub, np.nextafter(u16, np.float16(np.inf)), u16)
                l16 = lb.astype(np.float16)
                l16 = np.where(l16.astype(np.float64) > lb, np.nextafter(l16, np.float16(-np.inf)), l16)
                ubq, lbq = u16.astype(np.float64), l16.astype(np.float64)
            elif quant.startswith("rel"):  # relN:S -- N-bit codes over S x S-cell superblocks
                nbits, ssz = (int(v) for v in quant[3:].split(":"))
                k = ssz // BT
                ns = nb // k
                base = lb.reshape(ns, k, ns, k).min(axis=(1, 3))
                top = ub.reshape(ns, k, ns, k).max(axis=(1, 3))
                rng = np.maximum(top - base, 1e-30)
                step = 2.0 ** np.ceil(np.log2(rng / (2 ** nbits - 1)))  # a power of two
                bb = np.repeat(np.repeat(base, k, 0), k, 1)
                st = np.repeat(np.repeat(step, k, 0), k, 1)
                ubq = bb + np.ceil((ub - bb) / st) * st
                lbq = bb + np.floor((lb - bb) / st) * st
                assert (np.ceil((ub - bb) / st) <= 2 ** nbits - 1).all()
            elif quant == "u8":
                ubq = tmin + np.ceil((ub - tmin) / step) * step
                lbq = tmin + np.floor((lb - tmin) / step) * step
            else:
                ubq, lbq = ub, lb
            u = np.where(inr, ubq[iy // BT, ix // BT], 0.0)
            l_ = np.where(inr, lbq[iy // BT, ix // BT], 0.0)
            # known at issue time: off the raster, a constant block; with --p8 the code-3
            # records carry no terrain (8-B {phi, psi|flag} entries), else they do
            known = (~inr) | (u == l_) | ((cn == 3) & (not a.p8))
            # exact-known waypoints: their bounds are their value
            Tv = T.astype(np.float64)
            u = np.where(known, Tv, u)
            l_ = np.where(known, Tv, l_)
            pad = lambda v, fill: np.concatenate(
                [v, np.full((P, Wp - W), fill, v.dtype)], axis=1).reshape(P, nseg, G)
            U, L, K, TT = pad(u, -np.inf), pad(l_, -np.inf), pad(known, True), pad(Tv, -np.inf)
            # ideal: the group's maximum lower bound up front
            Lb = L.max(axis=2, keepdims=True)
            E = np.where(K, TT, -np.inf).max(axis=2, keepdims=True)
            f_ideal = (~K) & (U > E) & (U >= Lb)
            # chunked: bounds known chunk by chunk
            fch = np.zeros_like(K)
            Lrun = np.full((P, nseg, 1), -np.inf)
            Erun = np.full((P, nseg, 1), -np.inf)
            for c0 in range(0, G, CH):
                sl = slice(c0, min(G, c0 + CH))
                Lrun = np.maximum(Lrun, L[:, :, sl].max(axis=2, keepdims=True))
                Ec = np.maximum(Erun, np.where(K[:, :, sl], TT[:, :, sl], -np.inf)
                                .max(axis=2, keepdims=True))
                f = (~K[:, :, sl]) & (U[:, :, sl] > Ec) & (U[:, :, sl] >= Lrun)
                fch[:, :, sl] = f
                Erun = np.maximum(Ec, np.where(f, TT[:, :, sl], -np.inf).max(axis=2, keepdims=True))
            # sanity: the fetched + known set holds the group's exact maximum
            got = np.where(K | fch, TT, -np.inf).max(axis=2)
            assert np.array_equal(got, TT.max(axis=2)), "bound rule lost the maximum"
            fi = f_ideal.reshape(P, Wp)[:, :W]
            fc = fch.reshape(P, Wp)[:, :W]
            # path-level lower bounds: the maximum lb over every s-th waypoint of the whole path
            # (computed by the item from the unit-arc table, no memory request) seeds the chunked
            # rule's running bound
            for s_ in a.samples:
                lbp = l_[:, ::s_].max(axis=1) if s_ > 0 else l_.max(axis=1)
                Lrun = np.broadcast_to(lbp[:, None, None], (P, nseg, 1)).copy()
                Erun = np.full((P, nseg, 1), -np.inf)
                fs = np.zeros_like(K)
                pend = []  # fetched maxima not yet consumed (the pipeline's lag)
                for c0 in range(0, G, CH):
                    sl = slice(c0, min(G, c0 + CH))
                    Lrun = np.maximum(Lrun, L[:, :, sl].max(axis=2, keepdims=True))
                    Ec = np.maximum(Erun, np.where(K[:, :, sl], TT[:, :, sl], -np.inf)
                                    .max(axis=2, keepdims=True))
                    f = (~K[:, :, sl]) & (U[:, :, sl] > Ec) & (U[:, :, sl] >= Lrun)
                    fs[:, :, sl] = f
                    Erun = Ec
                    pend.append(np.where(f, TT[:, :, sl], -np.inf).max(axis=2, keepdims=True))
                    while len(pend) > a.lag:
                        Erun = np.maximum(Erun, pend.pop(0))
                print(f"    + path lower bound from every {s_ if s_ else 1}th waypoint: "
                      f"chunked fetches per waypoint {fs.reshape(P, Wp)[:, :W].mean():.4f}",
                      flush=True)
                if s_ == a.samples[-1] and a.use_sampled:
                    fc = fs.reshape(P, Wp)[:, :W]
            print(f"  bounds {BT:2d}^2 cells {quant:5s}: table {nb * nb} blocks; exact fetches "
                  f"per waypoint ideal {fi.mean():.4f}, chunked(CH={CH}) {fc.mean():.4f}; "
                  f"per group {fc.sum() / (P * nseg):.2f}", flush=True)
            results[(BT, quant)] = fc
    if a.no_l2:
        return

    so = "/tmp/libsiml2.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so,
                    os.path.join(ROOT, "tools", "sim_l2.c")], check=True)
    lib = ctypes.CDLL(so)
    lib.sim_lru.restype = ctypes.c_int64
    lib.sim_lru.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
    # line ids (disjoint ranges): the 8-B plane in 4x4 blocks, 16-B records row-major (1x8),
    # the 4-B Phi plane and the 4-B terrain plane in 4x8 blocks
    rec_line = (np.uint64(1) << np.uint64(28)) + (iy * (R // 8) + ix // 8).astype(np.uint64)
    p8_line = ((iy >> 2) * (R >> 2) + (ix >> 2)).astype(np.uint64)
    p4_line = (np.uint64(2) << np.uint64(28)) + ((iy >> 2) * (R >> 3) + (ix >> 3)).astype(np.uint64)
    t4_line = (np.uint64(3) << np.uint64(28)) + ((iy >> 2) * (R >> 3) + (ix >> 3)).astype(np.uint64)
    k2h = np.where(co == 3, rec_line, np.where(co == 1, p8_line, NONE)).astype(np.uint32)
    if a.p8:
        rec_line = (np.uint64(1) << np.uint64(28)) + ((iy >> 2) * (R >> 2) + (ix >> 2)).astype(np.uint64)
    phi4 = np.where(cn == 3, rec_line, np.where(cn == 1, p4_line, NONE)).astype(np.uint32)
    del rec_line, p8_line, p4_line

    items_p = np.repeat(np.arange(P), nseg)
    items_s = np.tile(np.arange(nseg), P)
    j0 = items_s * G
    j1 = np.minimum(j0 + G, W)
    mid = (j0 + j1 - 1) // 2
    mx, my, mi = ix[items_p, mid], iy[items_p, mid], inr[items_p, mid]
    last = (items_s == nseg - 1) & (W % G != 0)
    tb = a.tbits
    sh = int(np.log2(R)) - tb
    k = hilbert_index(tb, mx >> sh, my >> sh)
    k = np.where(mi, k + (last << (2 * tb)), 1 << (2 * tb + 1))
    perm = np.argsort(k, kind="stable")

    def misses(streams):
        n = perm.size
        nbk = (n + 255) // 256
        total, reqs = 0, 0
        for x in range(8):
            c0 = x * (nbk >> 3) + min(x, nbk & 7)
            c1 = c0 + (nbk >> 3) + (1 if x < (nbk & 7) else 0)
            its = perm[c0 * 256:min(c1 * 256, n)]
            out = []
            for w0 in range(0, its.size, a.window):
                win = its[w0:w0 + a.window]
                p, s0 = items_p[win], j0[win]
                Ln = j1[win] - s0
                for t in range(G):
                    ok = t < Ln
                    for s in streams:
                        out.append(s[p[ok], s0[ok] + t])
            st = np.ascontiguousarray(np.concatenate(out))
            reqs += int((st != NONE).sum())
            total += lib.sim_lru(st.ctypes.data, st.size, 2048, 16)
        return total, reqs

    m, r = misses([k2h])
    print(f"K2h layout (8-B plane, old codes): {m / 1e6:.2f}M misses, {r / 1e6:.2f}M requests",
          flush=True)
    m, r = misses([phi4])
    print(f"4-B Phi plane, new codes, no terrain: {m / 1e6:.2f}M misses, {r / 1e6:.2f}M requests",
          flush=True)
    for (BT, quant), fc in results.items():
        tl = np.where(fc, t4_line, NONE).astype(np.uint32)
        m, r = misses([phi4, tl])
        print(f"4-B Phi + terrain fetches (bounds {BT}^2 {quant}): {m / 1e6:.2f}M misses, "
              f"{r / 1e6:.2f}M requests", flush=True)


if __name__ == "__main__":
    main()
