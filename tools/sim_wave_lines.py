#!/usr/bin/env python3
"""Model: distinct 128-B p8 lines per K2h wave instruction (64 items of the sorted order, the
same slot t each) for the cfg3 batch at sort tiles of 2^tbits -- the L1 -> L2 requests per
waypoint the TCP has to hold (profiles/r06: 0.983 / 0.983 / 0.978 at tile bits 4 / 5 / 6;
measured 39.6M requests for 41.0M waypoints).  usage: python tools/sim_wave_lines.py [pairs]"""
import sys, numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from uam_path_planning_amd.arcs import arc_table
from uam_path_planning_amd.scenario import displacements
from uam_path_planning_amd.synthetic import random_pairs

def hilbert_d(bits, x, y):
    n = 1 << bits
    d = np.zeros_like(x, dtype=np.int64)
    x = x.astype(np.int64).copy(); y = y.astype(np.int64).copy()
    s = n >> 1
    while s > 0:
        rx = ((x & s) > 0).astype(np.int64); ry = ((y & s) > 0).astype(np.int64)
        d += s * s * ((3 * rx) ^ ry)
        # rotate
        m = ry == 0
        flip = m & (rx == 1)
        x = np.where(flip, s - 1 - x, x); y = np.where(flip, s - 1 - y, y)
        x2 = np.where(m, y, x); y2 = np.where(m, x, y)
        x, y = x2, y2
        s >>= 1
    return d

Q = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
R = 4096; N = 80; W = 82; G = 21; D = 5
pairs = random_pairs(100000, seed=0)[:Q]
ut = arc_table(N, displacements(D))  # [D][N][2]
P = Q * D
x0 = np.repeat(pairs[:, 0], D); y0 = np.repeat(pairs[:, 1], D)
xf = np.repeat(pairs[:, 2], D); yf = np.repeat(pairs[:, 3], D)
vx, vy = x0 - xf, y0 - yf; cx, cy = (xf + x0) * 0.5, (yf + y0) * 0.5
d = np.tile(np.arange(D), Q)
u = np.concatenate([np.stack([np.ones(D), np.zeros(D)], -1)[:, None], ut,
                    np.stack([-np.ones(D), np.zeros(D)], -1)[:, None]], axis=1)  # [D][W][2]
ux = u[d, :, 0]; uy = u[d, :, 1]
px = cx[:, None] + 0.5 * (vx[:, None] * ux - vy[:, None] * uy)
py = cy[:, None] + 0.5 * (vy[:, None] * ux + vx[:, None] * uy)
px[:, 0], py[:, 0] = x0, y0; px[:, -1], py[:, -1] = xf, yf
ix = np.floor(px * (R / 60.0)).astype(np.int64); iy = np.floor((20.0 - py) * (R / 60.0)).astype(np.int64)
inr = (ix >= 0) & (ix < R) & (iy >= 0) & (iy < R)
line = np.where(inr, (iy // 4) * (R // 4) + ix // 4, -1 - np.arange(P)[:, None] * 0)
nseg = (W + G - 1) // G
for tbits in (4, 5, 6):
    tshift = int(np.log2(R)) - tbits
    keys = []; items = []
    for s_ in range(nseg):
        j0, j1 = s_ * G, min(W, s_ * G + G)
        jm = (j0 + j1 - 1) // 2
        mx, my = ix[:, jm], iy[:, jm]
        ok = inr[:, jm]
        k = hilbert_d(tbits, np.clip(mx, 0, R - 1) >> tshift, np.clip(my, 0, R - 1) >> tshift)
        k = np.where(ok, k + (0 if (s_ < nseg - 1 or W % G == 0) else (1 << 2 * tbits)), 1 << 30)
        keys.append(k); items.append(np.arange(P) * nseg + s_)
    keys = np.concatenate(keys); items = np.concatenate(items)
    order = items[np.argsort(keys, kind='stable')]
    path = order // nseg; seg = order % nseg
    nw = len(order) // 64
    tot_req = 0; tot_wp = 0
    for t in range(G):
        j = seg * G + t
        valid = j < W
        jj = np.minimum(j, W - 1)
        ln = line[path, jj]
        ln = np.where(valid, ln, -2)
        L = ln[: nw * 64].reshape(nw, 64)
        Ls = np.sort(L, axis=1)
        uniq = (np.diff(Ls, axis=1) != 0).sum(1) + 1
        # drop invalid (-2) and off-raster (<0) as not requests
        has_neg = (Ls < 0)
        # count unique nonneg
        nn = np.where(Ls >= 0, Ls, -1)
        u2 = np.array([0])
        tot_req += ((np.diff(nn, axis=1) != 0) & (nn[:, 1:] >= 0)).sum() + (nn[:, 0] >= 0).sum()
        tot_wp += (L >= 0).sum()
    print(f"tbits {tbits}: requests per waypoint {tot_req / tot_wp:.4f}  ({tot_req} / {tot_wp})", flush=True)
