#!/usr/bin/env python3
"""Diagnostic: does a spatial order of the start/goal pairs (and an XCD-aware placement of the
ordered blocks) make the raster kernel K2 (k_eval_pairs<RASTER>) faster on cfg3?

The pairs are permuted on the host, so the kernel itself is unchanged: workgroup b evaluates
pairs [64 b, 64 b + 64) of the permuted array.  Workgroups are dispatched round-robin over the
8 XCDs (b -> XCD b % 8); the "xcd" placement gives XCD x a contiguous range of the ordered
chunks, so the paths in flight on one XCD (sharing one 4 MiB L2) are spatial neighbours.
Results are un-permuted and compared bit for bit with the unordered launch.
Prints one JSON line per order."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def spread(v, bits, stride):
    out = np.zeros_like(v, dtype=np.uint64)
    for b in range(bits):
        out |= ((v >> np.uint64(b)) & np.uint64(1)) << np.uint64(b * stride)
    return out


def quant(x, lo, hi, bits):
    q = np.floor((x - lo) / (hi - lo) * (1 << bits)).astype(np.int64)
    return np.clip(q, 0, (1 << bits) - 1).astype(np.uint64)


def morton(cols, bits):
    k = np.zeros(len(cols[0]), dtype=np.uint64)
    n = len(cols)
    for i, c in enumerate(cols):  # cols[0] gets the most significant bit of each group
        k |= spread(c, bits, n) << np.uint64(n - 1 - i)
    return k


def xcd_chunks(nb, n_xcd=8):
    """chunk index processed by block b when XCD x = b % n_xcd owns a contiguous chunk range"""
    counts = [len(range(x, nb, n_xcd)) for x in range(n_xcd)]
    start = np.concatenate([[0], np.cumsum(counts)[:-1]])
    b = np.arange(nb)
    return start[b % n_xcd] + b // n_xcd


def timed(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=99_968)  # a multiple of 64 (whole blocks)
    ap.add_argument("--R", type=int, default=4096)
    ap.add_argument("--bits", type=int, default=8)
    args = ap.parse_args()
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (build_region_map, canonical_params,
                                                canonical_spec, displacements, raster_geo)
    from uam_path_planning_amd.synthetic import LAND_BBOX, random_pairs, synthetic_dem

    Q, D = args.pairs, 5
    spec = canonical_spec(nfz_polygons=64)
    eng = Engine(0)
    eng.set_geometry(compile_map(build_region_map(spec)))
    eng.set_params(canonical_params(spec, N=80, altitude=320.0))
    ut = eng.tensor(arc_table(80, displacements(D)), torch.float64)
    raster = eng.raster_build(raster_geo(args.R),
                              eng.tensor(synthetic_dem(args.R), torch.float32))
    host = random_pairs(Q, seed=0)
    x0, x1, y0, y1 = LAND_BBOX
    b = args.bits
    qx0, qy0 = quant(host[:, 0], x0, x1, b), quant(host[:, 1], y0, y1, b)
    qxf, qyf = quant(host[:, 2], x0, x1, b), quant(host[:, 3], y0, y1, b)
    mx, my = quant((host[:, 0] + host[:, 2]) / 2, x0, x1, b), quant((host[:, 1] + host[:, 3]) / 2, y0, y1, b)
    orders = {
        "random": np.arange(Q),
        "morton4_goal_first": np.argsort(morton([qyf, qxf, qy0, qx0], b), kind="stable"),
        "morton4_start_first": np.argsort(morton([qx0, qy0, qxf, qyf], b), kind="stable"),
        "midpoint2": np.argsort(morton([my, mx], b), kind="stable"),
        "start2": np.argsort(morton([qy0, qx0], b), kind="stable"),
    }
    nb = Q // 64
    remap = xcd_chunks(nb)
    P = Q * D
    outs = eng.outputs(P, 82, n_pairs=Q)
    ref = None
    for name, perm in orders.items():
        for place in ("rr", "xcd"):
            if name == "random" and place == "xcd":
                continue
            p = perm.copy()
            if place == "xcd":
                p = p.reshape(nb, 64)[remap].reshape(-1)
            pairs = eng.tensor(host[p], torch.float64)
            med, best = timed(lambda: eng.eval_generated(pairs, ut, raster=raster,
                                                         outputs=outs))
            cost = outs[0]["cost"].cpu().numpy().reshape(Q, D)
            back = np.empty_like(cost)
            back[p] = cost
            if ref is None:
                ref = back
            same = bool(np.array_equal(back.view(np.uint64), ref.view(np.uint64)))
            print(json.dumps({"probe": "raster_order", "order": name, "placement": place,
                              "R": args.R, "pairs": Q, "kernel_ms_med": round(med, 4),
                              "kernel_ms_best": round(best, 4),
                              "paths_per_s": round(P / (med * 1e-3), 1),
                              "identical_to_random": same}), flush=True)


if __name__ == "__main__":
    main()
