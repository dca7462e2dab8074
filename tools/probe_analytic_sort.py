"""Does a spatial order of the pairs cut K3's (analytic mode) divergence?  Times
eval_generated in analytic mode on the cfg3 pairs in their random order and in a Morton order
of (x0, y0, xf, yf), and checks that the un-permuted outputs are identical (each path is
computed on its own, so the order cannot change a bit).
usage: python tools/probe_analytic_sort.py [--pairs 100000] [--reps 5]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402


def morton4(p, bits=8):
    lo, hi = p.min(0), p.max(0)
    q = ((p - lo) / np.maximum(hi - lo, 1e-12) * (2**bits - 1)).astype(np.uint64)
    key = np.zeros(len(p), np.uint64)
    for b in range(bits):
        for d in range(4):
            key |= ((q[:, d] >> np.uint64(b)) & np.uint64(1)) << np.uint64(4 * b + d)
    return key


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (CONFIGS, build_region_map, canonical_params,
                                                canonical_spec, displacements)
    from uam_path_planning_amd.synthetic import random_pairs

    cfg = CONFIGS["cfg3"]
    N, D = cfg["N"], cfg["D"]
    spec = canonical_spec(nfz_polygons=cfg["nfz_polygons"])
    eng = Engine(0)
    eng.set_geometry(compile_map(build_region_map(spec)))
    eng.set_params(canonical_params(spec, N=N, altitude=320.0))
    ut = eng.tensor(arc_table(N, displacements(D)), torch.float64)
    host = random_pairs(a.pairs, seed=0)
    order = np.argsort(morton4(host), kind="stable")
    # 4 bits per coordinate, ties in random order (what a 16-bit counting sort gives)
    rp = np.random.default_rng(1).permutation(len(host))
    o16 = rp[np.argsort(morton4(host[rp], bits=4), kind="stable")]
    # the device's key: shared x / y extents, x0 the most significant coordinate
    xs, ys = host[:, [0, 2]], host[:, [1, 3]]
    nx_ = (host[:, [0, 2]] - xs.min()) / (xs.max() - xs.min())
    ny_ = (host[:, [1, 3]] - ys.min()) / (ys.max() - ys.min())
    dev = np.stack([ny_[:, 1], nx_[:, 1], ny_[:, 0], nx_[:, 0]], 1)
    odev = rp[np.argsort(morton4(dev[rp], bits=4), kind="stable")]
    res = {}
    for name, arr in (("random", host), ("morton", host[order]), ("morton16", host[o16]),
                      ("device16", host[odev])):
        pairs = eng.tensor(np.ascontiguousarray(arr), torch.float64)
        out = eng.eval_generated(pairs, ut)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            out = eng.eval_generated(pairs, ut)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        res[name] = {k: v.cpu().numpy().copy() for k, v in out.items()
                     if isinstance(v, torch.Tensor)}
        print(f"{name}: {ms:.3f} ms per launch, {a.pairs * D / ms * 1e3:.3e} paths/s", flush=True)
    # un-permute the sorted run: pair order[i] was evaluated at position i
    inv = np.empty_like(order)
    inv[order] = np.arange(len(order))
    same = True
    for k, v in res["random"].items():
        w = res["morton"][k]
        if v.shape[0] == a.pairs * D:
            w = w.reshape(a.pairs, D, *w.shape[1:])[inv].reshape(v.shape)
        elif v.shape[0] == a.pairs:
            w = w[inv]
        else:
            continue
        eq = np.array_equal(v.view(np.uint8), w.view(np.uint8))
        same &= eq
        print(f"  {k}: identical={eq}")
    print("all identical:", same)


if __name__ == "__main__":
    main()
