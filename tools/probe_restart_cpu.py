#!/usr/bin/env python3
"""K6 restart probe on the CPU oracle (orc_refine): cfg3 map (5 balls, the reference polygon,
64 random polygons; N = 80), random pairs whose endpoints lie outside every no-fly shape, the 5
reference displacements per pair; the share of candidates (and of pairs' best candidates)
reaching sum g^2 <= 1e-3, with 0 and with n restarts (oracle refine_restart: the obstacle
holding most interior waypoints has them moved across the chord normal past its boundary).
usage: python tools/probe_restart_cpu.py [--pairs 40] [--restarts 0,2] [--margin 0.05]"""
import argparse
import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N = 80


def _setup():
    from oracle import oracle as O

    from uam_path_planning_amd.scenario import canonical_spec

    spec = canonical_spec(nfz_polygons=64)
    orc = O.Oracle(O.compile_spec(spec), N, spec["options"], spec["maxratio"], spec["maxalpha"],
                   spec["enlargement"], spec["weights"], anchor=tuple(spec["x_start"]))
    return O, orc


def work(args):
    wp, nres, margin, outer = args
    O, orc = _setup()
    rp = O.refine_params(n_restart=nres, restart_margin=margin, n_outer=outer)
    return orc.refine(wp, rp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=40)
    ap.add_argument("--restarts", default="0,2")
    ap.add_argument("--margin", type=float, default=0.05)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--outer", type=int, default=15)
    a = ap.parse_args()
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements
    from uam_path_planning_amd.synthetic import random_pairs

    O, orc = _setup()
    pairs = random_pairs(20 * a.pairs, seed=3)
    pts = orc.eval_points(pairs.reshape(-1, 2))
    ok = ((pts["psi_raw"] == 0) & (pts["collide"] == 0)).reshape(-1, 2).all(axis=1)
    pairs = pairs[ok][: a.pairs]
    ut = arc_table(N, displacements(5))
    wp0 = O.gen_paths(pairs, ut).reshape(-1, N + 2, 2)
    chunks = np.array_split(np.arange(wp0.shape[0]), a.procs * 2)
    for nres in [int(x) for x in a.restarts.split(",")]:
        t = time.time()
        with Pool(a.procs) as pool:
            res = pool.map(work, [(wp0[c].copy(), nres, a.margin, a.outer) for c in chunks])
        inf = np.concatenate([r["infeas"] for r in res])
        best = inf.reshape(-1, 5).min(axis=1)
        print(json.dumps({"restarts": nres, "margin": a.margin, "n_outer": a.outer,
                          "candidates": int(inf.size),
                          "share_candidates_le_1e-3": round(float((inf <= 1e-3).mean()), 4),
                          "share_candidates_le_1e-2": round(float((inf <= 1e-2).mean()), 4),
                          "share_pairs_best_le_1e-3": round(float((best <= 1e-3).mean()), 4),
                          "median_infeas": float(np.median(inf)),
                          "steps_mean": float(np.mean(np.concatenate([r["iters"] for r in res]))),
                          "wall_s": round(time.time() - t, 1)}), flush=True)


if __name__ == "__main__":
    main()
