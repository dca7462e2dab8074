"""Loaders for the committed golden fixtures (tests/golden/*, made by make_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def canonical():
    with open(os.path.join(GOLDEN, "canonical.json")) as f:
        meta = json.load(f)
    arr = dict(np.load(os.path.join(GOLDEN, "canonical.npz")))
    return meta, arr


def canonical_paths(meta, arr):
    xs = np.asarray(meta["map"]["x_start"], float)
    xg = np.asarray(meta["map"]["x_goal"], float)
    return np.stack([np.concatenate([xs, x, xg]).reshape(-1, 2) for x in arr["x_init"]])


def variants():
    return dict(np.load(os.path.join(GOLDEN, "variants.npz")))


def random_cases():
    with open(os.path.join(GOLDEN, "random_cases.json")) as f:
        return json.load(f)["cases"]


def arcs():
    return dict(np.load(os.path.join(GOLDEN, "arcs.npz")))


def grid():
    return dict(np.load(os.path.join(GOLDEN, "grid.npz")))


def errors():
    with open(os.path.join(GOLDEN, "errors.json")) as f:
        return {c["case"]: c for c in json.load(f)}


def waypoint_cells():
    """waypoint_cells.npz: pairs [Q, 4], displacements [D], N, and for R in (4096, 8192) the
    raster cell (iy * R + ix, -1 off the raster) of every waypoint of Solver.create_x_init's
    own paths, [Q * D, N + 2] int32 (stored as int16 differences of ix / iy along each path)."""
    a = dict(np.load(os.path.join(GOLDEN, "waypoint_cells.npz")))
    out = {"pairs": a["pairs"], "displacements": a["displacements"], "N": int(a["N"])}
    for R in (4096, 8192):
        ix = np.cumsum(a[f"dix{R}"].astype(np.int32), axis=1)
        iy = np.cumsum(a[f"diy{R}"].astype(np.int32), axis=1)
        out[f"cells{R}"] = np.where(ix >= 0, iy * R + ix, -1).astype(np.int32)
    return out
