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
