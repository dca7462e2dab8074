"""Randomized parity: configurations drawn from a seed, every output against the oracle bit for
bit.  Each case draws the map (no-fly polygon count and seed, region weights), the options
(length / penalty / obstacle / maxratio smoothing), the enlargement and turn limit, N, the
displacement count, the group length, the kernel-form options (terrain form, chunk length,
sort tile bits, rows per lane) and the batch, then checks one of

  * K1, the raster build (a raster geometry of its own: non-square, offset, any cell size)
    against orc_raster_build -- records, flags and all;
  * the generated raster evaluation -- the sorted forms (K2h, or K2g under maxratio_smooth),
    the form the library picks for the batch size, or the reference's sequential order
    (group 0: K2s / K2 / K2w), waypoint cells on some -- against orc_eval_generated_h /
    orc_eval_paths in the same group order;
  * the generated volume evaluation (K4h, or the sequential K4 when the form draw or the batch
    size selects it) against orc_eval_generated_h in volume mode / orc_eval_paths3d;
  * analytic mode (K3b or the small-batch forms) against the sequential orc_eval_paths.

The default run covers seeds 0-47; UAM_FUZZ_SEEDS=a:b widens it (profiles/r06 records a
long sweep).  Reference rules: as test_gpu_k2h.py / test_gpu_k4h.py / test_gpu_parity.py."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _seeds():
    v = os.environ.get("UAM_FUZZ_SEEDS", "0:48")
    a, b = (int(x) for x in v.split(":"))
    return list(range(a, b))


def _draw(seed):
    rng = np.random.default_rng(1000 + seed)
    c = {}
    c["kind"] = ["raster", "raster", "raster", "k1", "volume", "analytic"][seed % 6]
    c["nfz"] = int(rng.choice([0, 8, 32]))
    c["map_seed"] = int(rng.integers(0, 50))
    c["opts"] = {"length_smooth": bool(rng.integers(0, 2)),
                 "penalty_smooth": bool(rng.integers(0, 2)),
                 "obstacle_smooth": bool(rng.integers(0, 2)),
                 "maxratio_smooth": bool(rng.random() < 0.2) and c["kind"] == "raster"}
    c["enl"] = float(rng.choice([0.0, 0.1, 0.35]))
    c["maxratio"] = float(rng.choice([1.04, 1.25, 2.0]))
    c["maxalpha"] = float(np.pi / rng.choice([5.0, 10.0, 80.0]))
    c["wscale"] = rng.choice([0.0, 1.0, 1.0, 3.7])
    c["N"] = int(rng.choice([1, 2, 7, 40, 80, 120]))
    c["D"] = int(rng.choice([1, 2, 3, 5, 8, 16]))
    c["group"] = int(rng.integers(1, 65))
    c["Q"] = int(rng.integers(60, 3000))
    c["R"] = int(rng.choice([256, 384, 512, 1024]))
    c["terrain"] = int(rng.integers(0, 2))
    c["chunk"] = int(rng.choice([0, 6, 7, 8, 11]))
    c["tbits"] = int(rng.choice([0, 0, 3, 5]))
    c["k1_rows"] = int(rng.choice([1, 2, 4, 8]))
    c["nz"] = int(rng.choice([7, 16, 33]))
    c["geo"] = (int(rng.integers(120, 700)), int(rng.integers(120, 700)),
                float(rng.uniform(-5.0, 20.0)), float(rng.uniform(0.0, 25.0)),
                float(rng.uniform(0.02, 0.4)), float(rng.uniform(0.02, 0.4)))
    c["thr"] = float(rng.choice([0.0, 100.0, -9999.0]))
    c["pair_seed"] = int(rng.integers(0, 1 << 30))
    # raster: the sorted forms forced, the library's own choice by batch size, or the
    # reference's sequential order (group 0); waypoint cells on some
    c["form"] = str(rng.choice(["sorted", "sorted", "auto", "seq"]))
    c["cells"] = bool(rng.random() < 0.3)
    return c


def _setup(oracle_mod, c):
    from uam_path_planning_amd import build
    from uam_path_planning_amd.engine import Engine, PathParams
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import build_region_map, canonical_spec

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    build.build_library()
    e = Engine(0)
    e.set_option("group", 0 if c["form"] == "seq" else c["group"])
    if c["form"] != "auto":
        e.set_option("sorted_min_paths", 0)
        e.set_option("wave_max_paths", 0)
    e.set_option("k2h_terrain", c["terrain"])
    e.set_option("k4h_terrain", c["terrain"])
    e.set_option("k2g_chunk", c["chunk"])
    e.set_option("k2g_tile_bits", c["tbits"])
    e.set_option("k1_rows", c["k1_rows"])
    spec = canonical_spec(nfz_polygons=c["nfz"], seed=c["map_seed"])
    w = [float(x) * c["wscale"] for x in spec["weights"]]
    e.set_geometry(compile_map(build_region_map(spec)))
    e.set_params(PathParams(N=c["N"], **c["opts"], maxratio=c["maxratio"],
                            maxalpha=c["maxalpha"], enlargement=c["enl"], weights=tuple(w),
                            altitude=320.0))
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), c["N"], c["opts"], c["maxratio"],
                            c["maxalpha"], c["enl"], w, altitude=320.0)
    return e, orc


def _pairs(c, n3=False):
    from uam_path_planning_amd.synthetic import random_pairs, random_pairs3d

    if n3:
        pr = random_pairs3d(c["Q"], seed=c["pair_seed"])
        pr[::41, 2] = -50.0
        pr[::43, 5] = 900.0
        pr[::97, 0] += 70.0
        pr[min(11, c["Q"] - 1), 3:5] = pr[min(11, c["Q"] - 1), 0:2]
        return pr
    pr = random_pairs(c["Q"], seed=c["pair_seed"])
    pr[::97, 0] += 70.0
    pr[min(5, c["Q"] - 1), 1] = np.nan
    pr[min(11, c["Q"] - 1), 2:] = pr[min(11, c["Q"] - 1), :2]
    return pr


def _eq(gpu, ref, keys):
    for gk, ok in keys:
        np.testing.assert_array_equal(gpu[gk].cpu().numpy(), ref[ok], err_msg=gk)


KEYS = (("cost", "cost"), ("length_q", "lq"), ("length", "length"), ("kin_sum", "kin"),
        ("nfz_sum", "nfz"), ("nfz_hits", "nfz_hits"), ("offmap", "offmap"),
        ("min_clearance", "min_clearance"))


def _selection(gpu, ref, oracle_mod, D):
    np.testing.assert_array_equal(gpu["best_fval_idx"].cpu().numpy(),
                                  oracle_mod.argmin(ref["cost"], D, True))
    np.testing.assert_array_equal(gpu["best_length_idx"].cpu().numpy(),
                                  oracle_mod.argmin(ref["length"], D, False))


@pytest.mark.parametrize("seed", _seeds())
def test_fuzz_parity(oracle_mod, seed):
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import RasterGeo
    from uam_path_planning_amd.scenario import displacements, layer_weights, raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    c = _draw(seed)
    e, orc = _setup(oracle_mod, c)
    D, N = c["D"], c["N"]
    ut = arc_table(N, displacements(D))
    if c["kind"] == "k1":
        nx, ny, x0, yt, dx, dy = c["geo"]
        geo = RasterGeo(nx=nx, ny=ny, x0=x0, y_top=yt, dx=dx, dy=dy, nodata=-9999.0,
                        dem_threshold=c["thr"])
        dem = synthetic_dem(max(nx, ny))[:ny, :nx].copy()
        rec = e.raster_build(geo, dem, summary=False).rec.cpu().numpy()
        ref = orc.raster_build(oracle_mod.Oracle.raster_desc(nx, ny, x0, yt, dx, dy, -9999.0,
                                                             c["thr"]), dem)
        np.testing.assert_array_equal(rec, ref.view(np.int32))
        return
    if c["kind"] == "analytic":
        pairs = _pairs(c)
        gpu = e.eval_generated(pairs, ut, raster=None)
        ref = orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="analytic")
        _eq(gpu, ref, KEYS[:6])
        _selection(gpu, ref, oracle_mod, D)
        return
    if c["kind"] == "volume":
        R = min(c["R"], 512)
        geo = raster_geo(R)
        r2 = e.raster_build(geo, synthetic_dem(R))
        vol = e.volume_build(r2, c["nz"], 0.0, 640.0 / c["nz"], layer_weights(c["nz"]))
        e.volume_pack(vol)
        vd = oracle_mod.volume_desc(R, R, c["nz"], geo.x0, geo.y_top, geo.dx, geo.dy, 0.0,
                                    640.0 / c["nz"])
        host = (vol.vox.cpu().numpy().view(np.float32),
                vol.cols.cpu().numpy().view(np.float32))
        pairs = _pairs(c, n3=True)
        gpu = e.eval_generated3d(pairs, ut, vol)
        g, k = e.last_group(), e.last_kernel()
        if c["form"] == "sorted":
            assert k == "K4h+pack"
        if k.startswith("K4h"):
            ref = orc.eval_generated_h(pairs, ut, mode="volume", vdesc=vd, vol=host, group=g)
        else:   # the sequential lane-per-path K4
            assert g == 0, k
            ref = orc.eval_paths3d(oracle_mod.gen_paths3d(pairs, ut), vd, host)
        _eq(gpu, ref, KEYS + (("below_terrain", "below"),))
        _selection(gpu, ref, oracle_mod, D)
        return
    geo = raster_geo(c["R"])
    raster = e.raster_build(geo, synthetic_dem(c["R"]), summary=False)
    e.raster_summary(raster, 0, packed=True)
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy,
                                       geo.nodata, geo.dem_threshold)
    rec = raster.rec.cpu().numpy().view(np.float32)
    pairs = _pairs(c)
    gpu = e.eval_generated(pairs, ut, raster=raster, want_cells=c["cells"])
    g, k = e.last_group(), e.last_kernel()
    if c["form"] == "seq":
        assert g == 0
    elif c["form"] == "sorted" and not c["opts"]["maxratio_smooth"]:
        assert k == "K2h+pack"
    if k.startswith("K2h"):
        ref = orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=g,
                                   want_cells=c["cells"])
    else:   # K2g (maxratio_smooth) in group order, or a sequential-order form (group 0)
        ref = orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="raster", rdesc=rd,
                             rec=rec, group=g, want_cells=c["cells"])
    _eq(gpu, ref, KEYS + ((("cells", "cells"),) if c["cells"] else ()))
    _selection(gpu, ref, oracle_mod, D)
