"""BASELINE configs 4 and 5 at their full sizes, through the default kernels (tuning 0).

* cfg4: an 8192^2 synthetic DEM written as 225 x 150 Float32 GeoTIFF tiles in the layout of
  the reference mosaic (data/raw/nagasaki_geotiff/mergeLL.vrt:1-10: one ComplexSource +
  DstRect per tile, nodata -9999) -> DataManager.build_cost_raster (tile mosaic on the device +
  K1; the DEM read of map_generation/data_manager.py:12-17) -> eval_generated on one GPU's
  share of cfg4's 1M paths (25k pairs x 5 displacements = 1M / 8 GPUs).
* cfg5: the 1024 x 1024 x 64 (x, y, altitude) risk volume with 100k pairs x 5.

Checks: K1 records at 20k sampled cells == the oracle's formulas at the cell centres; an
oracle subsample of the paths bit-exact (every float64 output, counts, best indices); the
size-independent properties (pair permutation permutes the outputs bit for bit, a second
launch is bit-identical, argmin consistent with the costs).  Tolerance: exact equality (the
north_star bar is 1e-5 relative on cost, bit-exact on indices)."""
import numpy as np
import pytest

import kernel_ref

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

PATH_KEYS = (("cost", "cost"), ("length_q", "lq"), ("length", "length"), ("kin_sum", "kin"),
             ("nfz_sum", "nfz"), ("nfz_hits", "nfz_hits"), ("offmap", "offmap"),
             ("min_clearance", "min_clearance"))


@pytest.fixture(scope="module")
def eng():
    from uam_path_planning_amd.engine import Engine

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    return Engine(0)


def _np(t):
    return t.cpu().numpy()


def _oracle(oracle_mod, spec, N, altitude):
    return oracle_mod.Oracle(oracle_mod.compile_spec(spec), N, spec["options"],
                             spec["maxratio"], spec["maxalpha"], spec["enlargement"],
                             spec["weights"], altitude=altitude)


def _check_subsample(oracle_mod, gpu, ref, sub, D):
    idx = (sub[:, None] * D + np.arange(D)).reshape(-1)
    for gk, ok in PATH_KEYS:
        np.testing.assert_array_equal(_np(gpu[gk])[idx], ref[ok], err_msg=gk)
    np.testing.assert_array_equal(_np(gpu["best_fval_idx"])[sub],
                                  oracle_mod.argmin(ref["cost"], D, True))
    np.testing.assert_array_equal(_np(gpu["best_length_idx"])[sub],
                                  oracle_mod.argmin(ref["length"], D, False))


def _check_properties(eng, oracle_mod, launch, pairs, gpu, D):
    cost = _np(gpu["cost"])
    assert np.isfinite(cost).all()
    assert (cost >= (eng.params.N + 1) * _np(gpu["length_q"]) - 1e-9).all()
    perm = np.random.default_rng(9).permutation(len(pairs))
    gp = launch(pairs[perm])
    pidx = (perm[:, None] * D + np.arange(D)).reshape(-1)
    for k in ("cost", "nfz_sum", "min_clearance", "nfz_hits"):
        np.testing.assert_array_equal(_np(gp[k]), _np(gpu[k])[pidx], err_msg=k)
    np.testing.assert_array_equal(_np(gp["best_fval_idx"]), _np(gpu["best_fval_idx"])[perm])
    g2 = launch(pairs)
    for k in ("cost", "length", "nfz_sum", "min_clearance", "offmap"):
        np.testing.assert_array_equal(_np(g2[k]), _np(gpu[k]), err_msg=k)
    np.testing.assert_array_equal(_np(gpu["best_fval_idx"]), oracle_mod.argmin(cost, D, True))


def test_cfg4_geotiff_tiles_8192(eng, oracle_mod, tmp_path):
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.distributed import shard_range
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.map_generation import DataManager, write_tiled_dem
    from uam_path_planning_amd.scenario import (CONFIGS, build_region_map, canonical_params,
                                                canonical_spec, displacements, raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    cfg = CONFIGS["cfg4"]
    R, N, D = cfg["R"], cfg["N"], cfg["D"]
    assert R == 8192
    spec = canonical_spec(nfz_polygons=cfg["nfz_polygons"])
    params = canonical_params(spec, N=N, altitude=320.0)
    orc = _oracle(oracle_mod, spec, N, 320.0)
    geo = raster_geo(R)
    dem = synthetic_dem(R)
    gt = (geo.x0, geo.dx, 0.0, geo.y_top, 0.0, -geo.dy)
    vrt = write_tiled_dem(dem, gt, str(tmp_path / "tiles"))
    raster = DataManager(eng).build_cost_raster(vrt, compile_map(build_region_map(spec)),
                                                params)
    g = raster.geo
    assert (g.nx, g.ny, g.x0, g.y_top, g.dx, g.dy) == (R, R, geo.x0, geo.y_top, geo.dx, geo.dy)
    rec = _np(raster.rec)
    np.testing.assert_array_equal(rec[..., 2].view(np.float32), dem)   # tile mosaic == DEM
    # K1 records at sampled cells == the oracle's raster-build formulas at the cell centres
    rng = np.random.default_rng(5)
    iy, ix = rng.integers(0, R, 20_000), rng.integers(0, R, 20_000)
    xc = g.x0 + (ix.astype(np.float64) + 0.5) * g.dx
    yc = g.y_top - (iy.astype(np.float64) + 0.5) * g.dy
    pe = orc.eval_points(np.stack([xc, yc], 1))
    r = rec[iy, ix]
    np.testing.assert_array_equal(r[:, 0].view(np.float32), pe["phi"].astype(np.float32))
    np.testing.assert_array_equal(r[:, 1].view(np.float32), pe["psi_raw"].astype(np.float32))
    np.testing.assert_array_equal((r[:, 3] & 1) != 0, pe["collide"] != 0)
    assert ((r[:, 0].view(np.float32) != 0).mean() > 0.2) and ((r[:, 3] & 1).sum() > 0)
    # one GPU's share of cfg4's 1M paths (strong scaling over 8 GPUs, rank 0)
    lo, hi = shard_range(cfg["pairs"], 0, 8)
    pairs = random_pairs(cfg["pairs"], seed=0)[lo:hi]
    assert len(pairs) * D == 125_000
    ut = arc_table(N, displacements(D))

    def launch(pr):
        return eng.eval_generated(pr, ut, raster=raster)

    gpu = launch(pairs)
    sub = np.sort(np.random.default_rng(7).choice(len(pairs), 2000, replace=False))
    rd = oracle_mod.Oracle.raster_desc(g.nx, g.ny, g.x0, g.y_top, g.dx, g.dy, g.nodata,
                                       g.dem_threshold)
    ref = kernel_ref.raster_ref(oracle_mod, orc, eng.last_kernel(), eng.last_group(),
                                pairs[sub], ut, rd, rec.view(np.float32))
    _check_subsample(oracle_mod, gpu, ref, sub, D)
    assert (ref["nfz_hits"] > 0).any()
    _check_properties(eng, oracle_mod, launch, pairs, gpu, D)


def test_cfg5_volume_1024x1024x64(eng, oracle_mod):
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (CONFIGS, build_region_map, canonical_params,
                                                canonical_spec, displacements, layer_weights,
                                                raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs3d, synthetic_dem

    cfg = CONFIGS["cfg5"]
    R, nz, N, D, Q = cfg["R"], cfg["nz"], cfg["N"], cfg["D"], cfg["pairs"]
    assert (R, nz, Q) == (1024, 64, 100_000)
    spec = canonical_spec(nfz_polygons=cfg["nfz_polygons"])
    eng.set_geometry(compile_map(build_region_map(spec)))
    eng.set_params(canonical_params(spec, N=N, altitude=320.0))
    orc = _oracle(oracle_mod, spec, N, 320.0)
    geo = raster_geo(R)
    r2 = eng.raster_build(geo, synthetic_dem(R))
    lw = layer_weights(nz)
    vol = eng.volume_build(r2, nz, cfg["z0"], cfg["dz"], lw)
    vd = oracle_mod.volume_desc(R, R, nz, geo.x0, geo.y_top, geo.dx, geo.dy, cfg["z0"],
                                cfg["dz"])
    rec2 = _np(r2.rec).view(np.float32)
    ref_vol = oracle_mod.volume_build(vd, rec2, lw)
    np.testing.assert_array_equal(_np(vol.vox), ref_vol[0].view(np.int32))  # all 67M voxels
    np.testing.assert_array_equal(_np(vol.cols), ref_vol[1].view(np.int32))
    pairs = random_pairs3d(Q, seed=0)
    ut = arc_table(N, displacements(D))

    def launch(pr):
        return eng.eval_generated3d(pr, ut, vol)

    gpu = launch(pairs)
    sub = np.sort(np.random.default_rng(7).choice(Q, 2000, replace=False))
    ref = orc.eval_paths3d(oracle_mod.gen_paths3d(pairs[sub], ut), vd, ref_vol)
    _check_subsample(oracle_mod, gpu, ref, sub, D)
    idx = (sub[:, None] * D + np.arange(D)).reshape(-1)
    np.testing.assert_array_equal(_np(gpu["below_terrain"])[idx], ref["below"])
    _check_properties(eng, oracle_mod, launch, pairs, gpu, D)
    # K4h: the packed copy (one 16-B voxel per waypoint), the sorted grouped evaluation with
    # the similarity-form geometry -- bit-exact against its oracle statement on the subsample,
    # the reference's sequential per-segment sums within rounding
    eng.volume_pack(vol)
    gh = launch(pairs)
    assert eng.last_kernel() == "K4h+pack"
    refh = orc.eval_generated_h(pairs[sub], ut, mode="volume", vdesc=vd, vol=ref_vol,
                                group=eng.last_group())
    _check_subsample(oracle_mod, gh, refh, sub, D)
    np.testing.assert_array_equal(_np(gh["below_terrain"])[idx], refh["below"])
    for k in ("min_clearance", "nfz_hits", "offmap", "below_terrain"):
        np.testing.assert_array_equal(_np(gh[k]), _np(gpu[k]), err_msg=k)
    for k in ("cost", "length", "length_q", "nfz_sum"):
        np.testing.assert_allclose(_np(gh[k]), _np(gpu[k]), rtol=1e-12, err_msg=k)
    _check_properties(eng, oracle_mod, launch, pairs, gh, D)
