"""GPU parity: every kernel of libuampath against the CPU oracle (bit-exact: the kernels and
the oracle both compute in float64 with the reference's operation order and no FMA
contraction), and -- through the oracle -- against the reference's golden vectors.
Tolerances written here: exact equality for indices, counts, argmin and for every float64
output (the north_star bar is 1e-5 relative; we hold 0).  Raster-mode float32 record values
are compared exactly too (identical f64 -> f32 rounding)."""
import numpy as np
import pytest

import golden_io as G
import kernel_ref

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def eng():
    from uam_path_planning_amd import build
    from uam_path_planning_amd.engine import Engine

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    build.build_library()
    return Engine(0)


def _np(t):
    return t.cpu().numpy()


def _setup(eng, oracle_mod, spec, N, options, maxratio, maxalpha, enl, weights, anchor=None,
           altitude=150.0):
    from uam_path_planning_amd.engine import PathParams
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import build_region_map

    opts = {"length_smooth": False, "penalty_smooth": True, "obstacle_smooth": False,
            "maxratio_smooth": False}
    if options:
        opts.update(options)
    eng.set_geometry(compile_map(build_region_map(spec)))
    eng.set_params(PathParams(N=N, **opts, maxratio=maxratio, maxalpha=maxalpha,
                              enlargement=enl, weights=tuple(weights), anchor=anchor,
                              altitude=altitude))
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), N, opts, maxratio, maxalpha, enl,
                            weights, anchor=anchor, altitude=altitude)
    return orc


PATH_KEYS = (("cost", "cost"), ("length_q", "lq"), ("length", "length"), ("kin_sum", "kin"),
             ("nfz_sum", "nfz"), ("nfz_hits", "nfz_hits"), ("offmap", "offmap"))


def _assert_paths_equal(gpu, ref, raster=False):
    for gk, ok in PATH_KEYS:
        np.testing.assert_array_equal(_np(gpu[gk]), ref[ok], err_msg=gk)
    if raster:
        np.testing.assert_array_equal(_np(gpu["min_clearance"]), ref["min_clearance"])
    else:
        assert np.isnan(_np(gpu["min_clearance"])).all()


# ---- analytic mode (K3) vs oracle vs reference goldens ------------------------------------
def test_canonical_analytic(eng, oracle_mod):
    meta, arr = G.canonical()
    xs = tuple(meta["map"]["x_start"])
    orc = _setup(eng, oracle_mod, meta["map"], meta["N"], meta["options"], meta["maxratio"],
                 meta["maxalpha"], meta["enlargement"], meta["weights"], anchor=xs)
    wp = G.canonical_paths(meta, arr)
    gpu = eng.eval_waypoints(wp, want_g=True)
    ref = orc.eval_paths(wp, want_g=True)
    _assert_paths_equal(gpu, ref)
    np.testing.assert_array_equal(_np(gpu["g_rows"]), ref["g"])
    # and therefore the reference itself, bit for bit
    np.testing.assert_array_equal(_np(gpu["cost"]), arr["cost"])
    np.testing.assert_array_equal(_np(gpu["g_rows"]), arr["g"])
    np.testing.assert_array_equal(_np(gpu["length"]), arr["length"])
    pe = eng.eval_points(wp.reshape(-1, 2))
    np.testing.assert_array_equal(_np(pe["phi"]), arr["phi"].reshape(-1))
    np.testing.assert_array_equal(_np(pe["phi_regions"]),
                                  arr["phi_r"].transpose(0, 2, 1).reshape(-1, 3))
    np.testing.assert_array_equal(_np(pe["obs_norm"]), arr["obs_norm"].reshape(-1))
    np.testing.assert_array_equal(_np(pe["collide"]), arr["collide"].reshape(-1))


@pytest.mark.parametrize("ci", range(24))
def test_random_cases_analytic(eng, oracle_mod, ci):
    c = G.random_cases()[ci]
    orc = _setup(eng, oracle_mod, c["map"], c["N"], c["options"], c["maxratio"],
                 c["maxalpha"], c["enlargement"], c["weights"], anchor=tuple(c["map"]["x_start"]))
    wp = np.asarray(c["paths"]).reshape(len(c["paths"]), -1, 2)
    gpu = eng.eval_waypoints(wp, want_g=True)
    ref = orc.eval_paths(wp, want_g=True)
    for gk, ok in PATH_KEYS:
        np.testing.assert_array_equal(_np(gpu[gk]), ref[ok], err_msg=gk)
    np.testing.assert_array_equal(_np(gpu["g_rows"]), ref["g"])
    for i, o in enumerate(c["outputs"]):   # reference goldens (NaN where the reference is)
        np.testing.assert_allclose(_np(gpu["cost"])[i], o["cost"], rtol=1e-13, equal_nan=True)
    pts = wp.reshape(-1, 2)
    pe = eng.eval_points(pts)
    pr = orc.eval_points(pts)
    for k in ("phi", "phi_regions", "obs_norm", "psi_raw", "collide"):
        np.testing.assert_array_equal(_np(pe[k]), pr[k], err_msg=k)


def test_generated_analytic_and_argmin(eng, oracle_mod):
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.synthetic import random_pairs

    meta, arr = G.canonical()
    orc = _setup(eng, oracle_mod, meta["map"], meta["N"], meta["options"], meta["maxratio"],
                 meta["maxalpha"], meta["enlargement"], meta["weights"])
    ds = meta["displacements"]
    ut = arc_table(meta["N"], ds)
    pairs = np.concatenate([np.array([[*meta["map"]["x_start"], *meta["map"]["x_goal"]]]),
                            random_pairs(130, seed=5)])
    gpu = eng.eval_generated(pairs, ut)
    wp = oracle_mod.gen_paths(pairs, ut)
    np.testing.assert_array_equal(_np(eng.gen_paths(pairs, ut)), wp)
    ref = orc.eval_paths(wp)
    _assert_paths_equal(gpu, ref)
    # reference candidate costs (create_x_init arcs differ from the table by <= 1e-14)
    np.testing.assert_allclose(_np(gpu["cost"])[:5], arr["cost"], rtol=1e-12)
    bf = _np(eng.argmin(gpu["cost"], len(ds), True))
    bl = _np(eng.argmin(gpu["length"], len(ds), False))
    np.testing.assert_array_equal(bf, oracle_mod.argmin(ref["cost"], len(ds), True))
    np.testing.assert_array_equal(bl, oracle_mod.argmin(ref["length"], len(ds), False))
    assert bf[0] == 3


def test_argmin_semantics_gpu(eng):
    v = np.array([3.0, 1.0, 1.0, 2.0, np.nan, 5.0, 4.0, 4.0, 2.0, 0.0, 7.0, 9.0])
    assert _np(eng.argmin(v, 4, False)).tolist() == [1, 0, 2]


# ---- raster build (K1) --------------------------------------------------------------------
def test_raster_build_cell_centres_golden(eng, oracle_mod):
    from uam_path_planning_amd.engine import RasterGeo

    meta, _ = G.canonical()
    gr = G.grid()
    nx, ny, X0, Ytop, dx, dy = gr["geo"]
    geo = RasterGeo(int(nx), int(ny), X0, Ytop, dx, dy)
    for tag, opts, enl in (("a", {"penalty_smooth": True, "obstacle_smooth": True}, 0.0),
                           ("b", {"penalty_smooth": False, "obstacle_smooth": False}, 0.25)):
        _setup(eng, oracle_mod, meta["map"], 4, opts, 1.1, 0.3, enl, [200, 15000, 27000])
        rec = _np(eng.raster_build(geo).rec)
        np.testing.assert_array_equal(rec[..., 0].view(np.float32),
                                      gr[f"phi_{tag}"].astype(np.float32))
        np.testing.assert_array_equal(rec[..., 1].view(np.float32),
                                      gr[f"psi_{tag}"].astype(np.float32))
        np.testing.assert_array_equal(rec[..., 3] & 1, gr[f"collide_{tag}"])


@pytest.mark.parametrize("thr", [0.0, 100.0, -9999.0])
def test_raster_build_vs_oracle(eng, oracle_mod, thr):
    from uam_path_planning_amd.scenario import canonical_spec, raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    spec = canonical_spec(nfz_polygons=8)
    orc = _setup(eng, oracle_mod, spec, 80, spec["options"], spec["maxratio"], spec["maxalpha"],
                 spec["enlargement"], spec["weights"])
    geo = raster_geo(256, dem_threshold=thr)
    dem = synthetic_dem(256)
    rec = _np(eng.raster_build(geo, dem).rec)
    ref = orc.raster_build(oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top,
                                                         geo.dx, geo.dy, geo.nodata, thr), dem)
    np.testing.assert_array_equal(rec, ref.view(np.int32))


def test_raster_build_list_walk_and_partial_waves(eng, oracle_mod):
    """K1's wave walk without per-cell bitmasks (306 obstacles and a region table of more than
    256 shapes: the lists merged by their minimum head) on a 250^2 raster (waves span row ends;
    the last wave is partial)."""
    from uam_path_planning_amd.scenario import canonical_spec, raster_geo
    from uam_path_planning_amd.synthetic import random_convex_polygons, synthetic_dem

    spec = canonical_spec(nfz_polygons=300, seed=4)
    spec["regions"][1]["shapes"] = spec["regions"][1]["shapes"] + [
        {"kind": "polygon", "vertices": v} for v in random_convex_polygons(260, seed=6)]
    orc = _setup(eng, oracle_mod, spec, 80, spec["options"], spec["maxratio"], spec["maxalpha"],
                 spec["enlargement"], spec["weights"])
    geo = raster_geo(250)
    dem = synthetic_dem(250)
    rec = _np(eng.raster_build(geo, dem).rec)
    ref = orc.raster_build(oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top,
                                                         geo.dx, geo.dy, geo.nodata,
                                                         geo.dem_threshold), dem)
    np.testing.assert_array_equal(rec, ref.view(np.int32))
    assert (rec[..., 3] & 1).any()


@pytest.mark.parametrize("cpl", [1, 2, 4, 8])
@pytest.mark.parametrize("big", [False, True])
def test_raster_build_cells_per_lane(oracle_mod, cpl, big, monkeypatch):
    """K1 with 1 (single-cell kernel), 2, 4 and 8 rows per lane (UAM_OPT_K1_ROWS) on a
    333 x 251 raster: partial strips in both directions, lanes whose
    cells fall in different grid slots, the merged psi/contains walk (masks) and -- big: 306
    obstacles and a >256-shape region table -- the per-cell list cursors.  Non-smooth penalty
    and obstacle options take the other psi branch."""
    from uam_path_planning_amd.engine import Engine, RasterGeo
    from uam_path_planning_amd.scenario import canonical_spec
    from uam_path_planning_amd.synthetic import random_convex_polygons, synthetic_dem

    e2 = Engine(0)
    e2.set_option("k1_rows", cpl)
    spec = canonical_spec(nfz_polygons=300 if big else 64, seed=4)
    if big:
        spec["regions"][1]["shapes"] = spec["regions"][1]["shapes"] + [
            {"kind": "polygon", "vertices": v} for v in random_convex_polygons(260, seed=6)]
    geo = RasterGeo(nx=333, ny=251, x0=-1.0, y_top=21.0, dx=62.0 / 333, dy=62.0 / 251,
                    nodata=-9999.0, dem_threshold=0.0)
    dem = synthetic_dem(333)[:251].copy()
    for opts in ({}, {"penalty_smooth": False, "obstacle_smooth": True}):
        o = dict(spec["options"], **opts)
        orc = _setup(e2, oracle_mod, spec, 80, o, spec["maxratio"], spec["maxalpha"], 0.1,
                     spec["weights"])
        rec = _np(e2.raster_build(geo, dem).rec)
        ref = orc.raster_build(oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top,
                                                             geo.dx, geo.dy, geo.nodata,
                                                             geo.dem_threshold), dem)
        np.testing.assert_array_equal(rec, ref.view(np.int32))
    assert (rec[..., 3] & 1).any()


# ---- raster eval (K2) ---------------------------------------------------------------------
def _raster_case(eng, oracle_mod, R, Q, N, nfz, seed=0, D=5, geo=None):
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec, displacements, raster_geo
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    spec = canonical_spec(nfz_polygons=nfz)
    orc = _setup(eng, oracle_mod, spec, N, spec["options"], spec["maxratio"], spec["maxalpha"],
                 spec["enlargement"], spec["weights"], altitude=320.0)
    geo = geo or raster_geo(R)
    dem = synthetic_dem(geo.nx) if geo.nx == geo.ny else synthetic_dem(max(geo.nx, geo.ny))[
        :geo.ny, :geo.nx].copy()
    raster = eng.raster_build(geo, dem)
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy,
                                       geo.nodata, geo.dem_threshold)
    rec = _np(raster.rec).view(np.float32)
    pairs = random_pairs(Q, seed=seed)
    ut = arc_table(N, displacements(D))
    return orc, raster, rd, rec, pairs, ut


@pytest.mark.parametrize("R,Q,N", [(256, 300, 80), (2048, 200, 254), (512, 64, 1)])
def test_raster_eval_generated_vs_oracle(eng, oracle_mod, R, Q, N):
    """Both the wave-per-path kernel (what the default picks for these batch sizes) and the
    lane-per-path kernels (UAM_OPT_WAVE_MAX_PATHS = 0) against the oracle, generated and
    explicit paths."""
    orc, raster, rd, rec, pairs, ut = _raster_case(eng, oracle_mod, R, Q, N, nfz=4)
    wp = oracle_mod.gen_paths(pairs, ut)
    ref = orc.eval_paths(wp, mode="raster", rdesc=rd, rec=rec, want_cells=True)
    try:
        for wmax in (1 << 40, 0):
            eng.set_option("wave_max_paths", wmax)
            gpu = eng.eval_generated(pairs, ut, raster=raster, want_cells=True)
            _assert_paths_equal(gpu, ref, raster=True)
            np.testing.assert_array_equal(_np(gpu["cells"]), ref["cells"])
            np.testing.assert_array_equal(_np(gpu["best_fval_idx"]),
                                          oracle_mod.argmin(ref["cost"], 5, True))
            np.testing.assert_array_equal(_np(gpu["best_length_idx"]),
                                          oracle_mod.argmin(ref["length"], 5, False))
            # explicit-waypoint kernel on the same paths gives the same bits
            gpu2 = eng.eval_waypoints(wp, raster=raster, want_cells=True)
            _assert_paths_equal(gpu2, ref, raster=True)
            np.testing.assert_array_equal(_np(gpu2["cells"]), ref["cells"])
    finally:
        eng.set_option("wave_max_paths", 16384)


def test_raster_matches_reference_at_snapped_centres(eng, oracle_mod):
    """Raster-mode cost == analytic cost of the path snapped to its cells' centres, up to the
    f32 rounding of the stored record (|rel| <= 1e-6 <= the 1e-5 bar)."""
    orc, raster, rd, rec, pairs, ut = _raster_case(eng, oracle_mod, 512, 40, 80, nfz=0)
    gpu = eng.eval_generated(pairs, ut, raster=raster, want_cells=True)
    cells = _np(gpu["cells"])
    geo = raster.geo
    ix, iy = cells % geo.nx, cells // geo.nx
    snapped = np.stack([geo.x0 + (ix + 0.5) * geo.dx, geo.y_top - (iy + 0.5) * geo.dy], -1)
    ok = (cells >= 0).all(1)
    # the length terms use the true waypoints; only the penalty is read at the cell centre
    pen_gpu = _np(gpu["cost"]) - (orc.N + 1) * _np(gpu["length_q"])
    pts = snapped.reshape(-1, 2)
    phi = orc.eval_points(pts)["phi"].reshape(cells.shape)
    pen_ref = (phi / orc.N).sum(1)
    np.testing.assert_allclose(pen_gpu[ok], pen_ref[ok], rtol=1e-5, atol=1e-9)
    assert ok.sum() > 50


def test_offmap_and_empty(eng, oracle_mod):
    orc, raster, rd, rec, pairs, ut = _raster_case(eng, oracle_mod, 128, 8, 20, nfz=0)
    far = pairs.copy()
    far[:, 0] += 100.0           # starts far off the raster
    gpu = eng.eval_generated(far, ut, raster=raster, want_cells=True)
    ref = orc.eval_paths(oracle_mod.gen_paths(far, ut), mode="raster", rdesc=rd, rec=rec,
                         want_cells=True)
    _assert_paths_equal(gpu, ref, raster=True)
    assert (_np(gpu["offmap"]) > 0).all()
    empty = eng.eval_generated(np.zeros((0, 4)), ut, raster=raster)
    assert empty["cost"].numel() == 0
    e2 = eng.eval_waypoints(np.zeros((0, 22, 2)), raster=raster)
    assert e2["cost"].numel() == 0


def test_dem_mosaic(eng):
    rng = np.random.default_rng(3)
    tiles = rng.standard_normal((6, 9, 15)).astype(np.float32)
    xoff = np.array([0, 15, 30, 0, 15, 30], np.int32)
    yoff = np.array([0, 0, 0, 9, 9, 9], np.int32)
    dem = _np(eng.dem_mosaic(tiles, xoff, yoff, 40, 20))
    ref = np.full((20, 40), -9999.0, np.float32)
    for t in range(6):
        ys, xs = yoff[t], xoff[t]
        h, w = min(9, 20 - ys), min(15, 40 - xs)
        ref[ys:ys + h, xs:xs + w] = tiles[t, :h, :w]
    np.testing.assert_array_equal(dem, ref)


def test_full_size_cfg3_properties(eng, oracle_mod):
    """BASELINE config 3 at full size (4096^2 DEM + 69 no-fly shapes, 100k pairs x 5):
    oracle on a 2k-pair subsample (bit-exact), size-independent properties on the rest."""
    orc, raster, rd, rec, pairs, ut = _raster_case(eng, oracle_mod, 4096, 100_000, 80, nfz=64)
    gpu = eng.eval_generated(pairs, ut, raster=raster)
    assert eng.last_kernel() == "K2h+pack"     # the default for this batch size
    group = eng.last_group()
    assert group > 0
    sub = np.random.default_rng(7).choice(len(pairs), 2000, replace=False)
    sub.sort()
    wp = oracle_mod.gen_paths(pairs[sub], ut)
    ref = kernel_ref.raster_ref(oracle_mod, orc, eng.last_kernel(), group, pairs[sub], ut, rd,
                                rec)
    idx = (sub[:, None] * 5 + np.arange(5)).reshape(-1)
    for gk, ok in PATH_KEYS:
        np.testing.assert_array_equal(_np(gpu[gk])[idx], ref[ok], err_msg=gk)
    # against the reference's per-segment sequential sums: rounding only (bar 1e-5)
    seq = orc.eval_paths(wp, mode="raster", rdesc=rd, rec=rec)
    np.testing.assert_allclose(_np(gpu["cost"])[idx], seq["cost"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(_np(gpu["length"])[idx], seq["length"], rtol=1e-12, atol=0)
    # the whole batch through the sequential order (threads over pair shards; the C oracle
    # drops the GIL): the grouped sums move no selection on this batch (the
    # selection of the reference order, pinned at cfg3 size) and no cost by more than 1e-12
    import concurrent.futures
    bounds = np.linspace(0, len(pairs), 9).astype(int)

    def seq_part(k):
        sl = pairs[bounds[k]:bounds[k + 1]]
        r = orc.eval_paths(oracle_mod.gen_paths(sl, ut), mode="raster", rdesc=rd, rec=rec)
        return r["cost"], r["length"]

    with concurrent.futures.ThreadPoolExecutor(8) as ex:
        parts = list(ex.map(seq_part, range(8)))
    sc = np.concatenate([p_[0] for p_ in parts])
    sl_ = np.concatenate([p_[1] for p_ in parts])
    np.testing.assert_allclose(_np(gpu["cost"]), sc, rtol=1e-12, atol=0)
    assert (oracle_mod.argmin(sc, 5, True) != _np(gpu["best_fval_idx"])).sum() == 0
    assert (oracle_mod.argmin(sl_, 5, False) != _np(gpu["best_length_idx"])).sum() == 0
    cost, lq = _np(gpu["cost"]), _np(gpu["length_q"])
    assert np.isfinite(cost).all()
    assert (cost >= 81 * lq - 1e-9).all()                 # penalties are non-negative
    # permutation: shuffling pairs permutes outputs bit-for-bit (no cross-path coupling)
    perm = np.random.default_rng(9).permutation(len(pairs))
    gp = eng.eval_generated(pairs[perm], ut, raster=raster)
    pidx = (perm[:, None] * 5 + np.arange(5)).reshape(-1)
    np.testing.assert_array_equal(_np(gp["cost"]), cost[pidx])
    # determinism: a second launch is bit-identical
    g2 = eng.eval_generated(pairs, ut, raster=raster)
    np.testing.assert_array_equal(_np(g2["cost"]), cost)
    # argmin over the full batch vs the oracle's rule on the GPU costs
    bf = _np(eng.argmin(gpu["cost"], 5, True))
    np.testing.assert_array_equal(bf, oracle_mod.argmin(cost, 5, True))


# ---- drop-in API --------------------------------------------------------------------------
def test_dropin_problem_and_solver(eng):
    from uam_path_planning_amd.path_generation import Solver
    from uam_path_planning_amd.scenario import canonical_problem

    meta, arr = G.canonical()
    prob = canonical_problem()
    wp = G.canonical_paths(meta, arr)
    for i in range(5):
        z = wp[i].reshape(-1)
        assert prob.get_cost(z) == arr["cost"][i]
        np.testing.assert_array_equal(prob.get_nonlincon(z), arr["g"][i])
        assert prob.length_of(arr["x_init"][i]) == arr["length"][i]
        assert prob.length_of(z, prob.options["length_smooth"]) == arr["lq"][i]
    tp = prob.get_total_penalty_function()
    assert tp(wp[2, 10]) == arr["phi"][2, 10]
    pl = prob.get_penalty_function("Population")
    assert pl(wp[2, 10]) == arr["phi_r"][2, 1, 10]
    solver = Solver(prob, {})
    for i, d in enumerate(meta["displacements"]):
        np.testing.assert_allclose(solver.create_x_init(d), arr["x_init"][i], rtol=0,
                                   atol=1e-12)
    res = solver.evaluate_candidates(meta["displacements"])
    np.testing.assert_allclose(res["cost"], arr["cost"], rtol=1e-12)
    assert res["min_fval_index"] == 3
    with pytest.raises(ValueError):
        solver.create_x_init(1.5)
    with pytest.raises(ValueError):        # p vector of the wrong length (OpEn error 3003)
        solver.solve(np.zeros(2 * prob.N), [0.0])
    # shape primitives on the device
    m = prob.map
    assert m.collides(np.array([38.66652661075855, -9.203164091309498]))
    assert not m[(0.0, 0.0)]
    obs = m.obstacles[0]
    assert obs.contains([38.7, -9.2])
    assert obs.penalty_function(True, 0)([38.66652661075855, -9.203164091309498]) == 1.0


@pytest.mark.parametrize("D", [5, 3, 17])
def test_raster_kernels_bit_identical(eng, oracle_mod, D):
    """The raster forms return the same bits: the wave-per-path kernel, the lane-per-path K2
    (with the skip bitmap), K2s and K2g (against the grouped oracle), and the fused selection
    matches the oracle's rule; D = 17 exercises the fallback to the per-wave kernel + separate
    selection (K2d / K3d)."""
    orc, raster, rd, rec, pairs, ut = _raster_case(eng, oracle_mod, 512, 333, 80, nfz=4, D=D)
    wp = oracle_mod.gen_paths(pairs, ut)
    ref = orc.eval_paths(wp, mode="raster", rdesc=rd, rec=rec)
    seen = set()
    try:
        for wmax, smin, group, sim in ((1 << 40, 65536, 8, 1), (0, 65536, 8, 1), (0, 0, 0, 1),
                                       (0, 0, 8, 1), (0, 0, 8, 0)):
            eng.set_option("wave_max_paths", wmax)
            eng.set_option("sorted_min_paths", smin)
            eng.set_option("group", group)
            eng.set_option("k2g_sim", sim)
            gpu = eng.eval_generated(pairs, ut, raster=raster)
            seen.add(eng.last_kernel())
            r = ref if eng.last_group() == 0 else kernel_ref.raster_ref(
                oracle_mod, orc, eng.last_kernel(), eng.last_group(), pairs, ut, rd, rec)
            _assert_paths_equal(gpu, r, raster=True)
            np.testing.assert_array_equal(_np(gpu["best_fval_idx"]),
                                          oracle_mod.argmin(r["cost"], D, True))
            np.testing.assert_array_equal(_np(gpu["best_length_idx"]),
                                          oracle_mod.argmin(r["length"], D, False))
            ga = eng.eval_generated(pairs[:50], ut)      # analytic path of the same settings
            ra = orc.eval_paths(oracle_mod.gen_paths(pairs[:50], ut))
            _assert_paths_equal(ga, ra)
    finally:
        eng.set_option("wave_max_paths", 16384)
        eng.set_option("sorted_min_paths", 65536)
        eng.set_option("group", 21)
        eng.set_option("k2g_sim", 1)
    assert seen == ({"K2w", "K2d"} if D > 16 else
                    {"K2w", "K2+skip", "K2s+pack", "K2h+pack", "K2g+pack"})
    with pytest.raises(ValueError):
        eng.set_option("wave_max_paths", -1)


@pytest.mark.parametrize("enl", [-0.5, -1e-3, 0.0, 1e-3, 0.3, 2.0])
def test_culling_is_exact_near_boundaries(eng, oracle_mod, enl):
    """The kernels skip a shape outside a padded box of {h_i < e}; the oracle never skips.
    Points on vertices, on edges, just inside/outside and on the box margins must agree
    bit for bit for every output."""
    rng = np.random.default_rng(int(abs(enl) * 1000) + 11)
    shapes = [{"kind": "polygon", "vertices": [[0.0, 0.0], [3.0, 0.2], [2.5, 2.0], [0.4, 1.7]]},
              {"kind": "polygon", "vertices": [[5.0, 5.0], [5.001, 5.0], [5.0005, 5.002]]},
              {"kind": "ball", "center": [-3.0, 1.0], "r1": 1.5, "r2": 0.4},
              {"kind": "square", "center": [2.0, -3.0], "r1": 0.7, "r2": 1.9}]
    spec = {"obstacles": shapes, "regions": [{"name": "A", "color": "Red", "shapes": shapes}],
            "x_start": [0.0, 0.0], "x_goal": [1.0, 1.0]}
    pts = []
    for s in shapes:
        if s["kind"] == "polygon":
            v = np.asarray(s["vertices"])
            pts += list(v)
            for i in range(len(v)):
                a, b = v[i], v[(i + 1) % len(v)]
                for t in np.linspace(0, 1, 7):
                    m = a + t * (b - a)
                    pts += [m, m + rng.normal(scale=1e-9, size=2), m + rng.normal(scale=1e-3, size=2)]
        else:
            c = np.asarray(s["center"], float)
            pts += [c + rng.normal(scale=2.0, size=2) for _ in range(60)]
    lo, hi = np.min(pts, 0) - 3, np.max(pts, 0) + 3
    pts += list(rng.uniform(lo, hi, size=(2000, 2)))
    pts = np.asarray(pts, dtype=np.float64)
    for opts in ({"penalty_smooth": True, "obstacle_smooth": True},
                 {"penalty_smooth": False, "obstacle_smooth": False}):
        orc = _setup(eng, oracle_mod, spec, 4, opts, 1.1, 0.3, enl, [7.0])
        ge = eng.eval_points(pts)
        oe = orc.eval_points(pts)
        for k in ("phi", "phi_regions", "obs_norm", "psi_raw", "collide"):
            np.testing.assert_array_equal(_np(ge[k]), oe[k], err_msg=f"{k} opts={opts}")


@pytest.mark.parametrize("thr", [0.0, 250.0, -9999.0])
def test_vrt_ingest_and_dem_mask(eng, oracle_mod, tmp_path, thr):
    """VRT tile mosaic on the device == the DEM the tiles were cut from; the cost raster built
    from the tiles == the oracle's; the DEM mask == data_manager.py:14-17 semantics."""
    from uam_path_planning_amd.map_generation import DataManager, write_tiled_dem
    from uam_path_planning_amd.scenario import canonical_spec, raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    R = 512
    dem = synthetic_dem(R)
    geo = raster_geo(R, dem_threshold=thr)
    gt = (geo.x0, geo.dx, 0.0, geo.y_top, 0.0, -geo.dy)
    vrt = write_tiled_dem(dem, gt, str(tmp_path / "tiles"), deflate=(thr == 0.0))
    dm = DataManager(eng)
    d_dem, g2 = dm.load_dem(vrt, dem_threshold=thr)
    np.testing.assert_array_equal(_np(d_dem), dem)
    assert (g2.nx, g2.ny, g2.x0, g2.y_top, g2.dx, g2.dy) == \
        (geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy)
    spec = canonical_spec(nfz_polygons=4)
    orc = _setup(eng, oracle_mod, spec, 80, spec["options"], spec["maxratio"], spec["maxalpha"],
                 spec["enlargement"], spec["weights"])
    r = dm.build_cost_raster(vrt, eng.geometry, eng.params, dem_threshold=thr)
    ref = orc.raster_build(oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top,
                                                         geo.dx, geo.dy, -9999.0, thr), dem)
    np.testing.assert_array_equal(_np(r.rec), ref.view(np.int32))
    mask = dm.load_dem_mask(vrt, thr)
    np.testing.assert_array_equal(mask, (dem == -9999) if thr == -9999 else (dem > thr))


def test_load_tiles_chunked(eng, tmp_path):
    """uam_load_tiles (parallel native reader, ~32 MiB chunks through two page-locked buffers,
    each copied while the next is read): 544 tiles of 225 x 150 = three chunks, the last one
    partial, twice through the same context; the device tiles equal the Python reader's bit for
    bit.  A missing tile fails loudly with its path."""
    import os

    from uam_path_planning_amd.map_generation.vrt import (load_tiles, read_vrt, tile_layout,
                                                          write_tiled_dem)

    dem = np.random.default_rng(11).standard_normal((150 * 17, 225 * 32)).astype(np.float32)
    v = read_vrt(write_tiled_dem(dem, (0.0, 1.0, 0.0, 0.0, 0.0, -1.0), str(tmp_path)))
    paths, th, tw, xo, yo = tile_layout(v)
    assert len(paths) == 544
    ref, _, _ = load_tiles(v)
    for _ in range(2):
        got = eng.load_tiles(paths, th, tw, n_threads=8)
        np.testing.assert_array_equal(_np(got).view(np.int32), ref.view(np.int32))
    os.remove(paths[300])
    with pytest.raises(Exception, match=os.path.basename(paths[300])):
        eng.load_tiles(paths, th, tw)


def test_volume_mode_vs_oracle(eng, oracle_mod):
    """Config 5 (3-D risk volume, build-defined semantics): volume build and the volume path
    kernel bit-exact vs the oracle, incl. waypoints below/above the layer range."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import (canonical_spec, displacements, layer_weights,
                                                raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs3d, synthetic_dem

    spec = canonical_spec(nfz_polygons=8)
    orc = _setup(eng, oracle_mod, spec, 40, spec["options"], spec["maxratio"], spec["maxalpha"],
                 spec["enlargement"], spec["weights"])
    R, nz, z0, dz = 256, 64, 0.0, 10.0
    geo = raster_geo(R)
    dem = synthetic_dem(R)
    r2 = eng.raster_build(geo, dem)
    lw = layer_weights(nz)
    vol = eng.volume_build(r2, nz, z0, dz, lw)
    vd = oracle_mod.volume_desc(R, R, nz, geo.x0, geo.y_top, geo.dx, geo.dy, z0, dz)
    ref_vol = oracle_mod.volume_build(vd, _np(r2.rec).view(np.float32), lw)
    np.testing.assert_array_equal(_np(vol.vox), ref_vol[0].view(np.int32))
    np.testing.assert_array_equal(_np(vol.cols), ref_vol[1].view(np.int32))
    # the column bitmap: 8 x 8-column blocks at 256^2, set iff a column has terrain bits != 0
    # or the no-fly flag
    c = ref_vol[1].view(np.uint32)
    need = ((c[..., 0] != 0) | ((c[..., 1] & 1) != 0)).reshape(R // 8, 8, R // 8, 8)
    need = need.any(axis=(1, 3)).reshape(-1)
    bits = np.unpackbits(_np(vol.cbits)[: need.size // 32].view(np.uint8),
                         bitorder="little").astype(bool)
    np.testing.assert_array_equal(bits, need)
    assert 0 < need.sum() < need.size
    pairs = random_pairs3d(300, seed=4, zmin=-50.0, zmax=700.0)   # some outside [0, 640)
    ut = arc_table(40, displacements(5))
    ref = orc.eval_paths3d(oracle_mod.gen_paths3d(pairs, ut), vd, ref_vol)
    try:
        for wmax in (0, 1 << 40):   # lane-per-path, then wave-per-path (the auto pick here)
            eng.set_option("wave_max_paths", wmax)
            gpu = eng.eval_generated3d(pairs, ut, vol)
            for gk, ok in PATH_KEYS + (("below_terrain", "below"),
                                       ("min_clearance", "min_clearance")):
                np.testing.assert_array_equal(_np(gpu[gk]), ref[ok], err_msg=f"{gk} w{wmax}")
    finally:
        eng.set_option("wave_max_paths", 16384)
    assert (_np(gpu["offmap"]) > 0).any() and (_np(gpu["below_terrain"]) > 0).any()
    np.testing.assert_array_equal(_np(gpu["best_fval_idx"]), oracle_mod.argmin(ref["cost"], 5, True))


def test_shape_grid_index_is_exact(eng, oracle_mod):
    """The uniform-grid shape index (uam_set_params) must not change a bit: dense random
    points over and beyond the map (cfg3 geometry, 104 shapes), all polygon vertices, points
    on the map extent's edges, and NaN."""
    from uam_path_planning_amd.scenario import canonical_spec

    spec = canonical_spec(nfz_polygons=64)
    orc = _setup(eng, oracle_mod, spec, 10, {"obstacle_smooth": True}, 1.04, 0.04, 0.3,
                 spec["weights"])
    rng = np.random.default_rng(5)
    pts = [rng.uniform([-5, -45], [65, 25], size=(200_000, 2))]
    verts = np.array([v for s in spec["obstacles"] + [sh for r in spec["regions"]
                                                      for sh in r["shapes"]]
                      if s["kind"] == "polygon" for v in s["vertices"]], float)
    pts += [verts, verts + 1e-12, verts - 1e-12]
    lo, hi = verts.min(0), verts.max(0)
    t = np.linspace(0, 1, 101)[:, None]
    pts += [lo + t * [hi[0] - lo[0], 0], lo + t * [0, hi[1] - lo[1]], hi - t * [hi[0] - lo[0], 0]]
    pts += [np.array([[np.nan, 0.0], [1.0, np.nan]])]
    pts = np.vstack(pts)
    gpu = eng.eval_points(pts, want=("phi", "psi_raw", "collide"))
    ref = orc.eval_points(pts)
    np.testing.assert_array_equal(_np(gpu["phi"]), ref["phi"])
    np.testing.assert_array_equal(_np(gpu["psi_raw"]), ref["psi_raw"])
    np.testing.assert_array_equal(_np(gpu["collide"]), ref["collide"])


@pytest.mark.parametrize("order", ["1", "0"])
def test_generated_analytic_pair_order(oracle_mod, monkeypatch, order):
    """K3 evaluates batches of >= 4096 pairs in a spatial (Morton) order of the pairs
    (UAM_OPT_PAIR_ORDER, default on) and writes every result at its pair's own index: the outputs
    and the selection equal the oracle's, bit for bit, with the order on and off."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (CONFIGS, build_region_map, canonical_params,
                                                canonical_spec, displacements)
    from uam_path_planning_amd.synthetic import random_pairs

    e2 = Engine(0)
    e2.set_option("pair_order", int(order))
    spec = canonical_spec(nfz_polygons=CONFIGS["cfg3"]["nfz_polygons"])
    params = canonical_params(spec, N=40, altitude=320.0)
    e2.set_geometry(compile_map(build_region_map(spec)))
    e2.set_params(params)
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), params.N, spec["options"],
                            spec["maxratio"], spec["maxalpha"], spec["enlargement"],
                            spec["weights"], altitude=params.altitude)
    D = 5
    ut = arc_table(params.N, displacements(D))
    pairs = random_pairs(4500, seed=11)
    gpu = e2.eval_generated(pairs, ut)
    ref = orc.eval_paths(oracle_mod.gen_paths(pairs, ut))
    _assert_paths_equal(gpu, ref)
    np.testing.assert_array_equal(_np(gpu["best_fval_idx"]),
                                  oracle_mod.argmin(ref["cost"], D, True))
    np.testing.assert_array_equal(_np(gpu["best_length_idx"]),
                                  oracle_mod.argmin(ref["length"], D, False))


@pytest.mark.parametrize("order", ["1", "0"])
@pytest.mark.parametrize("weights", ["canonical", "zero"])
def test_raster_pair_order_and_gather_skip(oracle_mod, monkeypatch, order, weights):
    """K2 (raster, lane per path) with the spatial pair order + XCD placement on and off
    (UAM_OPT_PAIR_ORDER) and with the gather-skip bitmap at several block sizes and without it:
    every output, the cells and the selection equal the oracle's bit for bit.  With all region
    weights 0 and every land cell below sea level, Phi is +0 everywhere: the sea blocks are
    skipped (terrain +0.0 enters the maximum without a gather) while the below-sea-level land
    is gathered, and paths whose maximum is < 0 or exactly the skipped sea's +0.0 occur."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.scenario import canonical_spec, displacements, raster_geo
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    e2 = Engine(0)
    e2.set_option("pair_order", int(order))
    spec = canonical_spec(nfz_polygons=16)
    w = spec["weights"] if weights == "canonical" else [0.0] * len(spec["weights"])
    orc = _setup(e2, oracle_mod, spec, 40, spec["options"], spec["maxratio"], spec["maxalpha"],
                 spec["enlargement"], w, altitude=320.0)
    R = 1024
    geo = raster_geo(R)
    dem = synthetic_dem(R)
    if weights == "zero":
        dem = np.where(dem == -9999.0, dem, -np.abs(dem) - 1.0).astype(np.float32)
        dem[::97, ::89] = np.float32(np.nan)
    raster = e2.raster_build(geo, dem, summary=False)
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy,
                                       geo.nodata, geo.dem_threshold)
    rec = _np(raster.rec).view(np.float32)
    D = 5
    ut = arc_table(40, displacements(D))
    pairs = random_pairs(4500, seed=12)
    pairs[::97, 0] += 70.0            # some paths leave the raster
    ref = orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="raster", rdesc=rd, rec=rec,
                         want_cells=True)
    skipped = []
    for block in (None, 0, 4, 32):
        if block is None:
            raster.summary = None
        else:
            e2.raster_summary(raster, block)
            nb = (-(-R // raster.block)) ** 2
            bits = np.unpackbits(_np(raster.summary).view(np.uint8), bitorder="little")[:nb]
            skipped.append(float(bits.mean()))
        gpu = e2.eval_generated(pairs, ut, raster=raster, want_cells=True)
        _assert_paths_equal(gpu, ref, raster=True)
        np.testing.assert_array_equal(_np(gpu["cells"]), ref["cells"])
        np.testing.assert_array_equal(_np(gpu["best_fval_idx"]),
                                      oracle_mod.argmin(ref["cost"], D, True))
        np.testing.assert_array_equal(_np(gpu["best_length_idx"]),
                                      oracle_mod.argmin(ref["length"], D, False))
    assert max(skipped) > 0.2, skipped
    if weights == "zero":
        assert (ref["min_clearance"] > 320.0).any()    # maxima below sea level occur
        assert (ref["min_clearance"] == 320.0).any()   # maxima of exactly +0.0 (sea) occur


def test_raster_summary_table(eng, oracle_mod):
    """uam_raster_summary == its definition (numpy on the record raster): bit b set iff every
    cell of block b has phi == +-0, psi == +-0, no NFZ flag and a terrain reading +0.0 (a
    nodata cell or a +0.0f dem value; -0.0f, < 0 and NaN clear the bit); ragged edge blocks
    included; block sizes beyond the 65536-bit LDS bitmap are refused."""
    from uam_path_planning_amd.scenario import canonical_spec, raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    spec = canonical_spec(nfz_polygons=8)
    _setup(eng, oracle_mod, spec, 20, spec["options"], spec["maxratio"], spec["maxalpha"],
           spec["enlargement"], spec["weights"])
    geo = raster_geo(300)
    geo.nx, geo.ny = 300, 260
    dem = synthetic_dem(300)[:260].copy()
    dem[5, 7] = np.float32(np.nan)
    dem[200:204, 10:30] = np.float32(-3.0)
    dem[150:166, 0:64] = np.float32(0.0)      # +0.0 terrain: skippable where phi, psi are 0
    dem[170:186, 0:64] = np.float32(-0.0)     # -0.0 reads as 0 but is not +0.0: never set
    raster = eng.raster_build(geo, dem, summary=False)
    rec = _np(raster.rec)
    phi, psi = rec[..., 0].view(np.float32), rec[..., 1].view(np.float32)
    terr_bits = np.where(rec[..., 3] & 4, 0, rec[..., 2])    # nodata reads +0.0
    ok = (phi == 0) & (psi == 0) & ((rec[..., 3] & 1) == 0) & (terr_bits == 0)
    for block in (2, 4, 8, 32, 64, 128):   # (>= 8: one wave per block, k_raster_summary_w)
        eng.raster_summary(raster, block)
        nby, nbx = -(-260 // block), -(-300 // block)
        want = np.array([[ok[by * block:(by + 1) * block, bx * block:(bx + 1) * block].all()
                          for bx in range(nbx)] for by in range(nby)]).reshape(-1)
        got = np.unpackbits(_np(raster.summary).view(np.uint8), bitorder="little")
        assert got.size == 32 * (-(-want.size // 32))
        np.testing.assert_array_equal(got[:want.size].astype(bool), want, err_msg=f"B{block}")
        assert not got[want.size:].any()
        assert not want.all() and (want.any() or block > 32)
    big = raster_geo(4096)
    with pytest.raises(ValueError):
        eng.raster_summary(type(raster)(big, None), 8)


def test_raster_pack_table(eng, oracle_mod):
    """uam_raster_pack == its definition (uampath.hip, packed raster; test_gpu_k2h._check_pack:
    the 2-bit codes, the four planes at the blocked index, bounds holding every cell's terrain)
    on ragged edges (300 x 262 is no multiple of the 4 x 8-cell blocks or of the summary block),
    a NaN terrain cell (its superblock unbounded) and a strip of +0.0 terrain, summary blocks
    4, 16, 64 and 128."""
    from test_gpu_k2h import _check_pack
    from uam_path_planning_amd.scenario import canonical_spec, raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    spec = canonical_spec(nfz_polygons=8)
    _setup(eng, oracle_mod, spec, 20, spec["options"], spec["maxratio"], spec["maxalpha"],
           spec["enlargement"], spec["weights"])
    geo = raster_geo(300)
    geo.nx, geo.ny = 300, 262
    dem = synthetic_dem(300)[:262].copy()
    dem[5, 7] = np.float32(np.nan)
    dem[150:166, 0:64] = np.float32(0.0)
    raster = eng.raster_build(geo, dem, summary=False)
    rec = _np(raster.rec).view(np.float32).reshape(262, 300, 4)
    for block in (4, 16, 64, 128):   # (>= 8: one wave per block, k_raster_pack_map_w)
        eng.raster_summary(raster, block, packed=True)
        assert raster.block == block
        frac_bounded, _ = _check_pack(raster, rec)
        assert 0.0 < frac_bounded < 1.0  # the NaN cell's superblock is unbounded


@pytest.mark.parametrize("mode", ["analytic", "raster"])
def test_pair_order_two_streams(oracle_mod, mode):
    """The pair-order scratch is owned by the context: two batches of >= 4096 pairs
    enqueued on two streams of the same context, with no host synchronisation in between, must
    both come out exactly as the oracle says (a shared, unordered scratch would hand one launch
    the other's order: pairs evaluated twice or never)."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (CONFIGS, build_region_map, canonical_params,
                                                canonical_spec, displacements, raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    e = Engine(0)
    spec = canonical_spec(nfz_polygons=CONFIGS["cfg3"]["nfz_polygons"])
    params = canonical_params(spec, N=40, altitude=320.0)
    e.set_geometry(compile_map(build_region_map(spec)))
    e.set_params(params)
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), params.N, spec["options"],
                            spec["maxratio"], spec["maxalpha"], spec["enlargement"],
                            spec["weights"], altitude=params.altitude)
    D = 5
    ut = arc_table(params.N, displacements(D))
    kw, okw = {}, {}
    if mode == "raster":
        geo = raster_geo(512)
        raster = e.raster_build(geo, synthetic_dem(512))
        kw = {"raster": raster}
        okw = {"mode": "raster",
               "rdesc": oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx,
                                                      geo.dy, geo.nodata, geo.dem_threshold),
               "rec": raster.rec.cpu().numpy().view(np.float32)}
    pa, pb = random_pairs(6000, seed=31), random_pairs(4500, seed=32)
    ta = e.tensor(pa, torch.float64)
    tb = e.tensor(pb, torch.float64)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for _ in range(3):  # several rounds so the launches overlap
        with torch.cuda.stream(s1):
            ga = e.eval_generated(ta, ut, **kw)
        with torch.cuda.stream(s2):
            gb = e.eval_generated(tb, ut, **kw)
        outs.append((ga, gb))
    torch.cuda.synchronize()
    ra = orc.eval_paths(oracle_mod.gen_paths(pa, ut), **okw)
    rb = orc.eval_paths(oracle_mod.gen_paths(pb, ut), **okw)
    for ga, gb in outs:
        _assert_paths_equal(ga, ra, raster=mode == "raster")
        _assert_paths_equal(gb, rb, raster=mode == "raster")


@pytest.mark.parametrize("order", ["1", "0"])
def test_volume_pair_order(oracle_mod, monkeypatch, order):
    """Config 5's kernel with the raster pair order over the volume's x/y extent (batches of
    >= 4096 pairs; UAM_OPT_PAIR_ORDER on and off): every output and the selection bit-exact vs
    the oracle -- each pair is still read and written at its own index."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.scenario import (canonical_spec, displacements, layer_weights,
                                                raster_geo)
    from uam_path_planning_amd.synthetic import random_pairs3d, synthetic_dem

    e = Engine(0)
    e.set_option("pair_order", int(order))
    spec = canonical_spec(nfz_polygons=8)
    orc = _setup(e, oracle_mod, spec, 24, spec["options"], spec["maxratio"], spec["maxalpha"],
                 spec["enlargement"], spec["weights"])
    R, nz, z0, dz = 256, 32, 0.0, 20.0
    geo = raster_geo(R)
    r2 = e.raster_build(geo, synthetic_dem(R))
    lw = layer_weights(nz)
    vol = e.volume_build(r2, nz, z0, dz, lw)
    vd = oracle_mod.volume_desc(R, R, nz, geo.x0, geo.y_top, geo.dx, geo.dy, z0, dz)
    ref_vol = oracle_mod.volume_build(vd, _np(r2.rec).view(np.float32), lw)
    pairs = random_pairs3d(5000, seed=9, zmin=-50.0, zmax=700.0)
    ut = arc_table(24, displacements(5))
    ref = orc.eval_paths3d(oracle_mod.gen_paths3d(pairs, ut), vd, ref_vol)
    gpu = e.eval_generated3d(pairs, ut, vol)
    for gk, ok in PATH_KEYS + (("below_terrain", "below"), ("min_clearance", "min_clearance")):
        np.testing.assert_array_equal(_np(gpu[gk]), ref[ok], err_msg=gk)
    np.testing.assert_array_equal(_np(gpu["best_fval_idx"]),
                                  oracle_mod.argmin(ref["cost"], 5, True))
