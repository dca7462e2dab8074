"""K2h -- K2g's sort and grouped raster sums with the geometry terms in the similarity form
(the default for generated raster batches of >= UAM_OPT_SORTED_MIN_PATHS paths when
maxratio_smooth is off): get_cost's L, the true length and the kinematic rows from the unit
arc's sums scaled by |x0 - xf| / 2, once per path in the output launch; per (path, group) item
only the waypoints' points, cells and records.  Against the oracle's statement of it
(orc_eval_generated_h) bit for bit, and against the reference's sequential per-segment order
within rounding (north_star: 1e-5; here 1e-12).

Exercised: groups 1-64 (ragged last groups), D = 1-16, N = 1 and 80, canonical and all-zero
weights over a below-sea-level DEM with NaN cells, NaN pairs and a pair with start == goal
(h = 0), paths that leave the raster, a raster over part of the map, waypoint cells, chunk
lengths 6/7/8/11/16, two streams sharing one context, the fallback to K2g under
maxratio_smooth.  Reference rules: problem.py:38-44 (cost), 84-114 (rows), 130-146 (length_of),
solver.py:103-136 (the arcs), main.py:175-180 (selection)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

KEYS = (("cost", "cost"), ("length_q", "lq"), ("length", "length"), ("kin_sum", "kin"),
        ("nfz_sum", "nfz"), ("nfz_hits", "nfz_hits"), ("offmap", "offmap"),
        ("min_clearance", "min_clearance"))
ORDER_FREE = ("nfz_hits", "offmap", "min_clearance")


def _case(oracle_mod, group, N, weights="canonical", R=1024, nfz=16, geo=None, maxalpha=None,
          maxratio_smooth=False):
    from uam_path_planning_amd import build
    from uam_path_planning_amd.engine import Engine, PathParams
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import build_region_map, canonical_spec, raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    build.build_library()
    e = Engine(0)
    e.set_option("group", group)
    e.set_option("sorted_min_paths", 0)
    e.set_option("wave_max_paths", 0)
    spec = canonical_spec(nfz_polygons=nfz)
    w = spec["weights"] if weights == "canonical" else [0.0] * len(spec["weights"])
    opts = dict(spec["options"])
    opts["maxratio_smooth"] = maxratio_smooth
    ma = spec["maxalpha"] if maxalpha is None else maxalpha
    e.set_geometry(compile_map(build_region_map(spec)))
    e.set_params(PathParams(N=N, **opts, maxratio=spec["maxratio"], maxalpha=ma,
                            enlargement=spec["enlargement"], weights=tuple(w), altitude=320.0))
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), N, opts, spec["maxratio"],
                            ma, spec["enlargement"], w, altitude=320.0)
    geo = geo or raster_geo(R)
    dem = synthetic_dem(max(geo.nx, geo.ny))[:geo.ny, :geo.nx].copy()
    if weights == "zero":
        dem = np.where(dem == -9999.0, dem, -np.abs(dem) - 1.0).astype(np.float32)
        dem[::97, ::89] = np.float32(np.nan)
    raster = e.raster_build(geo, dem, summary=False)
    e.raster_summary(raster, 0, packed=True)
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy,
                                       geo.nodata, geo.dem_threshold)
    rec = raster.rec.cpu().numpy().view(np.float32)
    return e, orc, raster, rd, rec


def _check(gpu, ref, oracle_mod, D, seq=None):
    for gk, ok in KEYS:
        np.testing.assert_array_equal(gpu[gk].cpu().numpy(), ref[ok], err_msg=gk)
    np.testing.assert_array_equal(gpu["best_fval_idx"].cpu().numpy(),
                                  oracle_mod.argmin(ref["cost"], D, True))
    np.testing.assert_array_equal(gpu["best_length_idx"].cpu().numpy(),
                                  oracle_mod.argmin(ref["length"], D, False))
    if seq is not None:   # the reference's per-segment sequential sums: rounding only
        ok = np.isfinite(seq["cost"]) & (seq["length"] > 0)
        for gk, sk in KEYS:
            g = gpu[gk].cpu().numpy()
            if gk in ORDER_FREE:
                np.testing.assert_array_equal(g, seq[sk], err_msg=gk)
            elif gk == "kin_sum":
                np.testing.assert_allclose(g[ok], seq[sk][ok], rtol=1e-11, atol=1e-13,
                                           err_msg=gk)
            else:
                np.testing.assert_allclose(g[ok], seq[sk][ok], rtol=1e-12, atol=1e-300,
                                           err_msg=gk)


def _pairs(n, seed):
    from uam_path_planning_amd.synthetic import random_pairs

    pairs = random_pairs(n, seed=seed)
    pairs[::97, 0] += 70.0          # off the raster
    pairs[5, 1] = np.nan
    pairs[77] = np.nan
    pairs[11, 2:] = pairs[11, :2]   # start == goal: h = 0
    return pairs


@pytest.mark.parametrize("weights", ["canonical", "zero"])
@pytest.mark.parametrize("group", [1, 3, 8, 12, 16, 21])
def test_k2h_vs_oracle(oracle_mod, group, weights):
    """4500 pairs x 5 over a 1024^2 raster, N = 40 (W = 42); every output and both selections
    equal orc_eval_generated_h bit for bit, and the sequential per-segment oracle within
    rounding."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, raster, rd, rec = _case(oracle_mod, group, 40, weights)
    D = 5
    ut = arc_table(40, displacements(D))
    pairs = _pairs(4500, 12)
    ref = orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=group)
    seq = orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="raster", rdesc=rd, rec=rec)
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2h+pack" and e.last_group() == group
    _check(gpu, ref, oracle_mod, D, seq)
    if weights == "zero":
        assert (ref["min_clearance"] > 320.0).any()


@pytest.mark.parametrize("D", [1, 16])
@pytest.mark.parametrize("N", [1, 80])
def test_k2h_displacements_and_short_paths(oracle_mod, D, N):
    from uam_path_planning_amd.arcs import arc_table

    e, orc, raster, rd, rec = _case(oracle_mod, 21, N)
    ds = np.linspace(-1.0, 1.0, D) if D > 1 else np.array([0.3])
    ut = arc_table(N, ds)
    pairs = _pairs(1037 if D > 1 else 17037, 3)
    ref = orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=21)
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2h+pack"
    _check(gpu, ref, oracle_mod, D)


@pytest.mark.parametrize("maxalpha", [0.015, 0.3])
@pytest.mark.parametrize("chunk,group", [(6, 24), (7, 21), (8, 21), (8, 26), (11, 21), (11, 5),
                                         (16, 21), (16, 40), (21, 21), (21, 30), (21, 9),
                                         (0, 64)])
def test_k2h_chunks_and_turn_rows(oracle_mod, chunk, group, maxalpha):
    """The chunk length (gathers in flight) only changes how a group's waypoints are cut into
    load batches.  maxalpha 0.015 rad lies between the arcs' per-step turns (some turn rows
    positive, some +0); 0.3 keeps every row +0."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, raster, rd, rec = _case(oracle_mod, group, 80, maxalpha=maxalpha)
    e.set_option("k2g_chunk", chunk)
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = _pairs(2000, 9)
    ref = orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=group)
    if maxalpha < 0.1:
        assert (ref["kin"] > 0).any() and (ref["kin"] == 0).any()
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2h+pack" and e.last_group() == group
    _check(gpu, ref, oracle_mod, D)


@pytest.mark.parametrize("chunk,floor", [(11, 54000), (7, 90000), (21, 90000), (16, 60000)])
def test_k2h_lds_floor(oracle_mod, chunk, floor):
    """Fewer workgroups per CU (the setting K2h takes by default on rasters over 2^25 cells:
    54 000 B, 11 in flight) changes no bit."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, raster, rd, rec = _case(oracle_mod, 21, 80, maxalpha=0.015)
    e.set_option("k2g_chunk", chunk)
    e.set_option("k2g_lds_floor", floor)
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = _pairs(2000, 13)
    ref = orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=21)
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2h+pack"
    _check(gpu, ref, oracle_mod, D)


def test_k2h_partial_raster(oracle_mod):
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import RasterGeo
    from uam_path_planning_amd.scenario import displacements

    geo = RasterGeo(nx=1024, ny=512, x0=8.0, y_top=5.0, dx=40.0 / 1024, dy=40.0 / 1024,
                    nodata=-9999.0, dem_threshold=0.0)
    e, orc, raster, rd, rec = _case(oracle_mod, 21, 80, geo=geo)
    D = 3
    ut = arc_table(80, displacements(D))
    pairs = _pairs(3001, 5)
    ref = orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=21)
    assert (ref["offmap"] > 0).any() and (ref["offmap"] < 82).any()
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2h+pack"
    _check(gpu, ref, oracle_mod, D)


@pytest.mark.parametrize("tile,group,R,geo_kind", [(128, 21, 1024, "square"),
                                                  (64, 21, 1024, "square"),
                                                  (128, 7, 4096, "square"),
                                                  (64, 30, 1024, "partial"),
                                                  (128, 1, 1024, "partial")])
def test_k2h_tile_form(oracle_mod, tile, group, R, geo_kind):
    """The tile form (UAM_OPT_K2G_TILE_OWNER: one workgroup per T x T tile, its packed plane in
    LDS) changes where code-1 waypoints inside the tile are read, nothing else: every output
    equals orc_eval_generated_h bit for bit, with pairs off the raster (the off-raster bin's
    workgroup), NaN pairs, start == goal, a raster that is not a multiple of the tile (edge
    tiles zero-filled past the raster) and tiles without items."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import RasterGeo
    from uam_path_planning_amd.scenario import displacements

    geo = None
    if geo_kind == "partial":
        geo = RasterGeo(nx=1000, ny=700, x0=8.0, y_top=5.0, dx=40.0 / 1000, dy=40.0 / 1000,
                        nodata=-9999.0, dem_threshold=0.0)
    e, orc, raster, rd, rec = _case(oracle_mod, group, 80, R=R, nfz=64, geo=geo,
                                    maxalpha=0.015)
    e.set_option("k2g_tile_owner", tile)
    assert e.get_option("k2g_tile_owner") == tile
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = _pairs(3000, 41)
    ref = orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=group)
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2h-tile+pack" and e.last_group() == group
    _check(gpu, ref, oracle_mod, D)
    # with cells requested the launch is the cell-writing K2h, the same bits
    cells = e.eval_generated(pairs, ut, raster=raster, want_cells=True)
    assert e.last_kernel() == "K2h+pack"
    _check(cells, ref, oracle_mod, D)
    for bad in (1, 32, 256):
        with pytest.raises(ValueError):
            e.set_option("k2g_tile_owner", bad)


@pytest.mark.parametrize("group", [21, 5, 64])
def test_k2h_waypoint_cells(oracle_mod, group):
    """Waypoint cells from K2h at cfg3's geometry (4096^2, 70 no-fly shapes, N = 80) on a
    2k-pair subsample: every index (-1 off the raster) equals the oracle's, the other outputs
    equal those of the same batch without cells."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, raster, rd, rec = _case(oracle_mod, group, 80, R=4096, nfz=64)
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = _pairs(2000, 21)
    pairs[::53, 2] -= 80.0
    ref = orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=group, want_cells=True)
    assert (ref["cells"] == -1).any() and (ref["cells"] >= 0).mean() > 0.5
    gpu = e.eval_generated(pairs, ut, raster=raster, want_cells=True)
    assert e.last_kernel() == "K2h+pack"
    np.testing.assert_array_equal(gpu["cells"].cpu().numpy().reshape(ref["cells"].shape),
                                  ref["cells"])
    _check(gpu, ref, oracle_mod, D)
    gpu2 = e.eval_generated(pairs, ut, raster=raster)
    for gk, _ in KEYS:   # NaN pairs: NaN outputs compare equal here
        np.testing.assert_array_equal(gpu[gk].cpu().numpy(), gpu2[gk].cpu().numpy(), err_msg=gk)


def test_k2h_two_streams(oracle_mod):
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, raster, rd, rec = _case(oracle_mod, 21, 40)
    D = 5
    ut = arc_table(40, displacements(D))
    pa, pb = _pairs(6000, 31), _pairs(4500, 32)
    ta, tb = e.tensor(pa, torch.float64), e.tensor(pb, torch.float64)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for _ in range(3):
        with torch.cuda.stream(s1):
            ga = e.eval_generated(ta, ut, raster=raster)
        with torch.cuda.stream(s2):
            gb = e.eval_generated(tb, ut, raster=raster)
        outs.append((ga, gb))
    torch.cuda.synchronize()
    ra = orc.eval_generated_h(pa, ut, rdesc=rd, rec=rec, group=21)
    rb = orc.eval_generated_h(pb, ut, rdesc=rd, rec=rec, group=21)
    for ga, gb in outs:
        _check(ga, ra, oracle_mod, D)
        _check(gb, rb, oracle_mod, D)


def test_k2h_maxratio_smooth_runs_k2g(oracle_mod):
    """maxratio_smooth squares the norms inside the turn rows (problem.py:94,106), which are
    then not scale-free: such batches run K2g (per-segment geometry, grouped order)."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, raster, rd, rec = _case(oracle_mod, 21, 40, maxratio_smooth=True)
    D = 5
    ut = arc_table(40, displacements(D))
    pairs = _pairs(2000, 41)
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2g+pack"
    ref = orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="raster", rdesc=rd, rec=rec,
                         group=21)
    _check(gpu, ref, oracle_mod, D)
    with pytest.raises(ValueError):
        orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=21)
