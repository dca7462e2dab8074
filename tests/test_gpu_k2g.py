"""K2g -- the segment-grouped raster evaluation (launch_grouped: every (path, waypoint group)
item sorted once by the raster tile under its middle waypoint and evaluated in one launch,
per-group partial sums combined in group order by the output launch) -- against the CPU oracle
in the same grouped order (orc_eval_paths_g), bit for bit, and against the reference's
sequential order within rounding.

What is exercised: groups of 1, 3, 8, 12 and 16 waypoints (ragged last group; W = 3 and W = 42),
D = 1, 5 and 16, the packed raster with automatic and 4-cell blocks, all region weights 0 over
a below-sea-level DEM with NaN terrain cells (maxima < 0, exactly +0.0 from skipped sea), NaN
pairs, paths that leave the raster, a raster that covers only part of the map, two streams
sharing one context.  UAM_OPT_SORTED_MIN_PATHS = 0 makes K2g take these small batches;
BASELINE's cfg3 size runs through it by default (test_gpu_parity.py::
test_full_size_cfg3_properties).  Reference rule: problem.py:38-44 (cost), main.py:175-180
(selection)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

KEYS = (("cost", "cost"), ("length_q", "lq"), ("length", "length"), ("kin_sum", "kin"),
        ("nfz_sum", "nfz"), ("nfz_hits", "nfz_hits"), ("offmap", "offmap"),
        ("min_clearance", "min_clearance"))
# outputs the grouped order does not touch (exact against the sequential oracle)
ORDER_FREE = ("nfz_hits", "offmap", "min_clearance")


def _case(oracle_mod, group, N, weights="canonical", R=1024, nfz=16, geo=None, maxalpha=None):
    from uam_path_planning_amd import build
    from uam_path_planning_amd.engine import Engine, PathParams
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import build_region_map, canonical_spec, raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    build.build_library()
    e = Engine(0)
    e.set_option("k2g_sim", 0)   # K2g proper (the similarity form K2h: tests/test_gpu_k2h.py)
    e.set_option("group", group)
    e.set_option("sorted_min_paths", 0)
    e.set_option("wave_max_paths", 0)
    spec = canonical_spec(nfz_polygons=nfz)
    w = spec["weights"] if weights == "canonical" else [0.0] * len(spec["weights"])
    opts = spec["options"]
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
    if seq is not None:   # the reference's sequential order: rounding only (north_star: 1e-5)
        for gk, ok in KEYS:
            g = gpu[gk].cpu().numpy()
            if gk in ORDER_FREE:
                np.testing.assert_array_equal(g, seq[ok], err_msg=gk)
            else:
                np.testing.assert_allclose(g, seq[ok], rtol=1e-12, atol=1e-300, err_msg=gk)


@pytest.mark.parametrize("weights", ["canonical", "zero"])
@pytest.mark.parametrize("group", [1, 3, 8, 12, 16])
def test_k2g_vs_grouped_oracle(oracle_mod, group, weights):
    """4500 pairs x 5 over a 1024^2 raster, N = 40 (W = 42: groups of 1, 3 (14), 8 (5 + 2),
    12 (3 + 6), 16 (2 + 10)), packed copy with automatic and 4-cell blocks; some paths leave
    the raster and two pairs are NaN.  Every output and both selections equal the grouped
    oracle's bit for bit, and the sequential oracle's within rounding."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements
    from uam_path_planning_amd.synthetic import random_pairs

    e, orc, raster, rd, rec = _case(oracle_mod, group, 40, weights)
    D = 5
    ut = arc_table(40, displacements(D))
    pairs = random_pairs(4500, seed=12)
    pairs[::97, 0] += 70.0
    pairs[5, 1] = np.nan
    pairs[77] = np.nan
    wp = oracle_mod.gen_paths(pairs, ut)
    ref = orc.eval_paths(wp, mode="raster", rdesc=rd, rec=rec, group=group)
    seq = orc.eval_paths(wp, mode="raster", rdesc=rd, rec=rec)
    ok = np.isfinite(seq["cost"])
    for block in (0, 4):
        e.raster_summary(raster, block, packed=True)
        gpu = e.eval_generated(pairs, ut, raster=raster)
        assert e.last_kernel() == "K2g+pack"
        assert e.last_group() == group
        _check(gpu, ref, oracle_mod, D)
        np.testing.assert_allclose(gpu["cost"].cpu().numpy()[ok], seq["cost"][ok], rtol=1e-12)
    if weights == "zero":
        assert (ref["min_clearance"] > 320.0).any()    # maxima below sea level occur
    # without the packed copy the raster batch runs K2s (sequential sums)
    e.raster_summary(raster, 0, packed=False)
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2s+skip" and e.last_group() == 0
    _check(gpu, seq, oracle_mod, D)


@pytest.mark.parametrize("D", [1, 16])
@pytest.mark.parametrize("N", [1, 80])
def test_k2g_displacements_and_short_paths(oracle_mod, D, N):
    """D = 1 (blockDim 64 in the output launch) and 16 (1024), N = 1 (W = 3: one group) and
    N = 80 (cfg3's W = 82: 10 groups of 8 + 2), ragged pair counts."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.synthetic import random_pairs

    e, orc, raster, rd, rec = _case(oracle_mod, 8, N)
    e.raster_summary(raster, 0, packed=True)
    ds = np.linspace(-1.0, 1.0, D) if D > 1 else np.array([0.3])
    ut = arc_table(N, ds)
    pairs = random_pairs(1037 if D > 1 else 17037, seed=3)
    wp = oracle_mod.gen_paths(pairs, ut)
    ref = orc.eval_paths(wp, mode="raster", rdesc=rd, rec=rec, group=8)
    seq = orc.eval_paths(wp, mode="raster", rdesc=rd, rec=rec)
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2g+pack"
    _check(gpu, ref, oracle_mod, D, seq)


def test_k2g_partial_raster(oracle_mod):
    """A raster over part of the map (1024 x 512 cells, 40 km wide): many waypoints fall off it
    (the off-raster bin of the sort, offmap counts per group)."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import RasterGeo
    from uam_path_planning_amd.scenario import displacements
    from uam_path_planning_amd.synthetic import random_pairs

    geo = RasterGeo(nx=1024, ny=512, x0=8.0, y_top=5.0, dx=40.0 / 1024, dy=40.0 / 1024,
                    nodata=-9999.0, dem_threshold=0.0)
    e, orc, raster, rd, rec = _case(oracle_mod, 8, 80, geo=geo)
    e.raster_summary(raster, 0, packed=True)
    D = 3
    ut = arc_table(80, displacements(D))
    pairs = random_pairs(3001, seed=5)
    ref = orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="raster", rdesc=rd, rec=rec,
                         group=8)
    assert (ref["offmap"] > 0).any() and (ref["offmap"] < 82).any()
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2g+pack"
    _check(gpu, ref, oracle_mod, D)


def test_k2g_two_streams(oracle_mod):
    """Two K2g batches enqueued on two streams of one context without host synchronisation:
    keys, orders and partial slots live in the context's order scratch, so the second launch
    waits for the first one's last read -- both must come out exactly as the oracle says."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements
    from uam_path_planning_amd.synthetic import random_pairs

    e, orc, raster, rd, rec = _case(oracle_mod, 8, 40)
    e.raster_summary(raster, 0, packed=True)
    D = 5
    ut = arc_table(40, displacements(D))
    pa, pb = random_pairs(6000, seed=31), random_pairs(4500, seed=32)
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
    ra = orc.eval_paths(oracle_mod.gen_paths(pa, ut), mode="raster", rdesc=rd, rec=rec, group=8)
    rb = orc.eval_paths(oracle_mod.gen_paths(pb, ut), mode="raster", rdesc=rd, rec=rec, group=8)
    for ga, gb in outs:
        _check(ga, ra, oracle_mod, D)
        _check(gb, rb, oracle_mod, D)


def test_k2g_options(oracle_mod):
    """uam_set_option range checks and round trip."""
    from uam_path_planning_amd import build
    from uam_path_planning_amd.engine import Engine

    build.build_library()
    e = Engine(0)
    assert e.get_option("group") == 21
    for bad in (-1, 65):
        with pytest.raises(ValueError):
            e.set_option("group", bad)
    e.set_option("group", 12)
    assert e.get_option("group") == 12
    assert e.get_option("k2g_chunk") == 0
    for bad in (-1, 5, 9, 10, 12, 17, 20, 22):
        with pytest.raises(ValueError):
            e.set_option("k2g_chunk", bad)
    e.set_option("k2g_chunk", 7)
    assert e.get_option("k2g_chunk") == 7
    e.set_option("k2g_chunk", 11)
    assert e.get_option("k2g_chunk") == 11
    assert e.get_option("k2g_curve") == 1
    assert e.get_option("k2g_tile_bits") == 0  # automatic: tiles of ~256^2 cells
    for bad in (-1, 1, 2, 7):
        with pytest.raises(ValueError):
            e.set_option("k2g_tile_bits", bad)
    with pytest.raises(ValueError):
        e.set_option("k2g_curve", 2)
    assert e.get_option("k2g_sim") == 1   # K2h by default
    with pytest.raises(ValueError):
        e.set_option("k2g_sim", 2)


@pytest.mark.parametrize("chunk,group", [(6, 24), (7, 21), (8, 21), (8, 26), (11, 21), (11, 5), (6, 64), (16, 21), (16, 40)])
def test_k2g_chunk_lengths(oracle_mod, chunk, group):
    """The gathers in flight per lane (UAM_OPT_K2G_CHUNK) only change how a group's waypoints
    are cut into load batches (full and partial chunks, groups shorter than a chunk): every
    output equals the grouped oracle's."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements
    from uam_path_planning_amd.synthetic import random_pairs

    e, orc, raster, rd, rec = _case(oracle_mod, group, 80, maxalpha=0.015)
    e.set_option("k2g_chunk", chunk)
    e.raster_summary(raster, 0, packed=True)
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = random_pairs(2000, seed=9)
    pairs[5] = np.nan
    ref = orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="raster", rdesc=rd, rec=rec,
                         group=group)
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2g+pack" and e.last_group() == group
    _check(gpu, ref, oracle_mod, D)


@pytest.mark.parametrize("tbits,lds,curve", [(6, 0, 1), (4, 49152, 1), (3, 0, 1), (4, 0, 0),
                                             (5, 0, 0), (0, 0, 1)])
def test_k2g_tuning_knobs(oracle_mod, tbits, lds, curve):
    """The knobs that only move work between lanes -- the sort key's tile grid
    (UAM_OPT_K2G_TILE_BITS) and the evaluation's LDS floor (UAM_OPT_K2G_LDS_FLOOR) -- leave
    every output equal to the grouped oracle's; groups of 21 take two gather chunks; a
    turn limit of 0.015 rad (between the arcs' per-step turns) makes some kinematic rows
    nonzero and leaves others at +0 (kin_row's division skips)."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements
    from uam_path_planning_amd.synthetic import random_pairs

    e, orc, raster, rd, rec = _case(oracle_mod, 21, 80, maxalpha=0.015)
    e.set_option("k2g_tile_bits", tbits)
    e.set_option("k2g_lds_floor", lds)
    e.set_option("k2g_curve", curve)
    e.raster_summary(raster, 0, packed=True)
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = random_pairs(2000, seed=8)
    pairs[3] = np.nan
    ref = orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="raster", rdesc=rd, rec=rec,
                         group=21)
    assert (ref["kin"] > 0).any() and (ref["kin"] == 0).any()
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2g+pack" and e.last_group() == 21
    _check(gpu, ref, oracle_mod, D)


@pytest.mark.parametrize("group,chunk", [(21, 0), (8, 0), (5, 11), (64, 16)])
def test_k2g_waypoint_cells(oracle_mod, group, chunk):
    """K2g with waypoint indices requested (the reference's returned waypoints, solver.py:49,
    main.py:186-190, as raster cells): cfg3's geometry (4096^2, 70 no-fly shapes, N = 80) on a
    2k-pair subsample, paths leaving the raster and NaN pairs included.  Every cell index
    (-1 off the raster) equals the oracle's bit for bit, and the other outputs stay those of
    the grouped oracle (the cell-writing form takes CH = 8 whatever the chunk option)."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements
    from uam_path_planning_amd.synthetic import random_pairs

    e, orc, raster, rd, rec = _case(oracle_mod, group, 80, R=4096, nfz=64)
    e.set_option("k2g_chunk", chunk)
    e.raster_summary(raster, 0, packed=True)
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = random_pairs(2000, seed=21)
    pairs[::53, 2] -= 80.0
    pairs[7] = np.nan
    ref = orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="raster", rdesc=rd, rec=rec,
                         group=group, want_cells=True)
    assert (ref["cells"] == -1).any() and (ref["cells"] >= 0).mean() > 0.5
    gpu = e.eval_generated(pairs, ut, raster=raster, want_cells=True)
    assert e.last_kernel() == "K2g+pack" and e.last_group() == group
    np.testing.assert_array_equal(gpu["cells"].cpu().numpy().reshape(ref["cells"].shape),
                                  ref["cells"])
    _check(gpu, ref, oracle_mod, D)
    # the same batch without cells: identical outputs
    gpu2 = e.eval_generated(pairs, ut, raster=raster)
    for gk, _ in KEYS:   # NaN pairs: NaN outputs compare equal here
        np.testing.assert_array_equal(gpu[gk].cpu().numpy(), gpu2[gk].cpu().numpy(), err_msg=gk)
