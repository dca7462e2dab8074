"""K2s -- the segment-sorted raster evaluation (launch_segmented: paths cut into segments, each
segment index one launch over its items sorted by raster tile, per-path running sums carried in
HBM) -- against the CPU oracle, bit for bit, and against the lane-per-path K2
(UAM_OPT_SORTED_MIN_PATHS above the batch).  K2s is the fast form of the reference's
sequential sum order (UAM_OPT_GROUP = 0; the default K2g is tests/test_gpu_k2g.py).

What is exercised: 2, 3, 4 and 8 segments (UAM_OPT_K2S_SEGMENTS; ragged last segment; W = 3
where a segment is one waypoint), D = 1, 5 and 16, the gather-skip bitmap off / automatic / 4-cell blocks, the
packed raster (uam_raster_pack) or the 16-B records, all region
weights 0 over a below-sea-level DEM (maxima < 0 from gathered land, and exactly +0.0 from
skipped sea), NaN pairs and paths that leave the raster, and two streams sharing one
context.  UAM_OPT_SORTED_MIN_PATHS = 0 makes K2s take these small batches.  Reference rule:
problem.py:38-44 (cost), main.py:175-180 (selection)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

KEYS = (("cost", "cost"), ("length_q", "lq"), ("length", "length"), ("kin_sum", "kin"),
        ("nfz_sum", "nfz"), ("nfz_hits", "nfz_hits"), ("offmap", "offmap"),
        ("min_clearance", "min_clearance"))


def _case(oracle_mod, segs, N, weights="canonical", R=1024, nfz=16):
    from uam_path_planning_amd import build
    from uam_path_planning_amd.engine import Engine, PathParams
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import build_region_map, canonical_spec, raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    build.build_library()
    e = Engine(0)
    e.set_option("group", 0)   # K2s, not the segment-grouped K2g (tests/test_gpu_k2g.py)
    e.set_option("k2s_segments", segs)
    e.set_option("sorted_min_paths", 0)
    spec = canonical_spec(nfz_polygons=nfz)
    w = spec["weights"] if weights == "canonical" else [0.0] * len(spec["weights"])
    opts = spec["options"]
    e.set_geometry(compile_map(build_region_map(spec)))
    e.set_params(PathParams(N=N, **opts, maxratio=spec["maxratio"], maxalpha=spec["maxalpha"],
                            enlargement=spec["enlargement"], weights=tuple(w), altitude=320.0))
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), N, opts, spec["maxratio"],
                            spec["maxalpha"], spec["enlargement"], w, altitude=320.0)
    geo = raster_geo(R)
    dem = synthetic_dem(R)
    if weights == "zero":
        dem = np.where(dem == -9999.0, dem, -np.abs(dem) - 1.0).astype(np.float32)
        dem[::97, ::89] = np.float32(np.nan)
    raster = e.raster_build(geo, dem, summary=False)
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy,
                                       geo.nodata, geo.dem_threshold)
    rec = raster.rec.cpu().numpy().view(np.float32)
    return e, orc, raster, rd, rec


def _check(gpu, ref, oracle_mod, D):
    for gk, ok in KEYS:
        np.testing.assert_array_equal(gpu[gk].cpu().numpy(), ref[ok], err_msg=gk)
    np.testing.assert_array_equal(gpu["best_fval_idx"].cpu().numpy(),
                                  oracle_mod.argmin(ref["cost"], D, True))
    np.testing.assert_array_equal(gpu["best_length_idx"].cpu().numpy(),
                                  oracle_mod.argmin(ref["length"], D, False))


@pytest.mark.parametrize("weights", ["canonical", "zero"])
@pytest.mark.parametrize("segs", [2, 3, 4, 8])
def test_k2s_vs_oracle_and_k2(oracle_mod, segs, weights):
    """4500 pairs x 5 over a 1024^2 raster, N = 40 (W = 42: 21/21, 14 x 3, 11/11/11/9,
    6 x 7), pass 1 fused into segment 0's launch,
    skip bitmap off, automatic and 4-cell blocks, with and without the packed copy
    (uam_raster_pack: 8-B planes, 2-bit block codes); some paths leave the raster and two pairs
    are NaN.  Every output and both selections equal the oracle's, and K2's."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements
    from uam_path_planning_amd.synthetic import random_pairs

    e, orc, raster, rd, rec = _case(oracle_mod, segs, 40, weights)
    D = 5
    ut = arc_table(40, displacements(D))
    pairs = random_pairs(4500, seed=12)
    pairs[::97, 0] += 70.0
    pairs[5, 1] = np.nan
    pairs[77] = np.nan
    ref = orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="raster", rdesc=rd, rec=rec)
    from uam_path_planning_amd.engine import Engine

    k2 = Engine(0)
    k2.set_option("group", 0)
    k2.set_option("wave_max_paths", 0)     # the lane-per-path K2 at this batch size
    k2.set_geometry(e.geometry)
    k2.set_params(e.params)
    for block, pack in ((None, False), (0, False), (4, False), (0, True), (4, True)):
        if block is None:
            raster.summary = raster.packed = None
        else:
            e.raster_summary(raster, block, packed=pack)
        gpu = e.eval_generated(pairs, ut, raster=raster)
        assert e.last_kernel() == ("K2s" if block is None else
                                   "K2s+pack" if pack else "K2s+skip")
        _check(gpu, ref, oracle_mod, D)
        g2 = k2.eval_generated(pairs, ut, raster=raster)
        assert k2.last_kernel() == ("K2" if block is None else "K2+skip")
        for gk, _ in KEYS:
            np.testing.assert_array_equal(gpu[gk].cpu().numpy(), g2[gk].cpu().numpy(),
                                          err_msg=gk)
    if weights == "zero":
        assert (ref["min_clearance"] > 320.0).any()    # maxima below sea level occur


@pytest.mark.parametrize("D", [1, 16])
@pytest.mark.parametrize("N", [1, 80])
def test_k2s_displacements_and_short_paths(oracle_mod, D, N):
    """D = 1 (blockDim 64 in the output launch) and 16 (1024), N = 1 (W = 3: four segments
    become three of one waypoint) and N = 80 (cfg3's W = 82), ragged pair counts above the
    wave-per-path kernel's automatic range."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.synthetic import random_pairs

    e, orc, raster, rd, rec = _case(oracle_mod, 4, N)
    e.raster_summary(raster, 0, packed=True)
    ds = np.linspace(-1.0, 1.0, D) if D > 1 else np.array([0.3])
    ut = arc_table(N, ds)
    pairs = random_pairs(1037 if D > 1 else 17037, seed=3)  # above the wave kernel's 16384
    ref = orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="raster", rdesc=rd, rec=rec)
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2s+pack"
    _check(gpu, ref, oracle_mod, D)


def test_k2s_two_streams(oracle_mod):
    """Two K2s batches enqueued on two streams of one context without host synchronisation:
    the segment state, keys and orders live in the context's order scratch, so the second
    launch waits for the first one's last read -- both must come out exactly as the oracle
    says."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements
    from uam_path_planning_amd.synthetic import random_pairs

    e, orc, raster, rd, rec = _case(oracle_mod, 4, 40)
    e.raster_summary(raster, 0)
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
    ra = orc.eval_paths(oracle_mod.gen_paths(pa, ut), mode="raster", rdesc=rd, rec=rec)
    rb = orc.eval_paths(oracle_mod.gen_paths(pb, ut), mode="raster", rdesc=rd, rec=rec)
    for ga, gb in outs:
        _check(ga, ra, oracle_mod, D)
        _check(gb, rb, oracle_mod, D)
