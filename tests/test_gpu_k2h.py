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
lengths 6/7/8/11, two streams sharing one context, the fallback to K2g under
maxratio_smooth; the packed copy against its definition and the terrain-bound rule's sample
strides over DEMs with non-finite, flat and -0.0 terrain.  Reference rules: problem.py:38-44 (cost), 84-114 (rows), 130-146 (length_of),
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
          maxratio_smooth=False, obstacle_smooth=None, dem_edit=None):
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
    if obstacle_smooth is not None:
        opts["obstacle_smooth"] = obstacle_smooth
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
    if dem_edit == "nonfinite":   # unbounded superblocks
        dem[100:104, 300:302] = np.float32(np.inf)
        dem[::211, ::157] = np.float32(np.nan)
    elif dem_edit == "flat":      # a few values: many blocks of one value
        dem = np.where(dem == -9999.0, dem, np.round(dem / 200.0) * 200.0).astype(np.float32)
    elif dem_edit == "negzero":
        dem = np.where(np.abs(dem) < 40.0, np.float32(-0.0), dem).astype(np.float32)
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


@pytest.mark.parametrize("terrain", [1, 0])
@pytest.mark.parametrize("weights", ["canonical", "zero"])
@pytest.mark.parametrize("group", [1, 3, 8, 12, 16, 21])
def test_k2h_vs_oracle(oracle_mod, group, weights, terrain):
    """4500 pairs x 5 over a 1024^2 raster, N = 40 (W = 42); every output and both selections
    equal orc_eval_generated_h bit for bit, and the sequential per-segment oracle within
    rounding."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, raster, rd, rec = _case(oracle_mod, group, 40, weights)
    e.set_option("k2h_terrain", terrain)  # (1: the default, the terrain in the entry)
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


def _pack_dims(nx, ny, block):
    """The packed raster's sections (uampath.hip PackDims / uam_raster_pack_shape)."""
    nbx, nby = -(-nx // block), -(-ny // block)
    words = (nbx * nby * 2 + 31) // 32
    bsh = 3
    while (-(-nx // (1 << bsh))) * (-(-ny // (1 << bsh))) > 16384:
        bsh += 1
    bnbx, bnby = -(-nx // (1 << bsh)), -(-ny // (1 << bsh))
    w16 = lambda v: -(-v // 16) * 4
    bnd_off = w16(words * 4)
    sbt_off = bnd_off + w16(bnbx * bnby * 2)
    sbnbx, sbnby = -(-bnbx // 4), -(-bnby // 4)
    hwords = sbt_off + w16(sbnbx * sbnby * 8)
    a256 = lambda v: -(-v // 256) * 256
    nb8, lnby = -(-nx // 8), -(-ny // 4)
    off_p4 = a256(hwords * 4) + a256(bnbx * bnby * 8)
    off_t4 = off_p4 + a256(lnby * nb8 * 32 * 4)
    off_e8 = off_t4 + a256(lnby * nb8 * 32 * 4)
    off_r16 = off_e8 + a256(lnby * nb8 * 32 * 8)
    off_p8 = off_r16 + a256(lnby * nb8 * 32 * 16)
    nb4 = -(-nx // 4)
    return dict(words=words, bsh=bsh, bnbx=bnbx, bnby=bnby, bnd_off=bnd_off, sbt_off=sbt_off,
                sbnbx=sbnbx, sbnby=sbnby, hwords=hwords, nb8=nb8, nb4=nb4, off_p4=off_p4,
                off_t4=off_t4, off_e8=off_e8, off_r16=off_r16, off_p8=off_p8,
                bytes=off_p8 + a256(lnby * nb4 * 16 * 8))


def _check_pack(raster, rec):
    """uam_raster_pack against its definition (uampath.hip, packed raster): the block codes,
    the five planes bit for bit, and bounds that hold every cell's terrain."""
    ny, nx = rec.shape[:2]
    B = raster.block
    d = _pack_dims(nx, ny, B)
    raw = raster.packed.cpu().numpy().view(np.uint8).reshape(-1)
    bits = rec.view(np.uint32)
    phi, psi, fl = bits[..., 0], bits[..., 1], bits[..., 3]
    ter = np.where(fl & 4, np.float32(0.0), rec[..., 2]).astype(np.float32)
    # codes
    nbx, nby = -(-nx // B), -(-ny // B)
    cw = raw[:d["words"] * 4].view(np.uint32)
    for by in range(nby):
        for bx in range(nbx):
            sl = (slice(by * B, (by + 1) * B), slice(bx * B, (bx + 1) * B))
            need = ((psi[sl] & 0x7fffffff) != 0).any() or ((fl[sl] & 1) != 0).any()
            neg = (((psi[sl] >> 31) != 0) & (psi[sl] != 0x80000000)).any()
            nz = ((phi[sl] & 0x7fffffff) != 0).any() or (ter[sl].view(np.uint32) != 0).any()
            want = (3 if neg else 2) if need else (1 if nz else 0)
            b = by * nbx + bx
            assert ((int(cw[b >> 4]) >> ((b & 15) * 2)) & 3) == want, (bx, by)
    # planes
    iy, ix = np.mgrid[0:ny, 0:nx]
    a4 = (((iy >> 2) * d["nb8"] + (ix >> 3)) << 5) | ((iy & 3) << 3) | (ix & 7)
    p4 = raw[d["off_p4"]:d["off_t4"]].view(np.uint32)
    t4 = raw[d["off_t4"]:d["off_e8"]].view(np.float32)
    e8 = raw[d["off_e8"]:d["off_r16"]].view(np.uint32).reshape(-1, 2)
    r16 = raw[d["off_r16"]:d["off_p8"]].view(np.uint32).reshape(-1, 4)
    p8 = raw[d["off_p8"]:d["bytes"]].view(np.uint32).reshape(-1, 2)
    assert raw.size >= d["bytes"]
    np.testing.assert_array_equal(r16[a4], bits.reshape(ny, nx, 4))
    a44 = (((iy >> 2) * d["nb4"] + (ix >> 2)) << 4) | ((iy & 3) << 2) | (ix & 3)
    np.testing.assert_array_equal(p8[a44, 0], phi)
    np.testing.assert_array_equal(p8[a44, 1], ter.view(np.uint32))
    np.testing.assert_array_equal(p4[a4], phi)
    np.testing.assert_array_equal(t4[a4].view(np.uint32), ter.view(np.uint32))
    np.testing.assert_array_equal(e8[a4, 0], phi)
    np.testing.assert_array_equal(e8[a4, 1], (psi & 0x7fffffff) | ((fl & 1) << 31).astype(np.uint32))
    # bounds: decoded as the kernels decode them (f32: base + q * step)
    bnd = raw[d["bnd_off"] * 4:].view(np.uint16)[:d["bnbx"] * d["bnby"]]
    sbt = raw[d["sbt_off"] * 4:].view(np.float32)[:2 * d["sbnbx"] * d["sbnby"]].reshape(-1, 2)
    bx, by = ix >> d["bsh"], iy >> d["bsh"]
    e = bnd[by * d["bnbx"] + bx].astype(np.uint32)
    sb = sbt[(by >> 2) * d["sbnbx"] + (bx >> 2)]
    with np.errstate(invalid="ignore"):
        ub = sb[..., 0] + (e & 255).astype(np.float32) * sb[..., 1]
        lb = sb[..., 0] + (e >> 8).astype(np.float32) * sb[..., 1]
    assert ub.dtype == np.float32
    # a superblock is unbounded (NaN) exactly where it holds a non-finite terrain value
    bad = ~np.isfinite(ter)
    sbi = (by >> 2) * d["sbnbx"] + (bx >> 2)
    bad_sb = np.zeros(d["sbnbx"] * d["sbnby"], bool)
    np.logical_or.at(bad_sb, sbi.ravel(), bad.ravel())
    np.testing.assert_array_equal(np.isnan(sb[..., 0]), bad_sb[sbi])
    ok = ~bad_sb[sbi]
    assert (lb[ok] <= ter[ok]).all() and (ter[ok] <= ub[ok]).all()
    return ok.mean(), np.mean((ub - lb)[ok])


@pytest.mark.parametrize("R,block", [(1024, 0), (1024, 4), (1000, 8)])
def test_raster_pack_layout(oracle_mod, R, block):
    """The packed copy (uam_raster_pack) equals its definition; with a DEM holding NaN and
    +inf cells and obstacle_smooth off (negative psi: code-3 blocks) as well."""
    from uam_path_planning_amd.engine import RasterGeo

    geo = None
    if R == 1000:
        geo = RasterGeo(nx=1000, ny=700, x0=8.0, y_top=5.0, dx=40.0 / 1000, dy=40.0 / 1000,
                        nodata=-9999.0, dem_threshold=0.0)
    e, orc, raster, rd, rec = _case(oracle_mod, 21, 40, R=R, geo=geo)
    if block:
        e.raster_summary(raster, block, packed=True)
    frac, width = _check_pack(raster, rec)
    assert frac == 1.0 and width < 60.0
    e, orc, raster, rd, rec = _case(oracle_mod, 21, 40, weights="zero", R=R, geo=geo,
                                    obstacle_smooth=False, dem_edit="nonfinite")
    if block:
        e.raster_summary(raster, block, packed=True)
    codes = _check_pack(raster, rec)
    assert 0.0 < codes[0] < 1.0


@pytest.mark.parametrize("dem_edit", [None, "nonfinite", "flat", "negzero"])
@pytest.mark.parametrize("stride", [0, 1, 5, 8, 1024])
def test_k2h_terrain_bounds(oracle_mod, stride, dem_edit):
    """The terrain maximum through the bounds (h_item): only where a waypoint's bound could
    still be the path's maximum is its terrain fetched; min_clearance (and every other output)
    equals orc_eval_generated_h bit for bit for every sample stride of the path lower bound
    (1: every waypoint; 1024: p_0 only), with unbounded superblocks (NaN / +inf cells), a
    terrain of a few values (blocks whose bounds coincide), -0.0 terrain cells, and no-fly
    psi below zero (obstacle_smooth off: code-3 records carry the terrain)."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, raster, rd, rec = _case(oracle_mod, 21, 80, R=1024, nfz=64, maxalpha=0.015,
                                    dem_edit=dem_edit, obstacle_smooth=dem_edit != "flat")
    e.set_option("k2h_terrain", 0)  # the bound form
    e.set_option("k2h_lb_stride", stride)
    assert e.get_option("k2h_lb_stride") == stride
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = _pairs(3000, 43)
    ref = orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=21)
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2h+pack"
    _check(gpu, ref, oracle_mod, D)
    for bad in (-3, 1025):
        with pytest.raises(ValueError):
            e.set_option("k2h_lb_stride", bad)


@pytest.mark.parametrize("stride", [0, 8])
@pytest.mark.parametrize("dem_edit", [None, "nonfinite", "flat", "negzero"])
@pytest.mark.parametrize("chunk,group", [(6, 24), (7, 21), (8, 21), (11, 5), (0, 64)])
def test_k2h_terrain_in_entry(oracle_mod, chunk, group, dem_edit, stride):
    """UAM_OPT_K2H_TERRAIN 1: the terrain from the entry (8-B {phi, terrain} entries in code
    1, the 16-B records in codes 2 / 3; code 0 by the bound rule, with or without the path seed):
    the same outputs as the oracle bit for bit, with non-finite, constant and -0.0 terrain
    cells; 0 and 1 are the only values."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, raster, rd, rec = _case(oracle_mod, group, 80, R=1024, nfz=64, maxalpha=0.015,
                                    dem_edit=dem_edit)
    e.set_option("k2h_terrain", 1)
    e.set_option("k2g_chunk", chunk)
    e.set_option("k2h_lb_stride", stride)
    assert e.get_option("k2h_terrain") == 1
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = _pairs(3000, 47)
    ref = orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=group)
    gpu = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == "K2h+pack" and e.last_group() == group
    _check(gpu, ref, oracle_mod, D)
    for bad in (-1, 2):
        with pytest.raises(ValueError):
            e.set_option("k2h_terrain", bad)


@pytest.mark.parametrize("group,D,N", [(21, 5, 80), (5, 5, 80), (64, 5, 80), (7, 16, 80),
                                       (21, 4, 1), (3, 3, 2)])
def test_k2h_waypoint_cells(oracle_mod, group, D, N):
    """Waypoint cells from K2h at cfg3's geometry (4096^2, 70 no-fly shapes) on a 2k-pair
    subsample: every index (-1 off the raster) equals the oracle's, the other outputs equal
    those of the same batch without cells.  D N > 1024 (16 x 80) reads the arc rows from
    global memory instead of LDS; N = 1 / 2 (3 / 4 cells a path) wrap every lane's run of 4."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, raster, rd, rec = _case(oracle_mod, group, N, R=4096, nfz=64)
    ut = arc_table(N, displacements(D))
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


@pytest.mark.parametrize("sim", [1, 0])
def test_sorted_device_check_surfaces(oracle_mod, sim):
    """A failed sort check on the device (forced by the test-only UAM_OPT_TEST_SORT_FAULT)
    poisons every output of the batch -- NaN in the f64 outputs, -1 in the counts and both
    selections -- and surfaces on the host: Engine.synchronize (uam_synchronize) raises
    DeviceCheckError once, and the next call runs clean (K2h and, with k2g_sim 0, K2g)."""
    from uam_path_planning_amd import _lib
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, raster, rd, rec = _case(oracle_mod, 21, 40)
    e.set_option("k2g_sim", sim)
    D = 5
    ut = arc_table(40, displacements(D))
    pairs = _pairs(1500, 51)
    e.set_option("test_sort_fault", 1)
    bad = e.eval_generated(pairs, ut, raster=raster)
    assert e.last_kernel() == ("K2h+pack" if sim else "K2g+pack")
    with pytest.raises(_lib.DeviceCheckError):
        e.synchronize()
    for k in ("cost", "length_q", "length", "kin_sum", "nfz_sum", "min_clearance"):
        assert np.isnan(bad[k].cpu().numpy()).all(), k
    for k in ("nfz_hits", "offmap", "best_fval_idx", "best_length_idx"):
        assert (bad[k].cpu().numpy() == -1).all(), k
    e.synchronize()   # reported once
    e.set_option("test_sort_fault", 0)
    gpu = e.eval_generated(pairs, ut, raster=raster)
    e.synchronize()
    if sim:
        _check(gpu, orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=21), oracle_mod, D)
    else:
        _check(gpu, orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="raster", rdesc=rd,
                                   rec=rec, group=21), oracle_mod, D)


def test_device_check_reported_by_next_call(oracle_mod):
    """Without a synchronize in between, the next uam_eval_generated on the context reports
    the earlier call's failed check (once the failing call has completed)."""
    from uam_path_planning_amd import _lib
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, raster, rd, rec = _case(oracle_mod, 21, 40)
    ut = arc_table(40, displacements(5))
    pairs = _pairs(800, 52)
    e.set_option("test_sort_fault", 1)
    e.eval_generated(pairs, ut, raster=raster)
    torch.cuda.synchronize()
    e.set_option("test_sort_fault", 0)
    with pytest.raises(_lib.DeviceCheckError):
        e.eval_generated(pairs, ut, raster=raster)
    e.eval_generated(pairs, ut, raster=raster)
    e.synchronize()


@pytest.mark.parametrize("R", [4096, 8192])
@pytest.mark.parametrize("sorted_min", [0, 65536])
def test_k2h_cells_vs_create_x_init(oracle_mod, R, sorted_min):
    """Verdict r5 item 1: the returned waypoint cells of eval_generated(want_cells=True) equal
    the cells of the reference's own create_x_init waypoints (solver.py:103-136; fixture
    tests/golden/waypoint_cells.npz, first 2000 cfg3 pairs x 5 d, N = 80) at 4096^2 and 8192^2:
    0 mismatches over 820 000 waypoints, through K2h + k_cells (sorted_min 0) and through the
    lane-per-path form the default picks for a batch this small."""
    import golden_io as G
    from uam_path_planning_amd import build
    from uam_path_planning_amd.engine import Engine, PathParams
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import build_region_map, canonical_spec, raster_geo
    from uam_path_planning_amd.arcs import arc_table

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    build.build_library()
    w = G.waypoint_cells()
    e = Engine(0)
    e.set_option("sorted_min_paths", sorted_min)
    if sorted_min == 0:
        e.set_option("wave_max_paths", 0)
    spec = canonical_spec(nfz_polygons=16)
    e.set_geometry(compile_map(build_region_map(spec)))
    e.set_params(PathParams(N=w["N"], **spec["options"], maxratio=spec["maxratio"],
                            maxalpha=spec["maxalpha"], enlargement=spec["enlargement"],
                            weights=tuple(spec["weights"]), altitude=320.0))
    raster = e.raster_build(raster_geo(R), None)
    g = e.eval_generated(w["pairs"], arc_table(w["N"], w["displacements"]), raster=raster,
                         want_cells=True)
    e.synchronize()
    if sorted_min == 0:
        assert e.last_kernel() == "K2h+pack"
    cells = g["cells"].cpu().numpy().reshape(w[f"cells{R}"].shape)
    assert int((cells != w[f"cells{R}"]).sum()) == 0
    del raster
    torch.cuda.empty_cache()
