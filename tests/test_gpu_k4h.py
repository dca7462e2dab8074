"""K4h -- the volume (BASELINE config 5) in K2h's form: the packed copy (uam_volume_pack: one
4-B risk / 8-B risk+psi / 16-B voxel {risk, psi_nfz, terrain, flags} planes per layer in 4 x 8-
column blocks at one index, chosen per 8 x 8 columns by a code; the column terrain by bounds),
the (path, group) items sorted on the altitude band and x/y tile of their middle waypoint,
grouped partial sums, the geometry terms in the similarity form.  Against the oracle's
statement of it (orc_eval_generated_h, mode 2) bit for bit; against the sequential
lane-per-path K4 (orc_eval_paths3d) within rounding for the sums and exactly for the order-free
outputs (hits, off-volume counts, min clearance, below-terrain counts).  Reference rules as
K2h (no reference counterpart for the altitude terms)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

KEYS = (("cost", "cost"), ("length_q", "lq"), ("length", "length"), ("kin_sum", "kin"),
        ("nfz_sum", "nfz"), ("nfz_hits", "nfz_hits"), ("offmap", "offmap"),
        ("min_clearance", "min_clearance"), ("below_terrain", "below"))


def _case(oracle_mod, R, nz, N, group, maxalpha=None):
    from uam_path_planning_amd import build
    from uam_path_planning_amd.engine import Engine, PathParams
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (build_region_map, canonical_spec, layer_weights,
                                                raster_geo)
    from uam_path_planning_amd.synthetic import synthetic_dem

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    build.build_library()
    e = Engine(0)
    e.set_option("group", group)
    e.set_option("sorted_min_paths", 0)
    e.set_option("wave_max_paths", 0)
    spec = canonical_spec(nfz_polygons=16)
    ma = spec["maxalpha"] if maxalpha is None else maxalpha
    e.set_geometry(compile_map(build_region_map(spec)))
    e.set_params(PathParams(N=N, **spec["options"], maxratio=spec["maxratio"], maxalpha=ma,
                            enlargement=spec["enlargement"], weights=tuple(spec["weights"]),
                            altitude=320.0))
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), N, spec["options"],
                            spec["maxratio"], ma, spec["enlargement"], spec["weights"],
                            altitude=320.0)
    geo = raster_geo(R)
    r2 = e.raster_build(geo, synthetic_dem(R))
    lw = layer_weights(nz)
    vol = e.volume_build(r2, nz, 0.0, 640.0 / nz, lw)
    e.volume_pack(vol)
    vd = oracle_mod.volume_desc(R, R, nz, geo.x0, geo.y_top, geo.dx, geo.dy, 0.0, 640.0 / nz)
    host = (vol.vox.cpu().numpy().view(np.float32), vol.cols.cpu().numpy().view(np.float32))
    return e, orc, vol, vd, host


def _pairs3d(n, seed):
    from uam_path_planning_amd.synthetic import random_pairs3d

    pr = random_pairs3d(n, seed=seed)
    pr[::41, 2] = -50.0          # climbs in from below the volume
    pr[::43, 5] = 900.0          # leaves it at the top
    pr[::97, 0] += 70.0          # off the x/y grid
    pr[5, 1] = np.nan
    pr[11, 3:5] = pr[11, 0:2]    # start == goal (h = 0)
    return pr


def _check(gpu, ref, oracle_mod, D):
    for gk, ok in KEYS:
        np.testing.assert_array_equal(gpu[gk].cpu().numpy(), ref[ok], err_msg=gk)
    np.testing.assert_array_equal(gpu["best_fval_idx"].cpu().numpy(),
                                  oracle_mod.argmin(ref["cost"], D, True))
    np.testing.assert_array_equal(gpu["best_length_idx"].cpu().numpy(),
                                  oracle_mod.argmin(ref["length"], D, False))


@pytest.mark.parametrize("terrain", [1, 0])
@pytest.mark.parametrize("R,nz,group", [(256, 16, 21), (256, 64, 8), (512, 7, 21),
                                        (300, 33, 64), (256, 16, 1)])
def test_k4h_vs_oracle(oracle_mod, R, nz, group, terrain):
    """Volumes with nx not a multiple of the block width (300), odd layer counts (7, 33: the
    altitude bands' last band partial), groups of 1-64; every output equals orc_eval_generated_h
    bit for bit; against the sequential K4 form: exact for the order-free outputs, rounding
    for the sums."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, vol, vd, host = _case(oracle_mod, R, nz, 80, group)
    e.set_option("k4h_terrain", terrain)  # 0 (default): bounds; 1: the terrain in the entry
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = _pairs3d(3000, 17)
    ref = orc.eval_generated_h(pairs, ut, mode="volume", vdesc=vd, vol=host, group=group)
    assert (ref["offmap"] > 0).any() and (ref["below"] > 0).any()
    gpu = e.eval_generated3d(pairs, ut, vol)
    assert e.last_kernel() == "K4h+pack" and e.last_group() == group
    _check(gpu, ref, oracle_mod, D)
    seq = orc.eval_paths3d(oracle_mod.gen_paths3d(pairs, ut), vd, host)
    for k in ("nfz_hits", "offmap", "min_clearance", "below"):
        np.testing.assert_array_equal(ref[k], seq[k], err_msg=k)
    ok = np.isfinite(seq["cost"]) & (seq["length"] > 0)
    np.testing.assert_allclose(ref["cost"][ok], seq["cost"][ok], rtol=1e-12)


@pytest.mark.parametrize("terrain", [1, 0])
@pytest.mark.parametrize("chunk,floor", [(6, 0), (7, 0), (8, 0), (11, 0), (0, 0), (6, 28000),
                                         (11, 41000), (8, 90000), (16, 0), (21, 90000)])
def test_k4h_chunks(oracle_mod, chunk, floor, terrain):
    """Gathers in flight (chunk; 0 = the default 11) and workgroups per CU (the LDS floor; 0 =
    the default 60 000 B, 90 000 needs the raised dynamic-LDS attribute) only move work."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, vol, vd, host = _case(oracle_mod, 256, 16, 80, 21, maxalpha=0.015)
    e.set_option("k2g_chunk", chunk)
    e.set_option("k2g_lds_floor", floor)
    e.set_option("k4h_terrain", terrain)
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = _pairs3d(2000, 23)
    ref = orc.eval_generated_h(pairs, ut, mode="volume", vdesc=vd, vol=host, group=21)
    assert (ref["kin"] > 0).any()
    gpu = e.eval_generated3d(pairs, ut, vol)
    assert e.last_kernel() == "K4h+pack"
    _check(gpu, ref, oracle_mod, D)


@pytest.mark.parametrize("tile_bits,band", [(5, 0), (6, 0), (4, 2), (3, 16), (3, 1)])
def test_k4h_tile_bits_and_bands(oracle_mod, tile_bits, band):
    """The sort key's tiles (UAM_OPT_K2G_TILE_BITS, a raster setting: 5 and 6 give more
    (tile, band) bins than the sort holds at 64 layers, so the key takes the finest tiles that
    fit) and altitude bands (UAM_OPT_K4H_BAND: 1, 2, 16 layers) only move work."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, vol, vd, host = _case(oracle_mod, 256, 64, 80, 21, maxalpha=0.015)
    e.set_option("k2g_tile_bits", tile_bits)
    e.set_option("k4h_band", band)
    assert e.get_option("k4h_band") == band
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = _pairs3d(2000, 29)
    ref = orc.eval_generated_h(pairs, ut, mode="volume", vdesc=vd, vol=host, group=21)
    gpu = e.eval_generated3d(pairs, ut, vol)
    assert e.last_kernel() == "K4h+pack"
    _check(gpu, ref, oracle_mod, D)


def _vary_psi(e, vol):
    """Layer-varying psi in some columns (a psi of 0.25 at layer 3 only, every 13th row and
    37th column from 5, inside and outside the no-fly support): their 8 x 8-column blocks
    must take the 16-B table (code 3) although layer 0's psi is +0 in many of them; the packed
    copy is rebuilt."""
    vol.vox[::13, 5::37, 3, 1] = int(np.float32(0.25).view(np.int32))  # (int32 view)
    torch.cuda.synchronize()
    e.volume_pack(vol)


def test_k4h_pack_layout(oracle_mod):
    """uam_volume_pack against its definition (uampath.hip VpkDims / KVol4): the 4-B risk and
    8-B {risk, |psi| | nfz << 31} planes per layer (4 x 8-column blocks, one index), the 16-B
    voxels ({risk, psi} of the voxel, {terrain, flags} of the column; 4 x 2-column blocks), the
    8-B {risk, terrain} plane (4 x 4-column blocks), the column terrain (4 x 8), zero
    padding, the 2-bit code per 8 x 8 columns (3: a psi below zero in any
    layer; 2: another nonzero psi or the no-fly flag; 1: a nonzero risk; 0: none), and terrain
    bounds that hold every column."""
    from test_host_cpu import _vpk_sections

    e, orc, vol, vd, host = _case(oracle_mod, 300, 7, 10, 21)
    _vary_psi(e, vol)
    raw = vol.packed.cpu().numpy()
    ny, nx, nz = 300, 300, 7
    sec = _vpk_sections(nx, ny, nz)
    off = np.cumsum([0] + sec)
    assert raw.nbytes == off[-1]
    b = raw.view(np.uint8)
    nb8, lnby4 = (nx + 7) // 8, (ny + 3) // 4
    layer = lnby4 * nb8 * 32
    r4 = b[off[2]:off[2] + layer * nz * 4].view(np.uint32)
    t4 = b[off[3]:off[3] + layer * 4].view(np.float32)
    e8 = b[off[4]:off[4] + layer * nz * 8].view(np.uint32).reshape(-1, 2)
    nbx4, nby2 = (nx + 3) // 4, (ny + 1) // 2
    layer42 = nby2 * nbx4 * 8
    t16 = b[off[5]:off[5] + layer42 * nz * 16].view(np.int32).reshape(-1, 4)
    nb4 = (nx + 3) // 4
    layer44 = lnby4 * nb4 * 16
    q8 = b[off[6]:off[6] + layer44 * nz * 8].view(np.uint32).reshape(-1, 2)
    iz, iy, ix = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    vox = vol.vox.cpu().numpy()            # [ny, nx, nz, 2]
    cols = vol.cols.cpu().numpy()          # [ny, nx, 2]
    vz = vox.transpose(2, 0, 1, 3).reshape(-1, 2)
    cz = np.broadcast_to(cols, (nz, ny, nx, 2)).reshape(-1, 2)
    i4 = (((iz * lnby4 + iy // 4) * nb8 + ix // 8) * 32 + (iy % 4) * 8 + ix % 8).reshape(-1)
    i42 = ((iz * layer42) + ((iy // 2) * nbx4 + ix // 4) * 8 + (iy % 2) * 4 + ix % 4).reshape(-1)
    np.testing.assert_array_equal(t16[i42], np.concatenate([vz, cz], axis=1))
    np.testing.assert_array_equal(r4[i4], vz[:, 0].view(np.uint32))
    pz = (vz[:, 1].view(np.uint32) & 0x7fffffff) | ((cz[:, 1].view(np.uint32) & 1) << 31)
    np.testing.assert_array_equal(e8[i4], np.stack([vz[:, 0].view(np.uint32), pz], axis=1))
    it = (((iy[0] // 4) * nb8 + ix[0] // 8) * 32 + (iy[0] % 4) * 8 + ix[0] % 8)
    np.testing.assert_array_equal(t4[it].view(np.uint32), cols[:, :, 0].view(np.uint32))
    i44 = ((iz * layer44) + ((iy // 4) * nb4 + ix // 4) * 16 + (iy % 4) * 4 + ix % 4).reshape(-1)
    np.testing.assert_array_equal(q8[i44], np.stack([vz[:, 0].view(np.uint32),
                                                     cz[:, 0].view(np.uint32)], axis=1))
    for t, idx in ((t16, i42), (r4, i4), (e8, i4), (t4.view(np.uint32), it.reshape(-1)),
                   (q8, i44)):
        mask = np.ones(len(t), bool)
        mask[idx] = False
        assert (t[mask] == 0).all()
    # codes
    cnbx = cnby = (nx + 7) // 8
    cw = (cnbx * cnby + 15) // 16
    cm = b[:cw * 4].view(np.uint32)
    pb = vox[:, :, :, 1].view(np.uint32)
    rb = vox[:, :, :, 0].view(np.uint32)
    nfz = cols[:, :, 1].view(np.uint32) & 1

    def blk(a):
        full = np.zeros((cnby * 8, cnbx * 8), bool)
        full[:ny, :nx] = a
        return full.reshape(cnby, 8, cnbx, 8).any(axis=(1, 3)).reshape(-1)

    need = blk(((pb & 0x7fffffff) != 0).any(axis=2) | (nfz != 0))
    neg = blk((((pb >> 31) != 0) & (pb != 0x80000000)).any(axis=2))
    nzr = blk(((rb & 0x7fffffff) != 0).any(axis=2))
    want = np.where(need, np.where(neg, 3, 2), np.where(nzr, 1, 0))
    got = ((cm[:, None] >> (2 * np.arange(16))) & 3).reshape(-1)[:cnbx * cnby]
    np.testing.assert_array_equal(got, want)
    assert (want == 2).any() and (want == 1).any()
    # bounds hold every column's terrain
    bsh = 3
    bnbx = -(-nx // 8)
    w16 = lambda v: -(-v // 16) * 16
    bnd = b[w16(cw * 4):].view(np.uint16)[:bnbx * bnbx]
    sbo = w16(cw * 4) + w16(bnbx * bnbx * 2)
    sbnbx = -(-bnbx // 4)
    sbt = b[sbo:sbo + sbnbx * sbnbx * 8].view(np.float32).reshape(-1, 2)
    yy, xx = np.mgrid[0:ny, 0:nx]
    e = bnd[(yy >> bsh) * bnbx + (xx >> bsh)].astype(np.uint32)
    sb = sbt[((yy >> bsh) >> 2) * sbnbx + ((xx >> bsh) >> 2)]
    ub = sb[..., 0] + (e & 255).astype(np.float32) * sb[..., 1]
    lb = sb[..., 0] + (e >> 8).astype(np.float32) * sb[..., 1]
    ter = cols[:, :, 0].view(np.float32)
    assert (lb <= ter).all() and (ter <= ub).all()


@pytest.mark.parametrize("group", [21, 7])
def test_k4h_layer_varying_psi(oracle_mod, group):
    """A volume whose psi varies by layer in some columns, nonzero at layer 3 only in columns
    outside the no-fly support: their blocks must read the 16-B table, or the 8-B voxel's
    implied psi of +0 would drop the layer-3 terms; every output equals orc_eval_generated_h on
    the same voxels bit for bit."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, vol, vd, host = _case(oracle_mod, 256, 16, 80, group, maxalpha=0.015)
    _vary_psi(e, vol)
    host = (vol.vox.cpu().numpy().view(np.float32), vol.cols.cpu().numpy().view(np.float32))
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = _pairs3d(2000, 29)
    ref = orc.eval_generated_h(pairs, ut, mode="volume", vdesc=vd, vol=host, group=group)
    gpu = e.eval_generated3d(pairs, ut, vol)
    assert e.last_kernel() == "K4h+pack"
    _check(gpu, ref, oracle_mod, D)


def test_k4h_stale_pack_rebuilt(oracle_mod):
    """Voxels written in place after volume_pack (no explicit repack): eval_generated3d sees
    the buffer's version change and rebuilds the packed copy, so K4h evaluates the new voxels
    (every output equals orc_eval_generated_h on them)."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, vol, vd, host = _case(oracle_mod, 256, 16, 80, 21, maxalpha=0.015)
    old = vol.packed
    vol.vox[::7, 3::11, :, 0] = int(np.float32(2.5).view(np.int32))   # risk, every layer
    vol.vox[::13, 5::37, 3, 1] = int(np.float32(0.25).view(np.int32))
    torch.cuda.synchronize()
    host = (vol.vox.cpu().numpy().view(np.float32), vol.cols.cpu().numpy().view(np.float32))
    D = 5
    ut = arc_table(80, displacements(D))
    pairs = _pairs3d(2000, 31)
    ref = orc.eval_generated_h(pairs, ut, mode="volume", vdesc=vd, vol=host, group=21)
    gpu = e.eval_generated3d(pairs, ut, vol)
    assert e.last_kernel() == "K4h+pack" and vol.packed is not old
    _check(gpu, ref, oracle_mod, D)


def test_k4h_device_check_surfaces(oracle_mod):
    """K4h's failed sort check (forced, UAM_OPT_TEST_SORT_FAULT) poisons every output, the
    below-terrain count included, and raises DeviceCheckError at the next synchronize."""
    from uam_path_planning_amd import _lib
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements

    e, orc, vol, vd, host = _case(oracle_mod, 256, 16, 80, 21)
    ut = arc_table(80, displacements(5))
    pairs = _pairs3d(1000, 61)
    e.set_option("test_sort_fault", 1)
    bad = e.eval_generated3d(pairs, ut, vol)
    assert e.last_kernel() == "K4h+pack"
    with pytest.raises(_lib.DeviceCheckError):
        e.synchronize()
    for k in ("cost", "length_q", "length", "kin_sum", "nfz_sum", "min_clearance"):
        assert np.isnan(bad[k].cpu().numpy()).all(), k
    for k in ("nfz_hits", "offmap", "below_terrain", "best_fval_idx", "best_length_idx"):
        assert (bad[k].cpu().numpy() == -1).all(), k
    e.set_option("test_sort_fault", 0)
    gpu = e.eval_generated3d(pairs, ut, vol)
    e.synchronize()
    _check(gpu, orc.eval_generated_h(pairs, ut, mode="volume", vdesc=vd, vol=host, group=21),
           oracle_mod, 5)
