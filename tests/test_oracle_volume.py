"""CPU: the oracle's volume mode (config 5, build-defined; SURVEY §8(d)'s layout of 8-B voxels
{risk, psi_nfz} plus a column plane {terrain, flags}) against a pure-Python restatement on a
small volume: voxel and column contents, and per path the cost, no-fly sum and hits, the
off-volume count, the layer-centre below-terrain count and the minimum clearance."""
import math
import struct

import numpy as np


def _f32(x):
    return struct.unpack("f", struct.pack("f", x))[0]


def test_volume_build_and_eval_vs_python(oracle_mod):
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec, displacements, layer_weights

    nx, ny, nz, z0, dz = 12, 9, 6, -20.0, 50.0
    x0, y_top, dx, dy = 10.0, 18.0, 3.0, 4.0
    rng = np.random.default_rng(3)
    rec2 = np.zeros((ny, nx, 4), np.float32)
    rec2[..., 0] = rng.uniform(0.0, 5.0, (ny, nx))
    rec2[..., 1] = np.where(rng.random((ny, nx)) < 0.3, rng.uniform(0.0, 2.0, (ny, nx)), 0.0)
    rec2[..., 2] = rng.uniform(-15.0, 240.0, (ny, nx))
    flags = (rng.random((ny, nx)) < 0.2).astype(np.uint32) * 1          # NFZ
    flags |= (rng.random((ny, nx)) < 0.25).astype(np.uint32) * 4        # NODATA
    rec2[..., 3] = flags.view(np.float32)
    lw = layer_weights(nz)
    vd = oracle_mod.volume_desc(nx, ny, nz, x0, y_top, dx, dy, z0, dz)
    vox, cols = oracle_mod.volume_build(vd, rec2, lw)
    for iy in range(ny):
        for ix in range(nx):
            terrain = 0.0 if flags[iy, ix] & 4 else rec2[iy, ix, 2]
            assert cols[iy, ix, 0] == np.float32(terrain)
            assert cols[iy, ix, 1:].view(np.uint32)[0] == flags[iy, ix] & 7
            for iz in range(nz):
                assert vox[iy, ix, iz, 0] == np.float32(_f32(float(rec2[iy, ix, 0]) * lw[iz]))
                assert vox[iy, ix, iz, 1] == rec2[iy, ix, 1]

    spec = canonical_spec()
    N, D = 10, 3
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), N, spec["options"], spec["maxratio"],
                            spec["maxalpha"], spec["enlargement"], spec["weights"])
    pairs = np.column_stack([rng.uniform(8.0, 48.0, 40), rng.uniform(-20.0, 20.0, 40),
                             rng.uniform(-40.0, 330.0, 40), rng.uniform(8.0, 48.0, 40),
                             rng.uniform(-20.0, 20.0, 40), rng.uniform(-40.0, 330.0, 40)])
    ut = arc_table(N, displacements(D))
    wp3 = oracle_mod.gen_paths3d(pairs, ut).reshape(-1, N + 2, 3)
    ref = orc.eval_paths3d(wp3, vd, (vox, cols))
    geo2 = orc.eval_paths(wp3[..., :2].copy(), mode="analytic")    # shape-free terms below
    for p in range(wp3.shape[0]):
        c, ns, nh, off, bel, cm = (N + 1) * ref["lq"][p], 0.0, 0, 0, 0, math.inf
        for x, y, z in wp3[p]:
            fx = math.floor((x - x0) * (1.0 / dx))
            fy = math.floor((y_top - y) * (1.0 / dy))
            fz = math.floor((z - z0) * (1.0 / dz))
            if not (0 <= fx < nx and 0 <= fy < ny and 0 <= fz < nz):
                off += 1
                continue
            r = vox[fy, fx, fz]
            terrain = float(cols[fy, fx, 0])
            c = c + float(r[0]) / N
            ns = ns + float(r[1])
            nh += int(flags[fy, fx] & 1)
            bel += int(z0 + (fz + 0.5) * dz < terrain)
            cm = min(cm, z - terrain)
        assert ref["cost"][p] == c and ref["nfz"][p] == ns, p
        assert (ref["nfz_hits"][p], ref["offmap"][p], ref["below"][p]) == (nh, off, bel), p
        assert ref["min_clearance"][p] == cm, p
        assert ref["length"][p] == geo2["length"][p] and ref["kin"][p] == geo2["kin"][p]
    assert ref["offmap"].any() and ref["below"].any() and ref["nfz_hits"].any()


def test_volume_similarity_form_vs_sequential(oracle_mod):
    """orc_eval_generated_h in volume mode (K4h's definition): the order-free outputs (hits,
    off-volume and below-terrain counts, min clearance) equal orc_eval_paths3d's exactly; cost,
    L, length and the no-fly sum differ by rounding only (grouped raster sums, similarity-form
    geometry)."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec, displacements, layer_weights
    from uam_path_planning_amd.synthetic import random_pairs3d

    nx, ny, nz, z0, dz = 64, 48, 16, 0.0, 40.0
    x0, y_top, dx, dy = 0.0, 20.0, 60.0 / 64, 60.0 / 64
    rng = np.random.default_rng(5)
    rec2 = np.zeros((ny, nx, 4), np.float32)
    rec2[..., 0] = rng.uniform(0.0, 5.0, (ny, nx))
    rec2[..., 1] = np.where(rng.random((ny, nx)) < 0.3, rng.uniform(0.0, 2.0, (ny, nx)), 0.0)
    rec2[..., 2] = rng.uniform(-15.0, 400.0, (ny, nx))
    rec2[..., 3] = ((rng.random((ny, nx)) < 0.2).astype(np.uint32)).view(np.float32)
    vd = oracle_mod.volume_desc(nx, ny, nz, x0, y_top, dx, dy, z0, dz)
    vol = oracle_mod.volume_build(vd, rec2, layer_weights(nz))
    spec = canonical_spec(nfz_polygons=0)
    N = 40
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), N, spec["options"], spec["maxratio"],
                            spec["maxalpha"], spec["enlargement"], spec["weights"])
    ut = arc_table(N, displacements(5))
    pairs = random_pairs3d(300, seed=8)
    pairs[::17, 2] = -30.0
    seq = orc.eval_paths3d(oracle_mod.gen_paths3d(pairs, ut), vd, vol, want_cells=True)
    for G in (0, 7, 21):
        h = orc.eval_generated_h(pairs, ut, mode="volume", vdesc=vd, vol=vol, group=G,
                                 want_cells=True)
        for k in ("nfz_hits", "offmap", "below", "min_clearance", "cells"):
            np.testing.assert_array_equal(h[k], seq[k], err_msg=k)
        for k in ("cost", "lq", "length", "nfz"):
            np.testing.assert_allclose(h[k], seq[k], rtol=1e-12, atol=1e-300, err_msg=k)
    assert (seq["offmap"] > 0).any() and (seq["below"] > 0).any() and (seq["nfz"] > 0).any()
