"""Pin the CPU oracle (oracle/uam_oracle.c + oracle/geometry.py) against golden vectors that
tests/golden/make_golden.py recorded from the reference's own cost model
(problem.py get_cost/get_nonlincon/length_of/get_penalty_function, solver.py create_x_init)."""
import numpy as np
import pytest

import golden_io as G


def _oracle(O, meta):
    geom = O.compile_spec(meta["map"])
    return O.Oracle(geom, meta["N"], meta["options"], meta["maxratio"], meta["maxalpha"],
                    meta["enlargement"], meta["weights"])


def test_canonical_bit_exact(oracle_mod):
    meta, arr = G.canonical()
    orc = _oracle(oracle_mod, meta)
    wp = G.canonical_paths(meta, arr)
    out = orc.eval_paths(wp, want_g=True)
    np.testing.assert_array_equal(out["cost"], arr["cost"])
    np.testing.assert_array_equal(out["length"], arr["length"])
    np.testing.assert_array_equal(out["lq"], arr["lq"])
    np.testing.assert_array_equal(out["g"], arr["g"])
    np.testing.assert_array_equal(out["nfz_hits"], arr["collide"].sum(1))
    # the survey's quoted numbers
    np.testing.assert_allclose(out["cost"], [2497.86843688, 3226.73830892, 2565.28161896,
                                             2288.09556814, 3428.58186125], rtol=1e-11)
    assert int(np.argmin(np.sqrt(out["cost"]))) == 3
    # g sum split (kinematic + no-fly rows) equals the golden row sum
    np.testing.assert_allclose(out["kin"] + out["nfz"], arr["g"].sum(1), rtol=1e-13, atol=1e-13)


def test_canonical_points(oracle_mod):
    meta, arr = G.canonical()
    orc = _oracle(oracle_mod, meta)
    pts = G.canonical_paths(meta, arr).reshape(-1, 2)
    pe = orc.eval_points(pts)
    np.testing.assert_array_equal(pe["phi"], arr["phi"].reshape(-1))
    np.testing.assert_array_equal(pe["phi_regions"],
                                  arr["phi_r"].transpose(0, 2, 1).reshape(-1, 3))
    np.testing.assert_array_equal(pe["obs_norm"], arr["obs_norm"].reshape(-1))
    np.testing.assert_array_equal(pe["collide"], arr["collide"].reshape(-1))


def test_variants(oracle_mod):
    meta, arr = G.canonical()
    v = G.variants()
    m = dict(meta)
    m["enlargement"] = 0.5
    orc = _oracle(oracle_mod, m)
    out = orc.eval_paths(G.canonical_paths(meta, arr), want_g=True)
    np.testing.assert_array_equal(out["cost"], v["enl05_cost"])
    np.testing.assert_array_equal(out["g"], v["enl05_g"])
    # problem.py demo: N=10, default options, weights 4/13/45
    m2 = dict(meta)
    m2.update(N=10, options=None, maxratio=1.25, maxalpha=np.pi / 10, enlargement=0.0,
              weights=[4, 13, 45])
    orc2 = _oracle(oracle_mod, m2)
    xs, xg = np.asarray(meta["map"]["x_start"]), np.asarray(meta["map"]["x_goal"])
    wp = np.stack([np.concatenate([xs, x, xg]).reshape(-1, 2) for x in v["n10_x_init"]])
    out2 = orc2.eval_paths(wp, want_g=True)
    np.testing.assert_array_equal(out2["cost"], v["n10_cost"])
    np.testing.assert_array_equal(out2["g"], v["n10_g"])


@pytest.mark.parametrize("ci", range(24))
def test_random_cases(oracle_mod, ci):
    case = G.random_cases()[ci]
    orc = _oracle(oracle_mod, case)
    wp = np.asarray(case["paths"]).reshape(len(case["paths"]), -1, 2)
    out = orc.eval_paths(wp, want_g=True)
    for i, o in enumerate(case["outputs"]):
        np.testing.assert_allclose(out["cost"][i], o["cost"], rtol=1e-13, equal_nan=True)
        np.testing.assert_allclose(out["g"][i], np.asarray(o["g"], float), rtol=1e-13,
                                   atol=1e-300, equal_nan=True)
        np.testing.assert_allclose(out["length"][i], o["length"], rtol=1e-14)
        np.testing.assert_allclose(out["lq"][i], o["lq"], rtol=1e-14)
        pe = orc.eval_points(wp[i])
        np.testing.assert_allclose(pe["phi"], np.asarray(o["phi"], float), rtol=1e-13,
                                   equal_nan=True)
        np.testing.assert_allclose(pe["phi_regions"], np.asarray(o["phi_r"], float).T,
                                   rtol=1e-13, equal_nan=True)
        np.testing.assert_allclose(pe["obs_norm"], np.asarray(o["obs_norm"], float),
                                   rtol=1e-13, equal_nan=True)
        np.testing.assert_array_equal(pe["collide"], np.asarray(o["collide"]))


def test_arcs(oracle_mod):
    a = G.arcs()
    for pi, pr in enumerate(a["pairs"]):
        for N in a["Ns"]:
            ref = a[f"p{pi}_N{N}"]
            ut = oracle_mod.arc_table(int(N), a["ds"])
            got = oracle_mod.gen_paths(pr[None, :], ut)[:, 1:-1, :].reshape(len(a["ds"]), -1)
            scale = max(1.0, float(np.abs(pr).max()))
            for i, d in enumerate(a["ds"]):
                # the arc's radius (1+d^2)/(2|d|) sets the cancellation both formulas suffer
                rho = 1.0 if d == 0 else (1 + d * d) / (2 * abs(d))
                np.testing.assert_allclose(got[i], ref[i], rtol=0,
                                           atol=1e-14 * scale * max(1.0, rho) * 8)


def test_raster_cell_centres(oracle_mod):
    """Raster mode pin: a record computed at a cell centre equals the reference's Φ / ψ /
    collides evaluated at that centre (rounded to f32)."""
    meta, _ = G.canonical()
    gr = G.grid()
    nx, ny, X0, Ytop, dx, dy = gr["geo"]
    geom = oracle_mod.compile_spec(meta["map"])
    rd = oracle_mod.Oracle.raster_desc(nx, ny, X0, Ytop, dx, dy)
    for tag, opts, enl in (("a", {"penalty_smooth": True, "obstacle_smooth": True}, 0.0),
                           ("b", {"penalty_smooth": False, "obstacle_smooth": False}, 0.25)):
        orc = oracle_mod.Oracle(geom, 4, opts, 1.1, 0.3, enl, [200, 15000, 27000])
        rec = orc.raster_build(rd)
        np.testing.assert_array_equal(rec[..., 0], gr[f"phi_{tag}"].astype(np.float32))
        np.testing.assert_array_equal(rec[..., 1], gr[f"psi_{tag}"].astype(np.float32))
        flags = rec[..., 3].view(np.uint32)
        np.testing.assert_array_equal(flags & 1, gr[f"collide_{tag}"])


def test_argmin_semantics(oracle_mod):
    # strict '<', first index wins on ties, NaN never wins, sentinel-0 quirk (main.py:175-180)
    v = np.array([3.0, 1.0, 1.0, 2.0,
                  np.nan, 5.0, 4.0, 4.0,
                  2.0, 0.0, 7.0, 9.0])
    best = oracle_mod.argmin(v, 4, False)
    assert best.tolist() == [1, 0, 2]


def test_geometry_errors(oracle_mod):
    errs = G.errors()
    from oracle import geometry as og
    for case, pts in (("polygon_two_points", [[0.0, 0.0], [1.0, 0.0]]),
                      ("polygon_collinear", [[0.0, 0.0], [1.0, 0.0], [2.0, 0.0], [1.0, 1.0]]),
                      ("polygon_nonconvex", [[0.0, 0.0], [4.0, 0.0], [1.0, 1.0], [0.0, 4.0]])):
        with pytest.raises(ValueError) as ei:
            og.shape_from_spec({"kind": "polygon", "vertices": pts})
        assert str(ei.value) == errs[case]["message"]
    with pytest.raises(ValueError) as ei:
        oracle_mod.arc_table(4, [1.5])
    assert str(ei.value) == errs["arc_displacement_gt1"]["message"]


def _gsum(terms, init, G):
    """K2g's grouped order in plain Python: terms (index, value) in index order; the values of
    indices [kG, (k+1)G) summed from +0.0, the partials added to init in group order."""
    tot, part, grp = init, 0.0, 0
    for idx, v in terms:
        if idx // G != grp:
            tot, part, grp = tot + part, 0.0, idx // G
        part = part + v
    return tot + part


def _grouped_restatement(wp, rec, rd, N, group, p):
    """Pure-Python statement of the K2g sum order (independent of uam_oracle.c): each term is
    attached to a waypoint (Φ/N and ψ of waypoint j to j, the segment p_{j-1} -> p_j's length
    terms to j, get_cost's anchor term to 0, kinematic row k to k + 1).  Returns per path
    (cost, L, length, kinematic sum, no-fly sum)."""
    import math
    W = N + 2
    r = p["maxratio"] ** 2 if p["maxratio_smooth"] else p["maxratio"]
    mincos = math.cos(p["maxalpha"])

    def nrm(s, smooth):
        n = math.sqrt(s)
        return n * n if smooth else n

    def seg(z, j):
        dx, dy = z[j, 0] - z[j - 1, 0], z[j, 1] - z[j - 1, 1]
        return dx, dy, (0.0 + dx * dx) + dy * dy

    out = []
    for z in wp:
        tl = [(0, nrm(0.0, p["length_smooth"]))]          # anchor = the path's own p_0
        tl += [(j, nrm(seg(z, j)[2], p["length_smooth"])) for j in range(1, N + 1)]
        tlen = [(j, math.sqrt(seg(z, j)[2])) for j in range(1, N + 2)]
        tk = []
        for k in range(N):
            ax, ay, sa = seg(z, k + 1)
            bx, by, sb = seg(z, k + 2)
            dt = (0.0 + ax * bx) + ay * by
            na, nb = nrm(sa, p["maxratio_smooth"]), nrm(sb, p["maxratio_smooth"])
            tk += [(k + 1, max(0.0, nb - r * na)), (k + 1, max(0.0, na / r - nb)),
                   (k + 1, max(0.0, mincos - dt / (na * nb)))]
        tc, tn = [], []
        for j in range(W):
            fx = np.floor((z[j, 0] - rd.x0) * (1.0 / rd.dx))
            fy = np.floor((rd.y_top - z[j, 1]) * (1.0 / rd.dy))
            if not (0.0 <= fx < rd.nx and 0.0 <= fy < rd.ny):
                continue
            rc = rec[int(fy), int(fx)]
            tc.append((j, float(rc[0]) / float(N)))
            tn.append((j, float(rc[1])))
        L = _gsum(tl, 0.0, group)
        out.append((_gsum(tc, float(N + 1) * L, group), L, _gsum(tlen, 0.0, group),
                    _gsum(tk, 0.0, group), _gsum(tn, 0.0, group)))
    return out


@pytest.mark.parametrize("group", [1, 3, 8, 16, 21, 200])
def test_grouped_sum_order(oracle_mod, group):
    """The grouped order of the segment-grouped raster evaluation (K2g; orc_eval_paths_g):
    the C oracle equals a pure-Python statement of it bit for bit, and differs from the
    reference's sequential order (problem.py:38-44, 84-114, 130-146; orc_eval_paths) by
    rounding only, far inside the north_star's 1e-5 -- the order-free outputs (hits, off-raster
    counts, clearance) are identical."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec, displacements, raster_geo
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    spec = canonical_spec(nfz_polygons=8)
    N = 40
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), N, spec["options"], spec["maxratio"],
                            spec["maxalpha"], spec["enlargement"], spec["weights"],
                            altitude=320.0)
    geo = raster_geo(256)
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy,
                                       geo.nodata, geo.dem_threshold)
    rec = orc.raster_build(rd, synthetic_dem(256))
    pairs = random_pairs(60, seed=4)
    pairs[::7, 0] += 40.0          # some waypoints off the raster
    pairs[5, :2] = pairs[5, 2:] + [0.7, -0.4]   # a short path: kinematic rows are active
    wp = oracle_mod.gen_paths(pairs, arc_table(N, displacements(5)))
    seq = orc.eval_paths(wp, mode="raster", rdesc=rd, rec=rec)
    grp = orc.eval_paths(wp, mode="raster", rdesc=rd, rec=rec, group=group)
    opts = dict(spec["options"], maxratio=spec["maxratio"], maxalpha=spec["maxalpha"])
    py = _grouped_restatement(wp, rec, rd, N, group, opts)
    for i, (c, L, ln, k, n) in enumerate(py):
        assert (c, L, ln, k, n) == (grp["cost"][i], grp["lq"][i], grp["length"][i],
                                    grp["kin"][i], grp["nfz"][i]), i
    for k in ("nfz_hits", "offmap", "min_clearance"):
        np.testing.assert_array_equal(grp[k], seq[k], err_msg=k)
    for k in ("cost", "lq", "length", "kin", "nfz"):
        np.testing.assert_allclose(grp[k], seq[k], rtol=1e-12, atol=1e-300, err_msg=k)
    assert (seq["offmap"] > 0).any() and (seq["nfz"] > 0).any() and (seq["kin"] > 0).any()


def _similarity_restatement(pairs, ut, N, p):
    """Pure-Python statement of the similarity form (independent of uam_oracle.c): per
    displacement row the unit polyline u_0 = (1, 0), u_1..u_N = the table row, u_{N+1} =
    (-1, 0), its chord sums and row sums; per candidate h = |x0 - xf| / 2 scales them.
    Returns per path (L, length, kinematic sum)."""
    import math
    mincos, r = math.cos(p["maxalpha"]), p["maxratio"]
    ug = []
    for row in ut:
        pts = [(1.0, 0.0)] + [tuple(x) for x in row] + [(-1.0, 0.0)]
        s1n = s2n = s1a = s2a = e12 = e3 = 0.0
        pb = pdx = pdy = 0.0
        for k in range(1, N + 2):
            dx, dy = pts[k][0] - pts[k - 1][0], pts[k][1] - pts[k - 1][1]
            b = math.sqrt(dx * dx + dy * dy)
            if k <= N:
                s1n, s2n = s1n + b, s2n + b * b
            s1a, s2a = s1a + b, s2a + b * b
            if k >= 2:
                e12 = e12 + max(0.0, b - r * pb)
                e12 = e12 + max(0.0, pb / r - b)
                e3 = e3 + max(0.0, mincos - (pdx * dx + pdy * dy) / (pb * b))
            pb, pdx, pdy = b, dx, dy
        ug.append((s1n, s2n, s1a, s2a, e12, e3))
    out = []
    for x0, y0, xf, yf in pairs:
        vx, vy = x0 - xf, y0 - yf
        s = vx * vx + vy * vy
        h, h2 = math.sqrt(s) * 0.5, s * 0.25
        for s1n, s2n, s1a, s2a, e12, e3 in ug:
            L = 0.0 + (h2 * s2n if p["length_smooth"] else h * s1n)   # anchor = p_0: 0
            ks = h * e12 + e3 if (h > 0.0 and h < math.inf) else 0.0
            out.append((L, h * s1a, ks))
    return out


@pytest.mark.parametrize("maxalpha", [np.pi / 80, 0.015])
def test_similarity_form(oracle_mod, maxalpha):
    """K2h's definition (orc_eval_generated_h): the geometry terms from the unit arc's sums
    scaled by h = |x0 - xf| / 2 equal a pure-Python statement bit for bit, and the reference's
    per-segment sums (problem.py:100-107, 130-146; orc_eval_paths) within rounding; the raster
    terms are the grouped order's (orc_eval_paths_g) bit for bit: no-fly sums, hits, off-raster
    counts, clearance, waypoint cells."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec, displacements, raster_geo
    from uam_path_planning_amd.synthetic import random_pairs, synthetic_dem

    spec = canonical_spec(nfz_polygons=8)
    N = 80
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), N, spec["options"], spec["maxratio"],
                            maxalpha, spec["enlargement"], spec["weights"], altitude=320.0)
    geo = raster_geo(256)
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy,
                                       geo.nodata, geo.dem_threshold)
    rec = orc.raster_build(rd, synthetic_dem(256))
    pairs = random_pairs(80, seed=14)
    pairs[::7, 0] += 40.0
    pairs[5, :2] = pairs[5, 2:] + [0.7, -0.4]
    pairs[9, 2:] = pairs[9, :2]          # start == goal
    ut = arc_table(N, displacements(5))
    wp = oracle_mod.gen_paths(pairs, ut)
    seq = orc.eval_paths(wp, mode="raster", rdesc=rd, rec=rec, want_cells=True)
    for G in (0, 21):
        h = orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=G, want_cells=True)
        grp = orc.eval_paths(wp, mode="raster", rdesc=rd, rec=rec, group=G)
        opts = dict(spec["options"], maxratio=spec["maxratio"], maxalpha=maxalpha)
        py = _similarity_restatement(pairs, ut, N, opts)
        for i, (L, ln, ks) in enumerate(py):
            assert (L, ln, ks) == (h["lq"][i], h["length"][i], h["kin"][i]), i
        for k in ("nfz_hits", "offmap", "min_clearance", "cells"):
            np.testing.assert_array_equal(h[k], seq[k], err_msg=k)
        np.testing.assert_array_equal(h["nfz"], grp["nfz"])
        ok = seq["length"] > 0
        for k in ("cost", "lq", "length"):
            np.testing.assert_allclose(h[k][ok], seq[k][ok], rtol=1e-12, err_msg=k)
        np.testing.assert_allclose(h["kin"], seq["kin"], rtol=1e-11, atol=1e-13)
        assert (h["kin"] > 0).any() == (maxalpha < 0.02)


def test_similarity_form_canonical_goldens(oracle_mod):
    """The similarity form on the reference's own canonical scenario (main.py: N = 80, the 5
    displacements of main.py:160): L, the length and the kinematic rows' sum agree with the
    reference's recorded values (create_x_init's transcendental waypoints, per-segment sums)
    within 1e-12 -- the geometry does not depend on the raster, a small one serves."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import raster_geo

    meta, arr = G.canonical()
    orc = _oracle(oracle_mod, meta)
    geo = raster_geo(64)
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy,
                                       geo.nodata, geo.dem_threshold)
    rec = np.zeros((64, 64, 4), np.float32)
    xs, xg = meta["map"]["x_start"], meta["map"]["x_goal"]
    pair = np.array([[xs[0], xs[1], xg[0], xg[1]]])
    h = orc.eval_generated_h(pair, arc_table(meta["N"], meta["displacements"]), rdesc=rd,
                             rec=rec, group=21)
    np.testing.assert_allclose(h["lq"], arr["lq"], rtol=1e-12)
    np.testing.assert_allclose(h["length"], arr["length"], rtol=1e-12)
    N = meta["N"]
    np.testing.assert_allclose(h["kin"], arr["g"][:, :3 * N].sum(1), rtol=1e-12, atol=1e-12)


def test_waypoint_cells_vs_create_x_init(oracle_mod):
    """Verdict r5 item 1: waypoint-index parity against the reference's own generator.  The
    fixture holds the raster cells of Solver.create_x_init's waypoints (arctan / cos / sin,
    solver.py:103-136; linspace for d = 0) for the first 2000 cfg3 pairs x 5 displacements at
    N = 80 on the 4096^2 and 8192^2 grids.  The build's table-based generator (arcs.py, the
    oracle's and the GPU's arc formula) lands every one of the 820 000 waypoints in the same
    cell at both sizes: 0 mismatches (GPU side: test_gpu_k2h.py::test_k2h_cells_vs_create_x_init)."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.synthetic import random_pairs

    w = G.waypoint_cells()
    assert np.array_equal(w["pairs"], random_pairs(100_000, seed=0)[:2000])
    wp = oracle_mod.gen_paths(w["pairs"], arc_table(w["N"], w["displacements"]))
    for R in (4096, 8192):
        inv = 1.0 / (60.0 / R)
        fx = np.floor((wp[..., 0] - 0.0) * inv)
        fy = np.floor((20.0 - wp[..., 1]) * inv)
        ok = (fx >= 0) & (fx < R) & (fy >= 0) & (fy < R)
        cells = np.where(ok, fy * R + fx, -1).astype(np.int64)
        ref = w[f"cells{R}"]
        assert (ref == -1).sum() > 0 and (ref >= 0).sum() > 800_000
        assert int((cells != ref).sum()) == 0, R
