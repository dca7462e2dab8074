"""K3b -- analytic-mode evaluation with the block's waypoints sorted by shape-grid cell
(k_eval_pairs_k3b, the default for uam_eval_generated in analytic mode without g rows) -- against
the CPU oracle, bit for bit, and against the lane-per-path K3 (UAM_OPT_K3B_SEGMENT = 0).

What is exercised: segment lengths 2/4/8/16 with W not a multiple of the segment (ragged last
segment), D = 1, 5, 16 (blockDim 64..1024; the LDS picks a shorter segment at D = 16), the pair
order on (>= 4096 pairs) and off, ragged blocks (Q % 64 != 0), points with two or more nonzero
no-fly psi terms (overlapping obstacles; the non-smooth obstacle psi, whose terms are nonzero
outside the shapes, and the path's own lane re-walks those points), NaN pairs (no grid slot:
the per-point fallback) and pairs off the shape grid.  Reference rule evaluated:
problem.py:38-44 (cost), 49-82 (Phi), 109-112 (no-fly rows), Map.collides."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

KEYS = (("cost", "cost"), ("length_q", "lq"), ("length", "length"), ("kin_sum", "kin"),
        ("nfz_sum", "nfz"), ("nfz_hits", "nfz_hits"), ("offmap", "offmap"))


def _engine(monkeypatch, seg, spec, params, cpl=2):
    from uam_path_planning_amd import build
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import build_region_map

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    build.build_library()
    e = Engine(0)
    e.set_option("k3b_segment", seg)
    e.set_option("k3b_points_per_lane", cpl)
    e.set_geometry(compile_map(build_region_map(spec)))
    e.set_params(params)
    return e


def _oracle(O, spec, params):
    opts = {k: getattr(params, k) for k in ("length_smooth", "penalty_smooth",
                                            "obstacle_smooth", "maxratio_smooth")}
    return O.Oracle(O.compile_spec(spec), params.N, opts, params.maxratio, params.maxalpha,
                    params.enlargement, list(params.weights), anchor=params.anchor,
                    altitude=params.altitude)


def _check(gpu, ref, D):
    import oracle.oracle as O

    for gk, ok in KEYS:
        np.testing.assert_array_equal(gpu[gk].cpu().numpy(), ref[ok], err_msg=gk)
    np.testing.assert_array_equal(gpu["best_fval_idx"].cpu().numpy(),
                                  O.argmin(ref["cost"], D, True))
    np.testing.assert_array_equal(gpu["best_length_idx"].cpu().numpy(),
                                  O.argmin(ref["length"], D, False))


def _cfg3(N, **opt):
    from uam_path_planning_amd.scenario import CONFIGS, canonical_params, canonical_spec

    spec = canonical_spec(nfz_polygons=CONFIGS["cfg3"]["nfz_polygons"])
    params = canonical_params(spec, N=N, altitude=320.0)
    for k, v in opt.items():
        setattr(params, k, v)
    return spec, params


@pytest.mark.parametrize("cpl", [1, 2])
@pytest.mark.parametrize("seg", [2, 4, 8, 16])
@pytest.mark.parametrize("N", [40, 80])
def test_k3b_cfg3_segments(oracle_mod, monkeypatch, seg, N, cpl):
    """cfg3 geometry (104 shapes, overlapping random no-fly polygons), 4500 pairs x 5 (pair
    order on): every output and both selections equal the oracle's bit for bit."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import displacements
    from uam_path_planning_amd.synthetic import random_pairs

    spec, params = _cfg3(N)
    e = _engine(monkeypatch, seg, spec, params, cpl)
    D = 5
    ut = arc_table(N, displacements(D))
    pairs = random_pairs(4500, seed=21)
    gpu = e.eval_generated(pairs, ut)
    ref = _oracle(oracle_mod, spec, params).eval_paths(oracle_mod.gen_paths(pairs, ut))
    _check(gpu, ref, D)


@pytest.mark.parametrize("D", [1, 16])
@pytest.mark.parametrize("opts", [dict(obstacle_smooth=True), dict(penalty_smooth=False),
                                  dict(obstacle_smooth=False, enlargement=0.3)])
def test_k3b_options_nan_offgrid(oracle_mod, monkeypatch, D, opts):
    """D = 1 / 16, smooth / non-smooth penalties, enlargement: ragged batch (1000 pairs, order
    off) with NaN pairs and pairs far off the shape grid."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.synthetic import random_pairs

    spec, params = _cfg3(24, **opts)
    e = _engine(monkeypatch, 8, spec, params)
    ds = np.linspace(-1.0, 1.0, D) if D > 1 else np.array([0.4])
    ut = arc_table(24, ds)
    pairs = random_pairs(1000, seed=7)
    pairs[3, 0] = np.nan          # NaN start: every waypoint NaN
    pairs[10, 3] = np.nan         # NaN goal coordinate
    pairs[20] = [-200.0, -300.0, 250.0, 400.0]   # crosses far off the grid
    pairs[21] = [-200.0, -300.0, -150.0, -320.0]  # entirely off the grid
    gpu = e.eval_generated(pairs, ut)
    ref = _oracle(oracle_mod, spec, params).eval_paths(oracle_mod.gen_paths(pairs, ut))
    _check(gpu, ref, D)


def test_k3b_multi_psi_terms(oracle_mod, monkeypatch):
    """Three overlapping no-fly balls and a polygon over them, smooth obstacle psi: waypoints in
    the overlap carry 2-4 nonzero psi terms, which the path's lane re-walks in eval_path's
    order.  Checked against the oracle and against the lane-per-path K3."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec

    spec = canonical_spec()
    spec["obstacles"] = spec["obstacles"] + [
        {"kind": "ball", "center": [30.0, -10.0], "r1": 4.0, "r2": 3.0},
        {"kind": "ball", "center": [32.0, -9.0], "r1": 3.0, "r2": 3.0},
        {"kind": "ball", "center": [31.0, -11.0], "r1": 2.5, "r2": 2.0},
        {"kind": "polygon", "vertices": [[27.0, -14.0], [35.0, -14.0], [35.0, -6.0],
                                         [27.0, -6.0]]}]
    from uam_path_planning_amd.scenario import canonical_params

    params = canonical_params(spec, N=60, altitude=200.0)
    params.obstacle_smooth = True
    rng = np.random.default_rng(3)
    Q = 5000
    pairs = np.stack([rng.uniform(24, 38, Q), rng.uniform(-16, -4, Q),
                      rng.uniform(24, 38, Q), rng.uniform(-16, -4, Q)], axis=1)
    ut = arc_table(60, np.linspace(-1.0, 1.0, 5))
    ref = _oracle(oracle_mod, spec, params).eval_paths(oracle_mod.gen_paths(pairs, ut))
    assert np.count_nonzero(ref["nfz"]) > Q  # most paths cross the overlap
    e = _engine(monkeypatch, 8, spec, params)
    gpu = e.eval_generated(pairs, ut)
    _check(gpu, ref, 5)
    e0 = _engine(monkeypatch, 0, spec, params)   # lane-per-path K3
    g0 = e0.eval_generated(pairs, ut)
    for gk, _ in KEYS:
        np.testing.assert_array_equal(g0[gk].cpu().numpy(), gpu[gk].cpu().numpy(), err_msg=gk)


@pytest.mark.parametrize("ci", range(24))
def test_k3b_random_cases(oracle_mod, monkeypatch, ci):
    """The 24 golden random maps (polygons in shuffled vertex order, ellipses, squares, all 16
    option combinations, enlargements -0.2 / 0 / 0.3; NaN where the reference's normalisers are
    0/0) through K3b: 300 generated pairs over each map's extent x 5 displacements, every
    output bit-exact vs the oracle (NaN where the oracle has NaN)."""
    import golden_io as G

    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.engine import PathParams

    c = G.random_cases()[ci]
    params = PathParams(N=c["N"], **c["options"], maxratio=c["maxratio"],
                        maxalpha=c["maxalpha"], enlargement=c["enlargement"],
                        weights=tuple(c["weights"]), anchor=tuple(c["map"]["x_start"]))
    e = _engine(monkeypatch, 8, c["map"], params)
    rng = np.random.default_rng(100 + ci)
    Q = 300
    pairs = rng.uniform(-5.0, 5.0, size=(Q, 4))
    ut = arc_table(c["N"], np.linspace(-1.0, 1.0, 5))
    gpu = e.eval_generated(pairs, ut)
    ref = _oracle(oracle_mod, c["map"], params).eval_paths(oracle_mod.gen_paths(pairs, ut))
    _check(gpu, ref, 5)
