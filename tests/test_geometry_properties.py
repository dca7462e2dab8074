"""Property tests (hypothesis, CPU) of the geometry path: random convex polygons in random
vertex order, ellipses and squares, in random maps.  The product's geometry compiler
(uam_path_planning_amd.geometry, behind polygon()/ball()/square() of path_generation) must
produce the oracle compiler's tables bit for bit (oracle/geometry.py restates
polygon.py:7-143, ball.py:7-52, square.py:6-65), raise the same errors for degenerate input,
and the oracle's evaluation must satisfy the model's invariants (a convex polygon contains its
vertex mean; the smooth penalty is exactly 0 outside every shape and positive at a shape's
centre).  SURVEY.md §4 asks for these alongside the golden vectors."""
import math

import numpy as np
import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

SETTINGS = settings(max_examples=60, deadline=None,
                    suppress_health_check=[HealthCheck.too_slow])


@st.composite
def convex_polygon(draw, shuffle=True):
    k = draw(st.integers(3, 8))
    cx = draw(st.floats(-50.0, 50.0))
    cy = draw(st.floats(-50.0, 50.0))
    a = draw(st.floats(0.2, 5.0))
    b = draw(st.floats(0.2, 5.0))
    rot = draw(st.floats(0.0, math.pi))
    jit = draw(st.lists(st.floats(0.0, 0.6), min_size=k, max_size=k))
    pts = []
    for i in range(k):
        t = 2 * math.pi * (i + jit[i]) / k
        x, y = a * math.cos(t), b * math.sin(t)
        pts.append([cx + x * math.cos(rot) - y * math.sin(rot),
                    cy + x * math.sin(rot) + y * math.cos(rot)])
    if shuffle:
        pts = draw(st.permutations(pts))
    return {"kind": "polygon", "vertices": [list(p) for p in pts]}


@st.composite
def ellipse(draw):
    c = [draw(st.floats(-50.0, 50.0)), draw(st.floats(-50.0, 50.0))]
    r1 = draw(st.floats(0.1, 5.0))
    r2 = draw(st.one_of(st.none(), st.floats(0.1, 5.0)))
    s = {"kind": "ball", "center": c, "r1": r1}
    if r2 is not None:
        s["r2"] = r2
    return s


@st.composite
def axis_square(draw):
    c = [draw(st.floats(-50.0, 50.0)), draw(st.floats(-50.0, 50.0))]
    s = {"kind": "square", "center": c, "r1": draw(st.floats(0.1, 5.0))}
    if draw(st.booleans()):
        s["r2"] = draw(st.floats(0.1, 5.0))
    return s


shape = st.one_of(convex_polygon(), ellipse(), axis_square())


@st.composite
def region_map(draw):
    obstacles = draw(st.lists(shape, min_size=0, max_size=4))
    regions = [{"name": f"r{i}", "color": "red",
                "shapes": draw(st.lists(shape, min_size=1, max_size=4))}
               for i in range(draw(st.integers(1, 3)))]
    return {"obstacles": obstacles, "regions": regions, "x_start": [0.0, 0.0],
            "x_goal": [1.0, 1.0]}


def _compile_both(oracle_mod, spec):
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import build_region_map

    return compile_map(build_region_map(spec)), oracle_mod.compile_spec(spec)


@SETTINGS
@given(spec=region_map())
def test_compiler_matches_oracle_on_random_maps(oracle_mod, spec):
    ours, ref = _compile_both(oracle_mod, spec)
    for k in ("ineq_kind", "ineq_par", "shape_first", "shape_count", "shape_center",
              "region_first"):
        np.testing.assert_array_equal(getattr(ours, k), getattr(ref, k), err_msg=k)
    assert ours.n_obstacles == ref.n_obstacles and ours.n_regions == ref.n_regions


@SETTINGS
@given(pts=st.lists(st.tuples(st.integers(-4, 4), st.integers(-4, 4)), min_size=3, max_size=7,
                    unique=True).map(lambda ps: [[float(a), float(b)] for a, b in ps]))
def test_degenerate_polygons_fail_like_the_oracle(oracle_mod, pts):
    """Points on a small integer lattice: collinear triples and non-convex orders are common.
    The product's polygon() must accept exactly what the oracle accepts, with the same message
    (polygon.py:82,92,128,133), and compile to the same inequalities otherwise."""
    from oracle import geometry as OG
    from uam_path_planning_amd.path_generation import polygon

    ref_err = ours_err = None
    try:
        ref = OG._polygon(pts)
    except ValueError as e:
        ref_err = str(e)
    try:
        ours = polygon(*pts)
    except ValueError as e:
        ours_err = str(e)
    assert ours_err == ref_err
    if ref_err is None:
        spec = {"obstacles": [{"kind": "polygon", "vertices": pts}], "regions": [],
                "x_start": [0.0, 0.0], "x_goal": [1.0, 1.0]}
        a, b = _compile_both(oracle_mod, spec)
        np.testing.assert_array_equal(a.ineq_par, b.ineq_par)
        assert len(ours.inequalities) == len(ref[0])


@SETTINGS
@given(poly=convex_polygon(), far=st.floats(200.0, 1e4))
def test_penalty_invariants(oracle_mod, poly, far):
    """A convex polygon contains its vertex mean (Map.collides, map.py:41-43), the smooth
    no-fly psi is exactly 0 far outside, and the smooth normalised penalty of a region with
    that polygon is exactly 1 at the polygon's centre (psi(c)/psi(c), problem.py:76-79)."""
    spec = {"obstacles": [poly], "regions": [{"name": "r", "color": "red", "shapes": [poly]}],
            "x_start": [0.0, 0.0], "x_goal": [1.0, 1.0]}
    geom = oracle_mod.compile_spec(spec)
    orc = oracle_mod.Oracle(geom, 4,
                            {"length_smooth": False, "penalty_smooth": True,
                             "obstacle_smooth": True, "maxratio_smooth": False},
                            1.1, 0.3, 0.0, [1.0])
    c = geom.shape_center[0]  # the vertex mean as polygon.py:141 forms it
    pts = np.array([c, c + [far, 0.0], c + [0.0, -far]])
    out = orc.eval_points(pts)
    assert out["collide"][0] == 1 and out["collide"][1] == 0 and out["collide"][2] == 0
    assert out["psi_raw"][0] > 0.0
    assert out["psi_raw"][1] == 0.0 and out["psi_raw"][2] == 0.0
    assert out["phi"][0] == 1.0
    assert out["phi"][1] == 0.0 and out["phi"][2] == 0.0
