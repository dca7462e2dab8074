"""GPU refinement (uam_refine) against the oracle's orc_refine: the
refined waypoints, final cost, final infeasibility and step counts are compared with exact
equality (tolerance 0: same float64 operation order, no FMA contraction).  The reference's
OpEn solve itself is absent (parity unpinned vs the reference, see test_refine_cpu.py)."""
import dataclasses

import numpy as np
import pytest

import golden_io as G

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


def _setup(eng, oracle_mod, spec, N, options, maxratio, maxalpha, enl, weights, anchor):
    from uam_path_planning_amd.engine import PathParams
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import build_region_map

    eng.set_geometry(compile_map(build_region_map(spec)))
    eng.set_params(PathParams(N=N, **options, maxratio=maxratio, maxalpha=maxalpha,
                              enlargement=enl, weights=tuple(weights), anchor=anchor))
    return oracle_mod.Oracle(oracle_mod.compile_spec(spec), N, options, maxratio, maxalpha, enl,
                             weights, anchor=anchor)


def _check(eng, orc, oracle_mod, wp, **kw):
    gpu = eng.refine(wp, kw)
    ref = orc.refine(wp, oracle_mod.refine_params(**kw))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(gpu["iters"].cpu().numpy(), ref["iters"])
    np.testing.assert_array_equal(gpu["wp"].cpu().numpy(), ref["wp"])
    np.testing.assert_array_equal(gpu["cost"].cpu().numpy(), ref["cost"])
    np.testing.assert_array_equal(gpu["infeas"].cpu().numpy(), ref["infeas"])
    return gpu, ref


def test_refine_canonical_bit_exact(eng, oracle_mod):
    meta, arr = G.canonical()
    orc = _setup(eng, oracle_mod, meta["map"], meta["N"], meta["options"], meta["maxratio"],
                 meta["maxalpha"], meta["enlargement"], meta["weights"],
                 tuple(meta["map"]["x_start"]))
    wp = G.canonical_paths(meta, arr)
    gpu, ref = _check(eng, orc, oracle_mod, wp, n_outer=4, n_inner=12)
    assert (ref["iters"] > 0).all()
    before = eng.eval_waypoints(wp)["cost"].cpu().numpy()
    after = eng.eval_waypoints(gpu["wp"])["cost"].cpu().numpy()
    assert (after < before).all()


def test_refine_cfg3_geometry_bit_exact(eng, oracle_mod):
    """Generated candidates on the config-3 map (64 extra polygon no-fly zones, 69
    obstacle rows per waypoint) -- exercises the culled psi/psi_grad paths."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec, displacements
    from uam_path_planning_amd.synthetic import random_pairs

    spec = canonical_spec(nfz_polygons=64)
    N = 40
    opts = {"length_smooth": True, "penalty_smooth": True, "obstacle_smooth": True,
            "maxratio_smooth": False}
    orc = _setup(eng, oracle_mod, spec, N, opts, spec["maxratio"], spec["maxalpha"],
                 spec["enlargement"], spec["weights"], tuple(spec["x_start"]))
    ut = arc_table(N, displacements(5))
    wp = oracle_mod.gen_paths(random_pairs(24, seed=7), ut)
    _check(eng, orc, oracle_mod, wp, n_outer=3, n_inner=8)


def test_refine_edge_cases(eng, oracle_mod):
    from uam_path_planning_amd._lib import UamError

    meta, arr = G.canonical()
    opts = dict(meta["options"], maxratio_smooth=True)
    orc = _setup(eng, oracle_mod, meta["map"], meta["N"], opts, meta["maxratio"],
                 meta["maxalpha"], meta["enlargement"], meta["weights"],
                 tuple(meta["map"]["x_start"]))
    wp = G.canonical_paths(meta, arr)
    _check(eng, orc, oracle_mod, wp, n_outer=2, n_inner=6)          # smooth max-ratio rows
    _check(eng, orc, oracle_mod, wp[:0], n_outer=2, n_inner=6)      # empty batch
    _check(eng, orc, oracle_mod, wp, n_outer=0, n_inner=0)          # identity
    _check(eng, orc, oracle_mod, wp, n_outer=3, n_inner=10, memory=0)   # steepest descent
    _check(eng, orc, oracle_mod, wp, n_outer=3, n_inner=10, memory=3)   # ring wrap-around
    _check(eng, orc, oracle_mod, wp, n_outer=30, n_inner=60, inner_tol=1.0, delta=0.5)
    eng.set_params(dataclasses.replace(eng.params, obstacle_smooth=False))
    with pytest.raises((UamError, ValueError)):
        eng.refine(wp, {"n_outer": 1, "n_inner": 1})


def test_dropin_solver_solve(eng, oracle_mod):
    """Solver.solve(x_init, p) (solver.py:19-56 contract) = refinement of [x_start, x_init,
    x_goal] under p; fval = sqrt(get_cost(x)), length = length_of(x); bit-exact vs the oracle
    on the refined waypoints."""
    from uam_path_planning_amd.path_generation import Solver
    from uam_path_planning_amd.scenario import canonical_problem, canonical_spec

    spec = canonical_spec()
    prob = canonical_problem()
    solver = Solver(prob, {"refine": {"n_outer": 3, "n_inner": 10}})
    x_init = solver.create_x_init(0.25)
    params = list(spec["x_start"]) + list(spec["x_goal"]) + [
        spec["maxratio"], spec["maxalpha"], spec["enlargement"]] + list(spec["weights"])
    res = solver.solve(x_init, params)
    assert set(res) == {"x", "time", "fval", "length", "exit_status"}
    assert len(res["x"]) == 2 * prob.N
    z = np.concatenate([spec["x_start"], res["x"], spec["x_goal"]])
    assert res["fval"] == np.sqrt(prob.get_cost(z))
    assert res["length"] == prob.length_of(res["x"])
    assert res["exit_status"] in ("Converged", "NotConvergedIterations")
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), prob.N, spec["options"],
                            spec["maxratio"], spec["maxalpha"], spec["enlargement"],
                            spec["weights"], anchor=tuple(spec["x_start"]))
    wp0 = np.concatenate([spec["x_start"], x_init, spec["x_goal"]]).reshape(1, -1, 2)
    ref = orc.refine(wp0, oracle_mod.refine_params(n_outer=3, n_inner=10))
    np.testing.assert_array_equal(np.asarray(res["x"]), ref["wp"][0, 1:-1].reshape(-1))
    assert res["fval"] < np.sqrt(prob.get_cost(wp0.reshape(-1)))
    with pytest.raises(ValueError):
        solver.solve(x_init, params[:-1])


def test_dropin_solve_candidates_selection(eng):
    from uam_path_planning_amd.path_generation import Solver
    from uam_path_planning_amd.path_generation.solver import _select
    from uam_path_planning_amd.scenario import canonical_problem, canonical_spec

    spec = canonical_spec()
    prob = canonical_problem()
    solver = Solver(prob, {"refine": {"n_outer": 2, "n_inner": 8}})
    params = list(spec["x_start"]) + list(spec["x_goal"]) + [
        spec["maxratio"], spec["maxalpha"], spec["enlargement"]] + list(spec["weights"])
    res = solver.solve_candidates(params)
    assert res["x"].shape == (5, 2 * prob.N)
    assert res["min_fval_index"] == int(np.argmin(res["fval"]))
    assert res["min_length_index"] == int(np.argmin(res["length"]))
    one = solver.solve(solver.create_x_init(res["displacements"][2]), params)
    np.testing.assert_array_equal(np.asarray(one["x"]), res["x"][2])   # batch == single
    assert _select([3.0, 1.0, 1.0, 2.0]) == 1 and _select([0.0, 2.0]) == 1


def test_refine_large_paths_and_many_obstacles(eng, oracle_mod):
    """N = 254 (W = 256: 4 waypoints per lane, two waves per workgroup) and a map with more
    obstacles than the active-row masks hold (S > 256: the full-row fallback)."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec, displacements
    from uam_path_planning_amd.synthetic import random_pairs

    opts = {"length_smooth": True, "penalty_smooth": True, "obstacle_smooth": True,
            "maxratio_smooth": False}
    spec = canonical_spec(nfz_polygons=64)
    orc = _setup(eng, oracle_mod, spec, 254, opts, spec["maxratio"], spec["maxalpha"],
                 spec["enlargement"], spec["weights"], tuple(spec["x_start"]))
    wp = oracle_mod.gen_paths(random_pairs(3, seed=11), arc_table(254, displacements(5)))
    _check(eng, orc, oracle_mod, wp, n_outer=2, n_inner=5)
    many = canonical_spec(nfz_polygons=300, seed=4)          # 306 obstacles
    orc = _setup(eng, oracle_mod, many, 30, opts, many["maxratio"], many["maxalpha"],
                 many["enlargement"], many["weights"], tuple(many["x_start"]))
    wp = oracle_mod.gen_paths(random_pairs(8, seed=12), arc_table(30, displacements(5)))
    _check(eng, orc, oracle_mod, wp, n_outer=2, n_inner=6)


def test_refine_mask_widths_and_region_list_walk(eng, oracle_mod):
    """The wave-cooperative geometry walk in each of its forms: 106 obstacles (two active-row
    mask words per waypoint) and a region table of more than 256 shapes (no per-cell bitmask:
    the lanes' lists are merged by their minimum head)."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec, displacements
    from uam_path_planning_amd.synthetic import random_convex_polygons, random_pairs

    opts = {"length_smooth": True, "penalty_smooth": True, "obstacle_smooth": True,
            "maxratio_smooth": False}
    two = canonical_spec(nfz_polygons=100, seed=5)           # 106 obstacles
    orc = _setup(eng, oracle_mod, two, 40, opts, two["maxratio"], two["maxalpha"],
                 two["enlargement"], two["weights"], tuple(two["x_start"]))
    wp = oracle_mod.gen_paths(random_pairs(8, seed=13), arc_table(40, displacements(5)))
    _check(eng, orc, oracle_mod, wp, n_outer=3, n_inner=8)
    big = canonical_spec()
    big["regions"][1]["shapes"] = big["regions"][1]["shapes"] + [
        {"kind": "polygon", "vertices": v} for v in random_convex_polygons(260, seed=6)]
    assert sum(len(r["shapes"]) for r in big["regions"]) > 256
    orc = _setup(eng, oracle_mod, big, 40, opts, big["maxratio"], big["maxalpha"],
                 big["enlargement"], big["weights"], tuple(big["x_start"]))
    wp = oracle_mod.gen_paths(random_pairs(8, seed=14), arc_table(40, displacements(5)))
    _check(eng, orc, oracle_mod, wp, n_outer=3, n_inner=8)


def test_refine_restart_bit_exact(eng, oracle_mod):
    """n_restart > 0 (oracle refine_restart): a path that ends above delta is restarted with
    the waypoints inside the obstacle that holds most of them moved along the chord normal past
    its boundary; GPU == oracle bit for bit on the cfg3 map (70 no-fly shapes: polygons and
    balls, so both exit-distance forms run), and no path ends worse than without restarts (the
    first attempt is the no-restart run, the best attempt is kept)."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec, displacements
    from uam_path_planning_amd.synthetic import random_pairs

    spec = canonical_spec(nfz_polygons=64)
    N = 40
    orc = _setup(eng, oracle_mod, spec, N, spec["options"], spec["maxratio"], spec["maxalpha"],
                 spec["enlargement"], spec["weights"], tuple(spec["x_start"]))
    pairs = random_pairs(24, seed=5)
    wp = oracle_mod.gen_paths(pairs, arc_table(N, displacements(5))).reshape(-1, N + 2, 2)
    base = orc.refine(wp, oracle_mod.refine_params(n_outer=4, n_inner=12))
    gpu, ref = _check(eng, orc, oracle_mod, wp, n_outer=4, n_inner=12, n_restart=2,
                      restart_margin=0.05)
    assert (ref["infeas"] <= base["infeas"]).all()
    assert (ref["iters"] > base["iters"]).any()          # some paths were restarted
    assert (ref["infeas"] < base["infeas"]).any()        # and some came out better
