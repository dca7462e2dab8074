"""Refinement oracle (oracle/uam_oracle.c orc_refine) on the CPU.
The reference's own optimiser (OpEn/CasADi, solver.py:82-93) is a Rust build that is absent
here, so the refinement result is parity unpinned against the reference; what is pinned is
(a) its objective -- get_cost of the refined path is the golden-pinned cost function -- and
(b) GPU == oracle bit for bit (tests/test_gpu_refine.py).  These tests hold the optimiser's
own contract: endpoints fixed, cost and the augmented objective go down, determinism."""
import numpy as np
import pytest

import golden_io as G


def _canonical(oracle_mod, options=None):
    meta, arr = G.canonical()
    opts = dict(meta["options"])
    opts.update(options or {})
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(meta["map"]), meta["N"], opts,
                            meta["maxratio"], meta["maxalpha"], meta["enlargement"],
                            meta["weights"], anchor=tuple(meta["map"]["x_start"]))
    return orc, G.canonical_paths(meta, arr), arr


def test_refine_lowers_cost_and_keeps_endpoints(oracle_mod):
    orc, wp, arr = _canonical(oracle_mod)
    rp = oracle_mod.refine_params(n_outer=4, n_inner=10)
    out = orc.refine(wp, rp)
    z = out["wp"]
    np.testing.assert_array_equal(z[:, 0], wp[:, 0])
    np.testing.assert_array_equal(z[:, -1], wp[:, -1])
    assert (out["iters"] > 0).all()
    before = orc.eval_paths(wp)["cost"]
    after = orc.eval_paths(z)["cost"]
    np.testing.assert_array_equal(before, arr["cost"])        # the objective is the golden one
    assert (after < before).all(), (before, after)
    np.testing.assert_allclose(out["cost"], after, rtol=1e-12)
    again = orc.refine(wp, rp)
    np.testing.assert_array_equal(again["wp"], z)               # deterministic


def test_refine_needs_smooth_options(oracle_mod):
    orc, wp, _ = _canonical(oracle_mod, {"obstacle_smooth": False})
    with pytest.raises(ValueError):
        orc.refine(wp, oracle_mod.refine_params(n_outer=1, n_inner=1))


def test_refine_zero_iterations_is_identity(oracle_mod):
    orc, wp, arr = _canonical(oracle_mod)
    out = orc.refine(wp, oracle_mod.refine_params(n_outer=0, n_inner=0))
    np.testing.assert_array_equal(out["wp"], wp)
    np.testing.assert_allclose(out["cost"], arr["cost"], rtol=1e-12)
    assert (out["iters"] == 0).all()


def test_refine_defaults_match_engine(oracle_mod):
    import inspect

    from uam_path_planning_amd.engine import REFINE_DEFAULTS

    sig = inspect.signature(oracle_mod.refine_params)
    assert {k: v.default for k, v in sig.parameters.items()} == REFINE_DEFAULTS


def test_refine_lbfgs_beats_steepest_descent(oracle_mod):
    """Same step budget: L-BFGS memory reaches lower infeasibility than steepest descent on
    the canonical candidates (the convergence claim DESIGN.md makes)."""
    orc, wp, _ = _canonical(oracle_mod)
    sd = orc.refine(wp, oracle_mod.refine_params(n_outer=10, n_inner=20, memory=0))
    lb = orc.refine(wp, oracle_mod.refine_params(n_outer=10, n_inner=20, memory=8))
    assert np.sqrt(lb["infeas"]).sum() < 0.5 * np.sqrt(sd["infeas"]).sum()


def test_refine_restart_never_worse(oracle_mod):
    """oracle refine_restart: attempt 0 is the plain run and the best attempt by sum g^2 is
    kept, so no path ends worse with restarts; n_restart = 0 is the plain run bit for bit."""
    from uam_path_planning_amd.arcs import arc_table
    from uam_path_planning_amd.scenario import canonical_spec, displacements
    from uam_path_planning_amd.synthetic import random_pairs

    spec = canonical_spec(nfz_polygons=16)
    N = 24
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), N, spec["options"], spec["maxratio"],
                            spec["maxalpha"], spec["enlargement"], spec["weights"],
                            anchor=tuple(spec["x_start"]))
    wp = oracle_mod.gen_paths(random_pairs(6, seed=8),
                              arc_table(N, displacements(5))).reshape(-1, N + 2, 2)
    a = orc.refine(wp, oracle_mod.refine_params(n_outer=3, n_inner=8))
    b = orc.refine(wp, oracle_mod.refine_params(n_outer=3, n_inner=8, n_restart=0,
                                                restart_margin=0.3))
    np.testing.assert_array_equal(a["wp"], b["wp"])
    c = orc.refine(wp, oracle_mod.refine_params(n_outer=3, n_inner=8, n_restart=2))
    assert (c["infeas"] <= a["infeas"]).all()
    assert (c["iters"] >= a["iters"]).all()
