"""Candidate generator + batched candidate evaluation -- drop-in for the hot-path part of the
reference's ``Solver`` (geo_simulation_project/path_generation/solver.py:8-177).

  create_x_init(d)        solver.py:103-136, generated on the GPU (K4, arcs.arc_table)
  evaluate_candidates(ds) main.py:158-196 candidate loop + argmin, fused on the GPU:
                          every displacement evaluated in one launch, then the reference's
                          selection rule (main.py:175-180) on fval = sqrt(cost) and on length
  solve(x_init, params)   solver.py:19-56 -- the reference's OpEn ALM solve of
                          min get_cost s.t. get_nonlincon = 0 becomes the batched GPU
                          refinement (uam_refine; definition oracle/uam_oracle.c orc_refine):
                          same inputs (x_init [2N], p vector) and result dict
  solve_candidates(ds)    main.py:168-193 loop (create_x_init -> solve -> selection) with
                          every candidate refined in ONE launch
The refinement is this build's ALM (gradient inner solver with Armijo backtracking instead of
OpEn's PANOC),
so solutions are not OpEn's; the objective and constraints are the reference's.
"""
import dataclasses
import time

import numpy as np

from ..arcs import REFERENCE_DISPLACEMENTS, arc_table, check_displacement
from .problem import Problem


class Solver:
    def __init__(self, problem, opts):
        assert isinstance(problem, Problem)
        self.problem = problem
        self.x_sol = None
        self.x_init = None
        self.opts = opts
        self.verbose = True
        self.optimizer_name = None
        self.update_solver = False

    def _pair(self):
        m = self.problem.map
        x0 = np.asarray(m.x_start, dtype=np.float64).reshape(-1)
        xf = np.asarray(m.x_goal, dtype=np.float64).reshape(-1)
        return np.concatenate([x0, xf]).reshape(1, 4)

    def create_x_init(self, displacement=0):
        check_displacement(displacement)
        eng = self.problem.engine(need_enlargement=False)
        wp = eng.gen_paths(self._pair(), arc_table(self.problem.N, [displacement]))
        return wp[0, 1:-1, :].reshape(-1).cpu().numpy()

    # OpEn's default delta tolerance on the ALM infeasibility (|F1| <= 1e-4 -> "Converged")
    DELTA_TOLERANCE = 1e-4

    def _solve_params(self, params):
        """The OpEn parameter vector p = [x_start, x_goal, maxratio, maxalpha, enlargement,
        weights...] (solver.py:60-78) -> (PathParams, start, goal)."""
        names = self.problem.map.region_names()
        p = np.asarray(params, dtype=np.float64).reshape(-1)
        if p.size != 7 + len(names):
            raise ValueError(f"Vector `parameter` has wrong length: {p.size} != "
                             f"{7 + len(names)} (error 3003)")
        base = self.problem.path_params(need_kinematics=False, need_enlargement=False)
        pp = dataclasses.replace(base, maxratio=float(p[4]), maxalpha=float(p[5]),
                                 enlargement=float(p[6]),
                                 weights=tuple(float(w) for w in p[7:]))
        if not (pp.penalty_smooth and pp.obstacle_smooth):
            raise ValueError("refinement needs options penalty_smooth and obstacle_smooth "
                             "(the reference's main.py options)")
        return pp, p[0:2], p[2:4]

    def _refine(self, xs_init, params):
        from ..geometry import compile_map
        from ..engine import default_engine

        pp, xs, xg = self._solve_params(params)
        N = self.problem.N
        xi = np.asarray(xs_init, dtype=np.float64).reshape(-1, 2 * N)
        P = xi.shape[0]
        wp = np.empty((P, N + 2, 2))
        wp[:, 0] = xs
        wp[:, -1] = xg
        wp[:, 1:-1] = xi.reshape(P, N, 2)
        eng = default_engine()
        eng.set_geometry(compile_map(self.problem.map))
        eng.set_params(pp)
        t0 = time.perf_counter()
        out = eng.refine(wp, (self.opts or {}).get("refine"))
        ev = eng.eval_waypoints(out["wp"])
        eng.synchronize()
        elapsed = time.perf_counter() - t0
        z = out["wp"].cpu().numpy()
        res = {"wp": z, "x": z[:, 1:-1].reshape(P, -1), "time": elapsed,
               "cost": ev["cost"].cpu().numpy(), "length": ev["length"].cpu().numpy(),
               "infeasibility": np.sqrt(out["infeas"].cpu().numpy()),
               "iterations": out["iters"].cpu().numpy(),
               "nfz_hits": ev["nfz_hits"].cpu().numpy(), "kin_sum": ev["kin_sum"].cpu().numpy()}
        res["fval"] = np.sqrt(res["cost"])
        res["exit_status"] = ["Converged" if v <= self.DELTA_TOLERANCE
                              else "NotConvergedIterations" for v in res["infeasibility"]]
        return res

    def solve(self, x_init, params):
        """solver.py:19-56: refine x_init [2N] under p; returns x, time, fval = sqrt(cost),
        length (= length_of(x)), exit_status.  opts["refine"] overrides the ALM settings
        (engine.REFINE_DEFAULTS)."""
        self.x_init = x_init
        r = self._refine(x_init, params)
        self.x_sol = r["x"][0].tolist()
        return {"x": self.x_sol, "time": r["time"], "fval": float(r["fval"][0]),
                "length": self.problem.length_of(self.x_sol),
                "exit_status": r["exit_status"][0]}

    def solve_candidates(self, params, displacements=REFERENCE_DISPLACEMENTS):
        """main.py:168-193 -- every displacement's x_init refined in one launch, then the
        reference's selection rule (strict <, sentinel 0) on fval and on length."""
        ds = list(displacements)
        for d in ds:
            check_displacement(d)
        _, xs, xg = self._solve_params(params)
        eng = self.problem.engine(need_enlargement=False)
        pair = np.concatenate([xs, xg]).reshape(1, 4)
        x0 = eng.gen_paths(pair, arc_table(self.problem.N, ds))[:, 1:-1, :]
        r = self._refine(x0.reshape(len(ds), -1).cpu().numpy(), params)
        length = np.array([self.problem.length_of(x) for x in r["x"]])
        r["length"] = length
        r["min_fval_index"] = _select(r["fval"])
        r["min_length_index"] = _select(length)
        r["displacements"] = np.asarray(ds)
        return r

    def evaluate_candidates(self, displacements=REFERENCE_DISPLACEMENTS, raster=None):
        """Evaluate the map's start->goal candidates for every displacement in one launch.
        Returns numpy arrays per candidate plus the reference's two argmin indices."""
        ds = list(displacements)
        for d in ds:
            check_displacement(d)
        eng = self.problem.engine(need_kinematics=True)
        out = eng.eval_generated(self._pair(), arc_table(self.problem.N, ds), raster=raster)
        res = {k: v.cpu().numpy() for k, v in out.items()}
        res["fval"] = np.sqrt(res["cost"])
        res["min_fval_index"] = int(res.pop("best_fval_idx")[0])
        res["min_length_index"] = int(res.pop("best_length_idx")[0])
        res["displacements"] = np.asarray(ds)
        return res

    def get_error_code_explanation(self, error_code):
        error_codes = {
            1000: "Invalid request: Malformed or invalid JSON",
            1600: "Initial guess has incompatible dimensions",
            1700: "Wrong dimension of Langrange multipliers",
            2000: "Problem solution failed (solver error)",
            3003: "Vector `parameter` has wrong length",
        }
        return error_codes.get(error_code, "Error code not found")


def _select(values):
    """main.py:175-180: sentinel 0, strict < (first minimum wins)."""
    best, idx = 0, 0
    for i, v in enumerate(values):
        if best == 0 or v < best:
            best, idx = v, i
    return idx
