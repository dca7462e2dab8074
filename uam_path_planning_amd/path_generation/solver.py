"""Candidate generator + batched candidate evaluation -- drop-in for the hot-path part of the
reference's ``Solver`` (geo_simulation_project/path_generation/solver.py:8-177).

  create_x_init(d)        solver.py:103-136, generated on the GPU (K4, arcs.arc_table)
  evaluate_candidates(ds) main.py:158-196 candidate loop + argmin, fused on the GPU:
                          every displacement evaluated in one launch, then the reference's
                          selection rule (main.py:175-180) on fval = sqrt(cost) and on length
  solve()                 the OpEn PANOC/ALM optimiser (solver.py:19-101) -- out of scope
                          (code-generated Rust solver over TCP)
"""
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

    def solve(self, x_init, params):
        raise NotImplementedError(
            "Solver.solve runs the OpEn PANOC/ALM optimiser (code-generated Rust over TCP); it "
            "is outside the device hot path. Use evaluate_candidates() for the batched "
            "candidate costs.")

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
