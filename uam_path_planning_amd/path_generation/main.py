"""Driver -- the hot-path part of the reference's ``Main`` (path_generation/main.py:10-201):
the canonical Nagasaki map (setup_map 21-49, from the data files via the safe loader), the
N=80 problem (setup_problem 53-61), the parameter vector (main.py:128-150), and the candidate
loop + selection (run 158-196) -- except that every displacement is evaluated in ONE device
launch.  With --solve (main.py:168-193 solve loop) every candidate is refined in one launch by
the GPU ALM refinement (Solver.solve_candidates) and the printed fval/length are those of the
refined paths; without it they are those of the initial candidates.  Shapefile export and
plotting (main.py:92-116) are out of scope.

    python -m uam_path_planning_amd.path_generation.main [--solve]
"""
import sys

import numpy as np

from ..arcs import REFERENCE_DISPLACEMENTS
from ..scenario import build_region_map, canonical_spec
from .problem import Problem
from .solver import Solver


class Main:
    def __init__(self):
        self.map = None
        self.problem = None
        self.solver = None
        self.spec = canonical_spec()

    def setup_map(self):
        self.map = build_region_map(self.spec)
        self.map.map_version = "v1"

    def setup_problem(self):
        self.problem = Problem(self.map, self.spec["N"], dict(self.spec["options"]))

    def setup_solver_options(self):
        self.solver = Solver(self.problem, {})
        self.solver.optimizer_name = f"map_{self.map.map_version}_n{self.problem.N}"

    def check_options(self, maxratio, maxalpha):
        assert maxratio >= 1
        assert 0 <= maxalpha <= np.pi

    def run(self, displacements=REFERENCE_DISPLACEMENTS, verbose=True, solve=False):
        self.setup_map()
        self.setup_problem()
        self.setup_solver_options()
        x_start, x_goal = list(self.spec["x_start"]), list(self.spec["x_goal"])
        self.map.x_start, self.map.x_goal = x_start, x_goal
        maxratio, maxalpha, enlargement = (self.spec["maxratio"], self.spec["maxalpha"],
                                           self.spec["enlargement"])
        self.check_options(maxratio, maxalpha)
        self.problem.params.update({"maxratio": maxratio, "maxalpha": maxalpha,
                                    "enlargement": enlargement})
        for name, w in zip(self.map.region_names(), self.spec["weights"]):
            self.problem.set_weight(name, w)
        if solve:
            params = x_start + x_goal + [maxratio, maxalpha, enlargement] + \
                [self.problem.weights[n] for n in self.map.region_names()]
            res = self.solver.solve_candidates(params, displacements)
        else:
            res = self.solver.evaluate_candidates(displacements)
        if verbose:
            print("Start simulation: N =", self.problem.N)
            print("Solver" if solve else "Candidates", self.solver.optimizer_name,
                  "(GPU ALM refinement)" if solve else "(initial paths, no solve)")
            print("-------------------------------------")
            for i in range(len(displacements)):
                print("line", i + 1)
                if solve:
                    print(f"time: {res['time']} s (all lines)")
                print(f"fval: {res['fval'][i]}\nlength: {res['length'][i]} km")
                if solve:
                    print(f"exit_status: {res['exit_status'][i]}")
                print(f"nfz waypoints: {res['nfz_hits'][i]}\nkinematic violation: "
                      f"{res['kin_sum'][i]}")
                print("-------------------------------------")
            print("Min fval result: line", res["min_fval_index"] + 1)
            print("Min path length result: line", res["min_length_index"] + 1)
        return res


if __name__ == "__main__":
    Main().run(solve="--solve" in sys.argv[1:])
