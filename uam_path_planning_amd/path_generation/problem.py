"""Path cost model -- drop-in for the reference's ``Problem``
(geo_simulation_project/path_generation/problem.py:6-146), evaluated on the GPU.

Same constructor, ``options``/``params``/``weights`` dictionaries and method names:
  get_cost(z_)                    problem.py:38-44   -> K3 analytic path kernel
  get_total_penalty_function()    problem.py:49-56   -> point kernel (Φ)
  get_penalty_function(region)    problem.py:59-82   -> point kernel (weighted region / obstacles)
  get_nonlincon(z_)               problem.py:84-114  -> K3 with the full g vector
  length_of(x, smooth)            problem.py:130-146 -> length kernel
Inputs are numeric (numpy / list / torch).  CasADi symbols are not accepted: the symbolic
solver build is the OpEn optimiser, which is out of scope.
Batched extension: ``evaluate(waypoints [P, N+2, 2], raster=None)``.
"""
import numpy as np

from ..engine import PathParams, default_engine
from ..geometry import compile_map
from .region_map import RegionMap


def _numeric(z):
    try:
        import torch

        if isinstance(z, torch.Tensor):
            return z.detach().to("cpu", dtype=torch.float64).numpy()
    except ImportError:  # pragma: no cover
        pass
    a = np.asarray(z)
    if a.dtype == object:
        raise TypeError("Problem evaluates numeric inputs only (CasADi symbols belong to the "
                        "OpEn solver build, which is out of scope)")
    return a.astype(np.float64)


class Problem:
    def __init__(self, map, N, opts=None):
        assert isinstance(map, RegionMap)
        self.map = map
        self.N = N
        self.weights = {}
        self.options = {
            "length_smooth": False,
            "penalty_smooth": True,
            "obstacle_smooth": False,
            "maxratio_smooth": False,
        }
        self.params = {"maxratio": None, "maxalpha": None, "enlargement": None}
        if opts:
            self.options.update(opts)
        self.update_weights()
        self.altitude = 150.0

    def update_weights(self):
        for region_name in self.map.region_names():
            if region_name not in self.weights:
                self.weights[region_name] = 1

    def set_weight(self, region_name, w):
        assert region_name in self.map.regions
        self.weights[region_name] = w

    # -- device plumbing ---------------------------------------------------------------------
    def path_params(self, need_kinematics=False, need_enlargement=True):
        self.update_weights()
        p = self.params
        has_region_shapes = any(r["shapes"] for r in self.map.regions.values())
        if need_enlargement and has_region_shapes and p["enlargement"] is None:
            raise TypeError("unsupported operand type(s) for -: 'float' and 'NoneType' "
                            "(Problem.params['enlargement'] is None)")
        if need_kinematics and (p["maxratio"] is None or p["maxalpha"] is None):
            raise TypeError("Problem.params['maxratio'] / ['maxalpha'] is None")
        return PathParams(
            N=int(self.N),
            length_smooth=bool(self.options["length_smooth"]),
            penalty_smooth=bool(self.options["penalty_smooth"]),
            obstacle_smooth=bool(self.options["obstacle_smooth"]),
            maxratio_smooth=bool(self.options["maxratio_smooth"]),
            maxratio=1.0 if p["maxratio"] is None else float(p["maxratio"]),
            maxalpha=0.0 if p["maxalpha"] is None else float(p["maxalpha"]),
            enlargement=0.0 if p["enlargement"] is None else float(p["enlargement"]),
            weights=tuple(float(self.weights[r]) for r in self.map.region_names()),
            quirk_length=True,
            anchor=tuple(float(v) for v in np.asarray(self.map.x_start, float).reshape(-1)[:2]),
            altitude=float(self.altitude))

    def engine(self, **kw):
        eng = default_engine()
        eng.set_geometry(compile_map(self.map))
        eng.set_params(self.path_params(**kw))
        return eng

    def _path(self, z):
        a = _numeric(z).reshape(-1)
        W = self.N + 2
        if a.size != 2 * W:
            raise ValueError(f"z_ must hold 2*(N+2) = {2 * W} values (got {a.size})")
        return a.reshape(1, W, 2)

    # -- reference surface ---------------------------------------------------------------------
    def get_cost(self, z):
        out = self.engine().eval_waypoints(self._path(z))
        return float(out["cost"].cpu()[0])

    def get_total_penalty_function(self):
        def total_penalty(x):
            pts = _numeric(x).reshape(-1, 2)
            v = self.engine().eval_points(pts, want=("phi",))["phi"].cpu().numpy()
            return float(v[0]) if pts.shape[0] == 1 else v
        return total_penalty

    def get_penalty_function(self, region_name=None):
        if region_name is not None:
            self.update_weights()
            names = self.map.region_names()
            r = names.index(region_name)
        else:
            r = None

        def penalty(x):
            pts = _numeric(x).reshape(-1, 2)
            eng = self.engine()
            if r is None:
                v = eng.eval_points(pts, want=("obs_norm",))["obs_norm"]
            else:
                v = eng.eval_points(pts, want=("phi_regions",))["phi_regions"][:, r]
            v = v.cpu().numpy()
            return float(v[0]) if pts.shape[0] == 1 else v
        return penalty

    def get_nonlincon(self, z):
        out = self.engine(need_kinematics=True, need_enlargement=False).eval_waypoints(
            self._path(z), want_g=True)
        return out["g_rows"].cpu().numpy()[0]

    def length_of(self, x, smooth=False):
        a = _numeric(x).reshape(-1)
        y = np.concatenate([np.asarray(self.map.x_start, float).reshape(-1), a,
                            np.asarray(self.map.x_goal, float).reshape(-1)]).reshape(-1, 2)
        if y.shape[0] < self.N + 2:
            raise ValueError(f"length_of needs at least {2 * self.N} values (got {a.size})")
        eng = self.engine(need_enlargement=False)
        return float(eng.path_length(y[None], self.N + 1, smooth).cpu()[0])

    # -- batched extension -----------------------------------------------------------------------
    def evaluate(self, waypoints, raster=None, want_cells=False, want_g=False):
        """All paths at once: waypoints [P, N+2, 2] -> dict of device tensors (cost, length_q,
        length, kin_sum, nfz_sum, nfz_hits, min_clearance, offmap[, cells][, g_rows])."""
        eng = self.engine(need_kinematics=True)
        return eng.eval_waypoints(waypoints, raster=raster, want_cells=want_cells,
                                  want_g=want_g)
