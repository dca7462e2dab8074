"""Axis-aligned rectangle -- drop-in for the reference's ``square(center, r1, r2=None)``
(geo_simulation_project/path_generation/square.py:6-65): four half-planes right/left/top/bottom,
h = x0-c0-r1, -x0+c0-r1, x1-c1-r2, -x1+c1-r2 (square.py:29-51), centre = c, area 4 r1 r2.
Device form: ``(UAM_INEQ_AXIS, [k, c_k, r, s, 0, 0])`` with h = s*(x_k - c_k) - r; for s = -1 this
is bit-identical to the reference's -x_k + c_k - r (round-to-nearest is sign-symmetric)."""
import numpy as np

from .function import Function
from .quadratic_obstacle import QuadraticObstacle

AXIS = 2


def _side(k, c, r, s):
    def f(x):
        x = np.asarray(x, dtype=float).reshape(-1)
        return s * (x[k] - c) - r

    g = np.zeros(2)
    g[k] = s
    return Function(f, lambda x: g, np.zeros((2, 2)), spec=(AXIS, (float(k), c, r, s, 0.0, 0.0)))


def square(center, r1, r2=None):
    center = np.array(center).reshape(2)
    if r2 is None:
        r2 = r1
    c0, c1 = float(center[0]), float(center[1])
    obs = QuadraticObstacle(_side(0, c0, float(r1), 1.0), _side(0, c0, float(r1), -1.0),
                            _side(1, c1, float(r2), 1.0), _side(1, c1, float(r2), -1.0))
    obs.center = center
    obs.area = 4 * r1 * r2
    return obs
