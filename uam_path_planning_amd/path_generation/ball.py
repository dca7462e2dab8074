"""Elliptical shape -- drop-in for the reference's ``ball(center, r1=None, r2=None)``
(geo_simulation_project/path_generation/ball.py:7-52): h(x) = ((x0-c0)/r1)^2 + ((x1-c1)/r2)^2 - 1,
``ball(r)`` is a circle of radius r at the origin, ``ball(c, r)`` a circle, centre = c.
Device form: ``(UAM_INEQ_ELLIPSE, [c0, c1, r1, r2, 0, 0])``."""
import numpy as np

from .function import Function
from .quadratic_obstacle import QuadraticObstacle

ELLIPSE = 1


def ball(center, r1=None, r2=None):
    if r1 is None and r2 is None:
        r1 = center
        r2 = r1
        center = np.array([0.0, 0.0])
    elif r2 is None:
        r2 = r1
    center = np.array(center)
    assert center.shape == (2,)
    c0, c1 = float(center[0]), float(center[1])
    fr1, fr2 = float(r1), float(r2)

    def func(x):
        x = np.asarray(x, dtype=float).reshape(-1)
        a = (x[0] - c0) / fr1
        b = (x[1] - c1) / fr2
        return (0.0 + a * a) + b * b - 1

    def grad(x):
        x = np.asarray(x, dtype=float).reshape(-1)
        return 2 * np.array([(x[0] - c0) / fr1 ** 2, (x[1] - c1) / fr2 ** 2])

    f = Function(func, grad, np.array([[2 / fr1 ** 2, 0], [0, 2 / fr2 ** 2]]),
                 spec=(ELLIPSE, (c0, c1, fr1, fr2, 0.0, 0.0)))
    obs = QuadraticObstacle(f)
    obs.center = center
    obs.area = np.pi * r1 * r2
    return obs
