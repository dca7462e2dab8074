"""Convex polygon shape -- drop-in for the reference's ``polygon(*points)``
(geo_simulation_project/path_generation/polygon.py:7-143).

Same construction: starting at vertex 0, walk to the first remaining vertex b such that every
other vertex lies strictly on one side of the line a->b (``are_consecutive``, polygon.py:55-102),
one half-plane inequality per accepted edge, h(x) = -sgn * ((by-ay)(x0-ax) - (bx-ax)(x1-ay)),
then close back to vertex 0.  Same errors and messages (three aligned points, nonconvex,
couldn't close, fewer than 3 vertices).  Centre = vertex mean accumulated in the reference's
order (polygon.py:32-37, 141), area by the shoelace sum over the walk (120, 135, 140).
The device form of each edge is ``(UAM_INEQ_HALFPLANE, [ax, ay, bx-ax, by-ay, -sgn, 0])``.
"""
import numpy as np

from .function import Function
from .quadratic_obstacle import QuadraticObstacle

HALFPLANE = 0


def _edge_function(ax, ay, dx, dy, s):
    def f(x):
        x = np.asarray(x, dtype=float).reshape(-1)
        return s * (dy * (x[0] - ax) - dx * (x[1] - ay))

    # grad as the reference writes it (polygon.py:95-99: -sgn * [[by-ay], [bx-ax]])
    return Function(f, lambda x: s * np.array([[dy], [dx]]), np.zeros((2, 2)),
                    spec=(HALFPLANE, (ax, ay, dx, dy, s, 0.0)))


def polygon(*points):
    if len(points) < 3:
        raise ValueError(f"Only {len(points)} vertices given. At least 3 required")
    arrs = [np.array(p).reshape(2, 1) for p in points]
    n = len(arrs)
    center = arrs[0].copy()
    for b in range(1, n):
        center += arrs[b]          # same dtype behaviour as polygon.py:37
    xy = [(float(a[0, 0]), float(a[1, 0])) for a in arrs]

    def line(a, b, q):
        pa, pb = xy[a], xy[b]
        return (pb[1] - pa[1]) * (q[0] - pa[0]) - (pb[0] - pa[0]) * (q[1] - pa[1])

    def are_consecutive(a, b):
        sgn = 0.0
        for j in range(n):
            if j == a or j == b:
                continue
            s1 = float(np.sign(line(a, b, xy[j])))
            if s1 == 0:
                raise ValueError("Input contains three aligned points")
            if sgn == 0:
                sgn = s1
                continue
            if s1 != sgn:
                return False, None
        if sgn == 0:
            raise ValueError("The polygon is nonconvex")
        pa, pb = xy[a], xy[b]
        return True, _edge_function(pa[0], pa[1], pb[0] - pa[0], pb[1] - pa[1], -sgn)

    obs = QuadraticObstacle()
    remaining = list(range(1, n))
    a = 0
    area = 0.0
    while remaining:
        for i, b in enumerate(remaining):
            ok, f = are_consecutive(a, b)
            if ok:
                remaining.pop(i)
                area += xy[a][0] * xy[b][1] - xy[a][1] * xy[b][0]
                a = b
                obs.add(f)
                break
        else:
            raise ValueError("The polygon is nonconvex")
    ok, f = are_consecutive(a, 0)
    if not ok:
        raise ValueError("Couldn't close polygon")
    area += xy[a][0] * xy[0][1] - xy[a][1] * xy[0][0]
    obs.add(f)
    obs.area = abs(area) / 2
    obs.center = center / n
    obs.vertices = np.asarray(xy)
    return obs
