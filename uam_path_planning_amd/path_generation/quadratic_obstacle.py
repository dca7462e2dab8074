"""Convex shape as an intersection of inequalities h_i(x) <= 0.

Drop-in for the reference's ``QuadraticObstacle``
(geo_simulation_project/path_generation/quadratic_obstacle.py:7-149).  ``penalty_function``
(quadratic_obstacle.py:27-39) and ``contains`` (89-94) evaluate on the GPU through
libuampath (the shape is compiled to a one-shape device geometry); there is no host
evaluation of the penalty.
"""
import numpy as np

from .function import Function


class QuadraticObstacle:
    def __init__(self, *inequalities):
        self.inequalities = []
        self.xy_coords = None
        self.area = float("nan")
        self.center = float("nan")
        self.add(*inequalities)

    def add(self, *inequalities):
        for ineq in inequalities:
            assert isinstance(ineq, Function), f"Expected Function, got {type(ineq)}"
            assert ineq.is_quadratic, f"Function must be quadratic. is_quadratic: {ineq.is_quadratic}"
            assert ineq.n == 2, f"Function must be 2-dimensional, got {ineq.n}-dimensional"
            self.inequalities.append(ineq)

    # -- device-evaluated primitives ---------------------------------------------------------
    def penalty_function(self, smooth=True, enlargement=0):
        """psi(x) = prod_i min(h_i(x) - e, 0)^2 (smooth) or prod_i min(e - h_i(x), 0).
        Accepts one point (2,) or a batch (n, 2); evaluated on the GPU."""
        if enlargement is None:
            raise TypeError("unsupported operand type(s) for -: 'float' and 'NoneType'")
        from ..engine import shape_psi

        def psi(x):
            return shape_psi(self, x, bool(smooth), float(enlargement))

        return psi

    def contains(self, x):
        """All h_i(x) <= 1e-14 (quadratic_obstacle.py:89-94); GPU-evaluated."""
        from ..engine import shape_contains

        return shape_contains(self, x)

    # -- transforms: the reference's always fail ------------------------
    def linear_transform(self, A, b=None):
        A = np.asarray(A, dtype=float)
        if np.linalg.norm(A @ np.linalg.inv(A) - np.eye(2)) > 1e-8:
            print("Warning: Transformation matrix A is not invertible")
        if b is None:
            b = np.zeros(2)
        for h in self.inequalities:
            h.compose(A, b)

    def rotate(self, angle, center=None):
        if center is None:
            center = np.zeros(2)
        A = np.array([[np.cos(angle), -np.sin(angle)], [np.sin(angle), np.cos(angle)]])
        self.linear_transform(A, center - A @ center)

    def translate(self, v):
        self.linear_transform(np.eye(2), v)

    def rescale(self, rx, ry=None, center=None):
        if ry is None:
            ry = rx
        if center is None:
            center = np.zeros(2)
        elif isinstance(ry, np.ndarray):
            center, ry = ry, 1
        A = np.array([[rx, 0], [0, ry]])
        self.linear_transform(A, center - A @ center)

    def __len__(self):
        return len(self.inequalities)
