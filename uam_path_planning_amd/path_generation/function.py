"""Inequality function h(x) <= 0 of a convex shape.

Mirrors the reference's ``Function`` (geo_simulation_project/path_generation/function.py:4-194)
for what the hot path uses: a callable of a 2-D point, ``n``, ``grad``, ``hess`` and the
``is_quadratic`` / ``is_convex`` flags that ``QuadraticObstacle.add`` asserts
(quadratic_obstacle.py:9-15).  Every Function built by ``polygon``/``ball``/``square`` also
carries ``spec = (kind, params)``, the form the device kernels evaluate
(include/uampath.h UAM_INEQ_*).  A user Function without a spec can be held by a shape but is
rejected when the map is compiled for the device (the kernels only know the three kinds).
"""
import numpy as np


class Function:
    def __init__(self, f, grad=None, hess=None, n=2, spec=None):
        if not (callable(f) or isinstance(f, (int, float))):
            raise TypeError(f"Property must be numeric or callable; got '{type(f)}' instead")
        self._n = n
        self.f = (lambda x: f) if isinstance(f, (int, float)) else f
        self.grad = grad
        self.hess = hess
        self.spec = spec
        self._is_quadratic = True
        self._is_convex = True

    @property
    def n(self):
        return self._n if self._n is not None else 1

    @n.setter
    def n(self, dim):
        if not isinstance(dim, (int, float)) or dim <= 0 or int(dim) != dim:
            raise ValueError(f"Size should be a strictly positive integer (got '{dim}' instead)")
        self._n = int(dim)

    @property
    def is_quadratic(self):
        return self._is_quadratic

    @is_quadratic.setter
    def is_quadratic(self, value):
        self._is_quadratic = value

    @property
    def is_convex(self):
        return self._is_convex

    @is_convex.setter
    def is_convex(self, value):
        self._is_convex = value

    def __call__(self, x):
        return self.f(x)

    def compose(self, A, b=None):
        """In place, h(x) -> h(A x + b) with grad A^T grad h(A x + b) and hessian A H(x) A^T
        (the reference's own expression), as function.py:122-157 (a 1 x 1 A scales the identity; b defaults to
        0 and must be (m, 1), else the reference's ValueError).  The result is a host callable
        only: its device spec is dropped, so a shape holding it is rejected when a map is
        compiled for the device (the kernels evaluate the three shape kinds as built)."""
        A = np.asarray(A)
        m, n = A.shape
        if m == 1 and n == 1:
            m = len(b) if b is not None else self.n
            n = m
            A = A * np.eye(m)
        elif self._n is not None and self.n != m:
            raise ValueError(f"Size mismatch between function '{self.n}' and scaling matrix A "
                             f"'{A.shape}'")
        b = np.zeros((m, 1)) if b is None else b
        if np.asarray(b).shape != (m, 1):
            raise ValueError(f"Size mismatch between scaling matrix A '{A.shape}' and "
                             f"translation vector '{np.asarray(b).shape}'")
        f0, g0, h0 = self.f, self.grad, self.hess
        self.f = lambda x: f0(A @ x + b)
        if g0 is not None:
            self.grad = lambda x: A.T @ g0(A @ x + b)
            if h0 is not None:
                self.hess = (lambda x: A @ h0(x) @ A.T) if callable(h0) else A @ h0 @ A.T
        self._n = n
        self.spec = None
