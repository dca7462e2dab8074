"""Numeric stand-in for the subset of ``casadi`` (3.6.5, requirements.txt:3) that the
reference cost model calls.  TEST TOOLING ONLY: it exists so that
``tests/golden/make_golden.py`` can import the reference's pure-Python cost model in the
survey container (casadi is not installed and there is no network) and record golden
vectors.  Nothing in the product or on the GPU box imports it.

Every function is float64, operation-for-operation, mirroring CasADi's numeric runtime:
``casadi_dot`` accumulates ``r += x[i]*y[i]`` from 0 and ``casadi_norm_2`` is
``sqrt(casadi_dot(x, x))``.  ``fmin``/``fmax`` follow C ``fmin``/``fmax`` (a NaN operand
yields the other operand), like CasADi's ``OP_FMIN``/``OP_FMAX``.
"""
import math

import numpy as np

def _flat(x):
    return np.asarray(x, dtype=np.float64).reshape(-1)


def fmin(a, b):
    return np.fmin(a, b)


def fmax(a, b):
    return np.fmax(a, b)


def dot(a, b):
    a, b = _flat(a), _flat(b)
    r = 0.0
    for i in range(a.shape[0]):
        r = r + a[i] * b[i]
    return np.float64(r)


def sumsqr(a):
    return dot(a, a)


def norm_2(a):
    return np.float64(math.sqrt(dot(a, a)))


def sqrt(a):
    return np.sqrt(a)


def cos(a):
    if np.ndim(a) == 0:
        return math.cos(float(a))
    return np.cos(a)


def vertcat(*args):
    parts = [_flat(a) for a in args]
    if not parts:
        return np.zeros(0)
    return np.concatenate(parts)


def reshape(x, shape):
    return np.reshape(_flat(x), shape)


def DM(x):
    return np.asarray(x, dtype=np.float64)


class SX:
    @staticmethod
    def sym(*_a, **_k):
        raise NotImplementedError("symbolic SX is not available in the numeric stand-in")


class MX(SX):
    pass


from . import casadi  # noqa: E402,F401  (reference does ``import casadi.casadi as cs``)
