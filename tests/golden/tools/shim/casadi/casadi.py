"""``casadi.casadi`` alias of the numeric stand-in (reference polygon.py:5, solver.py:3)."""
from . import (DM, MX, SX, cos, dot, fmax, fmin, norm_2, reshape, sqrt,  # noqa: F401
               sumsqr, vertcat)
