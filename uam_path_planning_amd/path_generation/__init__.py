"""Drop-in for the reference's geo_simulation_project/path_generation call surface, evaluated
on MI355X through libuampath.  Same class and function names as the reference modules."""
from .ball import ball
from .function import Function
from .map import Map
from .polygon import polygon
from .problem import Problem
from .quadratic_obstacle import QuadraticObstacle
from .region_map import RegionMap
from .solver import Solver
from .square import square
from .utils import color2RGB, get_var_from_file

__all__ = ["Function", "QuadraticObstacle", "polygon", "ball", "square", "Map", "RegionMap",
           "Problem", "Solver", "color2RGB", "get_var_from_file"]
