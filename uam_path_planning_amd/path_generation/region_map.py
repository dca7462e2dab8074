"""Map with weighted penalty regions -- drop-in for the reference's ``RegionMap``
(path_generation/region_map.py:8-100): ordered ``regions`` {name: {'shapes', 'color'}},
``new_region`` / ``add_shape(s)_to_region`` / ``add_obstacle(s)`` / ``region_names`` with the
reference's errors.  Region order (insertion order) is the order of the Φ sum and of the
weights in the parameter vector (solver.py:61, 77-78)."""
from . import utils
from .map import Map
from .quadratic_obstacle import QuadraticObstacle


class RegionMap(Map):
    def __init__(self):
        super().__init__()
        self.regions = {}
        self.map_version = "v1"

    def add_obstacle(self, obstacle):
        self.add(obstacle)

    def add_obstacles(self, *obstacles):
        self.add(*obstacles)

    def new_region(self, name, color):
        if self.region_exists(name):
            raise ValueError(f"Name '{name}' already in use for areas")
        self.regions[name] = {"shapes": [], "color": utils.color2RGB(color)}

    def add_shape_to_region(self, region, obstacle):
        if not self.region_exists(region):
            raise ValueError(f"Unknown type '{region}' of penalty obstacles. Use new_region "
                             "method to define it")
        assert isinstance(obstacle, QuadraticObstacle)
        self.regions[region]["shapes"].append(obstacle)

    def add_shapes_to_region(self, region, *obstacles):
        for obstacle in obstacles:
            self.add_shape_to_region(region, obstacle)

    def region_names(self):
        return list(self.regions.keys())

    def region_exists(self, region):
        return region in self.regions
