"""Obstacle map -- drop-in for the reference's ``Map`` (path_generation/map.py:6-97).
``collides`` (map.py:41-43) and ``map[x, y]`` (91-97) evaluate on the GPU.  Plotting is out
of scope."""
import numpy as np

from .quadratic_obstacle import QuadraticObstacle


class Map:
    def __init__(self, *obstacles):
        self.obstacles = []
        self.x_goal = np.zeros(2)
        self.x_start = np.zeros(2)
        self.add(*obstacles)

    def add(self, *obstacles):
        for obstacle in obstacles:
            assert isinstance(obstacle, QuadraticObstacle), \
                "Obstacle must be a QuadraticObstacle object"
            self.obstacles.append(obstacle)

    def intersection(self, x0, direction):
        # map.py:19-39 calls QuadraticObstacle.intersection, which the reference comments out
        dist, p = float("inf"), None
        for obs in self.obstacles:
            obs.intersection(x0, direction)
        return p, dist

    def collides(self, x):
        """Any obstacle contains x (one point, or a batch (n, 2) -> bool array)."""
        from ..engine import map_collides

        return map_collides(self, x)

    def __len__(self):
        return len(self.obstacles)

    def __getitem__(self, key):
        if isinstance(key, tuple):
            return self.collides(np.array(key))
        elif isinstance(key, slice):
            return self.obstacles[key]
        else:
            raise TypeError("Invalid argument type.")
