"""Oracle-side geometry compiler.  TEST INFRASTRUCTURE, NOT PRODUCT.

Independent restatement (separate from the product's compiler in
uam_path_planning_amd/path_generation/) of how the reference turns shapes into inequalities,
producing the flat tables that oracle/uam_oracle.c consumes.  Keeping it separate means a bug
in the product's compiler shows up as a GPU-vs-oracle mismatch instead of cancelling out.

  polygon()  geo_simulation_project/path_generation/polygon.py:7-143 (convex walk from vertex 0,
             are_consecutive 55-102, edge h = -sgn*line 98, centre = vertex mean 141)
  ball()     ball.py:7-52  (h = ((x0-c0)/r1)^2 + ((x1-c1)/r2)^2 - 1, centre 49)
  square()   square.py:6-65 (four axis half-planes right/left/top/bottom, centre 63)
Map layout: obstacles (RegionMap.add_obstacles order, map.py:13-17) first, then region shapes
region-major in insertion order (region_map.py:22-61).
"""
import numpy as np

HALFPLANE, ELLIPSE, AXIS = 0, 1, 2
MAX_REGIONS = 16


def _polygon(vertices):
    pts = [(float(v[0]), float(v[1])) for v in vertices]
    n = len(pts)
    if n < 3:
        raise ValueError(f"Only {n} vertices given. At least 3 required")
    cx, cy = pts[0]
    for b in range(1, n):
        cx = cx + pts[b][0]
        cy = cy + pts[b][1]
    center = (cx / n, cy / n)

    def line(a, b, q):
        pa, pb = pts[a], pts[b]
        return (pb[1] - pa[1]) * (q[0] - pa[0]) - (pb[0] - pa[0]) * (q[1] - pa[1])

    def consecutive(a, b):
        sgn = 0.0
        for j in range(n):
            if j in (a, b):
                continue
            s1 = float(np.sign(line(a, b, pts[j])))
            if s1 == 0:
                raise ValueError("Input contains three aligned points")
            if sgn == 0:
                sgn = s1
                continue
            if s1 != sgn:
                return None
        if sgn == 0:
            raise ValueError("The polygon is nonconvex")
        pa, pb = pts[a], pts[b]
        return (pa[0], pa[1], pb[0] - pa[0], pb[1] - pa[1], -sgn)

    edges = []
    remaining = list(range(1, n))
    a = 0
    while remaining:
        for i, b in enumerate(remaining):
            e = consecutive(a, b)
            if e is not None:
                edges.append(e)
                remaining.pop(i)
                a = b
                break
        else:
            raise ValueError("The polygon is nonconvex")
    e = consecutive(a, 0)
    if e is None:
        raise ValueError("Couldn't close polygon")
    edges.append(e)
    ineqs = [(HALFPLANE, [ax, ay, dx, dy, s, 0.0]) for ax, ay, dx, dy, s in edges]
    return ineqs, center


def _ball(center, r1=None, r2=None):
    if r1 is None and r2 is None:
        r1, r2, center = center, center, [0.0, 0.0]
    elif r2 is None:
        r2 = r1
    c = [float(center[0]), float(center[1])]
    return [(ELLIPSE, [c[0], c[1], float(r1), float(r2), 0.0, 0.0])], (c[0], c[1])


def _square(center, r1, r2=None):
    if r2 is None:
        r2 = r1
    c0, c1 = float(center[0]), float(center[1])
    ineqs = [(AXIS, [0.0, c0, float(r1), 1.0, 0.0, 0.0]),
             (AXIS, [0.0, c0, float(r1), -1.0, 0.0, 0.0]),
             (AXIS, [1.0, c1, float(r2), 1.0, 0.0, 0.0]),
             (AXIS, [1.0, c1, float(r2), -1.0, 0.0, 0.0])]
    return ineqs, (c0, c1)


def shape_from_spec(s):
    if s["kind"] == "polygon":
        return _polygon(s["vertices"])
    if s["kind"] == "ball":
        return _ball(s["center"], s.get("r1"), s.get("r2"))
    if s["kind"] == "square":
        return _square(s["center"], s["r1"], s.get("r2"))
    raise ValueError(f"unknown shape kind {s['kind']}")


class FlatGeometry:
    """Flat SoA tables: ineq_kind[n_ineq] i32, ineq_par[n_ineq,6] f64, shape_first/count
    [n_shapes] i32, shape_center[n_shapes,2] f64, region_first[n_regions+1] i32."""

    def __init__(self, obstacles, regions):
        kinds, pars, first, count, centers = [], [], [], [], []

        def add(shape):
            ineqs, c = shape
            first.append(len(kinds))
            count.append(len(ineqs))
            centers.append(c)
            for k, p in ineqs:
                kinds.append(k)
                pars.append(p)

        for s in obstacles:
            add(s)
        region_first = [len(first)]
        for shapes in regions:
            for s in shapes:
                add(s)
            region_first.append(len(first))
        if len(regions) > MAX_REGIONS:
            raise ValueError("too many regions")
        self.n_obstacles = len(obstacles)
        self.n_regions = len(regions)
        self.ineq_kind = np.asarray(kinds, dtype=np.int32).reshape(-1)
        self.ineq_par = np.asarray(pars, dtype=np.float64).reshape(-1, 6)
        self.shape_first = np.asarray(first, dtype=np.int32)
        self.shape_count = np.asarray(count, dtype=np.int32)
        self.shape_center = np.asarray(centers, dtype=np.float64).reshape(-1, 2)
        self.region_first = np.asarray(region_first, dtype=np.int32)


def compile_spec(spec):
    obstacles = [shape_from_spec(s) for s in spec["obstacles"]]
    regions = [[shape_from_spec(s) for s in r["shapes"]] for r in spec["regions"]]
    return FlatGeometry(obstacles, regions)
