"""Golden-vector generator for the uam_path_planning hot path.  TEST TOOLING ONLY.

Runs ONLY in the survey/build container, where the reference is mounted read-only at
/root/reference.  It imports the reference's own pure-Python cost model
(geo_simulation_project/path_generation/{problem,region_map,map,quadratic_obstacle,polygon,
ball,square,function,solver}.py) under the numeric casadi stand-in in ./tools/shim, evaluates
it on fixed inputs, and writes small fixtures next to this file:

  canonical.npz / canonical.json  -- main.py scenario (main.py:21-49, 53-61, 122-160):
                                     N=80, 5 displacements, cost/length/g/per-waypoint Φ, ψ
  variants.npz                      -- enlargement 0.5, and the problem.py:211-272 N=10 demo
  random_cases.json                 -- random convex polygons / ellipses / squares, all 16
                                     option combinations, random waypoints, random params
  arcs.npz                          -- Solver.create_x_init (solver.py:103-136) for several N, d
  grid.npz                          -- reference Φ / ψ at raster cell centres (raster mode pin)
  waypoint_cells.npz                -- raster cells (4096^2, 8192^2) of Solver.create_x_init's
                                     own waypoints for the first 2000 cfg3 pairs x 5 d, N=80
  errors.json                       -- reference exception types + messages for bad inputs

Nothing here is copied reference source: the fixtures are inputs and the reference's outputs.
The reference never travels to the GPU box; only these fixtures do.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_ROOT = "/root/reference"
REF_PG = os.path.join(REF_ROOT, "geo_simulation_project", "path_generation")
REF_DATA = os.path.join(REF_ROOT, "data", "processed")

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(HERE, "tools", "shim"))
sys.path.insert(0, REF_PG)

import matplotlib  # noqa: E402

matplotlib.use("Agg")

import ball as ref_ball  # noqa: E402
import polygon as ref_polygon  # noqa: E402
import square as ref_square  # noqa: E402
import utils as ref_utils  # noqa: E402
from problem import Problem  # noqa: E402
from region_map import RegionMap  # noqa: E402
from solver import Solver  # noqa: E402

# ----------------------------------------------------------------------------------------
# canonical scenario constants (main.py:27-31, 48, 54-60, 390-407, 422)
NFZ_BALLS = [
    ([38.66652661075855, -9.203164091309498], 9),
    ([46.36137256675563, 3.9427562315386298], 2),
    ([19.846825121034392, 18.93411773399299], 2),
    ([26.037433469490207, 15.46710452712196], 2),
    ([46.87758543585609, -19.138710035318375], 2),
]
HIST_CENTER = ([33.874752, -24.981154], 1)
X_START = [35.590685, -27.711422]
X_GOAL = [26.478673, 9.564082]
DISPLACEMENTS = (np.arange(-2, 3) / 4).tolist()


def fl(x):
    return float(np.asarray(x, dtype=np.float64).reshape(-1)[0])


def read_vertices(name):
    """Vertex lists of a D1 text file, via the reference's own loader (utils.py:29-35),
    which builds reference polygons; we record the vertex lists it was given."""
    captured = []
    orig = ref_utils.polygon

    def spy(*pts):
        captured.append([[float(c) for c in p] for p in pts])
        return orig(*pts)

    ref_utils.polygon = spy
    try:
        shapes = ref_utils.get_var_from_file(os.path.join(REF_DATA, name), "vertices")
    finally:
        ref_utils.polygon = orig
    assert len(shapes) == len(captured)
    return shapes, captured


def build_from_spec(spec):
    """Build a reference RegionMap from our JSON map spec (shape kinds: polygon/ball/square)."""
    m = RegionMap()

    def mk(s):
        if s["kind"] == "polygon":
            return ref_polygon.polygon(*s["vertices"])
        if s["kind"] == "ball":
            return ref_ball.ball(s["center"], s["r1"], s.get("r2"))
        if s["kind"] == "square":
            return ref_square.square(s["center"], s["r1"], s.get("r2"))
        raise ValueError(s["kind"])

    m.add_obstacles(*[mk(s) for s in spec["obstacles"]])
    for reg in spec["regions"]:
        m.new_region(reg["name"], reg["color"])
        m.add_shapes_to_region(reg["name"], *[mk(s) for s in reg["shapes"]])
    m.x_start = list(spec["x_start"])
    m.x_goal = list(spec["x_goal"])
    return m


def canonical_spec():
    _, land = read_vertices("land_area.txt")
    _, pop = read_vertices("populated_area.txt")
    return {
        "obstacles": [{"kind": "ball", "center": c, "r1": r} for c, r in NFZ_BALLS],
        "regions": [
            {"name": "Land", "color": [0.9290, 0.6940, 0.1250],
             "shapes": [{"kind": "polygon", "vertices": v} for v in land]},
            {"name": "Population", "color": "Red",
             "shapes": [{"kind": "polygon", "vertices": v} for v in pop]},
            {"name": "HistCenter", "color": "Green",
             "shapes": [{"kind": "ball", "center": HIST_CENTER[0], "r1": HIST_CENTER[1]}]},
        ],
        "x_start": X_START,
        "x_goal": X_GOAL,
    }


def make_problem(m, N, opts, maxratio, maxalpha, enl, weights):
    p = Problem(m, N, opts)
    p.params.update({"maxratio": maxratio, "maxalpha": maxalpha, "enlargement": enl})
    for name, w in zip(m.region_names(), weights):
        p.set_weight(name, w)
    return p


def eval_path(problem, z_full):
    """Reference outputs for one path z_ = [p_0 .. p_{N+1}] (2(N+2) entries)."""
    N = problem.N
    W = N + 2
    m = problem.map
    cost = fl(problem.get_cost(z_full))
    g = np.asarray(problem.get_nonlincon(z_full), dtype=np.float64).reshape(-1)
    length = fl(problem.length_of(z_full[2:-2]))           # solver.py:49 reported length
    lq = fl(problem.length_of(z_full, problem.options["length_smooth"]))  # get_cost's term
    total = problem.get_total_penalty_function()
    per_region = [problem.get_penalty_function(r) for r in m.region_names()]
    obs_pen = problem.get_penalty_function(None)
    phi = np.zeros(W)
    phi_r = np.zeros((len(per_region), W))
    obs_norm = np.zeros(W)
    collide = np.zeros(W, dtype=np.int8)
    for j in range(W):
        x = z_full[2 * j:2 * j + 2]
        phi[j] = fl(total(x))
        for r, f in enumerate(per_region):
            phi_r[r, j] = fl(f(x))
        if m.obstacles:
            obs_norm[j] = fl(obs_pen(x))
        collide[j] = 1 if m.collides(np.asarray(x)) else 0
    return dict(cost=cost, g=g, length=length, lq=lq, phi=phi, phi_r=phi_r,
                obs_norm=obs_norm, collide=collide)


def arc(problem, d):
    s = Solver(problem, {})
    return np.asarray(s.create_x_init(d), dtype=np.float64)


def full_path(m, x_init):
    return np.concatenate([np.asarray(m.x_start, float), x_init, np.asarray(m.x_goal, float)])


# ----------------------------------------------------------------------------------------
def gen_canonical():
    spec = canonical_spec()
    m = build_from_spec(spec)
    N = 80
    opts = {"length_smooth": True, "penalty_smooth": True, "obstacle_smooth": True,
            "maxratio_smooth": False}
    params = dict(maxratio=1.04, maxalpha=np.pi / 80, enl=0.0, weights=[200, 15000, 27000])
    prob = make_problem(m, N, opts, params["maxratio"], params["maxalpha"], params["enl"],
                        params["weights"])
    out = {k: [] for k in ("x_init", "cost", "g", "length", "lq", "phi", "phi_r",
                           "obs_norm", "collide")}
    for d in DISPLACEMENTS:
        x = arc(prob, d)
        r = eval_path(prob, full_path(m, x))
        out["x_init"].append(x)
        for k in ("cost", "g", "length", "lq", "phi", "phi_r", "obs_norm", "collide"):
            out[k].append(r[k])
        print(f"canonical d={d:+.2f} cost={r['cost']:.10f} length={r['length']:.9f} "
              f"gsum={r['g'].sum():.6f} nfz_wp={int(r['collide'].sum())}")
    arrays = {k: np.asarray(v) for k, v in out.items()}
    arrays["displacements"] = np.asarray(DISPLACEMENTS)
    np.savez_compressed(os.path.join(HERE, "canonical.npz"), **arrays)
    meta = {"map": spec, "N": N, "options": opts, "maxratio": params["maxratio"],
            "maxalpha": params["maxalpha"], "enlargement": params["enl"],
            "weights": params["weights"], "displacements": DISPLACEMENTS,
            "source": "reference main.py:21-61,122-160 via problem.py get_cost/get_nonlincon"}
    with open(os.path.join(HERE, "canonical.json"), "w") as f:
        json.dump(meta, f, indent=1)
    return spec, m


def gen_variants(spec):
    res = {}
    # (a) canonical with enlargement 0.5
    m = build_from_spec(spec)
    opts = {"length_smooth": True, "penalty_smooth": True, "obstacle_smooth": True,
            "maxratio_smooth": False}
    prob = make_problem(m, 80, opts, 1.04, np.pi / 80, 0.5, [200, 15000, 27000])
    costs, gs = [], []
    for d in DISPLACEMENTS:
        z = full_path(m, arc(prob, d))
        costs.append(fl(prob.get_cost(z)))
        gs.append(np.asarray(prob.get_nonlincon(z), float).reshape(-1))
    res["enl05_cost"] = np.asarray(costs)
    res["enl05_g"] = np.asarray(gs)
    print("enl=0.5 costs", costs)
    # (b) problem.py:211-272 demo map/weights at N=10, default opts (problem.py:12-17)
    m2 = build_from_spec({"obstacles": spec["obstacles"], "regions": spec["regions"],
                          "x_start": X_START, "x_goal": X_GOAL})
    prob2 = make_problem(m2, 10, None, 1.25, np.pi / 10, 0.0, [4, 13, 45])
    costs, gs, xs = [], [], []
    for d in DISPLACEMENTS:
        x = arc(prob2, d)
        z = full_path(m2, x)
        xs.append(x)
        costs.append(fl(prob2.get_cost(z)))
        gs.append(np.asarray(prob2.get_nonlincon(z), float).reshape(-1))
    res["n10_cost"] = np.asarray(costs)
    res["n10_g"] = np.asarray(gs)
    res["n10_x_init"] = np.asarray(xs)
    print("N=10 default-opts costs", costs)
    np.savez_compressed(os.path.join(HERE, "variants.npz"), **res)


def rand_convex(rng, cx, cy, rmin, rmax, k):
    ang = np.sort(rng.uniform(0, 2 * np.pi, size=k))
    # keep angular gaps away from 0 so no three points are nearly collinear
    ang = np.linspace(0, 2 * np.pi, k, endpoint=False) + rng.uniform(0, 2 * np.pi / k * 0.6, k)
    a = rng.uniform(rmin, rmax)
    b = rng.uniform(rmin, rmax)
    rot = rng.uniform(0, np.pi)
    pts = []
    for t in ang:
        x, y = a * math.cos(t), b * math.sin(t)
        pts.append([cx + x * math.cos(rot) - y * math.sin(rot),
                    cy + x * math.sin(rot) + y * math.cos(rot)])
    order = rng.permutation(k)           # exercise polygon()'s convex-walk ordering
    return [[round(float(pts[i][0]), 6), round(float(pts[i][1]), 6)] for i in order]


def rand_shape(rng, kinds):
    kind = kinds[rng.integers(len(kinds))]
    cx, cy = rng.uniform(-4, 4), rng.uniform(-4, 4)
    if kind == "polygon":
        return {"kind": "polygon", "vertices": rand_convex(rng, cx, cy, 0.8, 3.0,
                                                           int(rng.integers(3, 9)))}
    if kind == "ball":
        r1 = float(rng.uniform(0.5, 3))
        r2 = float(rng.uniform(0.5, 3)) if rng.random() < 0.5 else None
        s = {"kind": "ball", "center": [float(cx), float(cy)], "r1": r1}
        if r2 is not None:
            s["r2"] = r2
        return s
    r1 = float(rng.uniform(0.5, 3))
    s = {"kind": "square", "center": [float(cx), float(cy)], "r1": r1}
    if rng.random() < 0.5:
        s["r2"] = float(rng.uniform(0.5, 3))
    return s


def gen_random_cases(n_cases=24, seed=12345):
    rng = np.random.default_rng(seed)
    cases = []
    for c in range(n_cases):
        n_obs = int(rng.integers(0, 4))
        n_reg = int(rng.integers(1, 4))
        spec = {"obstacles": [rand_shape(rng, ["ball", "polygon", "square"])
                              for _ in range(n_obs)],
                "regions": [], "x_start": [float(rng.uniform(-5, -3)), float(rng.uniform(-5, 5))],
                "x_goal": [float(rng.uniform(3, 5)), float(rng.uniform(-5, 5))]}
        for r in range(n_reg):
            spec["regions"].append({"name": f"R{r}", "color": "Red",
                                    "shapes": [rand_shape(rng, ["polygon", "ball", "square"])
                                               for _ in range(int(rng.integers(1, 4)))]})
        combo = c % 16
        opts = {"length_smooth": bool(combo & 1), "penalty_smooth": bool(combo & 2),
                "obstacle_smooth": bool(combo & 4), "maxratio_smooth": bool(combo & 8)}
        N = int(rng.integers(2, 14))
        maxratio = float(rng.uniform(1.0, 1.6))
        maxalpha = float(rng.uniform(0.05, 1.5))
        enl = float(rng.choice([0.0, 0.0, 0.3, -0.2]))
        weights = [float(rng.uniform(0.5, 50)) for _ in range(n_reg)]
        m = build_from_spec(spec)
        prob = make_problem(m, N, opts, maxratio, maxalpha, enl, weights)
        paths = []
        for _ in range(3):
            # random walk between start and goal, plus one arc
            t = np.linspace(0, 1, N + 2)[1:-1]
            base = np.outer(1 - t, spec["x_start"]) + np.outer(t, spec["x_goal"])
            z = base + rng.normal(scale=0.7, size=base.shape)
            paths.append(full_path(m, z.reshape(-1)))
        paths.append(full_path(m, arc(prob, float(rng.uniform(-0.9, 0.9)))))
        outs = []
        for z in paths:
            r = eval_path(prob, z)
            outs.append({"cost": r["cost"], "g": r["g"].tolist(), "length": r["length"],
                         "lq": r["lq"], "phi": r["phi"].tolist(),
                         "phi_r": r["phi_r"].tolist(), "obs_norm": r["obs_norm"].tolist(),
                         "collide": r["collide"].tolist()})
        cases.append({"map": spec, "N": N, "options": opts, "maxratio": maxratio,
                      "maxalpha": maxalpha, "enlargement": enl, "weights": weights,
                      "paths": [z.tolist() for z in paths], "outputs": outs})
    with open(os.path.join(HERE, "random_cases.json"), "w") as f:
        json.dump({"seed": seed, "cases": cases}, f)
    print(f"random cases: {len(cases)}")


def gen_arcs():
    res = {}
    m = RegionMap()
    pairs = [(X_START, X_GOAL), ([0.0, 0.0], [10.0, 0.0]), ([3.5, -1.25], [-7.0, 4.0])]
    Ns = [1, 4, 80, 254]
    ds = [-0.95, -0.5, -0.25, -1e-3, 0.0, 1e-3, 0.25, 0.5, 0.95, 1.0]
    for pi, (a, b) in enumerate(pairs):
        m.x_start, m.x_goal = list(a), list(b)
        for N in Ns:
            prob = Problem(m, N)
            res[f"p{pi}_N{N}"] = np.asarray([arc(prob, d) for d in ds])
    res["pairs"] = np.asarray([[*a, *b] for a, b in pairs])
    res["Ns"] = np.asarray(Ns)
    res["ds"] = np.asarray(ds)
    np.savez_compressed(os.path.join(HERE, "arcs.npz"), **res)


def gen_grid(spec):
    """Reference Φ and ψ at cell centres of a 48x40 raster over x∈[10,58], y∈[-40,0].
    Cell-centre convention (GeoTIFF, row 0 north): x = X0 + (ix+0.5)dx, y = Ytop-(iy+0.5)dy."""
    m = build_from_spec(spec)
    nx, ny, X0, Ytop, dx, dy = 48, 40, 10.0, 0.0, 1.0, 1.0
    res = {"geo": np.asarray([nx, ny, X0, Ytop, dx, dy], dtype=np.float64)}
    for tag, opts, enl in (("a", {"penalty_smooth": True, "obstacle_smooth": True}, 0.0),
                           ("b", {"penalty_smooth": False, "obstacle_smooth": False}, 0.25)):
        prob = make_problem(m, 4, opts, 1.1, 0.3, enl, [200, 15000, 27000])
        total = prob.get_total_penalty_function()
        obs = [o.penalty_function(opts["obstacle_smooth"]) for o in m.obstacles]
        phi = np.zeros((ny, nx))
        psi = np.zeros((ny, nx))
        col = np.zeros((ny, nx), dtype=np.int8)
        for iy in range(ny):
            for ix in range(nx):
                x = np.array([X0 + (ix + 0.5) * dx, Ytop - (iy + 0.5) * dy])
                phi[iy, ix] = fl(total(x))
                s = 0.0
                for f in obs:
                    s = s + fl(f(x))
                psi[iy, ix] = s
                col[iy, ix] = 1 if m.collides(x) else 0
        res[f"phi_{tag}"] = phi
        res[f"psi_{tag}"] = psi
        res[f"collide_{tag}"] = col
    np.savez_compressed(os.path.join(HERE, "grid.npz"), **res)


def gen_errors():
    cases = []

    def rec(label, fn):
        try:
            fn()
        except Exception as e:  # noqa: BLE001 - we record whatever the reference raises
            cases.append({"case": label, "type": type(e).__name__, "message": str(e)})
        else:
            cases.append({"case": label, "type": None, "message": None})

    rec("polygon_two_points", lambda: ref_polygon.polygon([0.0, 0.0], [1.0, 0.0]))
    rec("polygon_collinear", lambda: ref_polygon.polygon([0.0, 0.0], [1.0, 0.0], [2.0, 0.0],
                                                         [1.0, 1.0]))
    rec("polygon_nonconvex", lambda: ref_polygon.polygon([0.0, 0.0], [4.0, 0.0], [1.0, 1.0],
                                                         [0.0, 4.0]))
    rec("polygon_ok_square", lambda: ref_polygon.polygon([0.0, 0.0], [1.0, 0.0], [1.0, 1.0],
                                                         [0.0, 1.0]))
    m = RegionMap()
    m.x_start, m.x_goal = [0.0, 0.0], [1.0, 1.0]
    prob = Problem(m, 4)
    rec("arc_displacement_gt1", lambda: Solver(prob, {}).create_x_init(1.5))
    m.new_region("A", "Red")
    rec("region_duplicate", lambda: m.new_region("A", "Blue"))
    rec("region_unknown", lambda: m.add_shape_to_region("B", ref_ball.ball([0, 0], 1)))
    with open(os.path.join(HERE, "errors.json"), "w") as f:
        json.dump(cases, f, indent=1)


# cfg3's pairs (uam_path_planning_amd/synthetic.py random_pairs(100_000, seed=0): uniform in
# the land bbox) and raster extent (x in [0, 60] km, y in [-40, 20] km)
LAND_BBOX = (11.673387096774192, 46.75403225806451, -37.53246753246754, 19.204545454545457)


def cfg3_pairs(Q_total=100_000, take=2000):
    rng = np.random.default_rng(0)
    x = rng.uniform(LAND_BBOX[0], LAND_BBOX[1], size=(Q_total, 2))
    y = rng.uniform(LAND_BBOX[2], LAND_BBOX[3], size=(Q_total, 2))
    return np.stack([x[:, 0], y[:, 0], x[:, 1], y[:, 1]], axis=1)[:take].astype(np.float64)


def raster_cells(wp, R):
    """The raster cell of every waypoint (include/uampath.h uam_raster_desc): ix =
    floor((x - x0) * (1/dx)), iy = floor((y_top - y) * (1/dy)) in float64, ix = iy = -1 off
    the raster; x0 = 0, y_top = 20, dx = dy = 60 / R.  Stored as int16 differences along each
    path (the first waypoint's ix / iy as is), which compress: tests/golden_io.py
    waypoint_cells() rebuilds iy * R + ix."""
    inv = 1.0 / (60.0 / R)
    fx = np.floor((wp[..., 0] - 0.0) * inv)
    fy = np.floor((20.0 - wp[..., 1]) * inv)
    ok = (fx >= 0) & (fx < R) & (fy >= 0) & (fy < R)
    ix = np.where(ok, fx, -1.0).astype(np.int16)
    iy = np.where(ok, fy, -1.0).astype(np.int16)
    d = lambda a: np.concatenate([a[:, :1], np.diff(a, axis=1)], axis=1).astype(np.int16)
    return d(ix), d(iy)


def gen_waypoint_cells(take=2000, N=80):
    """Verdict r5 item 1: the reference's own waypoints (create_x_init, solver.py:103-136, with
    the pair's start and goal, main.py:160-171) as raster cells at 4096^2 and 8192^2, for the
    first `take` pairs of cfg3 x the 5 displacements of main.py:160.  Paths are pair-major
    (path = q * 5 + d), W = N + 2 cells each."""
    pairs = cfg3_pairs(take=take)
    m = RegionMap()
    wp = np.empty((take * len(DISPLACEMENTS), N + 2, 2))
    for q, pr in enumerate(pairs):
        m.x_start, m.x_goal = [pr[0], pr[1]], [pr[2], pr[3]]
        s = Solver(Problem(m, N), {})
        for di, d in enumerate(DISPLACEMENTS):
            x = np.asarray(s.create_x_init(d), dtype=np.float64).reshape(N, 2)
            p = q * len(DISPLACEMENTS) + di
            wp[p, 0] = pr[:2]
            wp[p, 1:N + 1] = x
            wp[p, N + 1] = pr[2:]
    res = {"pairs": pairs, "displacements": np.asarray(DISPLACEMENTS), "N": np.asarray(N)}
    for R in (4096, 8192):
        res[f"dix{R}"], res[f"diy{R}"] = raster_cells(wp, R)
    np.savez_compressed(os.path.join(HERE, "waypoint_cells.npz"), **res)
    print(f"waypoint cells: {wp.shape[0]} paths x {N + 2}")


if __name__ == "__main__":
    if not os.path.isdir(REF_PG):
        sys.exit("reference not mounted; golden fixtures are generated in the build container only")
    if sys.argv[1:] == ["cells"]:   # round 6: only the waypoint-cell fixture
        gen_waypoint_cells()
        sys.exit(0)
    spec, _ = gen_canonical()
    gen_variants(spec)
    gen_random_cases()
    gen_arcs()
    gen_grid(spec)
    gen_errors()
    gen_waypoint_cells()
    print("done")
