"""Synthetic inputs for the BASELINE configs.  The real Nagasaki DEM is a
Git-LFS pointer in the reference (data/raw/nagasaki_geotiff/merge_test.tif:1-3), so every
config runs on a synthetic DEM with the real one's statistics
(merge_test.tif.aux.xml:4-9): mean 129.48 m, std 112.59 m, range [-12.05, 557.52] m,
53.11 % valid cells (the rest nodata -9999 = sea)."""
import numpy as np

DEM_MEAN = 129.47586964714
DEM_STD = 112.58964659888
DEM_MIN = -12.046955108643
DEM_MAX = 557.51721191406
DEM_VALID = 0.5311
NODATA = -9999.0

# raster extent (km, EPSG:2443 plane): x in [0, 60], y in [-40, 20] (visualizer.py:12 limits)
EXTENT_X0, EXTENT_Y_TOP, EXTENT = 0.0, 20.0, 60.0

# bounding box of the Land polygons (data/processed/land_area.txt)
LAND_BBOX = (11.673387096774192, 46.75403225806451, -37.53246753246754, 19.204545454545457)


def _upsample(grid, R):
    """Bilinear upsampling of a (g+1)x(g+1) lattice to R x R cell centres (separable)."""
    g = grid.shape[0] - 1
    t = (np.arange(R, dtype=np.float64) + 0.5) / R * g
    i0 = np.clip(np.floor(t).astype(np.int64), 0, g - 1)
    f = t - i0
    M = np.zeros((R, g + 1))
    M[np.arange(R), i0] = 1.0 - f
    M[np.arange(R), i0 + 1] += f
    return M @ grid @ M.T


def synthetic_dem(R, seed=1, octaves=7, base=4):
    """R x R float32 DEM, row 0 = north, nodata -9999 on the 'sea' cells."""
    rng = np.random.default_rng(seed)
    field = np.zeros((R, R), dtype=np.float64)
    amp = 1.0
    g = base
    for _ in range(octaves):
        if g > R:
            break
        field += amp * _upsample(rng.standard_normal((g + 1, g + 1)), R)
        amp *= 0.55
        g *= 2
    sea_field = _upsample(rng.standard_normal((6, 6)), R) + \
        0.25 * _upsample(rng.standard_normal((17, 17)), R)
    thr = np.quantile(sea_field, 1.0 - DEM_VALID)
    land = sea_field >= thr
    vals = field[land]
    z = (field - vals.mean()) / vals.std() * DEM_STD + DEM_MEAN
    z = np.clip(z, DEM_MIN, DEM_MAX)
    return np.where(land, z, NODATA).astype(np.float32)


def random_pairs(Q, seed=0, bbox=LAND_BBOX):
    """Q start/goal pairs uniform in the Land bbox: [Q, 4] = (x0, y0, xf, yf)."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(bbox[0], bbox[1], size=(Q, 2))
    y = rng.uniform(bbox[2], bbox[3], size=(Q, 2))
    return np.stack([x[:, 0], y[:, 0], x[:, 1], y[:, 1]], axis=1).astype(np.float64)


def random_convex_polygons(K, seed=2, bbox=LAND_BBOX, rmin=0.5, rmax=3.0, kmin=4, kmax=8):
    """K random convex polygons (vertex lists in convex order), radii rmin..rmax km."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(K):
        k = int(rng.integers(kmin, kmax + 1))
        cx = rng.uniform(bbox[0], bbox[1])
        cy = rng.uniform(bbox[2], bbox[3])
        a, b = rng.uniform(rmin, rmax), rng.uniform(rmin, rmax)
        rot = rng.uniform(0, np.pi)
        ang = np.linspace(0, 2 * np.pi, k, endpoint=False) + rng.uniform(0, 2 * np.pi / k * 0.6, k)
        pts = []
        for t in ang:
            x, y = a * np.cos(t), b * np.sin(t)
            pts.append([round(float(cx + x * np.cos(rot) - y * np.sin(rot)), 6),
                        round(float(cy + x * np.sin(rot) + y * np.cos(rot)), 6)])
        out.append(pts)
    return out


def random_pairs3d(Q, seed=0, bbox=LAND_BBOX, zmin=100.0, zmax=500.0):
    """Q pairs with altitudes: [Q, 6] = (x0, y0, z0, xf, yf, zf), z in metres."""
    xy = random_pairs(Q, seed=seed, bbox=bbox)
    z = np.random.default_rng(seed + 1000).uniform(zmin, zmax, size=(Q, 2))
    return np.stack([xy[:, 0], xy[:, 1], z[:, 0], xy[:, 2], xy[:, 3], z[:, 1]], axis=1)
