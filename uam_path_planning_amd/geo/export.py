"""The reference's GIS exports, with the EPSG:2443 -> EPSG:4612
transform on the GPU (K7) and the shapefile layout of geopandas/OGR:

  make_result_line_shp(x, path)        path_generation/main.py:103-108 (km waypoints -> m,
                                        LineString start + waypoints + goal)
  save_points_to_shp(x, path)           path_generation/main.py:110-116 (one Point each)
  save_polygons_to_shapefile(polys, p)  map_generation/data_manager.py:83-86
  make_area_shp(polys, path)            map_generation/utils.py:81-84
  make_no_fly_zone_shp(path)            map_generation/utils.py:88-111 (Point.buffer circles)
  export_paths(wp, path)                batched: P refined / candidate paths [P, W, 2] km ->
                                        one shapefile of P LineStrings, one transform launch
"""
import numpy as np

from .crs import plane_to_geo
from .shapefile import POINT, POLYGON, POLYLINE, write_shapefile

# path_generation/main.py:103 / 110 defaults (metres, EPSG:2443)
START_POINT = (35590.685, -27711.422)
END_POINT = (26478.673, 9564.082)

# map_generation/utils.py:93-99: centre (m, EPSG:2443), radius (m)
NO_FLY_ZONES = {
    "air_port": ((38666.52661075855, -9203.164091309498), 9000),
    "defense_base1": ((46361.37256675563, 3942.7562315386298), 2000),
    "defense_base2": ((19846.825121034392, 18934.11773399299), 2000),
    "defense_base3": ((26037.433469490207, 15467.10452712196), 2000),
    "heli_port": ((46877.58543585609, -19138.710035318375), 2000),
}


def buffer_circle(center, radius, quad_segs=16):
    """shapely Point(center).buffer(radius): 4 * quad_segs segments, first vertex at angle 0,
    clockwise, closed (GEOS OffsetSegmentGenerator::createCircle)."""
    n = 4 * quad_segs
    th = -np.arange(n, dtype=np.float64) * (2.0 * np.pi / n)
    ring = np.c_[center[0] + radius * np.cos(th), center[1] + radius * np.sin(th)]
    return np.vstack([ring, ring[:1]])


def _path_points(x, start_point, end_point):
    a = np.asarray(x, dtype=np.float64).reshape(-1, 2) * 1000.0
    return np.vstack([np.asarray(start_point, np.float64).reshape(1, 2), a,
                      np.asarray(end_point, np.float64).reshape(1, 2)])


def _to_geo(pts_m, engine=None):
    pts = np.asarray(pts_m, dtype=np.float64).reshape(-1, 2)
    return plane_to_geo(pts, 1, engine).cpu().numpy() if len(pts) else pts


def make_result_line_shp(x, file_path, start_point=START_POINT, end_point=END_POINT,
                         engine=None):
    """main.py:103-108: x = [x1, y1, ...] (km) -> LineString shapefile in EPSG:4612."""
    return write_shapefile(file_path, [_to_geo(_path_points(x, start_point, end_point),
                                               engine)], POLYLINE)


def save_points_to_shp(x, output_path, start_point=START_POINT, end_point=END_POINT,
                       engine=None):
    """main.py:110-116: every waypoint (and the two endpoints) as a Point in EPSG:4612."""
    geo = _to_geo(_path_points(x, start_point, end_point), engine)
    return write_shapefile(output_path, list(geo), POINT)


def _polygons_to_geo(polygons, engine=None):
    rings = [np.asarray(p, dtype=np.float64).reshape(-1, 2) for p in polygons]
    if not rings:
        return []
    flat = _to_geo(np.vstack(rings), engine)
    out, o = [], 0
    for r in rings:
        out.append(flat[o:o + len(r)])
        o += len(r)
    return out


def save_polygons_to_shapefile(polygons, output_file, engine=None):
    """data_manager.py:83-86: polygons (vertex arrays, metres, EPSG:2443) -> EPSG:4612."""
    return write_shapefile(output_file, _polygons_to_geo(polygons, engine), POLYGON)


def make_area_shp(polygons, output_file, engine=None):
    """map_generation/utils.py:81-84 (same transform and layout)."""
    return save_polygons_to_shapefile(polygons, output_file, engine)


def make_no_fly_zone_shp(output_file, zones=NO_FLY_ZONES, engine=None):
    """map_generation/utils.py:88-111."""
    circles = [buffer_circle(c, r) for c, r in zones.values()]
    return write_shapefile(output_file, _polygons_to_geo(circles, engine), POLYGON)


def export_paths(wp_km, output_file, engine=None):
    """Batched export: wp [P, W, 2] (km, EPSG:2443) -> one EPSG:4612 shapefile with P
    LineStrings; all P*W waypoints go through one GPU transform launch."""
    import torch

    from ..engine import default_engine

    eng = engine if engine is not None else default_engine()
    wp = eng.tensor(wp_km, torch.float64)
    P, W = wp.shape[0], wp.shape[1]
    geo = eng.plane_to_geo((wp * 1000.0).reshape(-1, 2), 1).cpu().numpy().reshape(P, W, 2)
    return write_shapefile(output_file, list(geo), POLYLINE)
