"""EPSG:4612 / 6668 (geographic JGD2000 / JGD2011, lon-lat axis order as geopandas' to_crs
uses) <-> EPSG:2443..2461 (JGD2000 / Japan Plane Rectangular CS I..XIX, x = easting,
y = northing, metres), computed by the HIP kernel K7 (include/uampath.h uam_geo_to_plane).
The reference calls pyproj for exactly these pairs (map_generation/data_manager.py:24-26,
84-85; path_generation/main.py:106-115; map_generation/utils.py:81-111).  JGD2011 and JGD2000
share the GRS80 ellipsoid and PROJ applies no shift between them, so both map to the same
projection.  Parity: tests/golden/crs.npz (the reference's own shapefiles), <= 3e-14 deg."""
import numpy as np

GEOGRAPHIC_EPSG = (4612, 6668)
PLANE_EPSG = tuple(range(2443, 2462))   # zone = epsg - 2442


def _engine(engine):
    from ..engine import default_engine

    return engine if engine is not None else default_engine()


def _zone(epsg):
    if epsg not in PLANE_EPSG:
        raise ValueError(f"EPSG:{epsg} is not a JGD2000 plane rectangular CS (2443..2461)")
    return epsg - 2442


def geo_to_plane(lonlat, zone=1, engine=None):
    """[n, 2] (lon, lat) degrees -> [n, 2] (x, y) metres (device tensor)."""
    return _engine(engine).geo_to_plane(lonlat, zone)


def plane_to_geo(xy, zone=1, engine=None):
    """[n, 2] (x, y) metres -> [n, 2] (lon, lat) degrees (device tensor)."""
    return _engine(engine).plane_to_geo(xy, zone)


def to_crs(coords, src_epsg, dst_epsg, engine=None):
    """numpy [n, 2] in src_epsg -> numpy [n, 2] in dst_epsg (geopandas' to_crs for the pairs
    the reference uses)."""
    a = np.asarray(coords, dtype=np.float64).reshape(-1, 2)
    if src_epsg == dst_epsg:
        return a.copy()
    if src_epsg in GEOGRAPHIC_EPSG and dst_epsg in GEOGRAPHIC_EPSG:
        return a.copy()
    if len(a) == 0:
        return a.copy()
    if src_epsg in GEOGRAPHIC_EPSG:
        return geo_to_plane(a, _zone(dst_epsg), engine).cpu().numpy()
    if dst_epsg in GEOGRAPHIC_EPSG:
        return plane_to_geo(a, _zone(src_epsg), engine).cpu().numpy()
    eng = _engine(engine)
    return eng.geo_to_plane(eng.plane_to_geo(a, _zone(src_epsg)), _zone(dst_epsg)).cpu().numpy()
