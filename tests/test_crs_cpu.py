"""CRS transform + shapefile layout on the CPU.  The oracle's
transverse Mercator is pinned to the reference's own shapefiles (tests/golden/crs.npz, made
by tests/golden/make_crs_golden.py): inverse <= 5e-14 deg (float64 rounding of ~130 deg is
1.4e-14), forward <= 1e-8 m (the n^6 Krueger series is good to ~5 nm).  The writer's
layout is compared with the reference files' headers (crs_meta.json)."""
import datetime
import json
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN

TOL_DEG = 5e-14
TOL_M = 1e-8


@pytest.fixture(scope="module")
def crs():
    z = np.load(os.path.join(GOLDEN, "crs.npz"))
    with open(os.path.join(GOLDEN, "crs_meta.json")) as f:
        meta = json.load(f)
    return z, meta


def test_oracle_inverse_matches_reference_shapefiles(oracle_mod, crs):
    z, _ = crs
    got = oracle_mod.tm_inv(z["plane_xy"])
    err = np.abs(got - z["lonlat"]).max()
    assert err <= TOL_DEG, err


def test_oracle_forward_roundtrip(oracle_mod, crs):
    z, _ = crs
    xy = oracle_mod.tm_fwd(z["lonlat"])
    assert np.abs(xy - z["plane_xy"]).max() <= TOL_M


def test_oracle_zone_origins(oracle_mod):
    assert len(oracle_mod.JPRCS_ORIGINS) == 19
    for zone in (1, 9, 19):       # the origin maps to (0, 0) in its own zone
        tm = oracle_mod.tm_zone(zone)
        xy = oracle_mod.tm_fwd([[tm.lon0_deg, tm.lat0_deg]], tm)
        assert np.abs(xy).max() < 1e-8


def _split(z, name, meta):
    names = list(z["names"])
    si = names.index(name)
    sel = z["set"] == si
    ll, ring = z["lonlat"][sel], z["ring"][sel]
    return [ll[ring == r] for r in range(meta[name]["records"])]


@pytest.mark.parametrize("name", ["land", "populated", "nfz"])
def test_shapefile_writer_layout_matches_reference(tmp_path, crs, name):
    from uam_path_planning_amd.geo import shapefile as S

    z, meta = crs
    m = meta[name]
    rings = _split(z, name, meta)
    # feed half of the rings counter-clockwise: the writer must restore the ESRI orientation
    fed = [r[::-1].copy() if i % 2 else r for i, r in enumerate(rings)]
    path = S.write_shapefile(str(tmp_path / name), fed, S.POLYGON, date=datetime.date(2024, 12, 6))
    kind, geoms = S.read_shapefile(path)
    assert kind == m["shape_type"] == S.POLYGON
    assert [len(g[0]) for g in geoms] == m["vertices"]
    for g, r in zip(geoms, rings):
        np.testing.assert_array_equal(g[0], r)
    b = open(path, "rb").read()
    assert struct.unpack("<4d", b[36:68]) == tuple(m["bbox"])
    base = path[:-4]
    d = open(base + ".dbf", "rb").read()
    n, hlen, rlen = struct.unpack("<IHH", d[4:12])
    assert (n, hlen, rlen) == (m["dbf"]["n"], m["dbf"]["hlen"], m["dbf"]["rlen"])
    assert [d[32:43].split(b"\0")[0].decode(), chr(d[43]), d[48], d[49]] == m["dbf"]["field"]
    assert [d[hlen + i * rlen:hlen + (i + 1) * rlen].decode() for i in range(n)] == \
        m["dbf"]["rows"]
    assert d[-1:] == b"\x1a"
    assert open(base + ".prj").read() == m["prj"]
    assert open(base + ".cpg").read() == m["cpg"]
    x = open(base + ".shx", "rb").read()
    assert len(x) == 100 + 8 * n


def test_shapefile_points_and_lines_roundtrip(tmp_path):
    from uam_path_planning_amd.geo import shapefile as S

    pts = [(129.5, 33.0), (130.0, 32.5)]
    kind, g = S.read_shapefile(S.write_shapefile(str(tmp_path / "p"), pts, S.POINT))
    assert kind == S.POINT and g == pts
    line = np.array([[129.5, 33.0], [129.6, 33.1], [129.7, 33.0]])
    kind, g = S.read_shapefile(S.write_shapefile(str(tmp_path / "l"), [line], S.POLYLINE))
    assert kind == S.POLYLINE
    np.testing.assert_array_equal(g[0][0], line)          # lines keep their direction


def test_buffer_circle_matches_reference_vertex_order(oracle_mod, crs):
    from uam_path_planning_amd.geo.export import NO_FLY_ZONES, buffer_circle

    z, meta = crs
    rings = _split(z, "nfz", meta)
    for (c, r), ref in zip(NO_FLY_ZONES.values(), rings):
        got = oracle_mod.tm_inv(buffer_circle(c, r))
        assert np.abs(got - ref).max() <= TOL_DEG


def test_oracle_reprojection_properties(oracle_mod):
    """Nearest = the source pixel containing the inverse-transformed cell centre; bilinear
    reproduces a field linear in (u, v) exactly up to float32 rounding."""
    from uam_path_planning_amd.scenario import raster_geo

    geo = raster_geo(64)
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy)
    lon0, lat_top, dl = 129.4, 33.3, 0.002
    g = oracle_mod.geo_grid(400, 400, lon0, lat_top, dl, dl)
    iu, iv = np.meshgrid(np.arange(400), np.arange(400))
    src = (100.0 + 0.5 * iu + 0.25 * iv).astype(np.float32)
    near = oracle_mod.reproject(src, g, rd, resample=0)
    bil = oracle_mod.reproject(src, g, rd, resample=1)
    cx = geo.x0 + (np.arange(64) + 0.5) * geo.dx
    cy = geo.y_top - (np.arange(64) + 0.5) * geo.dy
    X, Y = np.meshgrid(cx, cy)
    ll = oracle_mod.tm_inv(np.c_[X.ravel() * 1000, Y.ravel() * 1000])
    u = (ll[:, 0] - lon0) / dl
    v = (lat_top - ll[:, 1]) / dl
    np.testing.assert_array_equal(near.ravel(), src[np.floor(v).astype(int), np.floor(u).astype(int)])
    lin = 100.0 + 0.5 * (u - 0.5) + 0.25 * (v - 0.5)
    np.testing.assert_allclose(bil.ravel(), lin, rtol=2e-7)
    g2 = oracle_mod.geo_grid(10, 10, 150.0, 40.0, dl, dl)                # no overlap
    assert (oracle_mod.reproject(src[:10, :10], g2, rd) == -9999.0).all()
