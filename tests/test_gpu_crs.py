"""GPU CRS transform, DEM reprojection and the GIS export (K7).
Tolerances: inverse transform vs the reference's shapefiles <= 5e-14 deg and vs the oracle
<= 2e-14 deg (device and host libm may differ by an ulp per transcendental); forward <= 1e-8 m
vs the reference inputs, <= 5e-9 m vs the oracle (one ulp of the conformal angle xi,
~1.1e-16 rad, is 7e-10 m after the k0*A = 6.4e6 m scale).  Reprojection: nearest is compared with
exact equality (an index can only move when a centre lies within ~1e-13 of a pixel edge),
bilinear within 1 float32 ulp."""
import datetime
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def eng():
    from uam_path_planning_amd import build
    from uam_path_planning_amd.engine import Engine

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    build.build_library()
    return Engine(0)


@pytest.fixture(scope="module")
def crs():
    z = np.load(os.path.join(GOLDEN, "crs.npz"))
    with open(os.path.join(GOLDEN, "crs_meta.json")) as f:
        meta = json.load(f)
    return z, meta


def test_gpu_transform_vs_reference_and_oracle(eng, oracle_mod, crs):
    z, _ = crs
    ll = eng.plane_to_geo(z["plane_xy"]).cpu().numpy()
    assert np.abs(ll - z["lonlat"]).max() <= 5e-14
    assert np.abs(ll - oracle_mod.tm_inv(z["plane_xy"])).max() <= 2e-14
    xy = eng.geo_to_plane(z["lonlat"]).cpu().numpy()
    assert np.abs(xy - z["plane_xy"]).max() <= 1e-8
    assert np.abs(xy - oracle_mod.tm_fwd(z["lonlat"])).max() <= 5e-9
    for zone in (2, 9, 13, 19):   # other zones: GPU == oracle on a grid around the origin
        tm = oracle_mod.tm_zone(zone)
        g = np.stack(np.meshgrid(np.linspace(tm.lon0_deg - 1.5, tm.lon0_deg + 1.5, 31),
                                 np.linspace(tm.lat0_deg - 2, tm.lat0_deg + 2, 41)), -1)
        g = g.reshape(-1, 2)
        p = eng.geo_to_plane(g, zone).cpu().numpy()
        assert np.abs(p - oracle_mod.tm_fwd(g, tm)).max() <= 5e-9
        back = eng.plane_to_geo(p, zone).cpu().numpy()
        assert np.abs(back - g).max() <= 1e-12
    assert eng.plane_to_geo(np.zeros((0, 2))).shape == (0, 2)
    with pytest.raises(ValueError):
        eng.geo_to_plane(z["lonlat"], 20)


@pytest.mark.parametrize("resample", [0, 1])
def test_gpu_reproject_vs_oracle(eng, oracle_mod, resample):
    """A lat/lon mosaic in the mergeLL.vrt layout (0.2 arc-second pixels) covering part of the
    plane raster (so some cells fall outside), with nodata holes."""
    from uam_path_planning_amd._lib import GeoGridDesc
    from uam_path_planning_amd.scenario import raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    geo = raster_geo(512)
    src = synthetic_dem(1024, seed=5)
    lon0, lat_top, d = 129.55, 33.2, 5.5555555555554013e-05 * 8
    gg = GeoGridDesc(1024, 1024, lon0, lat_top, d, d, -9999.0, 0)
    gpu = eng.reproject_dem(src, gg, geo, 1000.0, resample).cpu().numpy()
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy)
    ref = oracle_mod.reproject(src, oracle_mod.geo_grid(1024, 1024, lon0, lat_top, d, d), rd,
                               1000.0, resample)
    assert (ref == -9999.0).any() and (ref != -9999.0).any()
    if resample == 0:
        np.testing.assert_array_equal(gpu, ref)
    else:
        np.testing.assert_array_max_ulp(gpu, ref, maxulp=1)


def test_reprojected_dem_feeds_the_cost_raster(eng, oracle_mod):
    """lat/lon mosaic -> reproject (K7) -> raster build (K1) is the full-scale ingest chain of
    DataManager.load_dem_geographic; the record raster equals the oracle's build on the
    oracle's reprojected DEM."""
    from uam_path_planning_amd._lib import GeoGridDesc
    from uam_path_planning_amd.geometry import compile_map
    from uam_path_planning_amd.scenario import (build_region_map, canonical_params,
                                                canonical_spec, raster_geo)
    from uam_path_planning_amd.synthetic import synthetic_dem

    spec = canonical_spec()
    eng.set_geometry(compile_map(build_region_map(spec)))
    eng.set_params(canonical_params(spec))
    geo = raster_geo(256)
    src = synthetic_dem(512, seed=9)
    gg = GeoGridDesc(512, 512, 129.5, 33.25, 0.0015, 0.0015, -9999.0, 0)
    dem = eng.reproject_dem(src, gg, geo)
    rec = eng.raster_build(geo, dem).rec.cpu().numpy().view(np.float32)
    orc = oracle_mod.Oracle(oracle_mod.compile_spec(spec), spec["N"], spec["options"],
                            spec["maxratio"], spec["maxalpha"], spec["enlargement"],
                            spec["weights"])
    rd = orc.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy)
    odem = oracle_mod.reproject(src, oracle_mod.geo_grid(512, 512, 129.5, 33.25, 0.0015,
                                                         0.0015), rd)
    np.testing.assert_array_equal(dem.cpu().numpy(), odem)
    np.testing.assert_array_equal(rec.reshape(orc.raster_build(rd, odem).shape),
                                  orc.raster_build(rd, odem))


def _rings(z, meta, name):
    si = list(z["names"]).index(name)
    sel = z["set"] == si
    return ([z["plane_xy"][sel][z["ring"][sel] == r] for r in range(meta[name]["records"])],
            [z["lonlat"][sel][z["ring"][sel] == r] for r in range(meta[name]["records"])])


def test_export_no_fly_zone_and_polygons_match_reference_files(eng, crs, tmp_path):
    from uam_path_planning_amd.geo import export, shapefile as S

    z, meta = crs
    p = export.make_no_fly_zone_shp(str(tmp_path / "nfz" / "no_fly_zone.shp"), engine=eng)
    kind, geoms = S.read_shapefile(p)
    _, ref = _rings(z, meta, "nfz")
    assert kind == S.POLYGON and [len(g[0]) for g in geoms] == meta["nfz"]["vertices"]
    for g, r in zip(geoms, ref):
        assert np.abs(g[0] - r).max() <= 5e-14
    for name in ("land", "populated"):
        plane, ref = _rings(z, meta, name)
        # open rings; odd ones counter-clockwise with the same first vertex (the writer must
        # restore the ESRI orientation the reference files have)
        src = [pl[::-1][:-1] if i % 2 else pl[:-1] for i, pl in enumerate(plane)]
        p = export.save_polygons_to_shapefile(src, str(tmp_path / name / f"{name}.shp"),
                                              engine=eng)
        kind, geoms = S.read_shapefile(p)
        assert [len(g[0]) for g in geoms] == meta[name]["vertices"]
        for g, r in zip(geoms, ref):
            assert np.abs(g[0] - r).max() <= 5e-14
        assert open(p[:-4] + ".prj").read() == meta[name]["prj"]


def test_export_result_line_and_points(eng, oracle_mod, tmp_path):
    """main.py:103-116 on the canonical straight candidate; batched export of all 5."""
    import golden_io as G
    from uam_path_planning_amd.geo import export, shapefile as S

    meta, arr = G.canonical()
    x = arr["x_init"][2]
    p = export.make_result_line_shp(x, str(tmp_path / "line1.shp"), engine=eng)
    kind, geoms = S.read_shapefile(p)
    pts_m = export._path_points(x, export.START_POINT, export.END_POINT)
    assert kind == S.POLYLINE and len(geoms) == 1 and len(geoms[0][0]) == meta["N"] + 2
    assert np.abs(geoms[0][0] - oracle_mod.tm_inv(pts_m)).max() <= 2e-14
    p = export.save_points_to_shp(x, str(tmp_path / "line1_points.shp"), engine=eng)
    kind, geoms = S.read_shapefile(p)
    assert kind == S.POINT and len(geoms) == meta["N"] + 2
    wp = G.canonical_paths(meta, arr)
    p = export.export_paths(wp, str(tmp_path / "all.shp"), engine=eng)
    kind, geoms = S.read_shapefile(p)
    assert len(geoms) == 5
    for g, w in zip(geoms, wp):
        assert np.abs(g[0] - oracle_mod.tm_inv(w * 1000.0)).max() <= 2e-14


def test_load_dem_geographic_from_vrt_tiles(eng, oracle_mod, tmp_path):
    """VRT of Float32 GeoTIFF tiles in lon/lat (the mergeLL.vrt layout) -> device mosaic ->
    reprojection onto the plane grid == oracle reprojection of the same mosaic."""
    from uam_path_planning_amd.map_generation import DataManager
    from uam_path_planning_amd.map_generation.vrt import write_tiled_dem
    from uam_path_planning_amd.scenario import raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    src = synthetic_dem(600, seed=13)
    d = 5.5555555555554013e-05 * 10
    gt = (129.5, d, 0.0, 33.25, 0.0, -d)
    vrt = write_tiled_dem(src, gt, str(tmp_path / "tiles"), tile_w=225, tile_h=150)
    geo = raster_geo(256)
    dem, _ = DataManager(eng).load_dem_geographic(vrt, geo)
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy)
    ref = oracle_mod.reproject(src, oracle_mod.geo_grid(600, 600, 129.5, 33.25, d, d), rd)
    np.testing.assert_array_equal(dem.cpu().numpy(), ref)
