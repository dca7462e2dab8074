"""GPU land polygons (K8, uam_dem_polygons) against the oracle
(orc_dem_polygons): rectangles and their order bit-exact (integer metres).  The oracle is pinned
through test_polygons_cpu.py (its cv2 restatement on the reference's populated_area output, and
the DEM route == the vector route on exact polygons)."""
import numpy as np
import pytest

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


def _arr(rects):
    return np.asarray(rects, np.int64).reshape(-1, 4, 2)


@pytest.mark.parametrize("R,thr", [(512, 0.0), (1024, 0.0), (1024, 250.0), (1024, -9999.0)])
def test_dem_polygons_vs_oracle(eng, oracle_mod, R, thr):
    from uam_path_planning_amd.scenario import raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    geo = raster_geo(R)
    dem = synthetic_dem(R, seed=3)
    got = _arr(eng.dem_polygons(dem, geo, thr))
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy)
    ref = oracle_mod.dem_polygons(dem, rd, thr, 1000.0)
    assert len(ref) > 0
    np.testing.assert_array_equal(got, ref)


def test_dem_polygons_islands_and_dataprocessor(eng, oracle_mod, tmp_path):
    """The hand-built islands of test_polygons_cpu (divided L with a lake, small island,
    dropped islet) through DataManager / DataProcessor with the reference's call pattern
    (map_generation/main.py:27-35), from a GeoTIFF in metres."""
    import test_polygons_cpu as T
    from uam_path_planning_amd.map_generation import DataManager, write_geotiff
    from uam_path_planning_amd.map_generation.data_processor import DataProcessor

    dem = T._island_raster()
    gt = (T.X0_KM * 1000, T.DX_KM * 1000, 0.0, T.YTOP_KM * 1000, 0.0, -T.DX_KM * 1000)
    tif = str(tmp_path / "merge_test.tif")
    write_geotiff(tif, dem, gt)
    dm = DataManager(eng)
    polygons = dm.load_dem_polygons_from_geotiff(tif, 0)
    got = DataProcessor().process_polygons(polygons)
    rd = oracle_mod.Oracle.raster_desc(200, 200, T.X0_KM, T.YTOP_KM, T.DX_KM, T.DX_KM)
    np.testing.assert_array_equal(_arr(got), oracle_mod.dem_polygons(dem, rd, 0.0, 1000.0))
    vec = DataProcessor().process_polygons(T._island_polygons())
    assert T.as_multiset(got) == T.as_multiset(vec)
    path = str(tmp_path / "land_area.txt")
    dm.save_polygons([r for r in got], path)
    from uam_path_planning_amd.path_generation import utils as ut

    loaded = ut.get_var_from_file(path, "vertices")
    assert len(loaded) == len(got)


def test_dem_polygons_edge_cases(eng, oracle_mod):
    from uam_path_planning_amd.scenario import raster_geo

    geo = raster_geo(64)
    assert eng.dem_polygons(np.full((64, 64), -9999.0, np.float32), geo, 0.0) == []
    full = np.full((64, 64), 10.0, np.float32)          # one region = the whole raster
    got = _arr(eng.dem_polygons(full, geo, 0.0))
    rd = oracle_mod.Oracle.raster_desc(64, 64, geo.x0, geo.y_top, geo.dx, geo.dy)
    np.testing.assert_array_equal(got, oracle_mod.dem_polygons(full, rd, 0.0, 1000.0))
    assert len(got) == 25                               # 3600 km^2 -> divided into 5 x 5
    with pytest.raises(ValueError):
        eng.dem_polygons(full[:10], geo, 0.0)


def test_population_pipeline_reproduces_reference(eng, tmp_path):
    """map_generation/main.py:17-24 (process_population) end to end on the GPU transform:
    DID shapefile (EPSG:4612) -> load_polygons_from_shapefile (K7) -> process_polygons ->
    the reference's data/processed/populated_area.txt rectangles (tests/golden/polygons.npz):
    all 29 corner sets exact."""
    import os

    from conftest import GOLDEN
    from uam_path_planning_amd.geo.shapefile import POLYGON, write_shapefile
    from uam_path_planning_amd.map_generation import DataManager
    from uam_path_planning_amd.map_generation.data_processor import DataProcessor

    z = np.load(os.path.join(GOLDEN, "polygons.npz"))
    recs = []
    for r in range(len(z["ring_hole"])):
        ring = z["lonlat"][z["ring_start"][r]:z["ring_start"][r + 1]]
        if z["ring_hole"][r]:
            recs[-1].append(ring)
        else:
            recs.append([ring])
    shp = write_shapefile(str(tmp_path / "populated_area.shp"), recs, POLYGON)
    dm = DataManager(eng)
    polys = dm.load_polygons_from_shapefile(shp)
    got = DataProcessor().process_polygons(polys)
    sets = lambda rs: sorted(sorted(map(tuple, np.asarray(r).tolist())) for r in rs)
    assert sets(got) == sets(z["rects"])


@pytest.mark.parametrize("tiled", ["1", "0"])
@pytest.mark.parametrize("nx,ny,thr", [(700, 450, 0.0), (129, 1000, 150.0), (1000, 63, 0.0)])
def test_dem_polygons_tile_edges(oracle_mod, monkeypatch, tiled, nx, ny, thr):
    """Tile labelling (UAM_OPT_K8_TILED = 1, the default: 64 x 64 LDS tiles + edge joins) and the
    cell-parallel merge (0) on rasters that are not multiples of the tile: partial tiles on
    both edges, a single tile row, components crossing many tile edges, large regions split
    into box pieces (cuts inside and across tiles)."""
    from uam_path_planning_amd.engine import Engine, RasterGeo
    from uam_path_planning_amd.synthetic import synthetic_dem

    e2 = Engine(0)
    e2.set_option("k8_tiled", int(tiled))
    dx = 60.0 / max(nx, ny)
    geo = RasterGeo(nx=nx, ny=ny, x0=0.0, y_top=20.0, dx=dx, dy=dx, nodata=-9999.0,
                    dem_threshold=thr)
    dem = synthetic_dem(max(nx, ny), seed=3)[:ny, :nx].copy()
    got = _arr(e2.dem_polygons(dem, geo, thr))
    rd = oracle_mod.Oracle.raster_desc(nx, ny, geo.x0, geo.y_top, dx, dx)
    ref = oracle_mod.dem_polygons(dem, rd, thr, 1000.0)
    assert len(ref) > 0
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("streams", ["1", "2", "8"])
def test_dem_polygons_region_streams(oracle_mod, monkeypatch, streams):
    """The large regions spread over 1, 2 or 8 streams (UAM_OPT_K8_STREAMS; default 4): same
    rectangles in the same order as the oracle."""
    from uam_path_planning_amd.engine import Engine
    from uam_path_planning_amd.scenario import raster_geo
    from uam_path_planning_amd.synthetic import synthetic_dem

    e2 = Engine(0)
    e2.set_option("k8_streams", int(streams))
    geo = raster_geo(1024)
    dem = synthetic_dem(1024, seed=5)
    got = _arr(e2.dem_polygons(dem, geo, 0.0))
    rd = oracle_mod.Oracle.raster_desc(geo.nx, geo.ny, geo.x0, geo.y_top, geo.dx, geo.dy)
    ref = oracle_mod.dem_polygons(dem, rd, 0.0, 1000.0)
    assert len(ref) > 25  # several large regions
    np.testing.assert_array_equal(got, ref)
