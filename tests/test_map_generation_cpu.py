"""GeoTIFF / VRT tile IO (host side of the DEM ingest) and the D1 text writer."""
import numpy as np
import pytest


@pytest.mark.parametrize("deflate", [False, True])
def test_geotiff_roundtrip(tmp_path, deflate):
    from uam_path_planning_amd.map_generation import read_geotiff, write_geotiff

    rng = np.random.default_rng(0)
    a = rng.normal(100, 50, size=(150, 225)).astype(np.float32)
    a[3, 7] = -9999.0
    gt = (12.5, 0.0146484375, 0.0, 20.0, 0.0, -0.0146484375)
    p = tmp_path / "t.tif"
    write_geotiff(str(p), a, gt, deflate=deflate)
    b, gt2, nod = read_geotiff(str(p))
    np.testing.assert_array_equal(a, b)
    assert gt2 == gt and nod == -9999.0


def test_vrt_tiles_roundtrip(tmp_path):
    from uam_path_planning_amd.map_generation import load_tiles, read_vrt, write_tiled_dem
    from uam_path_planning_amd.synthetic import synthetic_dem

    dem = synthetic_dem(256)[:300 - 44, :500 - 260 + 16]   # non-multiple of the tile size
    gt = (0.0, 60 / 256, 0.0, 20.0, 0.0, -60 / 256)
    path = write_tiled_dem(dem, gt, str(tmp_path / "tiles"))
    v = read_vrt(path)
    assert (v.width, v.height) == (dem.shape[1], dem.shape[0])
    assert v.geotransform == gt and v.nodata == -9999.0
    tiles, xo, yo = load_tiles(v)
    assert tiles.shape[1:] == (150, 225)
    # place on the host (the device does this in k_dem_mosaic) and compare
    out = np.full(dem.shape, -9999.0, np.float32)
    for t, x, y in zip(tiles, xo, yo):
        h = min(150, dem.shape[0] - y)
        w = min(225, dem.shape[1] - x)
        out[y:y + h, x:x + w] = t[:h, :w]
    np.testing.assert_array_equal(out, dem)


def test_save_polygons_roundtrip(tmp_path):
    from uam_path_planning_amd.map_generation import DataManager
    from uam_path_planning_amd.path_generation.utils import parse_shapes_text

    polys = [[(1000.0, 2000.0), (3000.0, 2000.0), (2500.0, 4000.0), (1000.0, 2000.0)],
             [(0.0, 0.0), (500.0, 0.0), (500.0, 500.0), (0.0, 500.0)]]
    p = tmp_path / "area.txt"
    DataManager.save_polygons(polys, str(p))
    parsed = parse_shapes_text(p.read_text())["vertices"]
    assert [k for k, _, _ in parsed] == ["polygon", "polygon"]
    assert parsed[0][1] == [[1.0, 2.0], [3.0, 2.0], [2.5, 4.0]]
    assert parsed[1][1][2] == [0.5, 0.5]


@pytest.mark.parametrize("deflate", [False, True])
def test_native_tile_reader_matches_python(tmp_path, deflate):
    """uam_read_tiles (host C++, parallel) reads the same pixels as the Python GeoTIFF reader
    over a VRT tile set (225 x 150 tiles, strips of 9 rows, edge tiles padded with nodata),
    uncompressed and deflate, with 1 and 8 threads; a truncated tile and a tile of the wrong
    size fail the call with the tile's path in uam_last_error."""
    import ctypes
    import os

    from uam_path_planning_amd import _lib, build
    from uam_path_planning_amd.map_generation.vrt import (load_tiles, read_vrt, tile_layout,
                                                          write_tiled_dem)

    build.build_library()
    lib = _lib.load()
    dem = np.random.default_rng(5).standard_normal((400, 700)).astype(np.float32)
    dem[::13, ::7] = -9999.0
    v = read_vrt(write_tiled_dem(dem, (0.0, 1.0, 0.0, 0.0, 0.0, -1.0), str(tmp_path),
                                 deflate=deflate))
    paths, th, tw, xo, yo = tile_layout(v)
    ref, rxo, ryo = load_tiles(v)
    np.testing.assert_array_equal(xo, rxo)
    np.testing.assert_array_equal(yo, ryo)
    arr = (ctypes.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
    for threads in (1, 8):
        out = np.full((len(paths), th, tw), np.nan, np.float32)
        assert lib.uam_read_tiles(arr, len(paths), th, tw,
                                  out.ctypes.data_as(ctypes.c_void_p), threads) == 0
        np.testing.assert_array_equal(out.view(np.int32), ref.view(np.int32))
    # a truncated tile, then a size mismatch: UAM_E_INVALID naming the file
    with open(paths[3], "rb") as f:
        head = f.read(200)
    with open(paths[3], "wb") as f:
        f.write(head)
    out = np.empty((len(paths), th, tw), np.float32)
    assert lib.uam_read_tiles(arr, len(paths), th, tw, out.ctypes.data_as(ctypes.c_void_p),
                              4) == _lib.UAM_E_INVALID
    assert os.path.basename(paths[3]) in lib.uam_last_error().decode()
    assert lib.uam_read_tiles(arr, 2, th + 1, tw, out.ctypes.data_as(ctypes.c_void_p),
                              1) == _lib.UAM_E_INVALID
    assert "size" in lib.uam_last_error().decode()
