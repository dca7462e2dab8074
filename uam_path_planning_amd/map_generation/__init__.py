"""DEM / GeoTIFF-tile ingest and the cost-raster build (hot-path part of the reference's
map_generation; see data_manager.py)."""
from .data_manager import DataManager, geo_from_geotransform
from .geotiff import read_geotiff, write_geotiff
from .vrt import load_tiles, read_vrt, write_tiled_dem

__all__ = ["DataManager", "geo_from_geotransform", "read_geotiff", "write_geotiff",
           "read_vrt", "load_tiles", "write_tiled_dem"]
