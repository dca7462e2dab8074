"""Coordinate reference systems and GIS output.

* ``crs``: EPSG:4612 / 6668 (JGD2000 / JGD2011 lon-lat) <-> EPSG:2443..2461 (Japan Plane
  Rectangular CS, metres) on the GPU (uam_geo_to_plane / uam_plane_to_geo), and the DEM
  reprojection of the lat/lon tile mosaic onto the plane cost-raster grid (uam_reproject_dem).
* ``shapefile``: ESRI shapefile reader/writer (.shp/.shx/.dbf/.prj/.cpg) in the layout the
  reference's geopandas/OGR writes.
* ``export``: the reference's result and map exports (path_generation/main.py:103-116,
  map_generation/data_manager.py:83-86, map_generation/utils.py:81-111).
"""
from .crs import GEOGRAPHIC_EPSG, PLANE_EPSG, geo_to_plane, plane_to_geo, to_crs
from .shapefile import read_shapefile, write_shapefile

__all__ = ["GEOGRAPHIC_EPSG", "PLANE_EPSG", "geo_to_plane", "plane_to_geo", "to_crs",
           "read_shapefile", "write_shapefile"]
