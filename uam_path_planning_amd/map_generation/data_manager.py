"""DEM ingest and cost-raster build -- the hot-path part of the reference's
map_generation/data_manager.py (DataManager, 8-86).

* ``load_dem(path)``: a single GeoTIFF or a VRT tile mosaic (mergeLL.vrt layout); VRT tiles are
  placed by the device mosaic kernel.
* ``load_dem_mask(path, threshold_dem)``: the mask of load_dem_polygons_from_geotiff
  (data_manager.py:14-17): ``dem == -9999`` when threshold_dem == -9999, else ``dem > thr``,
  computed on the GPU as the MASK flag bit of the cost-raster build (K1).
* ``build_cost_raster(...)``: DEM -> device record raster {Φ, Σψ_nfz, dem, flags} (K1).
* ``load_dem_geographic(vrt, dst_geo)``: the full-scale ingest of SURVEY §8(f) rank 3 -- a
  lat/lon tile mosaic (mergeLL.vrt: JGD2011, 0.2" pixels, mergeLL.vrt:1-3) placed on the
  device (K0) and reprojected onto the plane cost-raster grid (K7, EPSG:2443 via the TM
  transform the reference delegates to pyproj, data_manager.py:24-26).
* ``save_polygons(vertex_lists, path)``: the D1 text format of data_manager.py:56-81
  (coordinates / 1000, m -> km), readable by path_generation.utils.get_var_from_file.
Shapefile output: ``uam_path_planning_amd.geo.export`` (save_polygons_to_shapefile).
"""
from ..engine import RasterGeo, default_engine
from .geotiff import read_geotiff
from .vrt import load_tiles, read_vrt, tile_layout


def geo_from_geotransform(width, height, gt, nodata=-9999.0, dem_threshold=0.0):
    x0, dx, rx, ytop, ry, ndy = gt
    if rx != 0 or ry != 0:
        raise ValueError("rotated geotransforms are not supported")
    if not (dx > 0 and ndy < 0):
        raise ValueError("expected north-up rasters (dx > 0, dy < 0)")
    return RasterGeo(nx=int(width), ny=int(height), x0=float(x0), y_top=float(ytop),
                     dx=float(dx), dy=float(-ndy), nodata=float(nodata),
                     dem_threshold=float(dem_threshold))


class DemRegions:
    """The DEM mask regions of load_dem_polygons_from_geotiff, kept on the device: the
    4-connected regions of (dem == -9999 if threshold == -9999 else dem > threshold)
    (data_manager.py:11-19).  DataProcessor.process_polygons labels and approximates them on
    the GPU (uam_dem_polygons)."""

    def __init__(self, engine, dem, geo, threshold, unit_m=1000.0):
        self.engine, self.dem, self.geo = engine, dem, geo
        self.threshold, self.unit_m = float(threshold), float(unit_m)


class DataManager:
    def __init__(self, engine=None):
        self._engine = engine

    @property
    def engine(self):
        return self._engine if self._engine is not None else default_engine()

    def load_dem(self, input_file, dem_threshold=0.0, n_threads=0):
        """-> (dem device tensor [ny][nx] float32, RasterGeo).  A VRT's tiles are read by the
        native parallel reader (n_threads host threads; 0 = up to 16) in chunks through the
        context's page-locked buffers, each chunk copied to the device while the next is read
        (uam_load_tiles; pageable reads and copies took 18-43 ms + 11-15 ms for cfg4's 2 035
        tiles against 9 + 5 ms page-locked, profiles/r03/ingest), then placed by the mosaic
        kernel (uam_dem_mosaic)."""
        eng = self.engine
        if input_file.lower().endswith(".vrt"):
            v = read_vrt(input_file)
            nod = -9999.0 if v.nodata is None else v.nodata
            paths, th, tw, xo, yo = tile_layout(v)
            tiles = eng.load_tiles(paths, th, tw, n_threads=n_threads)
            dem = eng.dem_mosaic(tiles, xo, yo, v.width, v.height, fill=nod)
            return dem, geo_from_geotransform(v.width, v.height, v.geotransform, nod,
                                              dem_threshold)
        data, gt, nod = read_geotiff(input_file)
        nod = -9999.0 if nod is None else nod
        import torch

        dem = eng.tensor(data, torch.float32)
        gt = gt or (0.0, 1.0, 0.0, float(data.shape[0]), 0.0, -1.0)
        return dem, geo_from_geotransform(data.shape[1], data.shape[0], gt, nod, dem_threshold)

    def load_dem_geographic(self, input_file, dst_geo, resample=0, zone=1, unit_m=1000.0):
        """Geographic (lon/lat) DEM mosaic -> plane DEM on ``dst_geo`` (RasterGeo in units of
        unit_m metres, JPRCS zone): device mosaic (K0) + reprojection (K7)."""
        from .._lib import GeoGridDesc

        eng = self.engine
        if input_file.lower().endswith(".vrt"):
            v = read_vrt(input_file)
            nod = -9999.0 if v.nodata is None else v.nodata
            tiles, xo, yo = load_tiles(v)
            src = eng.dem_mosaic(tiles, xo, yo, v.width, v.height, fill=nod)
            gt, w, h = v.geotransform, v.width, v.height
        else:
            data, gt, nod = read_geotiff(input_file)
            nod = -9999.0 if nod is None else nod
            import torch

            src = eng.tensor(data, torch.float32)
            h, w = data.shape
        lon0, dlon, rx, lat_top, ry, ndlat = gt
        if rx != 0 or ry != 0 or not (dlon > 0 and ndlat < 0):
            raise ValueError("expected a north-up geographic grid")
        grid = GeoGridDesc(int(w), int(h), float(lon0), float(lat_top), float(dlon),
                           float(-ndlat), float(nod), 0)
        dem = eng.reproject_dem(src, grid, dst_geo, unit_m, resample, zone)
        return dem, dst_geo

    def build_cost_raster(self, input_file, geometry, params, dem_threshold=0.0):
        eng = self.engine
        dem, geo = self.load_dem(input_file, dem_threshold)
        eng.set_geometry(geometry)
        eng.set_params(params)
        return eng.raster_build(geo, dem)

    def load_polygons_from_shapefile(self, input_file, src_epsg=4612, dst_epsg=2443):
        """data_manager.py:21-27: polygons of a shapefile in EPSG:4612 -> EPSG:2443 metres
        (GPU transform, K7).  -> list of (shell [n, 2], [holes]) with the ESRI ring roles
        (clockwise = shell, counter-clockwise = hole)."""
        import numpy as np

        from ..geo.crs import to_crs
        from ..geo.shapefile import POLYGON, read_shapefile

        kind, geoms = read_shapefile(input_file)
        if kind != POLYGON:
            raise ValueError(f"{input_file}: shape type {kind} is not Polygon")
        rings = [r for g in geoms if g for r in g]
        if not rings:
            return []
        flat = to_crs(np.vstack(rings), src_epsg, dst_epsg, self.engine)
        out, o = [], 0
        for g in geoms:
            if not g:
                continue
            for r in g:
                xy = flat[o:o + len(r)]
                o += len(r)
                x, y = r[:, 0], r[:, 1]
                if 0.5 * np.sum(x[:-1] * y[1:] - x[1:] * y[:-1]) > 0 and out:   # hole
                    out[-1][1].append(xy)
                else:
                    out.append((xy, []))
        return out

    def load_dem_polygons(self, dem, geo, threshold_dem=0, unit_m=1000.0):
        """Regions of an already-loaded DEM (device or host array on RasterGeo geo)."""
        return DemRegions(self.engine, dem, geo, threshold_dem, unit_m)

    def load_dem_mask(self, input_file, threshold_dem=0):
        """Boolean mask [rows][cols] of data_manager.py:14-17, evaluated on the GPU (K1)."""
        from ..engine import Engine, PathParams
        from ..geometry import compile_shapes

        eng = Engine(self.engine.device)
        dem, geo = DataManager(eng).load_dem(input_file, float(threshold_dem))
        eng.set_geometry(compile_shapes((), []))
        eng.set_params(PathParams(N=1))
        rec = eng.raster_build(geo, dem, summary=False, packed=False).rec  # only the flags
        return ((rec[..., 3] & 2) != 0).cpu().numpy()

    def load_dem_polygons_from_geotiff(self, input_file, threshold_dem=0):
        """data_manager.py:11-19: the mask regions of the DEM (plane raster, metres via the
        file's geotransform scale) as DemRegions for DataProcessor.process_polygons."""
        dem, geo = self.load_dem(input_file)
        return DemRegions(self.engine, dem, geo, threshold_dem, unit_m=1.0)

    @staticmethod
    def save_polygons(polygons, output_file):
        """polygons: list of vertex lists [[x, y], ...] in metres (closing vertex optional)."""
        with open(output_file, "w") as f:
            f.write("vertices = [")
            for i, pts in enumerate(polygons):
                pts = [tuple(p) for p in pts]
                if len(pts) > 1 and pts[0] == pts[-1]:
                    pts = pts[:-1]
                body = ", ".join("[" + str(x / 1000) + ", " + str(y / 1000) + "]"
                                 for x, y in pts)
                f.write("polygon(" + body + (")\n" if i == len(polygons) - 1 else "),\n"))
            f.write("]")

