"""GDAL VRT tile mosaics (the reference DEM is data/raw/nagasaki_geotiff/mergeLL.vrt:1-10:
18225 x 14250 Float32, one <ComplexSource> per 225 x 150 tile with a <DstRect>, nodata -9999).

read_vrt() parses the XML; load_tiles() reads every source tile (geotiff.read_geotiff) into one
[T][th][tw] stack with per-tile destination offsets, which the device mosaic kernel
(uam_dem_mosaic) places into the DEM plane.  write_tiled_dem() writes a DEM as such a tile set
+ VRT (used for the synthetic stand-in of the absent real tiles)."""
import gc
import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

from .geotiff import read_geotiff, write_geotiff


@dataclass
class VrtSource:
    filename: str
    src: tuple      # xOff, yOff, xSize, ySize
    dst: tuple
    nodata: float = None


@dataclass
class Vrt:
    width: int
    height: int
    geotransform: tuple
    nodata: float
    sources: list = field(default_factory=list)


def read_vrt(path):
    # a mosaic VRT holds thousands of sources: the cyclic collector adds 50 ms at random
    # points of the parse (profiles/r03/ingest), so it is paused for it
    gc_was = gc.isenabled()
    gc.disable()
    try:
        return _read_vrt(path)
    finally:
        if gc_was:
            gc.enable()


def _read_vrt(path):
    root = ET.parse(path).getroot()
    w, h = int(root.get("rasterXSize")), int(root.get("rasterYSize"))
    gt_el = root.find("GeoTransform")
    gt = tuple(float(v) for v in gt_el.text.replace(",", " ").split()) if gt_el is not None \
        else (0.0, 1.0, 0.0, 0.0, 0.0, -1.0)
    band = root.find("VRTRasterBand")
    if band is None or band.get("dataType", "Float32") != "Float32":
        raise ValueError("only one Float32 band is supported")
    nd_el = band.find("NoDataValue")
    nodata = float(nd_el.text) if nd_el is not None else None
    base = os.path.dirname(os.path.abspath(path))
    srcs = []
    for s in list(band.findall("ComplexSource")) + list(band.findall("SimpleSource")):
        fn_el = s.find("SourceFilename")
        fn = fn_el.text
        if fn_el.get("relativeToVRT", "0") == "1":
            fn = os.path.join(base, fn)

        def rect(tag):
            r = s.find(tag)
            return tuple(int(float(r.get(k))) for k in ("xOff", "yOff", "xSize", "ySize"))

        nd = s.find("NODATA")
        srcs.append(VrtSource(fn, rect("SrcRect"), rect("DstRect"),
                              float(nd.text) if nd is not None else None))
    return Vrt(w, h, gt, nodata, srcs)


def tile_layout(vrt):
    """-> (paths, th, tw, xoff [T] int32, yoff [T] int32) after the checks load_tiles makes on
    the VRT (equal-sized tiles, each whole source tile placed 1:1 at its DstRect)."""
    paths, xo, yo, shape = [], [], [], None
    for s in vrt.sources:
        if s.src[2:] != s.dst[2:] or s.src[:2] != (0, 0):
            raise ValueError(f"{s.filename}: resampling / partial SrcRect not supported")
        if shape is None:
            shape = (s.src[3], s.src[2])
        elif (s.src[3], s.src[2]) != shape:
            raise ValueError("tiles of different sizes")
        paths.append(s.filename)
        xo.append(s.dst[0])
        yo.append(s.dst[1])
    th, tw = shape if shape else (1, 1)
    return paths, th, tw, np.asarray(xo, np.int32), np.asarray(yo, np.int32)


def load_tiles(vrt):
    """-> tiles [T][th][tw] float32, xoff [T] int32, yoff [T] int32 (tiles equal-sized, whole
    source tile placed 1:1 at its DstRect -- the layout of the reference mosaic)."""
    tiles, xo, yo = [], [], []
    shape = None
    for s in vrt.sources:
        if s.src[2:] != s.dst[2:] or s.src[:2] != (0, 0):
            raise ValueError(f"{s.filename}: resampling / partial SrcRect not supported")
        data, _, _ = read_geotiff(s.filename)
        if data.shape != (s.src[3], s.src[2]):
            raise ValueError(f"{s.filename}: size {data.shape} != SrcRect {s.src}")
        if shape is None:
            shape = data.shape
        elif data.shape != shape:
            raise ValueError("tiles of different sizes")
        tiles.append(data)
        xo.append(s.dst[0])
        yo.append(s.dst[1])
    if not tiles:
        return np.zeros((0, 1, 1), np.float32), np.zeros(0, np.int32), np.zeros(0, np.int32)
    return np.stack(tiles), np.asarray(xo, np.int32), np.asarray(yo, np.int32)


def write_tiled_dem(dem, geotransform, out_dir, tile_w=225, tile_h=150, nodata=-9999.0,
                    name="mosaic.vrt", deflate=False):
    """Split dem [H][W] into tile_w x tile_h GeoTIFF tiles (strips of 9 rows) + a VRT.
    Edge tiles are padded with nodata (the VRT DstRect then hangs over the edge, as GDAL
    allows; the mosaic kernel clips)."""
    os.makedirs(out_dir, exist_ok=True)
    H, W = dem.shape
    x0, dx, _, ytop, _, ndy = geotransform
    root = ET.Element("VRTDataset", rasterXSize=str(W), rasterYSize=str(H))
    ET.SubElement(root, "GeoTransform").text = ", ".join(repr(float(v)) for v in geotransform)
    band = ET.SubElement(root, "VRTRasterBand", dataType="Float32", band="1")
    ET.SubElement(band, "NoDataValue").text = str(int(nodata)) if nodata == int(nodata) \
        else repr(nodata)
    k = 0
    for ty in range(0, H, tile_h):
        for tx in range(0, W, tile_w):
            t = np.full((tile_h, tile_w), nodata, np.float32)
            blk = dem[ty:ty + tile_h, tx:tx + tile_w]
            t[:blk.shape[0], :blk.shape[1]] = blk
            fn = f"tile_{k:05d}.tif"
            tgt = (x0 + tx * dx, dx, 0.0, ytop + ty * ndy, 0.0, ndy)
            write_geotiff(os.path.join(out_dir, fn), t, tgt, nodata=nodata, deflate=deflate)
            cs = ET.SubElement(band, "ComplexSource")
            ET.SubElement(cs, "SourceFilename", relativeToVRT="1").text = fn
            ET.SubElement(cs, "SourceBand").text = "1"
            ET.SubElement(cs, "SourceProperties", RasterXSize=str(tile_w),
                          RasterYSize=str(tile_h), DataType="Float32", BlockXSize=str(tile_w),
                          BlockYSize="9")
            ET.SubElement(cs, "SrcRect", xOff="0", yOff="0", xSize=str(tile_w),
                          ySize=str(tile_h))
            ET.SubElement(cs, "DstRect", xOff=str(tx), yOff=str(ty), xSize=str(tile_w),
                          ySize=str(tile_h))
            ET.SubElement(cs, "NODATA").text = str(int(nodata))
            k += 1
    path = os.path.join(out_dir, name)
    ET.ElementTree(root).write(path)
    return path
