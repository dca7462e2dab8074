"""Minimal single-band Float32 GeoTIFF reader/writer (no GDAL: rasterio 1.3.9 / GDAL 3.6.2 of
the reference, requirements.txt:31,13, are not installed).

Covers what the DEM path needs: the reference's tiles are 225 x 150 Float32 GeoTIFFs stored in
strips of 9 rows (data/raw/nagasaki_geotiff/mergeLL.vrt: BlockXSize=225, BlockYSize=9) with
nodata -9999.  Strips may be uncompressed (1) or Deflate (8 / 32946), horizontal predictor 1.
Georeferencing: ModelPixelScale (33550) + ModelTiepoint (33922) -> GDAL-style geotransform
(x0, dx, 0, y_top, 0, -dy); GDAL_NODATA (42113)."""
import struct
import zlib

import numpy as np

_TYPES = {1: ("B", 1), 2: ("s", 1), 3: ("H", 2), 4: ("I", 4), 12: ("d", 8), 16: ("Q", 8)}

T_WIDTH, T_LENGTH, T_BPS, T_COMPRESSION, T_PHOTOMETRIC = 256, 257, 258, 259, 262
T_STRIP_OFFSETS, T_SPP, T_ROWS_PER_STRIP, T_STRIP_BYTES = 273, 277, 278, 279
T_PLANAR, T_PREDICTOR, T_SAMPLE_FORMAT = 284, 317, 339
T_PIXEL_SCALE, T_TIEPOINT, T_NODATA = 33550, 33922, 42113


def write_geotiff(path, data, geotransform, nodata=-9999.0, rows_per_strip=9, deflate=False):
    """data: 2-D float32 array [rows][cols], row 0 north.  geotransform: (x0, dx, 0, y_top,
    0, -dy) (GDAL order)."""
    a = np.ascontiguousarray(data, dtype="<f4")
    h, w = a.shape
    strips = []
    for r0 in range(0, h, rows_per_strip):
        raw = a[r0:r0 + rows_per_strip].tobytes()
        strips.append(zlib.compress(raw, 6) if deflate else raw)
    x0, dx, _, ytop, _, ndy = geotransform
    nod = (repr(float(nodata)) if float(nodata) != int(nodata) else str(int(nodata))).encode()
    nod += b"\0"
    entries = []   # (tag, type, count, payload bytes)

    def add(tag, typ, vals):
        fmt, size = _TYPES[typ]
        if typ == 2:
            payload = vals
            count = len(vals)
        else:
            payload = struct.pack("<" + fmt * len(vals), *vals)
            count = len(vals)
        entries.append((tag, typ, count, payload))

    n = len(strips)
    add(T_WIDTH, 4, [w])
    add(T_LENGTH, 4, [h])
    add(T_BPS, 3, [32])
    add(T_COMPRESSION, 3, [8 if deflate else 1])
    add(T_PHOTOMETRIC, 3, [1])
    add(T_STRIP_OFFSETS, 4, [0] * n)          # patched below
    add(T_SPP, 3, [1])
    add(T_ROWS_PER_STRIP, 4, [rows_per_strip])
    add(T_STRIP_BYTES, 4, [len(s) for s in strips])
    add(T_PLANAR, 3, [1])
    add(T_SAMPLE_FORMAT, 3, [3])
    add(T_PIXEL_SCALE, 12, [float(dx), float(-ndy), 0.0])
    add(T_TIEPOINT, 12, [0.0, 0.0, 0.0, float(x0), float(ytop), 0.0])
    add(T_NODATA, 2, nod)
    entries.sort(key=lambda e: e[0])
    ifd_off = 8
    ifd_size = 2 + 12 * len(entries) + 4
    extra_off = ifd_off + ifd_size
    extra = bytearray()
    slots = []
    for tag, typ, count, payload in entries:
        if len(payload) <= 4:
            slots.append(payload.ljust(4, b"\0"))
        else:
            slots.append(struct.pack("<I", extra_off + len(extra)))
            extra += payload
            if len(extra) % 2:
                extra += b"\0"
    data_off = extra_off + len(extra)
    offsets, o = [], data_off
    for s in strips:
        offsets.append(o)
        o += len(s)
    # patch strip offsets payload
    for i, (tag, typ, count, payload) in enumerate(entries):
        if tag == T_STRIP_OFFSETS:
            newp = struct.pack("<" + "I" * n, *offsets)
            if len(newp) <= 4:
                slots[i] = newp.ljust(4, b"\0")
            else:
                pos = struct.unpack("<I", slots[i])[0] - extra_off
                extra[pos:pos + len(newp)] = newp
    with open(path, "wb") as f:
        f.write(b"II*\0" + struct.pack("<I", ifd_off))
        f.write(struct.pack("<H", len(entries)))
        for (tag, typ, count, _), slot in zip(entries, slots):
            f.write(struct.pack("<HHI", tag, typ, count) + slot)
        f.write(struct.pack("<I", 0))
        f.write(bytes(extra))
        for s in strips:
            f.write(s)


def _read_tags(buf):
    if buf[:4] != b"II*\0":
        raise ValueError("only little-endian classic TIFF is supported")
    (ifd,) = struct.unpack_from("<I", buf, 4)
    (n,) = struct.unpack_from("<H", buf, ifd)
    tags = {}
    for i in range(n):
        tag, typ, count = struct.unpack_from("<HHI", buf, ifd + 2 + 12 * i)
        if typ not in _TYPES:
            continue
        fmt, size = _TYPES[typ]
        nbytes = size * count
        off = ifd + 2 + 12 * i + 8
        if nbytes > 4:
            (off,) = struct.unpack_from("<I", buf, off)
        if typ == 2:
            tags[tag] = bytes(buf[off:off + count]).rstrip(b"\0").decode()
        else:
            tags[tag] = list(struct.unpack_from("<" + fmt * count, buf, off))
    return tags


def read_geotiff(path):
    """Returns (data float32 [rows][cols], geotransform, nodata or None)."""
    with open(path, "rb") as f:
        buf = f.read()
    t = _read_tags(buf)
    w, h = t[T_WIDTH][0], t[T_LENGTH][0]
    if t.get(T_BPS, [32])[0] != 32 or t.get(T_SAMPLE_FORMAT, [3])[0] != 3:
        raise ValueError("only Float32 samples are supported")
    if t.get(T_SPP, [1])[0] != 1:
        raise ValueError("only single-band rasters are supported")
    if t.get(T_PREDICTOR, [1])[0] != 1:
        raise ValueError("TIFF predictors are not supported")
    comp = t.get(T_COMPRESSION, [1])[0]
    rps = t.get(T_ROWS_PER_STRIP, [h])[0]
    out = np.empty((h, w), dtype="<f4")
    for i, (o, n) in enumerate(zip(t[T_STRIP_OFFSETS], t[T_STRIP_BYTES])):
        raw = bytes(buf[o:o + n])
        if comp in (8, 32946):
            raw = zlib.decompress(raw)
        elif comp != 1:
            raise ValueError(f"TIFF compression {comp} is not supported")
        r0 = i * rps
        rows = min(rps, h - r0)
        out[r0:r0 + rows] = np.frombuffer(raw, dtype="<f4", count=rows * w).reshape(rows, w)
    gt = None
    if T_PIXEL_SCALE in t and T_TIEPOINT in t:
        sx, sy = t[T_PIXEL_SCALE][:2]
        i, j, _, X, Y, _ = t[T_TIEPOINT][:6]
        gt = (X - i * sx, sx, 0.0, Y + j * sy, 0.0, -sy)
    nod = float(t[T_NODATA]) if T_NODATA in t else None
    return out.astype(np.float32), gt, nod
