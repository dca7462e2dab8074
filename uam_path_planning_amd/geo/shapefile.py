"""ESRI shapefile reader/writer in the layout the reference's geopandas/OGR output has
(data/processed/*/ *.shp): little/big-endian headers per the ESRI spec, outer polygon rings
closed and clockwise (a counter-clockwise input ring is reversed, its first vertex kept), one
dBase III attribute ``FID N(11,0)`` = 0..n-1, ``.cpg`` ISO-8859-1, ``.prj`` ESRI WKT.
Pure byte formatting: no GDAL/OGR, nothing executed from the files read."""
import datetime
import os
import struct

import numpy as np

POINT, POLYLINE, POLYGON = 1, 3, 5

# the .prj the reference's EPSG:4612 exports carry (ESRI WKT of JGD2000 geographic)
PRJ_4612 = ('GEOGCS["GCS_JGD_2000",DATUM["D_JGD_2000",SPHEROID["GRS_1980",6378137.0,'
            '298.257222101]],PRIMEM["Greenwich",0.0],UNIT["Degree",0.0174532925199433]]')


def _signed_area(ring):
    x, y = ring[:, 0], ring[:, 1]
    return 0.5 * float(np.sum(x[:-1] * y[1:] - x[1:] * y[:-1]))


def _close(ring):
    ring = np.asarray(ring, dtype=np.float64).reshape(-1, 2)
    if len(ring) and not np.array_equal(ring[0], ring[-1]):
        ring = np.vstack([ring, ring[:1]])
    return ring


def _orient_shell(ring):
    """Outer ring clockwise (ESRI); reversal keeps the first vertex."""
    ring = _close(ring)
    return ring[::-1].copy() if _signed_area(ring) > 0 else ring


def _record(kind, geom):
    if kind == POINT:
        x, y = (float(v) for v in np.asarray(geom, dtype=np.float64).reshape(2))
        return struct.pack("<i2d", POINT, x, y), (x, y, x, y)
    if kind == POLYLINE:
        parts = [np.asarray(geom, dtype=np.float64).reshape(-1, 2)]
    else:
        rings = geom if isinstance(geom, (list, tuple)) and len(geom) and \
            np.ndim(geom[0]) == 2 else [geom]
        parts = [_orient_shell(rings[0])] + [_close(r) for r in rings[1:]]
    pts = np.vstack(parts)
    box = (float(pts[:, 0].min()), float(pts[:, 1].min()), float(pts[:, 0].max()),
           float(pts[:, 1].max()))
    offs, o = [], 0
    for p in parts:
        offs.append(o)
        o += len(p)
    body = struct.pack("<i4d2i", kind, *box, len(parts), len(pts))
    body += struct.pack(f"<{len(parts)}i", *offs) + pts.astype("<f8").tobytes()
    return body, box


def _header(kind, words, box):
    return (struct.pack(">7i", 9994, 0, 0, 0, 0, 0, words) + struct.pack("<2i", 1000, kind) +
            struct.pack("<4d", *box) + struct.pack("<4d", 0.0, 0.0, 0.0, 0.0))


def write_shapefile(path, geometries, kind, prj=PRJ_4612, encoding="ISO-8859-1", date=None):
    """Write ``path``(.shp) + .shx/.dbf/.prj/.cpg.  geometries: points [2], polylines [n, 2],
    polygons [n, 2] (one shell) or [shell, hole, ...]."""
    base = path[:-4] if path.lower().endswith(".shp") else path
    d = os.path.dirname(base)
    if d:
        os.makedirs(d, exist_ok=True)
    recs, boxes = [], []
    for g in geometries:
        body, box = _record(kind, g)
        recs.append(body)
        boxes.append(box)
    if boxes:
        b = np.asarray(boxes)
        fbox = (b[:, 0].min(), b[:, 1].min(), b[:, 2].max(), b[:, 3].max())
    else:
        fbox = (0.0, 0.0, 0.0, 0.0)
    shp, shx, off = [], [], 50
    for i, body in enumerate(recs):
        words = len(body) // 2
        shp.append(struct.pack(">2i", i + 1, words) + body)
        shx.append(struct.pack(">2i", off, words))
        off += 4 + words
    with open(base + ".shp", "wb") as f:
        f.write(_header(kind, off, fbox) + b"".join(shp))
    with open(base + ".shx", "wb") as f:
        f.write(_header(kind, 50 + 4 * len(recs), fbox) + b"".join(shx))
    dt = date or datetime.date.today()
    n = len(recs)
    hdr = struct.pack("<4BIHH20x", 3, dt.year - 1900, dt.month, dt.day, n, 32 + 32 + 1, 12)
    field = b"FID".ljust(11, b"\0") + b"N" + b"\0" * 4 + bytes([11, 0]) + b"\0" * 14
    rows = b"".join(b" " + str(i).rjust(11).encode() for i in range(n))
    with open(base + ".dbf", "wb") as f:
        f.write(hdr + field + b"\r" + rows + b"\x1a")
    with open(base + ".prj", "w") as f:
        f.write(prj)
    with open(base + ".cpg", "w") as f:
        f.write(encoding)
    return base + ".shp"


def read_shapefile(path):
    """-> (kind, [geometry]) with points as (x, y) and polylines / polygons as lists of
    [n, 2] arrays (one per part)."""
    with open(path, "rb") as f:
        b = f.read()
    if struct.unpack(">i", b[:4])[0] != 9994:
        raise ValueError(f"{path}: not a shapefile")
    kind = struct.unpack("<i", b[32:36])[0]
    out, off = [], 100
    while off + 8 <= len(b):
        _, words = struct.unpack(">2i", b[off:off + 8])
        c = b[off + 8:off + 8 + 2 * words]
        off += 8 + 2 * words
        st = struct.unpack("<i", c[:4])[0]
        if st == 0:
            out.append(None)
        elif st == POINT:
            out.append(struct.unpack("<2d", c[4:20]))
        elif st in (POLYLINE, POLYGON):
            nparts, npts = struct.unpack("<2i", c[36:44])
            parts = list(struct.unpack(f"<{nparts}i", c[44:44 + 4 * nparts])) + [npts]
            p0 = 44 + 4 * nparts
            pts = np.frombuffer(c[p0:p0 + 16 * npts], dtype="<f8").reshape(-1, 2)
            out.append([pts[parts[i]:parts[i + 1]].copy() for i in range(nparts)])
        else:
            raise ValueError(f"{path}: shape type {st} not supported")
    return kind, out
