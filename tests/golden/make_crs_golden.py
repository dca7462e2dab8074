"""Golden vectors for the CRS transform and the GIS export, read
from data files the reference holds (run in the build container, where /root/reference
exists; the fixtures are committed, the reference never travels):

  land      data/raw/selected_polygons.txt (WKT, EPSG:2443 m)  ->
            data/processed/land/land_area.shp (EPSG:4612), written by
            map_generation/data_manager.py:83-86 (gpd.to_crs + to_file)
  populated data/processed/populated_area.txt (integer m / 1000, data_manager.py:56-81) ->
            data/processed/populated_area/populated_area.shp (map_generation/utils.py:81-84)
  nfz       the Point.buffer circles of map_generation/utils.py:93-104 ->
            data/processed/no_fly_zone/no_fly_zone.shp

Correspondence of vertices: the shapefile ring is the input ring closed and, when it was
counter-clockwise, reversed with its first vertex kept (OGR's ESRI orientation rule; TM is
conformal, so orientation is the same in both CRSs).  Parsing is struct / regex only.
Output: tests/golden/crs.npz (plane_xy, lonlat, set, ring) and crs_meta.json (per-shapefile
header: shape type, record count, bbox, vertices per record, dbf field)."""
import json
import os
import re
import struct

import numpy as np

REF = "/root/reference/data"
HERE = os.path.dirname(os.path.abspath(__file__))


def read_shp(path):
    b = open(path, "rb").read()
    kind = struct.unpack("<i", b[32:36])[0]
    box = struct.unpack("<4d", b[36:68])
    recs, off = [], 100
    while off < len(b):
        _, words = struct.unpack(">2i", b[off:off + 8])
        c = b[off + 8:off + 8 + 2 * words]
        off += 8 + 2 * words
        nparts, npts = struct.unpack("<2i", c[36:44])
        p0 = 44 + 4 * nparts
        recs.append(np.frombuffer(c[p0:p0 + 16 * npts], dtype="<f8").reshape(-1, 2).copy())
    return kind, box, recs


def dbf_meta(path):
    d = open(path, "rb").read()
    n, hlen, rlen = struct.unpack("<IHH", d[4:12])
    name = d[32:43].split(b"\0")[0].decode()
    return {"n": n, "hlen": hlen, "rlen": rlen, "field": [name, chr(d[43]), d[48], d[49]],
            "rows": [d[hlen + i * rlen:hlen + (i + 1) * rlen].decode() for i in range(n)]}


def orient(ring):
    ring = np.asarray(ring, dtype=np.float64)
    if not np.array_equal(ring[0], ring[-1]):
        ring = np.vstack([ring, ring[:1]])
    x, y = ring[:, 0], ring[:, 1]
    a = 0.5 * np.sum(x[:-1] * y[1:] - x[1:] * y[:-1])
    return ring[::-1].copy() if a > 0 else ring


def circle(c, r, n=64):
    th = -np.arange(n) * (2 * np.pi / n)
    ring = np.c_[c[0] + r * np.cos(th), c[1] + r * np.sin(th)]
    return np.vstack([ring, ring[:1]])


def main():
    sets = {}
    # land
    rings = []
    for line in open(f"{REF}/raw/selected_polygons.txt").read().strip().splitlines():
        body = re.search(r"\(\((.*)\)\)", line).group(1)
        rings.append(np.array([[float(v) for v in p.split()] for p in body.split(",")]))
    sets["land"] = (rings, f"{REF}/processed/land/land_area")
    # populated (integer metres, printed / 1000)
    txt = open(f"{REF}/processed/populated_area.txt").read()
    rings = []
    for body in re.findall(r"polygon\((.*?)\)(?=,\n|\n|$)", txt):
        pts = [[round(float(v) * 1000.0) for v in q.split(",")]
               for q in re.findall(r"\[([^\]]*)\]", body)]
        rings.append(np.array(pts, dtype=np.float64))
    sets["populated"] = (rings, f"{REF}/processed/populated_area/populated_area")
    # no-fly circles (map_generation/utils.py:93-99)
    locs = [((38666.52661075855, -9203.164091309498), 9000),
            ((46361.37256675563, 3942.7562315386298), 2000),
            ((19846.825121034392, 18934.11773399299), 2000),
            ((26037.433469490207, 15467.10452712196), 2000),
            ((46877.58543585609, -19138.710035318375), 2000)]
    sets["nfz"] = ([circle(c, r) for c, r in locs], f"{REF}/processed/no_fly_zone/no_fly_zone")

    plane, geo, set_id, ring_id, meta = [], [], [], [], {}
    for si, (name, (rings, base)) in enumerate(sets.items()):
        kind, box, recs = read_shp(base + ".shp")
        assert len(recs) == len(rings), (name, len(recs), len(rings))
        for ri, (r, g) in enumerate(zip(rings, recs)):
            o = orient(r)
            assert o.shape == g.shape, (name, ri, o.shape, g.shape)
            plane.append(o)
            geo.append(g)
            set_id += [si] * len(o)
            ring_id += [ri] * len(o)
        meta[name] = {"shape_type": kind, "records": len(recs), "bbox": list(box),
                      "vertices": [len(g) for g in recs], "dbf": dbf_meta(base + ".dbf"),
                      "prj": open(base + ".prj").read(), "cpg": open(base + ".cpg").read()}
    np.savez_compressed(os.path.join(HERE, "crs.npz"), plane_xy=np.vstack(plane),
                        lonlat=np.vstack(geo), set=np.array(set_id, np.int32),
                        ring=np.array(ring_id, np.int32), names=np.array(list(sets)))
    with open(os.path.join(HERE, "crs_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print({k: v["records"] for k, v in meta.items()}, len(set_id), "vertices")


if __name__ == "__main__":
    main()
