"""Golden vectors for DataProcessor.process_polygons, from data files the
reference holds (run in the build container; fixtures committed, the reference never travels):

  input   data/raw/populated_area/populated_area.shp -- the DID polygons (EPSG:4612), read by
          DataManager.load_polygons_from_shapefile (data_manager.py:21-27), to_crs(2443)
  output  data/processed/populated_area.txt -- process_polygons' 29 rectangles
          (map_generation/main.py:17-24, integer metres written / 1000 by save_polygons)

Rings keep their shapefile order and ESRI role (clockwise = shell, counter-clockwise = hole).
Output: tests/golden/polygons.npz (lonlat, ring_start, ring_hole, ring_record, rects [29,4,2]
int64 in the file's order and vertex order)."""
import os
import re
import struct

import numpy as np

REF = "/root/reference/data"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    b = open(f"{REF}/raw/populated_area/populated_area.shp", "rb").read()
    pts, starts, holes, recs = [], [0], [], []
    off, rec = 100, 0
    while off < len(b):
        _, words = struct.unpack(">2i", b[off:off + 8])
        c = b[off + 8:off + 8 + 2 * words]
        off += 8 + 2 * words
        nparts, npts = struct.unpack("<2i", c[36:44])
        parts = list(struct.unpack(f"<{nparts}i", c[44:44 + 4 * nparts])) + [npts]
        p0 = 44 + 4 * nparts
        xy = np.frombuffer(c[p0:p0 + 16 * npts], dtype="<f8").reshape(-1, 2)
        for i in range(nparts):
            r = xy[parts[i]:parts[i + 1]]
            x, y = r[:, 0], r[:, 1]
            a = 0.5 * np.sum(x[:-1] * y[1:] - x[1:] * y[:-1])
            pts.append(r)
            starts.append(starts[-1] + len(r))
            holes.append(1 if a > 0 else 0)    # ESRI: counter-clockwise ring = hole
            recs.append(rec)
        rec += 1
    txt = open(f"{REF}/processed/populated_area.txt").read()
    rects = []
    for body in re.findall(r"polygon\((.*?)\)(?=,\n|\n|$)", txt):
        rects.append([[round(float(v) * 1000.0) for v in q.split(",")]
                      for q in re.findall(r"\[([^\]]*)\]", body)])
    rects = np.array(rects, dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "polygons.npz"), lonlat=np.vstack(pts),
                        ring_start=np.array(starts, np.int64), ring_hole=np.array(holes, np.int32),
                        ring_record=np.array(recs, np.int32), rects=rects)
    print(rec, "records", len(holes), "rings", sum(holes), "holes", rects.shape, "rects")


if __name__ == "__main__":
    main()
