"""DataProcessor.process_polygons on the CPU: the library's host code
(uam_process_polygons) against the reference's own output.  Input: the DID polygons the
reference ships (data/raw/populated_area, EPSG:4612) transformed to EPSG:2443 (oracle TM, pinned
in test_crs_cpu.py); expected: data/processed/populated_area.txt (tests/golden/polygons.npz).
Tolerance 0: all 29 integer rectangles as exact corner sets (the list order of the reference's
output is GEOS' union order: compared as a multiset), and the cv2.boxPoints vertex order for
26 of them.  The other three are axis-aligned pieces of the divided polygon whose
minimum-area candidates tie exactly; there OpenCV's hull start -- and so the corner order --
follows the cyclic shift convexHull applies to the start of GEOS' clipped ring, which is not
reproduced (same rectangle, corners listed from another vertex)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def did():
    return np.load(os.path.join(GOLDEN, "polygons.npz"))


def did_polygons(z, xy):
    polys, cur = [], None
    for r in range(len(z["ring_hole"])):
        ring = xy[z["ring_start"][r]:z["ring_start"][r + 1]]
        if not z["ring_hole"][r]:
            cur = (ring, [])
            polys.append(cur)
        else:
            cur[1].append(ring)
    return polys


def as_multiset(rects):
    return sorted(tuple(map(tuple, np.asarray(r).tolist())) for r in rects)


def test_process_polygons_reproduces_reference_output(oracle_mod, did):
    from uam_path_planning_amd.map_generation.data_processor import DataProcessor

    xy = oracle_mod.tm_fwd(did["lonlat"])
    got = DataProcessor().process_polygons(did_polygons(did, xy))
    assert len(got) == 29
    sets = lambda rs: sorted(sorted(map(tuple, np.asarray(r).tolist())) for r in rs)
    assert sets(got) == sets(did["rects"])
    ordered = set(as_multiset(got)) & set(as_multiset(did["rects"]))
    assert len(ordered) >= 26


def test_process_polygons_edge_cases():
    from uam_path_planning_amd.map_generation.data_processor import DataProcessor

    dp = DataProcessor()
    assert dp.process_polygons([]) == []
    sq = np.array([[0, 0], [1000, 0], [1000, 1000], [0, 1000]], float)   # 1e6 m^2
    (r,) = dp.process_polygons([sq])
    assert sorted(map(tuple, r.tolist())) == [(0, 0), (0, 1000), (1000, 0), (1000, 1000)]
    # two squares sharing an edge merge (unary_union); touching at a corner they do not
    right = sq + [1000, 0]
    (r,) = dp.process_polygons([sq, right])
    assert sorted(map(tuple, r.tolist())) == [(0, 0), (0, 1000), (2000, 0), (2000, 1000)]
    diag = sq + [1000, 1000]
    assert len(dp.process_polygons([sq, diag])) == 2
    # small polygons are dropped; a hole lowers the area below min_area
    assert dp.process_polygons([sq * 0.5]) == []
    hole = np.array([[100, 100], [900, 100], [900, 900], [100, 900]], float)
    assert dp.process_polygons([(sq, [hole])]) == []
    # a large polygon is split into divisions^2 boxes: a 10 km square -> 25 2x2 km squares
    big = sq * 10
    rects = dp.process_polygons([big])
    assert len(rects) == 25
    for r in rects:
        r = np.asarray(r)
        assert r[:, 0].max() - r[:, 0].min() == 2000 and r[:, 1].max() - r[:, 1].min() == 2000
    with pytest.raises(ValueError):          # overlapping interiors are not a union input
        dp.process_polygons([sq, sq + [500, 0]])


def test_oracle_min_area_rect_reproduces_reference(oracle_mod, did):
    """The oracle's cv2.minAreaRect/boxPoints/np.intp restatement on the 12 DID polygons the
    reference approximates undivided: every rectangle and its vertex order."""
    xy = oracle_mod.tm_fwd(did["lonlat"])
    polys = did_polygons(did, xy)
    ref = set(as_multiset(did["rects"]))
    groups = [[0, 14], [12, 15]] + [[i] for i in range(18) if i not in (0, 14, 12, 15)]
    n = 0
    for g in groups:
        shells = [polys[i][0] for i in g]
        area = sum(abs(0.5 * np.sum(s[:-1, 0] * s[1:, 1] - s[1:, 0] * s[:-1, 1])) for s in shells)
        if area <= 750000 or area > 32e6:
            continue
        pts = np.vstack([np.vstack([polys[i][0]] + polys[i][1]) for i in g])
        box = oracle_mod.min_area_rect(pts)
        assert tuple(map(tuple, box.tolist())) in ref
        n += 1
    assert n == 12


# hand-built islands with pixel-aligned edges: raster and exact vector polygon both known
X0_KM, YTOP_KM, DX_KM = 0.0, 12.0, 0.06        # 60 m pixels


def _island_raster():
    dem = np.full((200, 200), -9999.0, np.float32)
    dem[30:170, 20:150] = 100.0          # L-shaped land mass (52.6 km^2 -> divided 5 x 5) ...
    dem[30:90, 90:150] = -9999.0
    dem[120:140, 40:60] = -9999.0        # ... with a lake
    dem[10:40, 170:190] = 50.0           # a small island (2.2 km^2)
    dem[100:105, 170:175] = 30.0         # a dropped islet (90 000 m^2 < min_area)
    return dem


def _to_m(cr):
    c, r = np.asarray(cr, float).T
    return np.c_[(X0_KM + c * DX_KM) * 1000.0, (YTOP_KM - r * DX_KM) * 1000.0]


def _island_polygons():
    shell = _to_m([(20, 30), (90, 30), (90, 90), (150, 90), (150, 170), (20, 170)])
    lake = _to_m([(40, 120), (60, 120), (60, 140), (40, 140)])
    small = _to_m([(170, 10), (190, 10), (190, 40), (170, 40)])
    islet = _to_m([(170, 100), (175, 100), (175, 105), (170, 105)])
    return [(shell, [lake]), small, islet]


def test_dem_route_matches_vector_route_on_exact_polygons(oracle_mod):
    """load_dem_polygons_from_geotiff + process_polygons on the raster (oracle: pixel
    labelling, box pieces on the refined grid) == process_polygons on the exact vector
    polygons (product host code: union, Weiler-Atherton pieces)."""
    from uam_path_planning_amd.map_generation.data_processor import DataProcessor

    dem = _island_raster()
    rd = oracle_mod.Oracle.raster_desc(200, 200, X0_KM, YTOP_KM, DX_KM, DX_KM)
    ras = oracle_mod.dem_polygons(dem, rd, 0.0, 1000.0)
    vec = DataProcessor().process_polygons(_island_polygons())
    assert len(ras) > 10                  # the divided L plus the small island
    assert as_multiset(ras) == as_multiset(vec)
    sea = oracle_mod.dem_polygons(dem, rd, -9999.0, 1000.0)   # threshold -9999: the sea
    assert len(sea) > 0 and as_multiset(sea) != as_multiset(ras)
