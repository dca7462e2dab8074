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
