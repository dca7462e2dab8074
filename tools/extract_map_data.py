"""Write uam_path_planning_amd/data/canonical_map.json from the reference's data files.

Data only (vertex coordinates), parsed without executing anything:
  data/processed/land_area.txt       Land region, 4 convex polygons (km, EPSG:2443 plane)
  data/processed/populated_area.txt  Population region, 29 polygons
  data/processed/no_fly_area.txt     one polygon no-fly zone (used by config 3)
and the scenario constants of geo_simulation_project/path_generation/main.py:
  no-fly balls main.py:27-31, HistCenter ball 48, N=80 54, options 55-60,
  start/goal 128, maxratio/maxalpha/enlargement 135, weights 145.
Run in the build container (needs /root/reference):  python tools/extract_map_data.py
"""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from uam_path_planning_amd.path_generation.utils import parse_shapes_text  # noqa: E402

REF_DATA = "/root/reference/data/processed"


def polys(name):
    with open(os.path.join(REF_DATA, name)) as f:
        parsed = parse_shapes_text(f.read())["vertices"]
    return [[[float(c) for c in p] for p in args] for kind, args, _ in parsed
            if kind == "polygon"]


def main():
    spec = {
        "source": "nomaporon/uam_path_planning data/processed/*.txt + path_generation/main.py",
        "units": "km, EPSG:2443 plane",
        "obstacles": [
            {"kind": "ball", "center": [38.66652661075855, -9.203164091309498], "r1": 9},
            {"kind": "ball", "center": [46.36137256675563, 3.9427562315386298], "r1": 2},
            {"kind": "ball", "center": [19.846825121034392, 18.93411773399299], "r1": 2},
            {"kind": "ball", "center": [26.037433469490207, 15.46710452712196], "r1": 2},
            {"kind": "ball", "center": [46.87758543585609, -19.138710035318375], "r1": 2},
        ],
        "regions": [
            {"name": "Land", "color": [0.929, 0.694, 0.125],
             "shapes": [{"kind": "polygon", "vertices": v} for v in polys("land_area.txt")]},
            {"name": "Population", "color": "Red",
             "shapes": [{"kind": "polygon", "vertices": v} for v in polys("populated_area.txt")]},
            {"name": "HistCenter", "color": "Green",
             "shapes": [{"kind": "ball", "center": [33.874752, -24.981154], "r1": 1}]},
        ],
        "no_fly_polygons": [{"kind": "polygon", "vertices": v} for v in polys("no_fly_area.txt")],
        "x_start": [35.590685, -27.711422],
        "x_goal": [26.478673, 9.564082],
        "N": 80,
        "options": {"length_smooth": True, "penalty_smooth": True, "obstacle_smooth": True,
                    "maxratio_smooth": False},
        "maxratio": 1.04,
        "maxalpha": math.pi / 80,
        "enlargement": 0.0,
        "weights": [200, 15000, 27000],
    }
    out = os.path.join(ROOT, "uam_path_planning_amd", "data", "canonical_map.json")
    with open(out, "w") as f:
        json.dump(spec, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
