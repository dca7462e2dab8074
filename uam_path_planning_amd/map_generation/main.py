"""Driver -- the reference's map_generation/main.py (Main.process_population 17-29,
process_land 32-44) on this build: polygons in EPSG:2443 metres, GPU transforms (K7) and GPU
DEM labelling (K8), host rectangle approximation (uam_process_polygons).  The interactive
selection and the plots (main.py:47-70, visualizer.py) are UI and out of scope.

    python -m uam_path_planning_amd.map_generation.main population <did.shp> <out.txt> [out.shp]
    python -m uam_path_planning_amd.map_generation.main land <dem.tif> <out.txt> [threshold]
"""
import sys

from ..geo.export import make_area_shp
from .data_manager import DataManager
from .data_processor import DataProcessor


class Main:
    def __init__(self, engine=None):
        self.data_manager = DataManager(engine)
        self.processor = DataProcessor()

    def process_population(self, shapefile, out_txt, out_shp=None):
        polygons = self.data_manager.load_polygons_from_shapefile(shapefile)
        processed = self.processor.process_polygons(polygons)
        self.data_manager.save_polygons(processed, out_txt)
        if out_shp:
            make_area_shp(processed, out_shp)
        return processed

    def process_land(self, dem_file, out_txt, threshold_dem=0):
        polygons = self.data_manager.load_dem_polygons_from_geotiff(dem_file, threshold_dem)
        processed = self.processor.process_polygons(polygons)
        self.data_manager.save_polygons(processed, out_txt)
        return processed


def main(argv):
    if len(argv) < 3 or argv[0] not in ("population", "land"):
        print(__doc__)
        return 2
    m = Main()
    if argv[0] == "population":
        out = m.process_population(argv[1], argv[2], argv[3] if len(argv) > 3 else None)
    else:
        out = m.process_land(argv[1], argv[2], float(argv[3]) if len(argv) > 3 else 0)
    print(f"{len(out)} rectangles -> {argv[2]}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
