// Polygon approximation shared by the vector path (uam_process_polygons) and the DEM path
// (uam_dem_polygons): DataProcessor.process_polygons of map_generation/data_processor.py:15-75.
#pragma once
#include <cstdint>
#include <vector>

// thread-local uam_last_error() text (defined in uampath.hip); returns code
int uam_fail_(int code, const char* fmt, ...);

namespace uampoly {

struct Pt {
    double x, y;
};
using Ring = std::vector<Pt>;  // open (first vertex not repeated)

// cv2.boxPoints(cv2.minAreaRect(float32 points)) truncated like np.intp (data_processor.py:
// 68-72); returns false for an empty input.
bool min_area_rect_box(const std::vector<Pt>& pts, int64_t box[8]);

// shapely Polygon(box).area of the integer rectangle (shoelace, float64)
double box_area(const int64_t box[8]);

}  // namespace uampoly
