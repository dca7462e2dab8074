// Polygon approximation shared by the vector path (uam_process_polygons) and the DEM path
// (uam_dem_polygons): DataProcessor.process_polygons of map_generation/data_processor.py:15-75.
#pragma once
#include <cstdint>
#include <vector>

#include <functional>

// thread-local uam_last_error() text (defined in uampath.hip); returns code
int uam_fail_(int code, const char* fmt, ...);

// tiles.cpp: read GeoTIFF tiles [0, n_tiles) in chunks of per_chunk on a thread pool: for chunk
// c, slot(c) gives its destination [per_chunk][th][tw] (nullptr: fail UAM_E_HIP), then
// filled(c, i0, i1) is called once tiles [i0, i1) are in (non-zero: stop with that code)
int tiles_stream(const char* const* paths, int32_t n_tiles, int32_t th, int32_t tw,
                 int32_t n_threads, int32_t per_chunk,
                 const std::function<float*(int32_t chunk)>& slot,
                 const std::function<int(int32_t chunk, int32_t i0, int32_t i1)>& filled);

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
