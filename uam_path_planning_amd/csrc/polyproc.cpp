// Host side of SURVEY §8(f) rank 2: DataProcessor.process_polygons
// (map_generation/data_processor.py:15-75) on polygons in plane metres.
//   unary_union  -> edge cancellation: rings oriented shell CCW / hole CW, every edge present
//                   in both directions removed, the rest re-linked into rings (leftmost turn
//                   at pinch vertices), holes assigned to the shell containing them.
//                   Interiors must be disjoint (shared boundaries are what unions merge in
//                   the reference data); overlapping inputs are rejected.
//   area filter  -> polygon.area > min_area (shell minus holes)
//   large split  -> divisions x divisions boxes over polygon.bounds; pieces of polygon n box by
//                   Weiler-Atherton chain linking (Liang-Barsky crossings, CCW box walk)
//   approximation-> cv2.minAreaRect + cv2.boxPoints on the float32 exterior coordinates,
//                   restated operation by operation (Andrew hull, rotating calipers in float32
//                   as OpenCV's rotcalipers.cpp, RotatedRect::points), np.intp truncation
//   final filter -> Polygon(box).area > min_approx_polygon_area
// Pinned: the reference's data/raw/populated_area -> data/processed/populated_area.txt
// (29/29 rectangles, vertex order included; tests/test_polygons_cpu.py).
//
// Attribution: calipers() and min_area_rect_box() below follow the rotating-calipers routine of
// OpenCV (modules/imgproc/src/rotcalipers.cpp, cv::minAreaRect / rotatingCalipers) step by
// step -- the same variable roles and control flow -- because float32 bit-parity with
// cv2.minAreaRect is the requirement.  OpenCV is distributed under the Apache License 2.0
// (4.5 and later; the 3-clause BSD license before): Copyright (C) 2000-2022 Intel
// Corporation, Willow Garage Inc., Itseez Inc., OpenCV Foundation and other contributors.
#include "polyproc.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <map>
#include <utility>

#include "../../include/uampath.h"

namespace uampoly {

// ---- cv2.minAreaRect restatement (float32) -----------------------------------------------
namespace {

struct P2f {
    float x, y;
};

double cross(const P2f& o, const P2f& a, const P2f& b) {
    return ((double)a.x - o.x) * ((double)b.y - o.y) - ((double)a.y - o.y) * ((double)b.x - o.x);
}

// convex hull as cv::convexHull(points, clockwise=false): strictly convex (collinear and
// duplicate points dropped), counter-clockwise, starting at the last point in (x, y) order
// (largest x, then largest y) -- the start matters for the calipers' tie-break
std::vector<P2f> hull(std::vector<P2f> p) {
    std::sort(p.begin(), p.end(), [](const P2f& a, const P2f& b) {
        return a.x < b.x || (a.x == b.x && a.y < b.y);
    });
    p.erase(std::unique(p.begin(), p.end(),
                        [](const P2f& a, const P2f& b) { return a.x == b.x && a.y == b.y; }),
            p.end());
    if (p.size() < 3) return p;
    std::vector<P2f> h(2 * p.size());
    size_t k = 0;
    for (size_t i = 0; i < p.size(); ++i) {
        while (k >= 2 && cross(h[k - 2], h[k - 1], p[i]) <= 0) --k;
        h[k++] = p[i];
    }
    for (size_t i = p.size() - 1, t = k + 1; i-- > 0;) {
        while (k >= t && cross(h[k - 2], h[k - 1], p[i]) <= 0) --k;
        h[k++] = p[i];
    }
    h.resize(k - 1);
    // Andrew's chain starts at the smallest (x, y); the upper chain starts at the largest
    size_t top = 0;
    for (size_t i = 1; i < h.size(); ++i)
        if (h[i].x > h[top].x || (h[i].x == h[top].x && h[i].y > h[top].y)) top = i;
    std::rotate(h.begin(), h.begin() + top, h.end());
    return h;
}

struct Rot {
    float cx, cy, w, h, angle;
};

// OpenCV rotatingCalipers(CALIPERS_MINAREARECT) + the tail of cv::minAreaRect
Rot calipers(const std::vector<P2f>& pts) {
    const int n = (int)pts.size();
    std::vector<P2f> vect(n);
    std::vector<float> inv(n);
    int left = 0, bottom = 0, right = 0, top = 0;
    float left_x = pts[0].x, right_x = pts[0].x, top_y = pts[0].y, bottom_y = pts[0].y;
    P2f pt0 = pts[0];
    for (int i = 0; i < n; ++i) {
        if (pt0.x < left_x) left_x = pt0.x, left = i;
        if (pt0.x > right_x) right_x = pt0.x, right = i;
        if (pt0.y > top_y) top_y = pt0.y, top = i;
        if (pt0.y < bottom_y) bottom_y = pt0.y, bottom = i;
        const P2f pt = pts[(i + 1) < n ? i + 1 : 0];
        const double dx = pt.x - pt0.x, dy = pt.y - pt0.y;  // float differences, widened
        vect[i].x = (float)dx;
        vect[i].y = (float)dy;
        inv[i] = (float)(1. / std::sqrt(dx * dx + dy * dy));
        pt0 = pt;
    }
    float orientation = 0;
    {
        double ax = vect[n - 1].x, ay = vect[n - 1].y;
        for (int i = 0; i < n; ++i) {
            const double bx = vect[i].x, by = vect[i].y;
            const double convexity = ax * by - ay * bx;
            if (convexity != 0) {
                orientation = (convexity > 0) ? 1.f : (-1.f);
                break;
            }
            ax = bx;
            ay = by;
        }
    }
    float base_a = orientation, base_b = 0;
    int seq[4] = {bottom, right, top, left};
    float minarea = FLT_MAX;
    int b_left = 0, b_bottom = 0;
    float b_a = 0, b_w = 0, b_b = 0, b_h = 0;
    for (int k = 0; k < n; ++k) {
        const float dp[4] = {
            +base_a * vect[seq[0]].x + base_b * vect[seq[0]].y,
            -base_b * vect[seq[1]].x + base_a * vect[seq[1]].y,
            -base_a * vect[seq[2]].x - base_b * vect[seq[2]].y,
            +base_b * vect[seq[3]].x - base_a * vect[seq[3]].y,
        };
        float maxcos = dp[0] * inv[seq[0]];
        int me = 0;
        for (int i = 1; i < 4; ++i) {
            const float cosalpha = dp[i] * inv[seq[i]];
            if (cosalpha > maxcos) {
                me = i;
                maxcos = cosalpha;
            }
        }
        const int pindex = seq[me];
        const float lead_x = vect[pindex].x * inv[pindex];
        const float lead_y = vect[pindex].y * inv[pindex];
        switch (me) {
            case 0: base_a = lead_x, base_b = lead_y; break;
            case 1: base_a = lead_y, base_b = -lead_x; break;
            case 2: base_a = -lead_x, base_b = -lead_y; break;
            default: base_a = -lead_y, base_b = lead_x; break;
        }
        seq[me] += 1;
        seq[me] = (seq[me] == n) ? 0 : seq[me];
        float dx = pts[seq[1]].x - pts[seq[3]].x;
        float dy = pts[seq[1]].y - pts[seq[3]].y;
        const float width = dx * base_a + dy * base_b;
        dx = pts[seq[2]].x - pts[seq[0]].x;
        dy = pts[seq[2]].y - pts[seq[0]].y;
        const float height = -dx * base_b + dy * base_a;
        const float area = width * height;
        if (area <= minarea) {
            minarea = area;
            b_left = seq[3];
            b_a = base_a;
            b_w = width;
            b_b = base_b;
            b_h = height;
            b_bottom = seq[0];
        }
    }
    const float A1 = b_a, B1 = b_b, A2 = -b_b, B2 = b_a;
    const float C1 = A1 * pts[b_left].x + pts[b_left].y * B1;
    const float C2 = A2 * pts[b_bottom].x + pts[b_bottom].y * B2;
    const float idet = 1.f / (A1 * B2 - A2 * B1);
    const float px = (C1 * B2 - C2 * B1) * idet;
    const float py = (A1 * C2 - A2 * C1) * idet;
    const float o1x = A1 * b_w, o1y = B1 * b_w, o2x = A2 * b_h, o2y = B2 * b_h;
    Rot r;
    r.cx = px + (o1x + o2x) * 0.5f;
    r.cy = py + (o1y + o2y) * 0.5f;
    r.w = (float)std::sqrt((double)o1x * o1x + (double)o1y * o1y);
    r.h = (float)std::sqrt((double)o2x * o2x + (double)o2y * o2y);
    r.angle = (float)std::atan2((double)o1y, (double)o1x);
    r.angle = (float)(r.angle * 180 / M_PI);
    return r;
}

}  // namespace

bool min_area_rect_box(const std::vector<Pt>& in, int64_t box[8]) {
    if (in.empty()) return false;
    std::vector<P2f> p(in.size());
    for (size_t i = 0; i < in.size(); ++i) p[i] = P2f{(float)in[i].x, (float)in[i].y};
    std::vector<P2f> h = hull(p);
    Rot r;
    if (h.size() > 2) {
        r = calipers(h);
    } else if (h.size() == 2) {  // cv::minAreaRect, two points
        r.cx = (h[0].x + h[1].x) * 0.5f;
        r.cy = (h[0].y + h[1].y) * 0.5f;
        const double dx = h[1].x - h[0].x, dy = h[1].y - h[0].y;
        r.w = (float)std::sqrt(dx * dx + dy * dy);
        r.h = 0;
        r.angle = (float)std::atan2(dy, dx);
        r.angle = (float)(r.angle * 180 / M_PI);
    } else {
        r.cx = h[0].x, r.cy = h[0].y, r.w = r.h = 0, r.angle = 0;
    }
    // RotatedRect::points
    const double ang = r.angle * M_PI / 180.;
    const float b = (float)std::cos(ang) * 0.5f;
    const float a = (float)std::sin(ang) * 0.5f;
    float pt[8];
    pt[0] = r.cx - a * r.h - b * r.w;
    pt[1] = r.cy + b * r.h - a * r.w;
    pt[2] = r.cx + a * r.h - b * r.w;
    pt[3] = r.cy - b * r.h - a * r.w;
    pt[4] = 2 * r.cx - pt[0];
    pt[5] = 2 * r.cy - pt[1];
    pt[6] = 2 * r.cx - pt[2];
    pt[7] = 2 * r.cy - pt[3];
    for (int i = 0; i < 8; ++i) box[i] = (int64_t)pt[i];  // np.intp: truncation toward zero
    return true;
}

double box_area(const int64_t b[8]) {
    double s = 0.0;
    for (int i = 0; i < 4; ++i) {
        const int j = (i + 1) & 3;
        s += (double)b[2 * i] * (double)b[2 * j + 1] - (double)b[2 * j] * (double)b[2 * i + 1];
    }
    return std::fabs(0.5 * s);
}

// ---- vector geometry --------------------------------------------------------------------
namespace {

double signed_area(const Ring& r) {
    double s = 0.0;
    for (size_t i = 0; i < r.size(); ++i) {
        const Pt& a = r[i];
        const Pt& b = r[(i + 1) % r.size()];
        s += a.x * b.y - b.x * a.y;
    }
    return 0.5 * s;
}

bool point_in_ring(const Ring& r, double x, double y) {
    bool in = false;
    for (size_t i = 0, j = r.size() - 1; i < r.size(); j = i++) {
        if (((r[i].y > y) != (r[j].y > y)) &&
            (x < (r[j].x - r[i].x) * (y - r[i].y) / (r[j].y - r[i].y) + r[i].x))
            in = !in;
    }
    return in;
}

struct Polygon {
    Ring shell;               // CCW
    std::vector<Ring> holes;  // CW
    double area() const {
        double a = signed_area(shell);
        for (const Ring& h : holes) a += signed_area(h);  // holes are negative
        return a;
    }
};

using Key = std::pair<double, double>;

// unary_union of polygons with disjoint interiors
bool union_polygons(std::vector<Ring> rings, const std::vector<int>& is_hole,
                    std::vector<Polygon>& out) {
    std::multimap<Key, Key> edges;  // from -> to
    double in_area = 0.0;
    for (size_t r = 0; r < rings.size(); ++r) {
        Ring& g = rings[r];
        if (g.size() >= 2 && g.front().x == g.back().x && g.front().y == g.back().y)
            g.pop_back();
        if (g.size() < 3) continue;
        const double a = signed_area(g);
        if ((a < 0) != (is_hole[r] != 0)) std::reverse(g.begin(), g.end());
        in_area += signed_area(g);
        for (size_t i = 0; i < g.size(); ++i) {
            const Pt& p = g[i];
            const Pt& q = g[(i + 1) % g.size()];
            if (p.x == q.x && p.y == q.y) continue;
            edges.emplace(Key{p.x, p.y}, Key{q.x, q.y});
        }
    }
    // cancel edges present in both directions
    std::multimap<Key, Key> keep;
    for (auto it = edges.begin(); it != edges.end(); ++it) {
        bool twin = false;
        auto rg = edges.equal_range(it->second);
        for (auto jt = rg.first; jt != rg.second; ++jt)
            if (jt->second == it->first) twin = true;
        if (!twin) keep.emplace(it->first, it->second);
    }
    // re-link: at each vertex take the outgoing edge with the smallest left turn from the
    // incoming direction (keeps faces to the left at pinch vertices)
    std::vector<Ring> outr;
    while (!keep.empty()) {
        auto it = keep.begin();
        const Key start = it->first;
        Key cur = it->second, prev = start;
        Ring ring{Pt{start.first, start.second}};
        keep.erase(it);
        size_t guard = 0;
        while (!(cur == start)) {
            ring.push_back(Pt{cur.first, cur.second});
            auto rg = keep.equal_range(cur);
            if (rg.first == rg.second) return false;  // open chain: not a valid union input
            auto best = rg.first;
            if (std::next(rg.first) != rg.second) {
                const double ix = cur.first - prev.first, iy = cur.second - prev.second;
                const double base = std::atan2(-iy, -ix);
                double bestang = 1e300;
                for (auto jt = rg.first; jt != rg.second; ++jt) {
                    double d = std::atan2(jt->second.second - cur.second,
                                          jt->second.first - cur.first) - base;
                    while (d <= 0) d += 2 * M_PI;
                    while (d > 2 * M_PI) d -= 2 * M_PI;
                    if (2 * M_PI - d < bestang) {  // most clockwise from the reverse = left face
                        bestang = 2 * M_PI - d;
                        best = jt;
                    }
                }
            }
            prev = cur;
            cur = best->second;
            keep.erase(best);
            if (++guard > edges.size()) return false;
        }
        outr.push_back(std::move(ring));
    }
    double out_area = 0.0;
    std::vector<Ring> shells, holes;
    for (Ring& r : outr) {
        const double a = signed_area(r);
        out_area += a;
        (a > 0 ? shells : holes).push_back(std::move(r));
    }
    if (std::fabs(out_area - in_area) > 1e-9 * std::max(1.0, std::fabs(in_area)))
        return false;  // overlapping interiors
    // interiors must be disjoint: no proper edge crossing between different shells and no
    // shell vertex strictly inside another shell
    auto bbox = [](const Ring& r, double b[4]) {
        b[0] = b[1] = 1e300, b[2] = b[3] = -1e300;
        for (const Pt& p : r)
            b[0] = std::min(b[0], p.x), b[1] = std::min(b[1], p.y), b[2] = std::max(b[2], p.x),
            b[3] = std::max(b[3], p.y);
    };
    auto orient = [](const Pt& a, const Pt& b, const Pt& c) {
        const double v = (b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x);
        return (v > 0) - (v < 0);
    };
    for (size_t i = 0; i < shells.size(); ++i) {
        double bi[4];
        bbox(shells[i], bi);
        for (size_t j = i + 1; j < shells.size(); ++j) {
            double bj[4];
            bbox(shells[j], bj);
            if (bi[2] < bj[0] || bj[2] < bi[0] || bi[3] < bj[1] || bj[3] < bi[1]) continue;
            const Ring &A = shells[i], &B = shells[j];
            for (size_t a = 0; a < A.size(); ++a) {
                const Pt &p1 = A[a], &p2 = A[(a + 1) % A.size()];
                for (size_t b = 0; b < B.size(); ++b) {
                    const Pt &q1 = B[b], &q2 = B[(b + 1) % B.size()];
                    const int o1 = orient(p1, p2, q1), o2 = orient(p1, p2, q2);
                    const int o3 = orient(q1, q2, p1), o4 = orient(q1, q2, p2);
                    if (o1 * o2 < 0 && o3 * o4 < 0) return false;  // proper crossing
                }
            }
            auto strictly_inside = [&](const Ring& outer, const Ring& inner) {
                for (const Pt& p : inner) {
                    bool on_boundary = false;
                    for (const Pt& q : outer)
                        if (q.x == p.x && q.y == p.y) on_boundary = true;
                    if (!on_boundary) return point_in_ring(outer, p.x, p.y);
                }
                return false;
            };
            if (strictly_inside(A, B) || strictly_inside(B, A)) return false;
        }
    }
    out.clear();
    for (Ring& s : shells) out.push_back(Polygon{std::move(s), {}});
    for (Ring& h : holes) {
        const Pt& p = h[0];
        int owner = -1;
        double best = 1e300;
        for (size_t i = 0; i < out.size(); ++i)
            if (point_in_ring(out[i].shell, p.x, p.y) && signed_area(out[i].shell) < best) {
                best = signed_area(out[i].shell);
                owner = (int)i;
            }
        if (owner >= 0) out[owner].holes.push_back(std::move(h));
    }
    return true;
}

struct Box {
    double x0, y0, x1, y1;
};

// pieces of (shell + holes) n box: Weiler-Atherton chain linking.  Each piece is returned as
// its boundary vertex list (only its convex hull is used).
std::vector<std::vector<Pt>> clip_pieces(const Polygon& pg, const Box& b) {
    const double w = b.x1 - b.x0, h = b.y1 - b.y0, per = 2 * w + 2 * h;
    auto inside = [&](const Pt& p) {
        return b.x0 <= p.x && p.x <= b.x1 && b.y0 <= p.y && p.y <= b.y1;
    };
    auto perim = [&](const Pt& p) {
        if (p.y == b.y0 && p.x >= b.x0 && p.x <= b.x1) return p.x - b.x0;
        if (p.x == b.x1) return w + (p.y - b.y0);
        if (p.y == b.y1) return w + h + (b.x1 - p.x);
        return 2 * w + h + (b.y1 - p.y);
    };
    std::vector<std::vector<Pt>> chains, pieces;
    bool any_inside_ring = false;
    std::vector<const Ring*> rings{&pg.shell};
    for (const Ring& r : pg.holes) rings.push_back(&r);
    for (size_t ri = 0; ri < rings.size(); ++ri) {
        const Ring& r = *rings[ri];
        const size_t n = r.size();
        size_t start = n;
        for (size_t i = 0; i < n; ++i)
            if (!inside(r[i])) {
                start = i;
                break;
            }
        if (start == n) {  // ring entirely in the box
            if (ri == 0) {
                pieces.push_back(r);
                any_inside_ring = true;
            }
            continue;
        }
        std::vector<Pt> cur;
        bool open = false;
        for (size_t k = 0; k < n; ++k) {
            const Pt p = r[(start + k) % n], q = r[(start + k + 1) % n];
            const double dx = q.x - p.x, dy = q.y - p.y;
            double t0 = 0.0, t1 = 1.0;
            bool ok = true;
            const double pp[4] = {-dx, dx, -dy, dy};
            const double qq[4] = {p.x - b.x0, b.x1 - p.x, p.y - b.y0, b.y1 - p.y};
            for (int e = 0; e < 4 && ok; ++e) {
                if (pp[e] == 0) {
                    if (qq[e] < 0) ok = false;
                } else {
                    const double t = qq[e] / pp[e];
                    if (pp[e] < 0)
                        t0 = std::max(t0, t);
                    else
                        t1 = std::min(t1, t);
                }
            }
            if (!ok || t0 >= t1) continue;
            if (t0 > 0) {
                cur.assign(1, Pt{p.x + t0 * dx, p.y + t0 * dy});
                open = true;
            }
            if (t1 < 1) {
                cur.push_back(Pt{p.x + t1 * dx, p.y + t1 * dy});
                if (open) chains.push_back(cur);
                cur.clear();
                open = false;
            } else if (open) {
                cur.push_back(q);
            }
        }
    }
    if (chains.empty()) {
        if (!any_inside_ring) {  // the box may lie entirely inside the polygon
            const double cx = 0.5 * (b.x0 + b.x1), cy = 0.5 * (b.y0 + b.y1);
            bool in = point_in_ring(pg.shell, cx, cy);
            for (const Ring& hr : pg.holes) in = in && !point_in_ring(hr, cx, cy);
            bool crosses = false;
            for (const Ring* r : rings)
                for (const Pt& p : *r)
                    if (p.x > b.x0 && p.x < b.x1 && p.y > b.y0 && p.y < b.y1) crosses = true;
            if (in && !crosses)
                pieces.push_back({{b.x0, b.y0}, {b.x1, b.y0}, {b.x1, b.y1}, {b.x0, b.y1}});
        }
        return pieces;
    }
    const Pt corner[4] = {{b.x0, b.y0}, {b.x1, b.y0}, {b.x1, b.y1}, {b.x0, b.y1}};
    const double ct[4] = {0.0, w, w + h, 2 * w + h};
    std::vector<double> tin(chains.size());
    for (size_t i = 0; i < chains.size(); ++i) tin[i] = perim(chains[i].front());
    std::vector<char> used(chains.size(), 0);
    for (size_t s = 0; s < chains.size(); ++s) {
        if (used[s]) continue;
        std::vector<Pt> piece;
        size_t c = s;
        while (!used[c]) {
            used[c] = 1;
            piece.insert(piece.end(), chains[c].begin(), chains[c].end());
            const double te = perim(chains[c].back());
            size_t nx = c;
            double bestd = 1e300;
            for (size_t i = 0; i < chains.size(); ++i) {
                double d = std::fmod(tin[i] - te + per, per);
                if (d < bestd) {
                    bestd = d;
                    nx = i;
                }
            }
            const double span = bestd > 0 ? bestd : per;
            std::vector<std::pair<double, int>> cs;
            for (int k = 0; k < 4; ++k) {
                const double d = std::fmod(ct[k] - te + per, per);
                if (d > 0 && d < span) cs.push_back({d, k});
            }
            std::sort(cs.begin(), cs.end());
            for (auto& ck : cs) piece.push_back(corner[ck.second]);
            c = nx;
        }
        pieces.push_back(std::move(piece));
    }
    return pieces;
}

}  // namespace

}  // namespace uampoly

using namespace uampoly;

// the rectangle-output step shared by both paths
static void emit(const std::vector<Pt>& pts, double min_approx, std::vector<int64_t>& out) {
    int64_t box[8];
    if (!min_area_rect_box(pts, box)) return;
    if (!(box_area(box) > min_approx)) return;
    out.insert(out.end(), box, box + 8);
}

extern "C" int uam_process_polygons(const double* xy, const int64_t* ring_start,
                                    int32_t n_rings, const int32_t* ring_hole,
                                    const uam_polyproc_params* prm, int64_t* rect_xy,
                                    int32_t max_rects, int32_t* n_rects) {
    if (!prm || !n_rects || (n_rings > 0 && (!xy || !ring_start || !ring_hole)))
        return uam_fail_(UAM_E_INVALID, "NULL argument");
    if (n_rings < 0 || prm->divisions < 1) return uam_fail_(UAM_E_INVALID, "bad arguments");
    std::vector<Ring> rings(n_rings);
    std::vector<int> hole(n_rings);
    for (int32_t r = 0; r < n_rings; ++r) {
        if (ring_start[r + 1] < ring_start[r]) return uam_fail_(UAM_E_INVALID, "ring_start");
        for (int64_t i = ring_start[r]; i < ring_start[r + 1]; ++i)
            rings[r].push_back(Pt{xy[2 * i], xy[2 * i + 1]});
        hole[r] = ring_hole[r];
    }
    std::vector<uampoly::Polygon> polys;
    if (!union_polygons(std::move(rings), hole, polys))
        return uam_fail_(UAM_E_INVALID,
                         "polygons overlap or do not close (union needs disjoint interiors)");
    std::vector<int64_t> out;
    for (const auto& pg : polys) {
        const double area = pg.area();
        if (!(area > prm->min_area)) continue;
        if (area > prm->large_area) {
            double minx = 1e300, miny = 1e300, maxx = -1e300, maxy = -1e300;
            for (const Pt& p : pg.shell) {
                minx = std::min(minx, p.x), maxx = std::max(maxx, p.x);
                miny = std::min(miny, p.y), maxy = std::max(maxy, p.y);
            }
            const int D = prm->divisions;
            const double dx = (maxx - minx) / D, dy = (maxy - miny) / D;
            for (int j = 0; j < D; ++j)
                for (int k = 0; k < D; ++k) {
                    const Box b{minx + j * dx, miny + k * dy, minx + (j + 1) * dx,
                                miny + (k + 1) * dy};
                    for (const auto& piece : clip_pieces(pg, b)) emit(piece, prm->min_approx_area, out);
                }
        } else {
            std::vector<Pt> ext(pg.shell.begin(), pg.shell.end());
            ext.push_back(pg.shell.front());  // exterior.coords is closed
            emit(ext, prm->min_approx_area, out);
        }
    }
    const int64_t n = (int64_t)out.size() / 8;
    *n_rects = (int32_t)n;
    if (rect_xy)
        for (int64_t i = 0; i < std::min<int64_t>(n, max_rects) * 8; ++i) rect_xy[i] = out[i];
    if (n > max_rects) return uam_fail_(UAM_E_INVALID, "%lld rectangles > max_rects %d",
                                        (long long)n, max_rects);
    return UAM_OK;
}
