// uampath.hip -- MI355X (gfx950) kernels + C ABI for batched candidate-path cost evaluation.
//
// Kernels (SURVEY.md §2 native inventory):
//   k_prepare        per-shape normaliser psi(centre) (problem.py:79 recomputes it per call)
//   k_eval_points    Φ / per-region / obstacle penalties + collides at arbitrary points
//   k_raster_build   K1: one 16-B record per DEM cell {Φ, Σψ_nfz, dem, flags}
//   k_dem_mosaic     VRT tile mosaic into the DEM plane
//   k_eval_paths     K2 (raster gather) / K3 (analytic) with K4 (arc generator) fused
//   k_argmin         K5: reference selection rule per candidate group
//   k_gen_paths, k_path_length  batched create_x_init / length_of
//
// Numerics: float64 throughout, compiled with -ffp-contract=off so every product and sum is a
// separately rounded IEEE operation in the reference's order (problem.py, quadratic_obstacle.py,
// polygon.py, ball.py, square.py); f64 sqrt and divide lower to gfx950's correctly rounded
// sequences.  Results are therefore bit-identical to the CPU oracle (oracle/uam_oracle.c).
//
// Thread mapping of the path kernels: one lane per path, waypoints walked in order, so the
// per-path sums keep the reference's sequential order with no cross-lane reduction.  In the
// fused-generator kernel each wave owns ONE displacement d (wave-uniform) and 64 start/goal
// pairs, so the unit-arc table row u[d][*] is read with scalar (SMEM) loads and the geometry
// tables are read with wave-uniform addresses (scalar cache) in the analytic mode.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <type_traits>
#include <string>
#include <thread>
#include <vector>

#include <dlfcn.h>
#include <rccl/rccl.h>

#include "../../include/uampath.h"
#include "polyproc.h"

// ---- Measurement-build knobs -------------------------------------------------------------
// Tuning experiments only (tools/build_variant.sh passes -D overrides into a separate .so that
// UAM_LIB_PATH loads); the shipped library is built with exactly these defaults, and no knob
// changes what any kernel computes.
#ifndef UAM_K1_TILE_ROWS
// raster rows per column of K1's strip order (0: row-major).  cfg3 map at 4096^2: row-major
// 0.225 ms, columns of 16 / 32 / 64 / 128 / 256 / 512 / 4096 rows 0.196 / 0.196 / 0.195 /
// 0.190 / 0.188 / 0.189 / 0.231 ms (the shape-free build 0.108 -> 0.118-0.130: the record
// rows' DRAM pages); profiles/r05/cc13, cc14
#define UAM_K1_TILE_ROWS 128
#endif
#ifndef UAM_K1_GRID_CAP
// K1's strip workgroups, cfg3 map at 4096^2 (32 768 strips): uncapped 0.185 ms, 16 384 0.179,
// 12 288 0.197, 8192 0.176, 6144 0.205, 4096 0.193, 2048 0.254 (profiles/r05/cc15, cc16)
#define UAM_K1_GRID_CAP 8192
#endif
#ifndef UAM_K1_NT
// K1's record stores: 1 nontemporal.  cfg3 map at 4096^2: 0.177 -> 0.158 ms, the shape-free
// build 0.108 -> 0.081 ms; 8192^2 0.649 -> 0.571 ms (profiles/r06/c13, c14; nontemporal DEM
// loads 0.171 ms and 7-8 waves per SIMD, which spill, were measured and dropped)
#define UAM_K1_NT 1
#endif
#ifndef UAM_RF_PREFETCH  // K6 refinement: 0 reads the L-BFGS pairs without prefetch
#define UAM_RF_PREFETCH 1
#endif
#ifndef UAM_RF_WAVES  // K6 refinement: waves per SIMD of k_refine's register budget
#define UAM_RF_WAVES 4
#endif
#ifndef UAM_RORD_BITS  // K2's raster pair order: 4^bits bins per key level
#define UAM_RORD_BITS 2
#endif
#ifndef UAM_G_NBK  // K2g / K2h / K4h counting sort: partitions (one 1024-thread block each)
#define UAM_G_NBK 256
#endif
#ifndef UAM_K2H_MINW  // K2h evaluation: waves per SIMD the register budget allows
#define UAM_K2H_MINW 4
#endif
#ifndef UAM_K2H_BS  // K2h evaluation: items per workgroup
#define UAM_K2H_BS 256
#endif
#ifndef UAM_SHAPE_GRID_N  // shape-grid index: cells per side
#define UAM_SHAPE_GRID_N 64
#endif
#ifndef UAM_GRID_REFINE  // shape-grid index: 0 lists every cell a shape's box meets
#define UAM_GRID_REFINE 1
#endif
// ---- end of the measurement-build knobs ---------------------------------------------------


namespace {

// ----------------------------------------------------------------------------------------
// device-side tables

struct alignas(16) DevIneq {  // 64 B: one s_load_dwordx16
    double p[6];
    int32_t kind;
    int32_t pad0;
    double pad1;
};

// Shape culling (see shape_box): outside box_pen / box_obs the smooth penalty of the shape is
// exactly +0 (some factor min(h_i - e, 0) is 0), so skipping it leaves every sum bit-identical.
enum : int32_t {
    SHAPE_BOX_PEN_OK = 1,   // host: box_pen bounds {h_i < enlargement for all i}
    SHAPE_BOX_OBS_OK = 2,   // host: box_obs bounds {h_i < 1e-14 for all i}
    SHAPE_CULL_PEN = 4,     // device: region penalty term may be skipped outside box_pen
    SHAPE_CULL_PSI = 8,     // device: raw obstacle psi may be skipped outside box_obs
    SHAPE_CULL_HIT = 16     // device: contains() may be skipped outside box_obs
};

struct alignas(16) DevShape {  // 128 B
    int32_t first, count, has_center, flags;
    double norm_pen;  // psi(centre; penalty_smooth, e)
    double norm_obs;  // psi(centre; obstacle_smooth, e)
    double cx, cy;
    double box_pen[4];  // xmin, xmax, ymin, ymax
    double box_obs[4];
    int32_t region;     // region of a region shape, -1 for obstacles
    int32_t pad0;
    double wreg;        // weight of its region (uam_set_params; 0 for obstacles)
};

__host__ __device__ __forceinline__ bool outside(const double* b, double x0, double x1) {
    return x0 < b[0] || x0 > b[1] || x1 < b[2] || x1 > b[3];  // NaN -> false (evaluate)
}

// Uniform-grid shape index (built by uam_set_params): for every cell the shapes whose culling
// box meets it, in ascending shape order, CSR-encoded; slot gx*gy lists the shapes that are
// never culled (what a point off the grid must evaluate).  Exact: a shape missing from a
// point's list has a box that does not contain the point, so box culling would skip it.
struct KShapeGrid {
    double x0, y0, x1, y1, inv_dx, inv_dy;
    int32_t gx, gy;
    const int32_t* start[3];  // 0 = region penalty (box_pen), 1 = psi, 2 = hit
    const int32_t* items[3];
    // the lists as per-slot bitmasks (bit i of word w: shape mbase + 64 w + i), mw words per
    // slot; null when the table spans more than 256 shapes
    const uint64_t* mask[3];
    int32_t mbase[3], mw[3];
};

struct KGeom {
    const DevIneq* __restrict__ ineq;
    const DevShape* __restrict__ shape;
    int32_t n_obstacles;
    int32_t n_regions;
    int32_t region_first[UAM_MAX_REGIONS + 1];
    KShapeGrid grid;  // grid.gx == 0: no index
};

// list slot of a point: its grid cell, gx*gy off the grid, -1 for NaN (no index: evaluate all)
__device__ __forceinline__ int grid_slot(const KShapeGrid& gr, double x, double y) {
    if (!(x == x) || !(y == y)) return -1;
    if (x < gr.x0 || x > gr.x1 || y < gr.y0 || y > gr.y1) return gr.gx * gr.gy;
    const int cx = min((int)floor((x - gr.x0) * gr.inv_dx), gr.gx - 1);
    const int cy = min((int)floor((y - gr.y0) * gr.inv_dy), gr.gy - 1);
    return cy * gr.gx + cx;
}

struct KParams {
    int32_t N;
    int32_t length_smooth, penalty_smooth, obstacle_smooth, maxratio_smooth;
    int32_t quirk_length, anchor_mode, pad;
    double anchor_x, anchor_y;
    double r_eff;      // maxratio, or maxratio**2 when maxratio_smooth (problem.py:95-96)
    double mincos;     // cos(maxalpha), computed on the host with libm (problem.py:98)
    double enlargement;
    double altitude;
    double weights[UAM_MAX_REGIONS];
};

struct KRaster {
    int32_t nx, ny;
    double x0, y_top, dx, dy, inv_dx, inv_dy;
    // K2 gather skip (uam_raster_summary): bitmap of 2^sshift x 2^sshift cell blocks, snbx
    // blocks per row, swords 32-bit words; null = gather every waypoint
    const uint32_t* __restrict__ sum;
    int32_t sshift, snbx, swords;
    // packed raster (uam_raster_pack; null = the sorted forms gather rec; layout: PackDims).
    // Header (hwords words, staged in LDS by K2h): the 2-bit code per summary block (pwords
    // words), the terrain bound table (one u16 per 2^bshift-square bound block, bnbx per row,
    // at word bnd_off) and the superblock table (float2 {base, step} per 4 x 4 bound blocks,
    // sbnbx per row, at word sbt_off).  Planes: p4 {phi} and t4 {terrain as read} in 4 x 8-cell
    // blocks (one 128-B line, nb8 per row), e8 {phi, psi | nfz << 31} in the same 4 x 8-cell
    // blocks (256 B: two lines of 2 x 8 cells), r16 (the records) in the same blocks (512 B),
    // all four at one index.
    const uint32_t* __restrict__ pmap;
    int32_t pwords, hwords, bnd_off, sbt_off;
    int32_t bshift, bnbx, sbnbx, nb8, nb4;  // (nb4: p8's 4 x 4-cell blocks per row)
    const uint32_t* __restrict__ p4;
    const float* __restrict__ t4;
    const uint2* __restrict__ e8;
    // K2h's addressing: the whole packed copy from one base by 32-bit byte offsets (the planes
    // p4 / e8 / r16 (the 16-B records, same blocks and index) and t4 at o4 / o8 / o16 / ot4);
    // null when the copy is 4 GiB or larger (K2h then stands aside)
    const char* __restrict__ pk;
    uint32_t o4, o8, o16, ot4, op8;  // (op8: the 8-B {phi, terrain} plane p8, p44_addr)
};

// volume (config 5): 8-B voxels {risk, psi_nfz} [ny][nx][nz], the 8-B column plane
// {terrain (+0 on nodata), flags} [ny][nx] and the column bitmap (one bit per 2^cshift-square
// block of columns: set unless every column reads {+0.0f, no NFZ}) of one buffer
// (uam_volume_shape)
struct KVolume {
    int32_t nx, ny, nz;
    double x0, y_top, z0, dz, inv_dx, inv_dy, inv_dz;
    const uint2* __restrict__ vox;
    const uint2* __restrict__ col;
    const uint32_t* __restrict__ cbits;
    int32_t cshift, cnbx, cwords;
};

struct KOut {
    double* cost;
    double* length_q;
    double* length;
    double* kin_sum;
    double* nfz_sum;
    int32_t* nfz_hits;
    double* min_clearance;
    int32_t* offmap;
    int32_t* cells;
    double* g_rows;
    int32_t* below_terrain;
};

// ----------------------------------------------------------------------------------------
// reference formulas (device)

__device__ __forceinline__ double ineq_h(const DevIneq* __restrict__ q, double x0, double x1) {
    const int kind = q->kind;
    if (kind == UAM_INEQ_HALFPLANE) {
        // polygon.py:69-71 line_F, h = -sgn * line (polygon.py:98)
        double line = q->p[3] * (x0 - q->p[0]) - q->p[2] * (x1 - q->p[1]);
        return q->p[4] * line;
    } else if (kind == UAM_INEQ_ELLIPSE) {
        // ball.py func: sumsqr(vertcat((x0-c0)/r1, (x1-c1)/r2)) - 1, sumsqr accumulates from 0
        double a = (x0 - q->p[0]) / q->p[2];
        double b = (x1 - q->p[1]) / q->p[3];
        double s = 0.0;
        s = s + a * a;
        s = s + b * b;
        return s - 1.0;
    } else {
        // square.py right/left/top/bottom: s*(x_k - c) - r
        double xk = (q->p[0] == 0.0) ? x0 : x1;
        return q->p[3] * (xk - q->p[1]) - q->p[2];
    }
}

// ineq_h at the CPL cells of one raster column (x0 shared, rows x1[k]), the same operations
// in the same order per cell.  The kind branch is taken once for all rows: with ineq_h called
// per row the compiler hoisted the ellipse's shared x division above the kind test, so every
// half-plane paid it (K1's inequality loop: ~14 f64 VALU per inequality).
template <int CPL>
__device__ __forceinline__ void ineq_h_col(const DevIneq& q, double x0, const double (&x1)[CPL],
                                           double (&h)[CPL]) {
    if (q.kind == UAM_INEQ_HALFPLANE) {
        const double ax = q.p[3] * (x0 - q.p[0]);
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const double line = ax - q.p[2] * (x1[k] - q.p[1]);
            h[k] = q.p[4] * line;
        }
    } else if (q.kind == UAM_INEQ_ELLIPSE) {
        const double a = (x0 - q.p[0]) / q.p[2];
        const double sa = 0.0 + a * a;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const double b = (x1[k] - q.p[1]) / q.p[3];
            const double s = sa + b * b;
            h[k] = s - 1.0;
        }
    } else if (q.p[0] == 0.0) {
        const double v = q.p[3] * (x0 - q.p[1]) - q.p[2];
#pragma unroll
        for (int k = 0; k < CPL; ++k) h[k] = v;
    } else {
#pragma unroll
        for (int k = 0; k < CPL; ++k) h[k] = q.p[3] * (x1[k] - q.p[1]) - q.p[2];
    }
}

// quadratic_obstacle.py:27-39
__device__ __forceinline__ double psi(const KGeom& g, const DevShape& sh, double x0, double x1,
                                      bool smooth, double e) {
    double r = 1.0;
    const int end = sh.first + sh.count;
    for (int i = sh.first; i < end; ++i) {
        double h = ineq_h(g.ineq + i, x0, x1);
        if (smooth) {
            double m = fmin(h - e, 0.0);
            r = r * (m * m);
        } else {
            r = r * fmin(e - h, 0.0);
        }
    }
    return r;
}

// quadratic_obstacle.py:89-94
__device__ __forceinline__ bool contains(const KGeom& g, const DevShape& sh, double x0,
                                         double x1) {
    const int end = sh.first + sh.count;
    bool in = true;
    for (int i = sh.first; i < end; ++i) in = in && !(ineq_h(g.ineq + i, x0, x1) > 1e-14);
    return in;
}

// problem.py:72-80 for region r (penalty_smooth, enlargement), weighted (problem.py:80)
__device__ __forceinline__ double region_penalty(const KGeom& g, const KParams& p, int r,
                                                 double x0, double x1) {
    double t = 0.0;
    const int s1 = g.region_first[r + 1];
    for (int s = g.region_first[r]; s < s1; ++s) {
        const DevShape& sh = g.shape[s];
        if ((sh.flags & SHAPE_CULL_PEN) && outside(sh.box_pen, x0, x1)) continue;  // adds +0
        double v = psi(g, sh, x0, x1, p.penalty_smooth != 0, p.enlargement);
        t = sh.has_center ? t + v / sh.norm_pen : t + v;
    }
    return p.weights[r] * t;
}

// problem.py:49-56.  With the grid index: the region shapes of the point's list, in ascending
// order; a region with no listed shape adds w_r * (+0), an exact no-op, so it is skipped.
__device__ __forceinline__ double total_penalty(const KGeom& g, const KParams& p, double x0,
                                                double x1) {
    const int slot = g.grid.gx ? grid_slot(g.grid, x0, x1) : -1;
    if (slot < 0) {
        double pen = 0.0;
        for (int r = 0; r < g.n_regions; ++r) pen = pen + region_penalty(g, p, r, x0, x1);
        return pen;
    }
    double pen = 0.0, t = 0.0;
    int rc = -1;
    const int k1 = g.grid.start[0][slot + 1];
    for (int k = g.grid.start[0][slot]; k < k1; ++k) {
        const DevShape& sh = g.shape[g.grid.items[0][k]];
        if (sh.region != rc) {
            if (rc >= 0) pen = pen + p.weights[rc] * t;
            rc = sh.region;
            t = 0.0;
        }
        if ((sh.flags & SHAPE_CULL_PEN) && outside(sh.box_pen, x0, x1)) continue;
        const double v = psi(g, sh, x0, x1, p.penalty_smooth != 0, p.enlargement);
        t = sh.has_center ? t + v / sh.norm_pen : t + v;
    }
    if (rc >= 0) pen = pen + p.weights[rc] * t;
    return pen;
}

__device__ __forceinline__ bool collides(const KGeom& g, double x0, double x1) {
    bool hit = false;
    const int slot = g.grid.gx ? grid_slot(g.grid, x0, x1) : -1;
    if (slot >= 0) {
        const int k1 = g.grid.start[2][slot + 1];
        for (int k = g.grid.start[2][slot]; k < k1; ++k) {
            const DevShape& sh = g.shape[g.grid.items[2][k]];
            if ((sh.flags & SHAPE_CULL_HIT) && outside(sh.box_obs, x0, x1)) continue;
            hit = hit || contains(g, sh, x0, x1);
        }
        return hit;
    }
    // a NaN coordinate makes every h(x) > 1e-14 test false (contains() is true) unless a finite
    // axis inequality decides: never cull such a point (slot -1 comes here)
    const bool nan = !(x0 == x0) || !(x1 == x1);
    for (int s = 0; s < g.n_obstacles; ++s) {
        const DevShape& sh = g.shape[s];
        if (!nan && (sh.flags & SHAPE_CULL_HIT) && outside(sh.box_obs, x0, x1)) continue;
        hit = hit || contains(g, sh, x0, x1);
    }
    return hit;
}

// Σ_o raw psi_o(x; obstacle_smooth, e = 0) -- the per-waypoint sum of the no-fly g rows
__device__ __forceinline__ double obstacle_psi_sum(const KGeom& g, const KParams& p, double x0,
                                                   double x1) {
    double acc = 0.0;
    const int slot = g.grid.gx ? grid_slot(g.grid, x0, x1) : -1;
    if (slot >= 0) {
        const int k1 = g.grid.start[1][slot + 1];
        for (int k = g.grid.start[1][slot]; k < k1; ++k) {
            const DevShape& sh = g.shape[g.grid.items[1][k]];
            if ((sh.flags & SHAPE_CULL_PSI) && outside(sh.box_obs, x0, x1)) continue;
            acc = acc + psi(g, sh, x0, x1, p.obstacle_smooth != 0, 0.0);
        }
        return acc;
    }
    for (int s = 0; s < g.n_obstacles; ++s) {
        const DevShape& sh = g.shape[s];
        if ((sh.flags & SHAPE_CULL_PSI) && outside(sh.box_obs, x0, x1)) continue;
        acc = acc + psi(g, sh, x0, x1, p.obstacle_smooth != 0, 0.0);
    }
    return acc;
}

// raw psi of obstacle s (a no-fly g row): exactly +0 when culled
__device__ __forceinline__ double obstacle_psi(const KGeom& g, const KParams& p, int s, double x0,
                                               double x1) {
    const DevShape& sh = g.shape[s];
    if ((sh.flags & SHAPE_CULL_PSI) && outside(sh.box_obs, x0, x1)) return 0.0;
    return psi(g, sh, x0, x1, p.obstacle_smooth != 0, 0.0);
}

// ----------------------------------------------------------------------------------------
// kernels

__global__ void k_prepare(KGeom g, KParams p, DevShape* __restrict__ shapes, int n_shapes) {
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_shapes) return;
    DevShape sh = shapes[s];
    sh.has_center = !(isnan(sh.cx) || isnan(sh.cy));
    sh.norm_pen = psi(g, sh, sh.cx, sh.cy, p.penalty_smooth != 0, p.enlargement);
    sh.norm_obs = psi(g, sh, sh.cx, sh.cy, p.obstacle_smooth != 0, p.enlargement);
    int32_t f = sh.flags & (SHAPE_BOX_PEN_OK | SHAPE_BOX_OBS_OK);
    // v / norm with v = +0 stays +0 only for a finite positive normaliser (0/0 = NaN must stay)
    const bool norm_ok = !sh.has_center || (isfinite(sh.norm_pen) && sh.norm_pen > 0.0);
    if ((f & SHAPE_BOX_PEN_OK) && p.penalty_smooth && norm_ok) f |= SHAPE_CULL_PEN;
    if ((f & SHAPE_BOX_OBS_OK) && p.obstacle_smooth) f |= SHAPE_CULL_PSI;
    if (f & SHAPE_BOX_OBS_OK) f |= SHAPE_CULL_HIT;
    sh.flags = f;
    shapes[s] = sh;
}

__global__ __launch_bounds__(256) void k_eval_points(KGeom g, KParams p,
                                                     const double* __restrict__ pts, int64_t n,
                                                     double* phi, double* phi_regions,
                                                     double* obs_norm, double* psi_raw,
                                                     int32_t* collide) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x0 = pts[2 * i], x1 = pts[2 * i + 1];
    if (phi) phi[i] = total_penalty(g, p, x0, x1);
    if (phi_regions)
        for (int r = 0; r < g.n_regions; ++r)
            phi_regions[i * g.n_regions + r] = region_penalty(g, p, r, x0, x1);
    if (obs_norm) {  // get_penalty_function(None): w = 1, obstacle_smooth, enlargement
        double t = 0.0;
        for (int s = 0; s < g.n_obstacles; ++s) {
            const DevShape sh = g.shape[s];
            double v = psi(g, sh, x0, x1, p.obstacle_smooth != 0, p.enlargement);
            t = sh.has_center ? t + v / sh.norm_obs : t + v;
        }
        obs_norm[i] = 1.0 * t;
    }
    if (psi_raw) psi_raw[i] = obstacle_psi_sum(g, p, x0, x1);
    if (collide) collide[i] = collides(g, x0, x1) ? 1 : 0;
}

// K1: record per cell.  One lane per cell, rows contiguous -> coalesced DEM reads and
// 16-B record stores (one global_store_dwordx4 per lane).
__global__ __launch_bounds__(256) void k_dem_mosaic(const float* __restrict__ tiles, int n_tiles,
                                                    int th, int tw,
                                                    const int32_t* __restrict__ xoff,
                                                    const int32_t* __restrict__ yoff,
                                                    float* __restrict__ dem, int nx, int ny) {
    const int64_t per = (int64_t)th * tw;
    const int64_t total = per * n_tiles;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int t = (int)(i / per);
        const int64_t r = i - t * per;
        const int y = (int)(r / tw), x = (int)(r - (int64_t)y * tw);
        const int gx = xoff[t] + x, gy = yoff[t] + y;
        if (gx >= 0 && gx < nx && gy >= 0 && gy < ny) dem[(int64_t)gy * nx + gx] = tiles[i];
    }
}

// Volume build (config 5): voxel (ix, iy, iz), iz fastest, from the 2-D record of its column:
// risk = Φ(column) * w[iz] (f64 product rounded to f32) and the column's psi_nfz; the layer's
// lane 0 also writes the column plane entry {terrain = column DEM (+0 for nodata = sea),
// NFZ | MASK | NODATA flags}.  BELOW_TERRAIN is not stored: the evaluation derives it from the
// layer centre z0 + (iz + 0.5) dz and the column's terrain.
__global__ __launch_bounds__(256) void k_volume_build(const uint4* __restrict__ rec2, int nx,
                                                      int ny, int nz,
                                                      const double* __restrict__ layer_w,
                                                      uint2* __restrict__ vox,
                                                      uint2* __restrict__ col) {
    const int64_t total = (int64_t)nx * ny * nz;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < total;
         v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = v / nz;
        const int iz = (int)(v - c * nz);
        const uint4 r = rec2[c];
        const float risk = (float)((double)__uint_as_float(r.x) * layer_w[iz]);
        vox[v] = make_uint2(__float_as_uint(risk), r.y);
        if (iz == 0) {
            const uint32_t terrain = (r.w & UAM_FLAG_NODATA) ? 0u : r.z;  // +0.0f bits
            col[c] = make_uint2(terrain, r.w & (UAM_FLAG_NFZ | UAM_FLAG_MASK | UAM_FLAG_NODATA));
        }
    }
}

// a volume waypoint's voxel and column (in: inside the volume); r = {risk, psi, terrain, flags}.
// With the column bitmap (sbits, in LDS) a column of a clear block is not read: it is
// {+0.0f, 0} by the bitmap's definition, so every output is the same.
__device__ __forceinline__ uint4 vol_fetch(const KVolume& vs, const uint32_t* sbits, double x0,
                                           double x1, double z, bool& in, int64_t& v) {
    const double fx = floor((x0 - vs.x0) * vs.inv_dx);
    const double fy = floor((vs.y_top - x1) * vs.inv_dy);
    const double fz = floor((z - vs.z0) * vs.inv_dz);
    in = (fx >= 0.0) && (fx < (double)vs.nx) && (fy >= 0.0) && (fy < (double)vs.ny) &&
         (fz >= 0.0) && (fz < (double)vs.nz);
    const int32_t ix = in ? (int32_t)fx : 0, iy = in ? (int32_t)fy : 0;
    const int64_t c = (int64_t)iy * vs.nx + ix;
    v = c * vs.nz + (in ? (int64_t)fz : (int64_t)0);
    const uint2 a = vs.vox[v];
    uint2 b = make_uint2(0u, 0u);
    const int32_t blk = (iy >> vs.cshift) * vs.cnbx + (ix >> vs.cshift);
    if (!sbits || ((sbits[blk >> 5] >> (blk & 31)) & 1u)) b = vs.col[c];
    return make_uint4(a.x, a.y, b.x, b.y);
}

// the column bitmap: one lane per block of 2^shift x 2^shift columns, set when a column of it
// has terrain bits != +0.0f or the no-fly flag; the wave's ballot gives two words
__global__ __launch_bounds__(256) void k_volume_colbits(const uint2* __restrict__ col, int nx,
                                                        int ny, int shift, int nbx, int n_blocks,
                                                        int n_words, uint32_t* __restrict__ out) {
    const int32_t blk = blockIdx.x * blockDim.x + threadIdx.x;
    bool need = false;
    if (blk < n_blocks) {
        const int bx = blk % nbx, by = blk / nbx;
        const int x0 = bx << shift, y0 = by << shift;
        const int x1 = min(x0 + (1 << shift), nx), y1 = min(y0 + (1 << shift), ny);
        for (int iy = y0; iy < y1 && !need; ++iy)
            for (int ix = x0; ix < x1; ++ix) {
                const uint2 c = col[(int64_t)iy * nx + ix];
                if (c.x != 0u || (c.y & UAM_FLAG_NFZ)) {
                    need = true;
                    break;
                }
            }
    }
    const uint64_t m = __ballot(need);
    const int lane = threadIdx.x & 63;
    const int32_t w0 = (blk - lane) >> 5;  // the wave's first block is a multiple of 64
    if (lane == 0 && w0 < n_words) out[w0] = (uint32_t)m;
    if (lane == 32 && w0 + 1 < n_words) out[w0 + 1] = (uint32_t)(m >> 32);
}

// below the column's terrain: the layer centre z0 + (iz + 0.5) dz of altitude z
__device__ __forceinline__ bool vol_below(const KVolume& vs, double z, uint32_t terrain_bits) {
    const double fz = floor((z - vs.z0) * vs.inv_dz);
    const double hc = vs.z0 + (fz + 0.5) * vs.dz;
    return hc < (double)__uint_as_float(terrain_bits);
}

// candidate point k (1..N) of pair pr: solver.py:121-136 restated as
// p = C + 0.5*[[vx,-vy],[vy,vx]] u, v = x0 - xf, C = (xf + x0)/2
__device__ __forceinline__ void arc_point(double x0, double y0, double xf, double yf, double ux,
                                          double uy, double& px, double& py) {
    const double vx = x0 - xf, vy = y0 - yf;
    const double cx = (xf + x0) * 0.5, cy = (yf + y0) * 0.5;
    px = cx + 0.5 * (vx * ux - vy * uy);
    py = cy + 0.5 * (vy * ux + vx * uy);
}

// Source of a path's waypoints: explicit [P][W][2] or generated from (pair, u[d]).
template <bool GEN>
struct PathSrc {
    const double* __restrict__ wp;  // explicit: this path's W points
    double x0, y0, xf, yf;          // generated: the pair
    const double* __restrict__ u;   // generated: u[d][0..N-1][2] (wave-uniform address)
    double za, zb;                  // volume mode: altitude at p_0 and p_{N+1} (m)
    int W;
    // volume mode altitude profile: z_j = za + (zb - za) * (j / (N+1))
    __device__ __forceinline__ double alt(int j) const {
        return za + (zb - za) * ((double)j / (double)(W - 1));
    }
    __device__ __forceinline__ void at(int j, double& px, double& py) const {
        if (GEN) {
            if (j == 0) {
                px = x0;
                py = y0;
            } else if (j == W - 1) {
                px = xf;
                py = yf;
            } else {
                arc_point(x0, y0, xf, yf, u[2 * (j - 1)], u[2 * (j - 1) + 1], px, py);
            }
        } else {
            const double2 v = reinterpret_cast<const double2*>(wp)[j];
            px = v.x;
            py = v.y;
        }
    }
};

// Per-path results, in the reference's summation order (see eval_path).
struct PathAcc {
    double cost, L, len, ksum, nsum, hmax, cmin;
    int32_t nh, off, below;
};

// Gathers of one chunk of C consecutive waypoints (issued together, consumed together).
template <int C>
struct Chunk {
    uint4 r[C];
    bool in[C];
};

template <bool GEN, int C>
__device__ __forceinline__ void issue_chunk(const KRaster& rs, const uint4* __restrict__ rec,
                                            const PathSrc<GEN>& src, int j0, int W,
                                            int32_t* cells, Chunk<C>& ch) {
#pragma unroll
    for (int t = 0; t < C; ++t) {
        const int j = j0 + t;
        ch.in[t] = false;
        ch.r[t] = make_uint4(0, 0, 0, 0);
        if (j < W) {
            double x0, x1;
            src.at(j, x0, x1);
            // uampath.h raster convention: float64 floor of the scaled offset
            const double fx = floor((x0 - rs.x0) * rs.inv_dx);
            const double fy = floor((rs.y_top - x1) * rs.inv_dy);
            const bool in = (fx >= 0.0) && (fx < (double)rs.nx) && (fy >= 0.0) &&
                            (fy < (double)rs.ny);
            const int64_t cell = in ? (int64_t)fy * rs.nx + (int64_t)fx : (int64_t)0;
            ch.in[t] = in;
            ch.r[t] = rec[cell];  // unconditional: off-raster lanes read cell 0 (cached)
            if (cells) cells[j] = in ? (int32_t)cell : -1;
        }
    }
}

template <int C>
__device__ __forceinline__ void consume_chunk(const Chunk<C>& ch, int j0, int W, double dN,
                                              PathAcc& a) {
#pragma unroll
    for (int t = 0; t < C; ++t) {
        if (j0 + t >= W) break;
        if (!ch.in[t]) {
            ++a.off;
            a.hmax = fmax(a.hmax, 0.0);  // off-raster counts as sea level
            continue;
        }
        a.cost = a.cost + (double)__uint_as_float(ch.r[t].x) / dN;
        a.nsum = a.nsum + (double)__uint_as_float(ch.r[t].y);
        a.nh += (ch.r[t].w & UAM_FLAG_NFZ) ? 1 : 0;
        const double terrain =
            (ch.r[t].w & UAM_FLAG_NODATA) ? 0.0 : (double)__uint_as_float(ch.r[t].z);
        a.hmax = fmax(a.hmax, terrain);
    }
}

// ---- K2 gather skip (uam_raster_summary; build-defined, no reference counterpart) --------
// A bitmap with one bit per B x B cell block, set when every cell of the block has phi == +-0,
// psi == +-0, no no-fly flag and a terrain that reads +0.0 (a nodata cell, as consume_chunk
// reads it, or a DEM value of +0.0f: open sea).  A waypoint in a set block adds exactly nothing
// to the cost and no-fly sums (x + (+-0) == x for every accumulator, none of which is ever -0)
// and nothing to nfz_hits, and its terrain is exactly +0.0, so the path maximum takes
// fmax(hmax, +0.0) with no memory request.  K2 holds the bitmap in LDS (<= 8 KiB), so the test
// costs no memory request either; it gathers only the other waypoints.  Every output is
// bit-identical to gathering every waypoint.  (Round 2's first form also set the bit over
// terrain < 0 and re-fetched the skipped records of paths whose gathered maximum stayed < 0;
// those re-walks cost K2s 50-60 us per cfg3 launch and are gone with the +0.0 rule.)
constexpr int SKIP_MAX_BITS = 65536;  // 8 KiB of LDS

// raster cell of a point (uampath.h convention: float64 floor of the scaled offset; -1 off the
// raster) and whether its block's bit is set (false off the raster)
__device__ __forceinline__ int32_t raster_cell_skip(const KRaster& rs, const uint32_t* bits,
                                                   double x0, double x1, bool& skip) {
    const double fx = floor((x0 - rs.x0) * rs.inv_dx);
    const double fy = floor((rs.y_top - x1) * rs.inv_dy);
    skip = false;
    if (!((fx >= 0.0) && (fx < (double)rs.nx) && (fy >= 0.0) && (fy < (double)rs.ny))) return -1;
    const int32_t ix = (int32_t)fx, iy = (int32_t)fy;
    const int32_t b = (iy >> rs.sshift) * rs.snbx + (ix >> rs.sshift);
    skip = (bits[b >> 5] >> (b & 31)) & 1u;
    return iy * rs.nx + ix;
}

// Pass 2 of a raster path with the gather skip (bits: the bitmap in LDS); chunks of 8 gathers
// in flight, consumed in waypoint order exactly as consume_chunk does.  (Compacting each chunk
// to the lane's next 8 needed waypoints measured 3x slower: the per-slot forward scans
// diverge.)
// (chunks of 4-16 at 4-8 waves per SIMD measured 4-36% slower on cfg3, r02)
constexpr int SKIP_CHUNK = 8;  // gathers per chunk
constexpr int SKIP_MINW = 5;   // waves per SIMD the skip kernel is compiled for (6 spills)
template <bool GEN>
__device__ __forceinline__ void raster_pass2_skip(const KRaster& rs, const uint4* __restrict__ rec,
                                                  const uint32_t* bits, const PathSrc<GEN>& src,
                                                  int W, int32_t* cells, double dN, PathAcc& a) {
    constexpr int CH = SKIP_CHUNK;
    for (int j0 = 0; j0 < W; j0 += CH) {
        uint4 r[CH];
        uint32_t inb = 0, need = 0;
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            if (j0 + t < W) {
                double x0, x1;
                src.at(j0 + t, x0, x1);
                bool sk;
                const int32_t cl = raster_cell_skip(rs, bits, x0, x1, sk);
                if (cells) cells[j0 + t] = cl;
                if (cl >= 0) {
                    inb |= 1u << t;
                    if (!sk) {
                        need |= 1u << t;
                        r[t] = rec[cl];
                    }
                }
            }
        }
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            if (j0 + t >= W) break;
            if (!((inb >> t) & 1u)) {
                ++a.off;
                a.hmax = fmax(a.hmax, 0.0);  // off-raster counts as sea level
                continue;
            }
            if (!((need >> t) & 1u)) {  // phi, psi +-0 (exact no-ops), terrain +0.0
                a.hmax = fmax(a.hmax, 0.0);
                continue;
            }
            a.cost = a.cost + (double)__uint_as_float(r[t].x) / dN;
            a.nsum = a.nsum + (double)__uint_as_float(r[t].y);
            a.nh += (r[t].w & UAM_FLAG_NFZ) ? 1 : 0;
            const double terrain =
                (r[t].w & UAM_FLAG_NODATA) ? 0.0 : (double)__uint_as_float(r[t].z);
            a.hmax = fmax(a.hmax, terrain);
        }
    }
}

// one thread per B x B block (B = 2^shift, row-major blocks); bit b of word b / 32
__global__ __launch_bounds__(256) void k_raster_summary(const uint4* __restrict__ rec, int32_t nx,
                                                        int32_t ny, int32_t shift, int32_t nbx,
                                                        int32_t n_blocks,
                                                        uint32_t* __restrict__ out) {
    const int32_t blk = blockIdx.x * blockDim.x + threadIdx.x;
    bool skip = false;
    if (blk < n_blocks) {
        const int B = 1 << shift;
        const int bx = blk % nbx, by = blk / nbx;
        const int x0 = bx << shift, y0 = by << shift;
        const int x1 = min(x0 + B, (int)nx), y1 = min(y0 + B, (int)ny);
        skip = true;
        for (int iy = y0; iy < y1 && skip; ++iy)
            for (int ix = x0; ix < x1; ++ix) {
                const uint4 r = rec[(int64_t)iy * nx + ix];
                const uint32_t t = (r.w & UAM_FLAG_NODATA) ? 0u : r.z;  // +0.0f bits
                if ((r.x & 0x7fffffffu) || (r.y & 0x7fffffffu) || (r.w & UAM_FLAG_NFZ) || t) {
                    skip = false;
                    break;
                }
            }
    }
    const uint64_t m = __ballot(skip);
    const int lane = threadIdx.x & 63;
    const int32_t w = blk >> 5;  // lanes 0 and 32 write the wave's two words
    if ((lane & 31) == 0 && blk < n_blocks)
        out[w] = (uint32_t)(lane ? (m >> 32) : m);
}

// the same bits with one wave per block (blocks of >= 8 x 8 cells): the wave reads the block's
// rows as coalesced runs of min(B, 64) records, stops at the first row step with a non-skippable
// cell, and lane 0 sets the block's bit (the words zeroed by the caller).  The thread-per-block
// kernel above reads each lane's block serially, 16 B at a stride of B records across the lanes.
__global__ __launch_bounds__(256) void k_raster_summary_w(const uint4* __restrict__ rec,
                                                          int32_t nx, int32_t ny, int32_t shift,
                                                          int32_t nbx, int32_t n_blocks,
                                                          uint32_t* __restrict__ out) {
    const int32_t blk = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    if (blk >= n_blocks) return;
    const int lane = threadIdx.x & 63;
    const int B = 1 << shift, lpr = B < 64 ? B : 64, rpi = 64 / lpr;
    const int bx = blk % nbx, by = blk / nbx;
    const int x0 = bx << shift, y0 = by << shift;
    const int x1 = min(x0 + B, (int)nx), y1 = min(y0 + B, (int)ny);
    const int lc = lane & (lpr - 1), lr = lane / lpr;
    bool skip = true;
    for (int r0 = y0; r0 < y1 && skip; r0 += rpi) {
        bool bad = false;
        const int iy = r0 + lr;
        for (int c0 = x0; c0 < x1; c0 += lpr) {
            const int ix = c0 + lc;
            if (iy < y1 && ix < x1) {
                const uint4 r = rec[(int64_t)iy * nx + ix];
                const uint32_t t = (r.w & UAM_FLAG_NODATA) ? 0u : r.z;  // +0.0f bits
                bad = bad || (r.x & 0x7fffffffu) || (r.y & 0x7fffffffu) ||
                      (r.w & UAM_FLAG_NFZ) || t;
            }
        }
        skip = __ballot(bad) == 0;
    }
    if (skip && lane == 0) atomicOr(out + (blk >> 5), 1u << (blk & 31));
}

// ---- Packed raster (uam_raster_pack; build-defined, no reference counterpart) --------------
// The sorted forms are bound by 128-B lines; a 16-B record uses one eighth of its line, and most
// waypoints need less of it.  The packed copy (layout: PackDims) keeps what each block needs in
// the narrowest entry, with a 2-bit code per summary block saying which one a waypoint reads:
//   0  nothing: every cell has phi == +-0, psi == +-0, no no-fly flag and a terrain that reads
//      +0.0 (the phi and psi terms are exact no-ops on accumulators that are never -0, the hit
//      count adds 0, the terrain is exactly +0.0);
//   1  the 4-B phi plane p4 (psi == +-0 and no flag over the block), 32 cells per line;
//   2  the 8-B plane e8 {phi, |psi| with the no-fly flag in the sign bit}, 16 cells per line:
//      every psi of the block is >= +0 or -0 (its decoded +0 adds exactly what -0 adds);
//   3  the whole 16-B record from rec (a psi of the block is negative or a sign-bit NaN).
// The terrain (as the evaluation reads it: +0.0 on a nodata cell) is out of codes 0-2: it feeds
// only the order-free path maximum, so K2h fetches it from the 4-B plane t4 only for waypoints
// whose block's upper bound could still be that maximum (h_item), and the forms without the
// bound rule read t4 for every in-raster waypoint outside code 3.  Bounds: per bound block
// (2^bshift cells square) a u16 {ub code, lb code << 8}, decoded ub = base + q * step in f32
// (the superblock's {base, step}, step a power of two, so q * step is exact and the sum rounds
// once, the same operations here and in the kernels); every cell's terrain lies in [lb, ub].  A
// superblock holding a non-finite terrain value stores {NaN, NaN}: its bounds decode to NaN,
// which the evaluation reads as "no bound" (always fetched, no lower bound).
constexpr int PK_BOUND_MAX = 16384;  // bound blocks at most (32 KiB of u16 in LDS)

// (index products by 24-bit multiplies, full rate: cells and block counts are < 2^24,
// uam_raster_pack's limits)
__device__ __forceinline__ int32_t p4_addr(const KRaster& rs, int32_t ix, int32_t iy) {
    return (int32_t)(((__umul24((uint32_t)(iy >> 2), (uint32_t)rs.nb8) + (uint32_t)(ix >> 3)) << 5) |
                     (((uint32_t)iy & 3u) << 3) | ((uint32_t)ix & 7u));
}

// p8's index: 4 x 4-cell blocks (16 entries of 8 B, one 128-B line, a square of cells)
__device__ __forceinline__ int32_t p44_addr(const KRaster& rs, int32_t ix, int32_t iy) {
    return (int32_t)(((__umul24((uint32_t)(iy >> 2), (uint32_t)rs.nb4) + (uint32_t)(ix >> 2)) << 4) |
                     (((uint32_t)iy & 3u) << 2) | ((uint32_t)ix & 3u));
}

// the summary-block index of cell (ix, iy) (its 2-bit code: word b >> 4, bits 2 (b & 15))
__device__ __forceinline__ int32_t pk_block(const KRaster& rs, int32_t ix, int32_t iy) {
    return (int32_t)(__umul24((uint32_t)(iy >> rs.sshift), (uint32_t)rs.snbx) +
                     (uint32_t)(ix >> rs.sshift));
}

// the bound entry (u16) and superblock {base, step} of cell (ix, iy) from a header copy
__device__ __forceinline__ void pk_bound_raw(const KRaster& rs, const uint32_t* __restrict__ hdr,
                                             int32_t ix, int32_t iy, uint32_t& e, float2& sb) {
    const uint32_t bx = (uint32_t)(ix >> rs.bshift), by = (uint32_t)(iy >> rs.bshift);
    e = reinterpret_cast<const uint16_t*>(hdr + rs.bnd_off)[__umul24(by, (uint32_t)rs.bnbx) + bx];
    sb = reinterpret_cast<const float2*>(hdr + rs.sbt_off)[__umul24(by >> 2, (uint32_t)rs.sbnbx) +
                                                           (bx >> 2)];
}

// decode: base + q * step with q * step exact (step a power of two), so the fused form rounds
// once exactly as the separate one (k_raster_bounds' check)
__device__ __forceinline__ void pk_bound_decode(uint32_t e, float2 sb, float& ub, float& lb) {
    ub = fmaf((float)(e & 255u), sb.y, sb.x);
    lb = fmaf((float)(e >> 8), sb.y, sb.x);
}

// the raster cell of a generated point (arc_point's or the pair's coordinates; uampath.h's float64
// floor): false off the raster or NaN, with (ix, iy) = (0, 0) then (a valid header index)
__device__ __forceinline__ bool gen_cell_g(double gx0, double gy_top, double inv_dx,
                                           double inv_dy, int32_t nx, int32_t ny, double x0,
                                           double x1, int32_t& ix, int32_t& iy) {
    const double tx = (x0 - gx0) * inv_dx;
    const double ty = (gy_top - x1) * inv_dy;
    // (bitwise: no short-circuit branches)
    const bool in = (tx >= 0.0) & (tx < (double)nx) & (ty >= 0.0) & (ty < (double)ny);
    ix = in ? (int32_t)tx : 0;
    iy = in ? (int32_t)ty : 0;
    return in;
}

__device__ __forceinline__ bool gen_cell(const KRaster& rs, double x0, double x1, int32_t& ix,
                                         int32_t& iy) {
    return gen_cell_g(rs.x0, rs.y_top, rs.inv_dx, rs.inv_dy, rs.nx, rs.ny, x0, x1, ix, iy);
}

// a chunk's per-slot entry kinds: the code (2 bits) and the cell's first component in the
// aligned 16 B (sub, 2 bits), one bit mask per bit so the consume selects components with
// independent conditions (a select on bits of one index folds into a dynamic vector index,
// which put the chunk's loads in scratch memory)
struct PkSlots {
    uint32_t c0 = 0, c1 = 0, s0 = 0, s1 = 0;
    __device__ __forceinline__ void set(int t, uint32_t v) {  // v = code | sub << 2
        c0 |= (v & 1u) << t;
        c1 |= ((v >> 1) & 1u) << t;
        s0 |= ((v >> 2) & 1u) << t;
        s1 |= ((v >> 3) & 1u) << t;
    }
};
#define PK_CODES_CHECK(CH) static_assert((CH) <= 32, "one bit per slot in 32")

// spread the 16 low bits of v to the even bits of the result
__device__ __forceinline__ uint32_t spread16(uint32_t v) {
    v &= 0xffffu;
    v = (v | (v << 8)) & 0x00ff00ffu;
    v = (v | (v << 4)) & 0x0f0f0f0fu;
    v = (v | (v << 2)) & 0x33333333u;
    v = (v | (v << 1)) & 0x55555555u;
    return v;
}

// the generic reads of an in-raster waypoint (the forms without the bound rule: K2s+pack, K2g):
// its value entry vp (rec in code 3, the aligned 16 B of e8 / p4 holding its cell in codes 2 / 1,
// left at the caller's dummy line in code 0) and its terrain tp (t4 outside code 3, left at the
// caller's dummy otherwise); returns cs = code | sub << 2 for pk_terms (sub: the cell's first
// component in the 16 B)
__device__ __forceinline__ uint32_t pk_locate(const KRaster& rs, const uint4* __restrict__ rec,
                                              const uint32_t* __restrict__ map, int32_t ix,
                                              int32_t iy, const uint4*& vp, const float*& tp) {
    const int32_t b = pk_block(rs, ix, iy);
    const uint32_t code = (map[b >> 4] >> ((b & 15) * 2)) & 3u;
    if (code == 3u) {
        vp = rec + (iy * rs.nx + ix);
        return 3u;
    }
    const int32_t a4 = p4_addr(rs, ix, iy);
    tp = rs.t4 + a4;
    uint32_t sub = 0;
    if (code == 2u) {
        vp = reinterpret_cast<const uint4*>(rs.e8 + (a4 & ~1));
        sub = (uint32_t)(a4 & 1) * 2u;
    } else if (code == 1u) {
        vp = reinterpret_cast<const uint4*>(rs.p4 + (a4 & ~3));
        sub = (uint32_t)(a4 & 3);
    }
    return code | (sub << 2);
}

// the terms of slot t's located waypoint from its 16 B r: phi and psi bits (+0 where the code
// holds none), the no-fly hit, and the record's terrain as read (meaningful in code 3 only)
__device__ __forceinline__ void pk_terms(const uint4& r, const PkSlots& k, int t, uint32_t& phi,
                                         uint32_t& psi, uint32_t& hit, float& rter) {
    const bool c0 = (k.c0 >> t) & 1u, c1 = (k.c1 >> t) & 1u;
    const bool s0 = (k.s0 >> t) & 1u, s1 = (k.s1 >> t) & 1u;
    const uint32_t lo = s0 ? r.y : r.x, hi = s0 ? r.w : r.z;
    phi = (c0 || c1) ? (s1 ? hi : lo) : 0u;
    // psi and the flag: code 2 at its cell's second word (sub 0 or 2), code 3 the record's y
    const uint32_t praw = c1 ? (s1 ? r.w : r.y) : 0u;
    psi = (c1 && !c0) ? (praw & 0x7fffffffu) : praw;
    hit = (c1 && !c0) ? (praw >> 31) : (c1 && c0 && (r.w & UAM_FLAG_NFZ)) ? 1u : 0u;
    rter = (r.w & UAM_FLAG_NODATA) ? 0.0f : __uint_as_float(r.z);
}

// pk_terms of one slot's kind word k = code | word << 2 (K2h: one register per slot)
__device__ __forceinline__ void pk_terms_k(const uint4& r, uint32_t k, uint32_t& phi,
                                           uint32_t& psi, uint32_t& hit, float& rter) {
    PkSlots s;
    s.set(0, k);
    pk_terms(r, s, 0, phi, psi, hit, rter);
}

// one thread per cell, rows coalesced: the five planes at their blocked addresses (e8 and r16
// are written everywhere, read only in code-2 / code-3 blocks; p8 {phi, terrain as read} only
// by K2h's terrain-in-entry form)
__global__ __launch_bounds__(256) void k_raster_pack(const uint4* __restrict__ rec, KRaster rs,
                                                     uint32_t* __restrict__ p4,
                                                     float* __restrict__ t4,
                                                     uint2* __restrict__ e8,
                                                     uint4* __restrict__ r16,
                                                     uint2* __restrict__ p8) {
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= (int64_t)rs.nx * rs.ny) return;
    const int32_t iy = (int32_t)(c / rs.nx), ix = (int32_t)(c - (int64_t)iy * rs.nx);
    const uint4 r = rec[c];
    const int32_t a4 = p4_addr(rs, ix, iy);
    p4[a4] = r.x;
    t4[a4] = (r.w & UAM_FLAG_NODATA) ? 0.0f : __uint_as_float(r.z);
    e8[a4] =
        make_uint2(r.x, (r.y & 0x7fffffffu) | ((r.w & UAM_FLAG_NFZ) ? 0x80000000u : 0u));
    r16[a4] = r;
    p8[p44_addr(rs, ix, iy)] = make_uint2(r.x, (r.w & UAM_FLAG_NODATA) ? 0u : r.z);
}

// one thread per summary block: its 2-bit code; lanes 0/16/32/48 write the wave's 4 words
__global__ __launch_bounds__(256) void k_raster_pack_map(const uint4* __restrict__ rec,
                                                         int32_t nx, int32_t ny, int32_t shift,
                                                         int32_t nbx, int32_t n_blocks,
                                                         uint32_t* __restrict__ out) {
    const int32_t blk = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t code = 0;
    if (blk < n_blocks) {
        const int B = 1 << shift;
        const int bx = blk % nbx, by = blk / nbx;
        const int x0 = bx << shift, y0 = by << shift;
        const int x1 = min(x0 + B, (int)nx), y1 = min(y0 + B, (int)ny);
        bool need = false, neg = false, nz = false;
        for (int iy = y0; iy < y1; ++iy)
            for (int ix = x0; ix < x1; ++ix) {
                const uint4 r = rec[(int64_t)iy * nx + ix];
                if ((r.y & 0x7fffffffu) || (r.w & UAM_FLAG_NFZ)) need = true;
                if ((r.y >> 31) && r.y != 0x80000000u) neg = true;  // negative, or a -NaN
                // a phi to add, or a terrain other than +0.0 as read
                if ((r.x & 0x7fffffffu) || ((r.w & UAM_FLAG_NODATA) ? 0u : r.z)) nz = true;
            }
        code = need ? (neg ? 3u : 2u) : nz ? 1u : 0u;
    }
    const uint64_t lo = __ballot(code & 1u), hi = __ballot(code >> 1);
    const int lane = threadIdx.x & 63;
    if ((lane & 15) == 0 && blk < n_blocks) {
        const int sh = lane;  // this lane's 16 blocks are bits [lane, lane + 16) of the ballots
        out[blk >> 4] = spread16((uint32_t)(lo >> sh)) | (spread16((uint32_t)(hi >> sh)) << 1);
    }
}

// the same codes with one wave per block (blocks of >= 8 x 8 cells): coalesced runs of the
// block's rows, a stop once a negative psi decides code 3, lane 0 ORs the code into the map
// (zeroed by uam_raster_pack's memset)
__global__ __launch_bounds__(256) void k_raster_pack_map_w(const uint4* __restrict__ rec,
                                                           int32_t nx, int32_t ny, int32_t shift,
                                                           int32_t nbx, int32_t n_blocks,
                                                           uint32_t* __restrict__ out) {
    const int32_t blk = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    if (blk >= n_blocks) return;
    const int lane = threadIdx.x & 63;
    const int B = 1 << shift, lpr = B < 64 ? B : 64, rpi = 64 / lpr;
    const int bx = blk % nbx, by = blk / nbx;
    const int x0 = bx << shift, y0 = by << shift;
    const int x1 = min(x0 + B, (int)nx), y1 = min(y0 + B, (int)ny);
    const int lc = lane & (lpr - 1), lr = lane / lpr;
    bool need = false, neg = false, nz = false;
    for (int r0 = y0; r0 < y1 && !neg; r0 += rpi) {
        const int iy = r0 + lr;
        for (int c0 = x0; c0 < x1; c0 += lpr) {
            const int ix = c0 + lc;
            if (iy < y1 && ix < x1) {
                const uint4 r = rec[(int64_t)iy * nx + ix];
                need = need || (r.y & 0x7fffffffu) || (r.w & UAM_FLAG_NFZ);
                neg = neg || ((r.y >> 31) && r.y != 0x80000000u);  // negative, or a -NaN
                nz = nz || (r.x & 0x7fffffffu) || ((r.w & UAM_FLAG_NODATA) ? 0u : r.z);
            }
        }
        neg = __ballot(neg) != 0;
    }
    need = __ballot(need) != 0;
    nz = __ballot(nz) != 0;
    const uint32_t code = need ? (neg ? 3u : 2u) : nz ? 1u : 0u;
    if (code && lane == 0) atomicOr(out + (blk >> 4), code << ((blk & 15) * 2));
}

// one wave per bound block: {min, max} of its terrain as read, from the 4-B terrain plane (4 x 8-
// cell blocks, nb8 per row: the raster's t4, the volume's column terrain); min = NaN when the
// block holds a non-finite value
__global__ __launch_bounds__(256) void k_t4_bminmax(const float* __restrict__ t4, int32_t nx,
                                                    int32_t ny, int32_t nb8, int32_t bshift,
                                                    int32_t bnbx, int32_t nbb,
                                                    float2* __restrict__ scr) {
    const int32_t blk = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (blk >= nbb) return;  // (whole waves)
    const int B = 1 << bshift;
    const int bx = blk % bnbx, by = blk / bnbx;
    const int x0 = bx << bshift, y0 = by << bshift;
    const int w = min(B, nx - x0), h = min(B, ny - y0);
    float mn = INFINITY, mx = -INFINITY;
    bool bad = false;
    for (int k = lane; k < w * h; k += 64) {
        const int iy = y0 + k / w, ix = x0 + k % w;
        const float t = t4[((((iy >> 2) * nb8 + (ix >> 3)) << 5) | ((iy & 3) << 3) | (ix & 7))];
        if (!__builtin_isfinite(t)) bad = true;
        mn = fminf(mn, t);
        mx = fmaxf(mx, t);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, o));
        mx = fmaxf(mx, __shfl_xor(mx, o));
    }
    bad = __any(bad);
    if (lane == 0) scr[blk] = make_float2(bad ? __builtin_nanf("") : mn, mx);
}

// one thread per bound block: its superblock's {base, step} from the members' {min, max} (every
// member forms the same ones; the member at (0, 0) stores them) and its own u16 codes
__global__ __launch_bounds__(256) void k_raster_bounds(const float2* __restrict__ scr,
                                                       int32_t bnbx, int32_t bnby,
                                                       int32_t sbnbx,
                                                       uint16_t* __restrict__ bnd,
                                                       float2* __restrict__ sbt) {
    const int32_t blk = blockIdx.x * 256 + threadIdx.x;
    if (blk >= bnbx * bnby) return;
    const int bx = blk % bnbx, by = blk / bnbx;
    const int sx = bx >> 2, sy = by >> 2;
    float base = INFINITY, top = -INFINITY;
    bool bad = false;
    for (int yy = sy * 4; yy < min(sy * 4 + 4, bnby); ++yy)
        for (int xx = sx * 4; xx < min(sx * 4 + 4, bnbx); ++xx) {
            const float2 m = scr[yy * bnbx + xx];
            if (!(m.x == m.x)) bad = true;
            base = fminf(base, m.x);
            top = fmaxf(top, m.y);
        }
    float step = 1.0f;
    if (!bad) {  // the smallest power of two with (top - base) / step <= 253 (2 codes of margin)
        const double range = (double)top - (double)base;
        int e = -126;
        while (e < 127 && ldexp(253.0, e) < range) ++e;
        step = ldexpf(1.0f, e);
    }
    const bool lead = ((bx & 3) == 0) && ((by & 3) == 0);
    if (bad) {
        if (lead) sbt[sy * sbnbx + sx] = make_float2(__builtin_nanf(""), __builtin_nanf(""));
        bnd[blk] = 0;
        return;
    }
    if (lead) sbt[sy * sbnbx + sx] = make_float2(base, step);
    const float2 m = scr[blk];
    // the kernels' decode: base + (float)q * step (q * step exact, one rounding)
    int qu = (int)ceil(((double)m.y - (double)base) / (double)step);
    qu = min(max(qu, 0), 255);
    while (qu < 255 && base + (float)qu * step < m.y) ++qu;
    int ql = (int)floor(((double)m.x - (double)base) / (double)step);
    ql = min(max(ql, 0), 255);
    while (ql > 0 && base + (float)ql * step > m.x) --ql;
    bnd[blk] = (uint16_t)(qu | (ql << 8));
}

// Raster mode with the gather skip (internal; KRaster::sum set, raster_pass2_skip): its own
// kernel instantiation, so the plain raster kernel keeps its register budget.
constexpr int MODE_RASTER_SKIP = 4;

// Volume mode (BASELINE config 5, no reference counterpart): the waypoint's voxel
// (ix, iy as in raster mode, iz = floor((z - z0) / dz)) holds {risk f32, psi_nfz f32} (risk
// already carries the altitude-layer weight) and its column {terrain f32, flags}.
template <bool GEN, int C>
__device__ __forceinline__ void issue_chunk_vol(const KVolume& vs, const uint32_t* sbits,
                                                const PathSrc<GEN>& src, int j0, int W,
                                                int32_t* cells, Chunk<C>& ch) {
#pragma unroll
    for (int t = 0; t < C; ++t) {
        const int j = j0 + t;
        ch.in[t] = false;
        ch.r[t] = make_uint4(0, 0, 0, 0);
        if (j < W) {
            double x0, x1;
            src.at(j, x0, x1);
            bool in;
            int64_t v;
            ch.r[t] = vol_fetch(vs, sbits, x0, x1, src.alt(j), in, v);
            ch.in[t] = in;
            if (cells) cells[j] = in ? (int32_t)v : -1;
        }
    }
}

template <bool GEN, int C>
__device__ __forceinline__ void consume_chunk_vol(const KVolume& vs, const Chunk<C>& ch,
                                                  const PathSrc<GEN>& src, int j0, int W,
                                                  double dN, PathAcc& a) {
#pragma unroll
    for (int t = 0; t < C; ++t) {
        const int j = j0 + t;
        if (j >= W) break;
        if (!ch.in[t]) {
            ++a.off;
            continue;
        }
        a.cost = a.cost + (double)__uint_as_float(ch.r[t].x) / dN;
        a.nsum = a.nsum + (double)__uint_as_float(ch.r[t].y);
        a.nh += (ch.r[t].w & UAM_FLAG_NFZ) ? 1 : 0;
        const double z = src.alt(j);
        a.below += vol_below(vs, z, ch.r[t].z) ? 1 : 0;
        a.cmin = fmin(a.cmin, z - (double)__uint_as_float(ch.r[t].z));
    }
}

// Kinematic row k of problem.py:100-107 from the norms pn, nk of segments k and k + 1 (the
// squared norms when maxratio_smooth) and their dot product dt:
//   c1 = max(0, nk - r pn), c2 = max(0, pn / r - nk), c3 = max(0, mincos - dt / (pn nk)).
// The two f64 divisions (~10 VALU instructions each) are skipped where their outcome is
// provably +0, which is every row of a path that keeps to the ratio and turn limits:
//   c2: t = RN(nk r); pn <= RN(t (1 - 2^-50)) implies pn < nk r exactly, so pn / r < nk,
//       RN(pn / r) <= nk and the difference is <= 0: c2 = +0;
//   c3: q = RN(pn nk) in [1e-200, 1e200], mincos > 1e-100, dt >= RN(RN(mincos q) (1 + 2^-50))
//       implies dt > mincos q exactly, so RN(dt / q) >= mincos and c3 = +0.
// (RN's relative error is <= 2^-53 in that range, well inside the 2^-50 margins.)  Otherwise
// the formula runs as written; NaN and infinite operands fail both tests.  Every value is
// bit-identical to the plain formula.
__device__ __forceinline__ void kin_row(const KParams& p, double pn, double nk, double dt,
                                        double& c1, double& c2, double& c3) {
    c1 = fmax(0.0, nk - p.r_eff * pn);
    const double t2 = nk * p.r_eff;
    c2 = (pn <= t2 * (1.0 - 0x1p-50)) ? 0.0 : fmax(0.0, pn / p.r_eff - nk);
    const double q = pn * nk;
    bool fast3 = false;
    if (q >= 1e-200 && q <= 1e200 && p.mincos > 1e-100) {
        const double t3 = p.mincos * q;
        fast3 = dt >= t3 * (1.0 + 0x1p-50);
    }
    c3 = fast3 ? 0.0 : fmax(0.0, p.mincos - dt / q);
}

// Pass 1 of a path: get_cost's length term L (problem.py:130-146 with the quirk), the true
// length (length_of, solver.py:49) and the sum of the 3N kinematic rows (problem.py:100-107),
// optionally storing the rows.  Shared by every path kernel, so their bits agree.
template <bool GEN>
__device__ __forceinline__ void path_pass1(const KParams& p, const PathSrc<GEN>& src,
                                           double* grow, PathAcc& a) {
    const int N = p.N, W = N + 2;
    const bool ls = p.length_smooth != 0, ms = p.maxratio_smooth != 0;
    double px, py;
    src.at(0, px, py);
    double L = 0.0;
    if (p.quirk_length) {  // y_0 = anchor (map.x_start), y_1 = p_0 (problem.py:137-140)
        const double ax = p.anchor_mode ? p.anchor_x : px;
        const double ay = p.anchor_mode ? p.anchor_y : py;
        const double dx = px - ax, dy = py - ay;
        double s = 0.0;
        s = s + dx * dx;
        s = s + dy * dy;
        const double n = sqrt(s);
        L = L + (ls ? n * n : n);
    }
    double len = 0.0, ksum = 0.0;
    double pdx = 0.0, pdy = 0.0, pn = 0.0;
    for (int j = 1; j < W; ++j) {
        double qx, qy;
        src.at(j, qx, qy);
        const double dx = qx - px, dy = qy - py;
        double s = 0.0;
        s = s + dx * dx;
        s = s + dy * dy;
        const double n = sqrt(s);  // norm_2 = sqrt(dot) (casadi_norm_2)
        len = len + n;
        if (!p.quirk_length || j <= N) L = L + (ls ? n * n : n);
        const double nk = ms ? n * n : n;
        if (j >= 2) {  // kinematic row k = j-2 (problem.py:100-107)
            double dt = 0.0;
            dt = dt + pdx * dx;
            dt = dt + pdy * dy;
            double c1, c2, c3;
            kin_row(p, pn, nk, dt, c1, c2, c3);
            ksum = ksum + c1;
            ksum = ksum + c2;
            ksum = ksum + c3;
            if (grow) {
                grow[3 * (j - 2)] = c1;
                grow[3 * (j - 2) + 1] = c2;
                grow[3 * (j - 2) + 2] = c3;
            }
        }
        pdx = dx;
        pdy = dy;
        pn = nk;
        px = qx;
        py = qy;
    }
    a.L = L;
    a.len = len;
    a.ksum = ksum;
}

// One path: pass 1 = geometry-only terms (length_of, true length, kinematic rows), pass 2 =
// per-waypoint penalty (analytic formulas or the record gather).  C = gathers per chunk.
template <int MODE, bool GEN, int C>
__device__ __forceinline__ PathAcc eval_path(const KGeom& g, const KParams& p, const KRaster& rs,
                                             const KVolume& vs, const uint4* __restrict__ rec,
                                             const PathSrc<GEN>& src, int64_t path,
                                             const KOut& out, const uint32_t* sbits = nullptr) {
    const int N = p.N, W = N + 2;
    const int n_rows = 3 * N + g.n_obstacles * W;
    double* grow =
        (MODE == UAM_MODE_ANALYTIC && out.g_rows) ? out.g_rows + path * n_rows : nullptr;
    PathAcc a;
    path_pass1<GEN>(p, src, grow, a);

    // ---- pass 2: cost = (N+1) L + sum_j phi(p_j)/N  (problem.py:41-43) ------------------
    a.cost = (double)(N + 1) * a.L;
    a.nsum = 0.0;
    a.nh = 0;
    a.off = 0;
    a.below = 0;
    a.hmax = -INFINITY;
    a.cmin = INFINITY;
    const double dN = (double)N;
    if (MODE == UAM_MODE_VOLUME) {
        int32_t* cells = out.cells ? out.cells + path * W : nullptr;
        for (int j0 = 0; j0 < W; j0 += C) {
            Chunk<C> ch;
            issue_chunk_vol<GEN, C>(vs, sbits, src, j0, W, cells, ch);
            consume_chunk_vol<GEN, C>(vs, ch, src, j0, W, dN, a);
        }
    } else if (MODE == UAM_MODE_ANALYTIC) {
        for (int j = 0; j < W; ++j) {
            double x0, x1;
            src.at(j, x0, x1);
            a.cost = a.cost + total_penalty(g, p, x0, x1) / dN;
            const int slot = (g.grid.gx && !grow) ? grid_slot(g.grid, x0, x1) : -1;
            if (slot >= 0) {  // listed obstacles only: the others add +0 (exact no-op)
                const int k1 = g.grid.start[1][slot + 1];
                for (int k = g.grid.start[1][slot]; k < k1; ++k) {
                    const DevShape& sh = g.shape[g.grid.items[1][k]];
                    if ((sh.flags & SHAPE_CULL_PSI) && outside(sh.box_obs, x0, x1)) continue;
                    a.nsum = a.nsum + psi(g, sh, x0, x1, p.obstacle_smooth != 0, 0.0);
                }
            } else {
                for (int s = 0; s < g.n_obstacles; ++s) {
                    const double v = obstacle_psi(g, p, s, x0, x1);
                    a.nsum = a.nsum + v;
                    if (grow) grow[3 * N + s * W + j] = v;
                }
            }
            a.nh += collides(g, x0, x1) ? 1 : 0;
        }
    } else if (MODE == MODE_RASTER_SKIP) {
        raster_pass2_skip<GEN>(rs, rec, sbits, src, W, out.cells ? out.cells + path * W : nullptr,
                               dN, a);
    } else {
        int32_t* cells = out.cells ? out.cells + path * W : nullptr;
        for (int j0 = 0; j0 < W; j0 += C) {
            Chunk<C> ch;
            issue_chunk<GEN, C>(rs, rec, src, j0, W, cells, ch);
            consume_chunk<C>(ch, j0, W, dN, a);
        }
    }
    return a;
}

// raster: cruise altitude - highest terrain under the waypoints; volume: min over waypoints of
// (waypoint altitude - terrain of its column); analytic: NaN (no DEM)
__device__ __forceinline__ double clearance(const KParams& p, int mode, const PathAcc& a) {
    return (mode == UAM_MODE_RASTER || mode == MODE_RASTER_SKIP)
               ? p.altitude - a.hmax
                                   : (mode == UAM_MODE_VOLUME ? a.cmin : (double)NAN);
}

__device__ __forceinline__ void write_path(const KOut& out, const KParams& p, int mode,
                                           int64_t path, const PathAcc& a) {
    if (out.cost) out.cost[path] = a.cost;
    if (out.length_q) out.length_q[path] = a.L;
    if (out.length) out.length[path] = a.len;
    if (out.kin_sum) out.kin_sum[path] = a.ksum;
    if (out.nfz_sum) out.nfz_sum[path] = a.nsum;
    if (out.nfz_hits) out.nfz_hits[path] = a.nh;
    if (out.offmap) out.offmap[path] = a.off;
    if (out.min_clearance) out.min_clearance[path] = clearance(p, mode, a);
    if (out.below_terrain) out.below_terrain[path] = a.below;
}

// main.py:175-180 selection over D values (see uam_argmin)
__device__ __forceinline__ int select_best(const double* v, int stride, int D, bool take_sqrt) {
    int bi = 0;
    double bv = 0.0;
    for (int d = 0; d < D; ++d) {
        const double x = take_sqrt ? sqrt(v[d * stride]) : v[d * stride];
        if (bv == 0.0 || x < bv) {
            bv = x;
            bi = d;
        }
    }
    return bi;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_eval_waypoints(KGeom g, KParams p, KRaster rs,
                                                        const uint4* __restrict__ rec,
                                                        const double* __restrict__ wp,
                                                        int64_t n_paths, KOut out) {
    const int64_t path = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (path >= n_paths) return;
    PathSrc<false> src;
    src.W = p.N + 2;
    src.wp = wp + path * (int64_t)src.W * 2;
    src.u = nullptr;
    src.x0 = src.y0 = src.xf = src.yf = 0.0;
    src.za = src.zb = 0.0;
    const KVolume vs{};
    const PathAcc a = eval_path<MODE, false, 8>(g, p, rs, vs, rec, src, path, out);
    write_path(out, p, MODE, path, a);
}

// D > 16 (the block-of-pairs kernels hold all D waves of a pair in one workgroup): global wave
// w -> displacement d = w % D (wave-uniform), pairs [(w / D)*64, +64); outputs stored straight
// from registers (stride-D stores), selection by k_argmin afterwards.
template <int MODE>
__global__ __launch_bounds__(256) void k_eval_generated(KGeom g, KParams p, KRaster rs,
                                                        const uint4* __restrict__ rec,
                                                        const double* __restrict__ pairs,
                                                        int64_t n_pairs,
                                                        const double* __restrict__ utab, int D,
                                                        int64_t n_waves, KOut out) {
    const int64_t wave = __builtin_amdgcn_readfirstlane(
        (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    if (wave >= n_waves) return;
    const int lane = threadIdx.x & 63;
    const int d = (int)(wave % D);
    const int64_t q = (wave / D) * 64 + lane;
    if (q >= n_pairs) return;
    const double4 pr = reinterpret_cast<const double4*>(pairs)[q];
    PathSrc<true> src;
    src.W = p.N + 2;
    src.wp = nullptr;
    src.x0 = pr.x;
    src.y0 = pr.y;
    src.xf = pr.z;
    src.yf = pr.w;
    src.u = utab + (int64_t)d * p.N * 2;
    src.za = src.zb = 0.0;
    const KVolume vs{};
    const PathAcc a = eval_path<MODE, true, 8>(g, p, rs, vs, rec, src, q * D + d, out);
    write_path(out, p, MODE, q * D + d, a);
}

// Ordered chunk evaluated by workgroup b of nb: XCD x = b % 8 owns the contiguous chunk range
// [x * (nb / 8) + min(x, nb % 8), ...) and walks it in dispatch order (a bijection on [0, nb)).
__device__ __forceinline__ int64_t xcd_chunk(int64_t b, int64_t nb) {
    const int64_t x = b & 7, k = b >> 3;
    return x * (nb >> 3) + (x < (nb & 7) ? x : (nb & 7)) + k;
}

// Variant 2+: one workgroup = one block of 64 pairs x all D displacements (wave = d,
// lane = pair).  Results are staged in LDS and written with unit-stride (coalesced) stores
// over the block's contiguous path range [b*64*D, (b+1)*64*D); the candidate selection
// (main.py:175-180) runs in the same launch on the staged costs / lengths.
template <int MODE, int MINW>
__global__ __launch_bounds__(1024, MINW) void k_eval_pairs(KGeom g, KParams p, KRaster rs,
                                                           KVolume vs,
                                                           const uint4* __restrict__ rec,
                                                           const double* __restrict__ pairs,
                                                           int64_t n_pairs,
                                                           const double* __restrict__ utab,
                                                           int D, KOut out,
                                                           int32_t* __restrict__ best_f,
                                                           int32_t* __restrict__ best_l,
                                                           const int32_t* __restrict__ order) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int BP = 64 * D;                     // paths per block
    double* s_cost = smem;
    double* s_L = s_cost + BP;
    double* s_len = s_L + BP;
    double* s_k = s_len + BP;
    double* s_n = s_k + BP;
    double* s_clr = s_n + BP;
    int32_t* s_nh = reinterpret_cast<int32_t*>(s_clr + BP);
    int32_t* s_off = s_nh + BP;
    int32_t* s_bel = s_off + BP;
    uint32_t* s_bits = reinterpret_cast<uint32_t*>(s_bel + BP);  // gather-skip bitmap
    if (MODE == MODE_RASTER_SKIP) {
        for (int i = threadIdx.x; i < rs.swords; i += blockDim.x) s_bits[i] = rs.sum[i];
        __syncthreads();
    } else if (MODE == UAM_MODE_VOLUME) {  // the column bitmap
        for (int i = threadIdx.x; i < vs.cwords; i += blockDim.x) s_bits[i] = vs.cbits[i];
        __syncthreads();
    }

    const int d = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    // order (optional): slot -> pair, a spatial order of the pairs (pair_order).  Block b takes
    // the ordered chunk xcd_chunk(b): workgroups are dispatched round-robin over the 8 XCDs,
    // so the chunks of XCD b % 8 form one contiguous range of the order and the paths sharing
    // an XCD's L2 are spatial neighbours.  Every pair is still read and written at its own
    // index, so results do not depend on the order.
    const bool ordered = order != nullptr;
    const int64_t q0 = 64 * (ordered ? xcd_chunk(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x);
    const bool in = q0 + lane < n_pairs;
    const int64_t q = (ordered && in) ? (int64_t)order[q0 + lane] : q0 + lane;
    const int slot = d * 64 + lane;
    if (in) {
        PathSrc<true> src;
        src.W = p.N + 2;
        src.wp = nullptr;
        if (MODE == UAM_MODE_VOLUME) {  // pairs [Q][6] = (x0, y0, z0, xf, yf, zf)
            const double* pr = pairs + 6 * q;
            src.x0 = pr[0], src.y0 = pr[1], src.za = pr[2];
            src.xf = pr[3], src.yf = pr[4], src.zb = pr[5];
        } else {
            const double4 pr = reinterpret_cast<const double4*>(pairs)[q];
            src.x0 = pr.x, src.y0 = pr.y, src.xf = pr.z, src.yf = pr.w;
            src.za = src.zb = 0.0;
        }
        src.u = utab + (int64_t)d * p.N * 2;
        const PathAcc a =
            eval_path<MODE, true, 8>(g, p, rs, vs, rec, src, q * D + d, out, s_bits);
        s_cost[slot] = a.cost;
        s_L[slot] = a.L;
        s_len[slot] = a.len;
        s_k[slot] = a.ksum;
        s_n[slot] = a.nsum;
        s_clr[slot] = clearance(p, MODE, a);
        s_nh[slot] = a.nh;
        s_off[slot] = a.off;
        s_bel[slot] = a.below;
    }
    __syncthreads();
    // stores staged through LDS: thread t -> block-local path (pair t / D, displacement t % D),
    // so the D paths of a pair are D consecutive threads and D consecutive addresses
    const int t = threadIdx.x;
    const int qi = t / D, di = t - qi * D;
    if (q0 + qi < n_pairs) {
        const int64_t gp = (ordered ? (int64_t)order[q0 + qi] : q0 + qi) * D + di;
        const int s = di * 64 + qi;
        if (out.cost) out.cost[gp] = s_cost[s];
        if (out.length_q) out.length_q[gp] = s_L[s];
        if (out.length) out.length[gp] = s_len[s];
        if (out.kin_sum) out.kin_sum[gp] = s_k[s];
        if (out.nfz_sum) out.nfz_sum[gp] = s_n[s];
        if (out.min_clearance) out.min_clearance[gp] = s_clr[s];
        if (out.nfz_hits) out.nfz_hits[gp] = s_nh[s];
        if (out.offmap) out.offmap[gp] = s_off[s];
        if (out.below_terrain) out.below_terrain[gp] = s_bel[s];
    }
    if (d == 0 && in) {
        if (best_f) best_f[q] = select_best(s_cost + lane, 64, D, true);
        if (best_l) best_l[q] = select_best(s_len + lane, 64, D, false);
    }
}

// ----------------------------------------------------------------------------------------
// K6: batched refinement.  One 64-lane wavefront per path, lane l owning
// waypoints j = l, l+64, ...; the path's points z, gradient gr and kinematic multipliers live
// in the wave's LDS slice, obstacle multipliers [S][W] in the workspace (row s*W + j touched
// only by the lane owning j).  Definition and operation order: oracle/uam_oracle.c
// orc_refine (GPU == oracle bit for bit; path sums = per-lane sums + xor butterfly).  The
// reference solves min get_cost(z) s.t. get_nonlincon(z) in {0} with OpEn (solver.py:82-93).

struct KRefine {
    int32_t n_outer, n_inner, max_backtrack, memory;
    double c0, rho, c_max, alpha0, armijo, theta, max_step, inner_tol, delta;
    int32_t n_restart;
    double restart_margin;
};
constexpr int RF_MAXM = 8;  // L-BFGS memory bound (uam_refine_params.memory)

__device__ __forceinline__ void ineq_grad(const DevIneq* __restrict__ q, double x0, double x1,
                                          double& gx, double& gy) {
    const int kind = q->kind;
    if (kind == UAM_INEQ_HALFPLANE) {
        gx = q->p[4] * q->p[3];
        gy = -(q->p[4] * q->p[2]);
    } else if (kind == UAM_INEQ_ELLIPSE) {
        const double a = (x0 - q->p[0]) / q->p[2];
        const double b = (x1 - q->p[1]) / q->p[3];
        gx = (2.0 * a) / q->p[2];
        gy = (2.0 * b) / q->p[3];
    } else {
        gx = (q->p[0] == 0.0) ? q->p[3] : 0.0;
        gy = (q->p[0] == 0.0) ? 0.0 : q->p[3];
    }
}

// smooth psi = prod m_i^2 (== psi(.., smooth, e) bit for bit) and, when want, its gradient
// sum_i (2 psi / m_i) grad h_i (nonzero only where psi != 0)
__device__ __forceinline__ double psi_vg(const KGeom& g, const DevShape& sh, double x0,
                                         double x1, double e, bool want, double& dx,
                                         double& dy) {
    double v = 1.0;
    const int end = sh.first + sh.count;
    for (int i = sh.first; i < end; ++i) {
        const double m = fmin(ineq_h(g.ineq + i, x0, x1) - e, 0.0);
        v = v * (m * m);
    }
    dx = 0.0;
    dy = 0.0;
    if (want && v != 0.0) {
        double ox = 0.0, oy = 0.0;
        for (int i = sh.first; i < end; ++i) {
            const double m = fmin(ineq_h(g.ineq + i, x0, x1) - e, 0.0);
            const double coef = (2.0 * v) / m;
            double hx, hy;
            ineq_grad(g.ineq + i, x0, x1, hx, hy);
            ox = ox + coef * hx;
            oy = oy + coef * hy;
        }
        dx = ox;
        dy = oy;
    }
    return v;
}

// Phi (== total_penalty bit for bit) and, when want, grad Phi
__device__ double phi_vg(const KGeom& g, const KParams& p, double x0, double x1, bool want,
                         double& dx, double& dy) {
    double pen = 0.0, gx = 0.0, gy = 0.0;
    const int slot = g.grid.gx ? grid_slot(g.grid, x0, x1) : -1;
    if (slot >= 0) {  // grid-listed region shapes, regions in order (see total_penalty)
        double t = 0.0, tx = 0.0, ty = 0.0;
        int rc = -1;
        const int k1 = g.grid.start[0][slot + 1];
        for (int k = g.grid.start[0][slot]; k < k1; ++k) {
            const DevShape& sh = g.shape[g.grid.items[0][k]];
            if (sh.region != rc) {
                if (rc >= 0) {
                    pen = pen + p.weights[rc] * t;
                    gx = gx + p.weights[rc] * tx;
                    gy = gy + p.weights[rc] * ty;
                }
                rc = sh.region;
                t = tx = ty = 0.0;
            }
            if ((sh.flags & SHAPE_CULL_PEN) && outside(sh.box_pen, x0, x1)) continue;
            double ex, ey;
            const double v = psi_vg(g, sh, x0, x1, p.enlargement, want, ex, ey);
            if (sh.has_center) {
                t = t + v / sh.norm_pen;
                if (want && v != 0.0) {
                    tx = tx + ex / sh.norm_pen;
                    ty = ty + ey / sh.norm_pen;
                }
            } else {
                t = t + v;
                if (want && v != 0.0) {
                    tx = tx + ex;
                    ty = ty + ey;
                }
            }
        }
        if (rc >= 0) {
            pen = pen + p.weights[rc] * t;
            gx = gx + p.weights[rc] * tx;
            gy = gy + p.weights[rc] * ty;
        }
        dx = gx;
        dy = gy;
        return pen;
    }
    for (int r = 0; r < g.n_regions; ++r) {
        double t = 0.0, tx = 0.0, ty = 0.0;
        const int s1 = g.region_first[r + 1];
        for (int s = g.region_first[r]; s < s1; ++s) {
            const DevShape& sh = g.shape[s];
            if ((sh.flags & SHAPE_CULL_PEN) && outside(sh.box_pen, x0, x1)) continue;  // psi = 0
            double ex, ey;
            const double v = psi_vg(g, sh, x0, x1, p.enlargement, want, ex, ey);
            if (sh.has_center) {
                t = t + v / sh.norm_pen;
                if (want && v != 0.0) {
                    tx = tx + ex / sh.norm_pen;
                    ty = ty + ey / sh.norm_pen;
                }
            } else {
                t = t + v;
                if (want && v != 0.0) {
                    tx = tx + ex;
                    ty = ty + ey;
                }
            }
        }
        pen = pen + p.weights[r] * t;
        gx = gx + p.weights[r] * tx;
        gy = gy + p.weights[r] * ty;
    }
    dx = gx;
    dy = gy;
    return pen;
}

// kinematic rows of (p_k, p_k+1, p_k+2); q in {0,1,2}: d row / d p_k+q, q < 0: values only
__device__ __forceinline__ void kin_col(double pkx, double pky, double p1x, double p1y,
                                        double p2x, double p2y, double r, double mincos,
                                        bool ms, int q, double (&cv)[3], double (&dq)[3][2]) {
    const double ax = p1x - pkx, ay = p1y - pky;
    const double bx = p2x - p1x, by = p2y - p1y;
    double sa = 0.0, sb = 0.0, dt = 0.0;
    sa = sa + ax * ax;
    sa = sa + ay * ay;
    sb = sb + bx * bx;
    sb = sb + by * by;
    dt = dt + ax * bx;
    dt = dt + ay * by;
    const double ra = sqrt(sa), rb = sqrt(sb);
    const double na = ms ? ra * ra : ra, nb = ms ? rb * rb : rb;
    cv[0] = fmax(0.0, nb - r * na);
    cv[1] = fmax(0.0, na / r - nb);
    const double den = na * nb;
    cv[2] = fmax(0.0, mincos - dt / den);
    if (q < 0) return;
    const double gax = ms ? 2.0 * ax : ax / ra, gay = ms ? 2.0 * ay : ay / ra;
    const double gbx = ms ? 2.0 * bx : bx / rb, gby = ms ? 2.0 * by : by / rb;
    double da[3][2], db[3][2];
    da[0][0] = -(r * gax), da[0][1] = -(r * gay), db[0][0] = gbx, db[0][1] = gby;
    da[1][0] = gax / r, da[1][1] = gay / r, db[1][0] = -gbx, db[1][1] = -gby;
    const double d2 = den * den;
    const double qax = bx / den - ((dt * nb) * gax) / d2, qay = by / den - ((dt * nb) * gay) / d2;
    const double qbx = ax / den - ((dt * na) * gbx) / d2, qby = ay / den - ((dt * na) * gby) / d2;
    da[2][0] = -qax, da[2][1] = -qay, db[2][0] = -qbx, db[2][1] = -qby;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        if (q == 0) {
            dq[t][0] = -da[t][0];
            dq[t][1] = -da[t][1];
        } else if (q == 1) {
            dq[t][0] = da[t][0] - db[t][0];
            dq[t][1] = da[t][1] - db[t][1];
        } else {
            dq[t][0] = db[t][0];
            dq[t][1] = db[t][1];
        }
    }
}

// LDS visibility between the lanes of one wave (wave-private slice, no block barrier)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// v of lane l ^ OFF (whole wave active).  32 / 16: gfx950's permlane swaps; 8: DPP row_ror:8
// (= xor 8 inside a 16-lane row); 4: row_ror:4 reads lane l^4 or l^4^8, which hold the same
// value once the xor-8 stage has run (wave_sum only); 2 / 1: DPP quad_perm.  All VALU, no
// LDS round trip (ds_bpermute) per stage.
template <int OFF>
__device__ __forceinline__ uint32_t lane_xor_u32(uint32_t v) {
    if constexpr (OFF == 32 || OFF == 16) {
        const auto a = OFF == 32 ? __builtin_amdgcn_permlane32_swap(v, v, false, false)
                                 : __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (threadIdx.x & OFF) != 0 ? a[0] : a[1];  // a[0]: partner below, a[1]: above
    } else {
        constexpr int ctrl = OFF == 8 ? 0x128 : (OFF == 4 ? 0x124 : (OFF == 2 ? 0x4E : 0xB1));
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, ctrl, 0xf, 0xf, false);
    }
}

template <int OFF>
__device__ __forceinline__ double lane_xor(double v) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = lane_xor_u32<OFF>((uint32_t)u), hi = lane_xor_u32<OFF>((uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// wave-wide min / or (whole wave active; order-free, so the xor-4 stage may read l^4^8)
__device__ __forceinline__ int32_t wave_min_i32(int32_t v) {
    v = min(v, (int32_t)lane_xor_u32<32>((uint32_t)v));
    v = min(v, (int32_t)lane_xor_u32<16>((uint32_t)v));
    v = min(v, (int32_t)lane_xor_u32<8>((uint32_t)v));
    v = min(v, (int32_t)lane_xor_u32<4>((uint32_t)v));
    v = min(v, (int32_t)lane_xor_u32<2>((uint32_t)v));
    v = min(v, (int32_t)lane_xor_u32<1>((uint32_t)v));
    return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ uint64_t wave_or_u64(uint64_t v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo |= lane_xor_u32<32>(lo), hi |= lane_xor_u32<32>(hi);
    lo |= lane_xor_u32<16>(lo), hi |= lane_xor_u32<16>(hi);
    lo |= lane_xor_u32<8>(lo), hi |= lane_xor_u32<8>(hi);
    lo |= lane_xor_u32<4>(lo), hi |= lane_xor_u32<4>(hi);
    lo |= lane_xor_u32<2>(lo), hi |= lane_xor_u32<2>(hi);
    lo |= lane_xor_u32<1>(lo), hi |= lane_xor_u32<1>(hi);
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    return ((uint64_t)hi << 32) | lo;
}

// xor butterfly 32..1 (the oracle's wsum tree); every lane ends with the same value
__device__ __forceinline__ double wave_sum(double v) {
    v = v + lane_xor<32>(v);
    v = v + lane_xor<16>(v);
    v = v + lane_xor<8>(v);
    v = v + lane_xor<4>(v);
    v = v + lane_xor<2>(v);
    v = v + lane_xor<1>(v);
    return v;
}

struct RfPath {
    const double* z;   // LDS [W][2]
    double* gr;        // LDS [W][2] gradient (waypoint-indexed; endpoints unused)
    const double* dr;  // LDS [W][2] search direction
    const double* yk;  // LDS [3N]
    const double* yo;  // global [S][W]
    const uint64_t* act;  // LDS [W][nmw]: rows with a nonzero multiplier (null: no masks)
    int N, W, nmw;
    __device__ __forceinline__ void pt(int j, double a, double& x, double& y) const {
        x = z[2 * j];
        y = z[2 * j + 1];
        if (a != 0.0 && j >= 1 && j <= N) {
            x = x + a * dr[2 * j];
            y = y + a * dr[2 * j + 1];
        }
    }
};

// path dot product over interior waypoints (lane-owned entries), lane-tree order
__device__ __forceinline__ double wdot(const double* u, const double* v, int N, int lane) {
    double s = 0.0;
    for (int j = lane; j < N + 2; j += 64) {
        const double t = (j >= 1 && j <= N) ? u[2 * j] * v[2 * j] + u[2 * j + 1] * v[2 * j + 1]
                                             : 0.0;
        s = s + t;
    }
    return wave_sum(s);
}

// Candidate no-fly rows of a waypoint: the obstacles the grid index lists at its position
// (psi may be nonzero there) or whose multiplier is nonzero (act); every other row adds
// (c/2)(0 + 0/c)^2 = +0 to L and nothing to the gradient, so skipping it is exact.  Rows are
// visited in ascending order.  No index / NaN point: all rows.
constexpr int RF_MASKW = 4;  // bitmask words per waypoint: S <= 256 uses the masks

// mask words per waypoint for S obstacles (0: no masks); sizes the wave's LDS slice, so maps
// with <= 64 obstacles keep 6 waves per SIMD resident
__host__ __device__ __forceinline__ int rf_mask_words(int S) {
    return (S > 0 && S <= 64 * RF_MASKW) ? (S + 63) >> 6 : 0;
}

__device__ __forceinline__ uint64_t pick_word(const uint64_t (&cw)[RF_MASKW], int w) {
    return w == 0 ? cw[0] : (w == 1 ? cw[1] : (w == 2 ? cw[2] : cw[3]));  // no dynamic index
}

__device__ __forceinline__ void rf_candidates(const KGeom& g, double x, double y,
                                              const uint64_t* act, int nmw,
                                              uint64_t (&cw)[RF_MASKW]) {
    const int S = g.n_obstacles;
    const int slot = g.grid.gx ? grid_slot(g.grid, x, y) : -1;
#pragma unroll
    for (int w = 0; w < RF_MASKW; ++w) cw[w] = (act && w < nmw) ? act[w] : 0ull;
    if (slot < 0) {
#pragma unroll
        for (int w = 0; w < RF_MASKW; ++w) {
            const int lo = 64 * w;
            cw[w] = S >= lo + 64 ? ~0ull : (S > lo ? ((1ull << (S - lo)) - 1ull) : 0ull);
        }
        return;
    }
    if (g.grid.mask[1]) {  // mbase[1] == 0: bit s is obstacle s
        const uint64_t* m = g.grid.mask[1] + (int64_t)slot * g.grid.mw[1];
#pragma unroll
        for (int w = 0; w < RF_MASKW; ++w)
            if (w < g.grid.mw[1]) cw[w] |= m[w];
        return;
    }
    const int k1 = g.grid.start[1][slot + 1];
    for (int k = g.grid.start[1][slot]; k < k1; ++k) {
        const int sh = g.grid.items[1][k];
#pragma unroll
        for (int w = 0; w < RF_MASKW; ++w)
            if ((sh >> 6) == w) cw[w] |= 1ull << (sh & 63);
    }
}

__device__ __forceinline__ double seg_term(double px, double py, double qx, double qy, bool ls,
                                           double sc, bool want, double& vx, double& vy) {
    const double dx = qx - px, dy = qy - py;
    double s = 0.0;
    s = s + dx * dx;
    s = s + dy * dy;
    const double n = sqrt(s);
    if (want) {
        vx = ls ? sc * (2.0 * dx) : sc * (dx / n);
        vy = ls ? sc * (2.0 * dy) : sc * (dy / n);
    }
    return ls ? n * n : n;
}

// Read-only table entry at a wave-uniform index through the constant address space: the
// geometry tables do not change during a launch, and this lets the compiler use scalar loads
// (s_load) even though the kernel stores to global memory (which rules out its noclobber
// proof for plain global loads).
template <typename T>
__device__ __forceinline__ T uload(const T* base, int i) {
    static_assert(sizeof(T) % 4 == 0, "dword records");
    using CW = const __attribute__((address_space(4))) uint32_t;
    CW* src = (CW*)(base + i);
    T out;
    uint32_t* dst = reinterpret_cast<uint32_t*>(&out);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) dst[k] = src[k];
    return out;
}

// psi_vg for a wave-uniform shape (records through uload); same operations as psi_vg
__device__ __forceinline__ double psi_vg_u(const KGeom& g, const DevShape& sh, double x0,
                                           double x1, double e, bool want, double& dx,
                                           double& dy) {
    double v = 1.0;
    const int end = sh.first + sh.count;
    for (int i = sh.first; i < end; ++i) {
        const DevIneq q = uload(g.ineq, i);
        const double m = fmin(ineq_h(&q, x0, x1) - e, 0.0);
        v = v * (m * m);
    }
    dx = 0.0;
    dy = 0.0;
    if (want && v != 0.0) {
        double ox = 0.0, oy = 0.0;
        for (int i = sh.first; i < end; ++i) {
            const DevIneq q = uload(g.ineq, i);
            const double m = fmin(ineq_h(&q, x0, x1) - e, 0.0);
            const double coef = (2.0 * v) / m;
            double hx, hy;
            ineq_grad(&q, x0, x1, hx, hy);
            ox = ox + coef * hx;
            oy = oy + coef * hy;
        }
        dx = ox;
        dy = oy;
    }
    return v;
}

// Phi and grad Phi at every lane's point, computed by the wave together (uniform control flow,
// whole wave active; lanes with !valid contribute nothing).  Each lane walks its own grid list
// in ascending order exactly as phi_vg does, so its sums are bit-identical to phi_vg; the wave
// visits the union of the lanes' lists in ascending order (the minimum of the lane heads), so
// the shape index is wave-uniform and the shape and inequality records come through scalar
// loads instead of per-lane dependent gathers.  No index or a NaN point: phi_vg itself.
__device__ __forceinline__ double phi_vg_wave(const KGeom& g, const KParams& p, double x0,
                                              double x1, bool valid, bool want, double& dx,
                                              double& dy) {
    const int slot = valid ? (g.grid.gx ? grid_slot(g.grid, x0, x1) : -1) : -2;
    double pen = 0.0, gx = 0.0, gy = 0.0;
    int k = 0, k1 = 0;
    if (slot >= 0) {
        k = g.grid.start[0][slot];
        k1 = g.grid.start[0][slot + 1];
    }
    double t = 0.0, tx = 0.0, ty = 0.0;
    int rc = -1;
    // the lane's list as bitmask words (ascending bits = ascending shapes), or -- tables over
    // 256 shapes -- a cursor into the list
    const int mw = g.grid.mask[0] ? g.grid.mw[0] : 0;
    uint64_t lm[RF_MASKW] = {0ull, 0ull, 0ull, 0ull};
    if (mw && slot >= 0) {
        const uint64_t* m = g.grid.mask[0] + (int64_t)slot * mw;
#pragma unroll
        for (int w = 0; w < RF_MASKW; ++w)
            if (w < mw) lm[w] = m[w];
    }
    int w = 0;
    uint64_t ub = mw ? wave_or_u64(lm[0]) : 0ull;
    for (;;) {
        int s, cand;
        if (mw) {  // next set bit of the union, wave-uniform
            while (!ub && ++w < mw) ub = wave_or_u64(pick_word(lm, w));
            if (!ub) break;
            const int bit = __builtin_ctzll(ub);
            ub &= ub - 1;
            s = g.grid.mbase[0] + 64 * w + bit;
            cand = ((pick_word(lm, w) >> bit) & 1ull) ? s : INT32_MAX;
        } else {
            cand = k < k1 ? g.grid.items[0][k] : INT32_MAX;
            s = wave_min_i32(cand);  // wave-uniform
            if (s == INT32_MAX) break;
        }
        if (cand == s) {
            ++k;
            const DevShape sh = uload(g.shape, s);
            if (sh.region != rc) {
                if (rc >= 0) {
                    pen = pen + p.weights[rc] * t;
                    gx = gx + p.weights[rc] * tx;
                    gy = gy + p.weights[rc] * ty;
                }
                rc = sh.region;
                t = tx = ty = 0.0;
            }
            if (!((sh.flags & SHAPE_CULL_PEN) && outside(sh.box_pen, x0, x1))) {
                double ex, ey;
                const double v = psi_vg_u(g, sh, x0, x1, p.enlargement, want, ex, ey);
                if (sh.has_center) {
                    t = t + v / sh.norm_pen;
                    if (want && v != 0.0) {
                        tx = tx + ex / sh.norm_pen;
                        ty = ty + ey / sh.norm_pen;
                    }
                } else {
                    t = t + v;
                    if (want && v != 0.0) {
                        tx = tx + ex;
                        ty = ty + ey;
                    }
                }
            }
        }
    }
    if (rc >= 0) {
        pen = pen + p.weights[rc] * t;
        gx = gx + p.weights[rc] * tx;
        gy = gy + p.weights[rc] * ty;
    }
    if (slot == -1) pen = phi_vg(g, p, x0, x1, want, gx, gy);
    dx = gx;
    dy = gy;
    return pen;
}

// Walk the union of the lanes' grid lists of table L (0 penalty, 1 psi, 2 hit) in ascending
// shape order, wave-uniformly (uniform control flow, whole wave active): body(s, mine) with s
// wave-uniform and mine = s is in this lane's list (slot < 0: empty list).  Each lane thus
// sees exactly its own list, in its order; the wave's shape index is uniform, so the records
// come through scalar loads.  Per-cell bitmasks when the table has them, else the lists
// merged by their minimum head.
template <int L, class F>
__device__ __forceinline__ void wave_walk(const KGeom& g, int slot, F&& body) {
    const int mw = g.grid.mask[L] ? g.grid.mw[L] : 0;
    if (mw) {
        uint64_t lm[RF_MASKW] = {0ull, 0ull, 0ull, 0ull};
        if (slot >= 0) {
            const uint64_t* m = g.grid.mask[L] + (int64_t)slot * mw;
#pragma unroll
            for (int w = 0; w < RF_MASKW; ++w)
                if (w < mw) lm[w] = m[w];
        }
#pragma unroll 1
        for (int w = 0; w < mw; ++w) {
            const uint64_t mine = pick_word(lm, w);
            for (uint64_t b = wave_or_u64(mine); b; b &= b - 1) {
                const int bit = __builtin_ctzll(b);
                body(g.grid.mbase[L] + 64 * w + bit, ((mine >> bit) & 1ull) != 0);
            }
        }
        return;
    }
    int k = 0, k1 = 0;
    if (slot >= 0) {
        k = g.grid.start[L][slot];
        k1 = g.grid.start[L][slot + 1];
    }
    for (;;) {
        const int cand = k < k1 ? g.grid.items[L][k] : INT32_MAX;
        const int s = wave_min_i32(cand);
        if (s == INT32_MAX) break;
        const bool mine = cand == s;
        if (mine) ++k;
        body(s, mine);
    }
}

// psi / contains of a wave-uniform shape (records through uload); same operations as psi /
// contains
__device__ __forceinline__ double psi_u(const KGeom& g, const DevShape& sh, double x0, double x1,
                                        bool smooth, double e) {
    double r = 1.0;
    const int end = sh.first + sh.count;
    for (int i = sh.first; i < end; ++i) {
        const DevIneq q = uload(g.ineq, i);
        const double h = ineq_h(&q, x0, x1);
        if (smooth) {
            const double m = fmin(h - e, 0.0);
            r = r * (m * m);
        } else {
            r = r * fmin(e - h, 0.0);
        }
    }
    return r;
}

__device__ __forceinline__ bool contains_u(const KGeom& g, const DevShape& sh, double x0,
                                           double x1) {
    const int end = sh.first + sh.count;
    bool in = true;
    for (int i = sh.first; i < end; ++i) {
        const DevIneq q = uload(g.ineq, i);
        in = in && !(ineq_h(&q, x0, x1) > 1e-14);
    }
    return in;
}

// K1: one 16-B record per DEM cell {Phi, sum psi_nfz, dem, flags} (data_manager.py:14-17 mask,
// problem.py:49-56 Phi, the no-fly g rows' psi, Map.collides).  A wave covers 64 consecutive
// cells of a row, which nearly always share one grid cell: the three shape tables are walked
// by the whole wave (wave_walk), each lane adding exactly what total_penalty /
// obstacle_psi_sum / collides add, in their order -- records bit-identical to those
// functions.  Cells with no index slot (no grid, NaN) use the per-lane functions.
__global__ __launch_bounds__(256) void k_raster_build(KGeom g, KParams p, KRaster rs,
                                                      const float* __restrict__ dem,
                                                      float nodata, float thr,
                                                      uint4* __restrict__ rec) {
    const int64_t total = (int64_t)rs.nx * rs.ny;
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); base < total;
         base += stride) {  // wave-uniform trip count
        const int64_t c = base + lane;
        const bool valid = c < total;
        double xc = 0.0, yc = 0.0;
        float z = 0.0f;
        if (valid) {
            const int64_t iy = c / rs.nx, ix = c - iy * rs.nx;
            xc = rs.x0 + ((double)ix + 0.5) * rs.dx;
            yc = rs.y_top - ((double)iy + 0.5) * rs.dy;
            z = dem ? dem[c] : 0.0f;
        }
        const int slot = valid ? (g.grid.gx ? grid_slot(g.grid, xc, yc) : -1) : -2;
        double pen = 0.0, t = 0.0;
        int rc = -1;
        wave_walk<0>(g, slot, [&](int s, bool mine) {
            if (!mine) return;
            const DevShape sh = uload(g.shape, s);
            if (sh.region != rc) {
                if (rc >= 0) pen = pen + p.weights[rc] * t;
                rc = sh.region;
                t = 0.0;
            }
            if ((sh.flags & SHAPE_CULL_PEN) && outside(sh.box_pen, xc, yc)) return;
            const double v = psi_u(g, sh, xc, yc, p.penalty_smooth != 0, p.enlargement);
            t = sh.has_center ? t + v / sh.norm_pen : t + v;
        });
        if (rc >= 0) pen = pen + p.weights[rc] * t;
        double acc = 0.0;
        wave_walk<1>(g, slot, [&](int s, bool mine) {
            if (!mine) return;
            const DevShape sh = uload(g.shape, s);
            if ((sh.flags & SHAPE_CULL_PSI) && outside(sh.box_obs, xc, yc)) return;
            acc = acc + psi_u(g, sh, xc, yc, p.obstacle_smooth != 0, 0.0);
        });
        bool hit = false;
        wave_walk<2>(g, slot, [&](int s, bool mine) {
            if (!mine) return;
            const DevShape sh = uload(g.shape, s);
            if ((sh.flags & SHAPE_CULL_HIT) && outside(sh.box_obs, xc, yc)) return;
            hit = hit || contains_u(g, sh, xc, yc);
        });
        if (slot == -1) {
            pen = total_penalty(g, p, xc, yc);
            acc = obstacle_psi_sum(g, p, xc, yc);
            hit = collides(g, xc, yc);
        }
        if (valid) {
            uint32_t fl = 0;
            if (hit) fl |= UAM_FLAG_NFZ;
            if (thr == -9999.0f ? (z == -9999.0f) : (z > thr)) fl |= UAM_FLAG_MASK;
            if (z == nodata) fl |= UAM_FLAG_NODATA;
            rec[c] = make_uint4(__float_as_uint((float)pen), __float_as_uint((float)acc),
                                __float_as_uint(z), fl);
        }
    }
}

// ---- K1 with CPL cells (rows) per lane ------------------------------------------------------
// The single-cell K1 spends most of its issue slots in the scalar walk (measured: 357 SALU,
// 499 VALU and 53 SMEM instructions per 64-cell wave on the cfg3 map, profiles/r01/k1/): the
// union walk, the shape and inequality records and the loop control are paid once per wave.
// Here a wave covers a strip of 64 columns x CPL rows, one column per lane, so each walk step
// and each scalar record load serves CPL cells; each inequality is evaluated once for all the
// lane's cells, and the no-fly psi and contains tables are walked together (one h per
// inequality for both).  Every cell still adds exactly its own list's terms in its own order.

// table-L walk over CPL cells per lane: body(s, mine), mine = bit k set iff s is in cell k's
// list; s ascending and wave-uniform (see wave_walk)
template <int L, int CPL, class F>
__device__ __forceinline__ void wave_walk_cells(const KGeom& g, const int (&slot)[CPL],
                                                F&& body) {
    const int mw = g.grid.mask[L] ? g.grid.mw[L] : 0;
    if (mw) {
#pragma unroll 1
        for (int w = 0; w < mw; ++w) {
            uint64_t mk[CPL], any = 0ull;
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                mk[k] = slot[k] >= 0 ? g.grid.mask[L][(int64_t)slot[k] * mw + w] : 0ull;
                any |= mk[k];
            }
            for (uint64_t b = wave_or_u64(any); b; b &= b - 1) {
                const int bit = __builtin_ctzll(b);
                uint32_t mine = 0;
#pragma unroll
                for (int k = 0; k < CPL; ++k) mine |= (uint32_t)((mk[k] >> bit) & 1ull) << k;
                body(g.grid.mbase[L] + 64 * w + bit, mine);
            }
        }
        return;
    }
    int kk[CPL], k1[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        kk[k] = k1[k] = 0;
        if (slot[k] >= 0) {
            kk[k] = g.grid.start[L][slot[k]];
            k1[k] = g.grid.start[L][slot[k] + 1];
        }
    }
    for (;;) {
        int cand[CPL], lmin = INT32_MAX;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            cand[k] = kk[k] < k1[k] ? g.grid.items[L][kk[k]] : INT32_MAX;
            lmin = min(lmin, cand[k]);
        }
        const int s = wave_min_i32(lmin);
        if (s == INT32_MAX) break;
        uint32_t mine = 0;
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            if (cand[k] == s) {
                mine |= 1u << k;
                ++kk[k];
            }
        body(s, mine);
    }
}

// the two obstacle tables (1: psi, 2: contains) in one ascending walk when both have masks:
// body(s, mine_psi, mine_hit)
template <int CPL, class F>
__device__ __forceinline__ void wave_walk_obs_cells(const KGeom& g, const int (&slot)[CPL],
                                                    F&& body) {
    const int mw = g.grid.mask[1] ? g.grid.mw[1] : 0;
    if (mw && g.grid.mask[2] && g.grid.mw[2] == mw && g.grid.mbase[2] == g.grid.mbase[1]) {
#pragma unroll 1
        for (int w = 0; w < mw; ++w) {
            uint64_t m1[CPL], m2[CPL], any = 0ull;
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const bool on = slot[k] >= 0;
                m1[k] = on ? g.grid.mask[1][(int64_t)slot[k] * mw + w] : 0ull;
                m2[k] = on ? g.grid.mask[2][(int64_t)slot[k] * mw + w] : 0ull;
                any |= m1[k] | m2[k];
            }
            for (uint64_t b = wave_or_u64(any); b; b &= b - 1) {
                const int bit = __builtin_ctzll(b);
                uint32_t a1 = 0, a2 = 0;
#pragma unroll
                for (int k = 0; k < CPL; ++k) {
                    a1 |= (uint32_t)((m1[k] >> bit) & 1ull) << k;
                    a2 |= (uint32_t)((m2[k] >> bit) & 1ull) << k;
                }
                body(g.grid.mbase[1] + 64 * w + bit, a1, a2);
            }
        }
        return;
    }
    wave_walk_cells<1, CPL>(g, slot, [&](int s, uint32_t m) { body(s, m, 0u); });
    wave_walk_cells<2, CPL>(g, slot, [&](int s, uint32_t m) { body(s, 0u, m); });
}

template <int CPL>
__global__ __launch_bounds__(256) void k_raster_build_cells(KGeom g, KParams p, KRaster rs,
                                                            const float* __restrict__ dem,
                                                            float nodata, float thr,
                                                            uint4* __restrict__ rec) {
    constexpr int K1_SPT = UAM_K1_TILE_ROWS / CPL;  // strips per column of the strip order
    const int sxn = (rs.nx + 63) / 64, sny = (rs.ny + CPL - 1) / CPL;
    const int lane = threadIdx.x & 63;
    // strip order: row-major, or (K1_SPT > 0) down columns of K1_SPT strips so that a
    // workgroup's waves and the workgroups an XCD runs in a row cover one 64-column tile of the
    // shape grid (the same shape lists: scalar-cache hits), the 8 XCDs taking contiguous ranges
    const int64_t n_virt = K1_SPT ? (int64_t)sxn * ((sny + K1_SPT - 1) / K1_SPT) * K1_SPT
                                  : (int64_t)sxn * sny;
    int64_t blk = blockIdx.x;
    if (K1_SPT) blk = (int64_t)(blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const int64_t w0 = __builtin_amdgcn_readfirstlane((int)((blk * blockDim.x + threadIdx.x) >> 6));
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const bool pen_smooth = p.penalty_smooth != 0, obs_smooth = p.obstacle_smooth != 0;
    // the strip's first row and column block (a strip of the last tile row past the raster
    // gets rows >= ny: every cell invalid, nothing walked or stored)
    auto strip_of = [&](int64_t st, int& sy, int& sx) {
        if (K1_SPT) {
            const int64_t tile = st / K1_SPT;
            const int ty = (int)(tile / sxn);
            sx = (int)(tile - (int64_t)ty * sxn);
            sy = ty * K1_SPT + (int)(st - tile * K1_SPT);
        } else {
            sy = (int)(st / sxn), sx = (int)(st - (int64_t)sy * sxn);
        }
    };
    auto load_z = [&](int sy, int sx, float (&zz)[CPL]) {
        const int ix = sx * 64 + lane;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const int iy = sy * CPL + k;
            zz[k] = (ix < rs.nx && iy < rs.ny && dem) ? dem[(int64_t)iy * rs.nx + ix] : 0.0f;
        }
    };
    int sy = 0, sx = 0;
    float z[CPL];
    if (w0 < n_virt) {
        strip_of(w0, sy, sx);
        load_z(sy, sx, z);
    }
    for (int64_t st = w0; st < n_virt; st += nw) {  // wave-uniform strip index
        // the next strip's DEM loads issued before this strip's walks (a grid smaller than
        // the strip count: each wave loops)
        int nsy = 0, nsx = 0;
        float zn[CPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k) zn[k] = 0.0f;
        if (st + nw < n_virt) {
            strip_of(st + nw, nsy, nsx);
            load_z(nsy, nsx, zn);
        }
        const int ix = sx * 64 + lane;
        const double xc = rs.x0 + ((double)ix + 0.5) * rs.dx;
        double yc[CPL];
        int slot[CPL];
        bool valid[CPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const int iy = sy * CPL + k;
            valid[k] = ix < rs.nx && iy < rs.ny;
            yc[k] = rs.y_top - ((double)iy + 0.5) * rs.dy;
            slot[k] = valid[k] ? (g.grid.gx ? grid_slot(g.grid, xc, yc[k]) : -1) : -2;
        }
        // Φ: total_penalty's region loop, per cell
        double pen[CPL], t[CPL], wc[CPL];  // wc: the weight of the cell's current region
        int rc[CPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k) pen[k] = t[k] = wc[k] = 0.0, rc[k] = -1;
        wave_walk_cells<0, CPL>(g, slot, [&](int s, uint32_t mine) {
            if (!mine) return;
            const DevShape sh = uload(g.shape, s);
            uint32_t need = 0;
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                if (!((mine >> k) & 1u)) continue;
                if (sh.region != rc[k]) {
                    if (rc[k] >= 0) pen[k] = pen[k] + wc[k] * t[k];
                    rc[k] = sh.region;
                    wc[k] = sh.wreg;  // p.weights[sh.region], from the shape record
                    t[k] = 0.0;
                }
                if (!((sh.flags & SHAPE_CULL_PEN) && outside(sh.box_pen, xc, yc[k])))
                    need |= 1u << k;
            }
            if (!need) return;
            double r[CPL];
#pragma unroll
            for (int k = 0; k < CPL; ++k) r[k] = 1.0;
            const int end = sh.first + sh.count;
            for (int i = sh.first; i < end; ++i) {  // psi_u, one record load for all cells
                const DevIneq q = uload(g.ineq, i);
                double hk[CPL];
                ineq_h_col<CPL>(q, xc, yc, hk);
#pragma unroll
                for (int k = 0; k < CPL; ++k) {
                    const double h = hk[k];
                    if (pen_smooth) {
                        const double m = fmin(h - p.enlargement, 0.0);
                        r[k] = r[k] * (m * m);
                    } else {
                        r[k] = r[k] * fmin(p.enlargement - h, 0.0);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < CPL; ++k)
                if ((need >> k) & 1u)
                    t[k] = sh.has_center ? t[k] + r[k] / sh.norm_pen : t[k] + r[k];
        });
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            if (rc[k] >= 0) pen[k] = pen[k] + wc[k] * t[k];
        // Σψ_nfz (obstacle_psi_sum, e = 0) and Map.collides, one h per inequality for both
        double acc[CPL];
        bool hit[CPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k) acc[k] = 0.0, hit[k] = false;
            wave_walk_obs_cells<CPL>(g, slot, [&](int s, uint32_t m1, uint32_t m2) {
            if (!(m1 | m2)) return;
            const DevShape sh = uload(g.shape, s);
            uint32_t n1 = 0, n2 = 0;
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const bool out = outside(sh.box_obs, xc, yc[k]);
                if (((m1 >> k) & 1u) && !((sh.flags & SHAPE_CULL_PSI) && out)) n1 |= 1u << k;
                if (((m2 >> k) & 1u) && !((sh.flags & SHAPE_CULL_HIT) && out)) n2 |= 1u << k;
            }
            if (!(n1 | n2)) return;
            double r[CPL];
            bool in[CPL];
#pragma unroll
            for (int k = 0; k < CPL; ++k) r[k] = 1.0, in[k] = true;
            const int end = sh.first + sh.count;
            for (int i = sh.first; i < end; ++i) {
                const DevIneq q = uload(g.ineq, i);
                double hk[CPL];
                ineq_h_col<CPL>(q, xc, yc, hk);
#pragma unroll
                for (int k = 0; k < CPL; ++k) {
                    const double h = hk[k];
                    if (obs_smooth) {
                        const double m = fmin(h - 0.0, 0.0);
                        r[k] = r[k] * (m * m);
                    } else {
                        r[k] = r[k] * fmin(0.0 - h, 0.0);
                    }
                    in[k] = in[k] && !(h > 1e-14);
                }
            }
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                if ((n1 >> k) & 1u) acc[k] = acc[k] + r[k];
                if ((n2 >> k) & 1u) hit[k] = hit[k] || in[k];
            }
        });
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            if (slot[k] == -1) {  // no index slot (no grid, NaN): the per-point functions
                pen[k] = total_penalty(g, p, xc, yc[k]);
                acc[k] = obstacle_psi_sum(g, p, xc, yc[k]);
                hit[k] = collides(g, xc, yc[k]);
            }
            if (valid[k]) {
                uint32_t fl = 0;
                if (hit[k]) fl |= UAM_FLAG_NFZ;
                if (thr == -9999.0f ? (z[k] == -9999.0f) : (z[k] > thr)) fl |= UAM_FLAG_MASK;
                if (z[k] == nodata) fl |= UAM_FLAG_NODATA;
                uint4* dst = rec + (int64_t)(sy * CPL + k) * rs.nx + ix;
                if (UAM_K1_NT) {
                    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                    const v4u w = {__float_as_uint((float)pen[k]), __float_as_uint((float)acc[k]),
                                   __float_as_uint(z[k]), fl};
                    __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(dst));
                } else {
                    *dst = make_uint4(__float_as_uint((float)pen[k]),
                                      __float_as_uint((float)acc[k]), __float_as_uint(z[k]), fl);
                }
            }
        }
        sy = nsy, sx = nsx;
#pragma unroll
        for (int k = 0; k < CPL; ++k) z[k] = zn[k];
    }
}

// The inequalities of a wave-uniform shape in ascending order, their records through scalar
// loads two at a time (one wait per pair instead of one per record): f(q) per inequality.
template <class F>
__device__ __forceinline__ void for_ineqs_u(const KGeom& g, const DevShape& sh, F&& f) {
    int i = sh.first;
    const int end = sh.first + sh.count;
    for (; i + 1 < end; i += 2) {
        const DevIneq q0 = uload(g.ineq, i);
        const DevIneq q1 = uload(g.ineq, i + 1);
        f(q0);
        f(q1);
    }
    if (i < end) f(uload(g.ineq, i));
}

// ---- K3b: analytic evaluation with cell-sorted waypoints ----------------------------------
// k_eval_pairs<ANALYTIC> runs one lane per path, so at each step a wave's 64 lanes evaluate 64
// points that lie kilometres apart: 64 different shape-grid lists, walked with per-lane
// dependent loads of the shape and inequality records (profiles/r02: 75% of wave cycles
// parked on s_waitcnt, 7% VALU).  K3b keeps the block layout (wave = displacement, lane =
// pair; pass 1 and every ordered sum stay with the path's own lane) but evaluates the
// waypoints in segments of S steps: the block's 64 D S points of a segment are counting-sorted
// in LDS by the Morton code of their grid cell, and each wave evaluates 64 CPL consecutive
// sorted points at a time (CPL per lane) -- the same or adjacent cells -- walking the union of
// their lists wave-uniformly, with the shape and inequality records through scalar loads as
// K1 does.  Each point's results go to LDS: Phi (f64), its nonzero no-fly psi terms in list
// order (appended to a term list), their count and the collision bit.  The path's lane then
// adds them in waypoint order exactly as eval_path does: Phi / N into the cost chain, the psi
// terms into the no-fly chain (a +-0 term, which the list omits, is an exact no-op on an
// accumulator that is never -0), the hit count.  A point with more than K3B_KT terms, or whose
// terms do not fit the segment's term list, is re-walked by its lane (eval_path's own loop).
// Outputs are bit-identical to k_eval_pairs.
constexpr int K3B_BINS = 1024 + 2;  // grid cell mod 1024, off-grid, no slot
constexpr int K3B_KT = 3;           // psi terms a point keeps in registers (more: re-walk)
constexpr uint8_t K3B_HIT = 1, K3B_REWALK = 7;  // flags: bit 0 hit, bits 1-3 term count

__device__ __forceinline__ int k3b_key(int slot, int gx) {
    if (slot < 0) return 1025;
    if (slot >= gx * gx) return 1024;
    return slot & 1023;  // row-major cell; cells 1024 apart share a bin (only coherence suffers)
}

// exclusive scan of h[0..n) in place by the whole block (nt threads, nt % 64 == 0); returns
// the total.  part: >= nt / 64 + 1 ints of scratch.
__device__ __forceinline__ int block_excl_scan(int32_t* h, int n, int32_t* part) {
    const int t = threadIdx.x, nt = blockDim.x, per = (n + nt - 1) / nt;
    const int lo = min(n, t * per), hi = min(n, lo + per);
    int32_t sum = 0;
    for (int i = lo; i < hi; ++i) sum += h[i];
    int32_t inc = sum;  // inclusive wave scan
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t v = __shfl_up(inc, o, 64);
        if ((t & 63) >= o) inc += v;
    }
    if ((t & 63) == 63) part[t >> 6] = inc;
    __syncthreads();
    if (t == 0) {
        int32_t run = 0;
        for (int w = 0; w < nt / 64; ++w) {
            const int32_t v = part[w];
            part[w] = run;
            run += v;
        }
        part[nt / 64] = run;
    }
    __syncthreads();
    int32_t run = part[t >> 6] + inc - sum;
    for (int i = lo; i < hi; ++i) {
        const int32_t v = h[i];
        h[i] = run;
        run += v;
    }
    const int32_t total = part[nt / 64];
    __syncthreads();
    return total;
}

// Per-point results of the evaluation phase.
template <int CPL>
struct K3bRes {
    double pen[CPL];
    double tm[CPL][K3B_KT];  // the first nonzero obstacle psi terms, list order
    int cnt[CPL];            // nonzero terms (may exceed K3B_KT)
    bool hit[CPL];
};

// Phi, the nonzero obstacle psi terms and the collision bit of each lane's CPL points (whole
// wave active, uniform control flow; slot -2 = no point).  Same terms in the same order as
// total_penalty / eval_path's psi loop / collides (the walk of k_raster_build_cells).
template <int CPL>
__device__ __forceinline__ void k3b_points(const KGeom& g, const KParams& p,
                                           const double (&x)[CPL], const double (&y)[CPL],
                                           const int (&slot)[CPL], K3bRes<CPL>& R) {
    const bool pen_smooth = p.penalty_smooth != 0, obs_smooth = p.obstacle_smooth != 0;
    double t[CPL], wc[CPL];  // wc: the weight of the lane's current region (rc)
    int rc[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) R.pen[k] = t[k] = wc[k] = 0.0, rc[k] = -1;
    const int(&slot0)[CPL] = slot;
    const int(&slot1)[CPL] = slot;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        R.cnt[k] = 0;
        R.hit[k] = false;
#pragma unroll
        for (int m = 0; m < K3B_KT; ++m) R.tm[k][m] = 0.0;
    }
    auto k3b_finish_pen = [&]() {
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            if (rc[k] >= 0) R.pen[k] = R.pen[k] + wc[k] * t[k];
    };
    auto add_term = [&](int k, double v) {  // v nonzero or NaN: a term the no-fly chain adds
#pragma unroll
        for (int m = 0; m < K3B_KT; ++m)
            if (R.cnt[k] == m) R.tm[k][m] = v;
        ++R.cnt[k];
    };
    auto body0 = [&](int s, uint32_t mine) {
        if (!mine) return;
        const DevShape sh = uload(g.shape, s);
        uint32_t need = 0;
        const double wnew = sh.wreg;  // the region's weight, in the same record load
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            if (!((mine >> k) & 1u)) continue;
            if (sh.region != rc[k]) {
                if (rc[k] >= 0) R.pen[k] = R.pen[k] + wc[k] * t[k];
                rc[k] = sh.region;
                wc[k] = wnew;
                t[k] = 0.0;
            }
            if (!((sh.flags & SHAPE_CULL_PEN) && outside(sh.box_pen, x[k], y[k])))
                need |= 1u << k;
        }
        if (!need) return;
        double r[CPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k) r[k] = 1.0;
        for_ineqs_u(g, sh, [&](const DevIneq& q) {
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const double h = ineq_h(&q, x[k], y[k]);
                if (pen_smooth) {
                    const double m = fmin(h - p.enlargement, 0.0);
                    r[k] = r[k] * (m * m);
                } else {
                    r[k] = r[k] * fmin(p.enlargement - h, 0.0);
                }
            }
        });
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            if ((need >> k) & 1u) t[k] = sh.has_center ? t[k] + r[k] / sh.norm_pen : t[k] + r[k];
    };

    auto body1 = [&](int s, uint32_t m1, uint32_t m2) {
        if (!(m1 | m2)) return;
        const DevShape sh = uload(g.shape, s);
        uint32_t n1 = 0, n2 = 0;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const bool out = outside(sh.box_obs, x[k], y[k]);
            if (((m1 >> k) & 1u) && !((sh.flags & SHAPE_CULL_PSI) && out)) n1 |= 1u << k;
            if (((m2 >> k) & 1u) && !((sh.flags & SHAPE_CULL_HIT) && out)) n2 |= 1u << k;
        }
        if (!(n1 | n2)) return;
        double r[CPL];
        bool in[CPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k) r[k] = 1.0, in[k] = true;
        for_ineqs_u(g, sh, [&](const DevIneq& q) {
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const double h = ineq_h(&q, x[k], y[k]);
                if (obs_smooth) {
                    const double m = fmin(h - 0.0, 0.0);
                    r[k] = r[k] * (m * m);
                } else {
                    r[k] = r[k] * fmin(0.0 - h, 0.0);
                }
                in[k] = in[k] && !(h > 1e-14);
            }
        });
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            if (((n1 >> k) & 1u) && !(r[k] == 0.0)) add_term(k, r[k]);
            if ((n2 >> k) & 1u) R.hit[k] = R.hit[k] || in[k];
        }
    };
    // mask words of all three tables loaded at once, before either walk (tables of <= 128
    // shapes with masks); otherwise the generic walkers
    const KShapeGrid& gr = g.grid;
    const bool fast = gr.mask[0] && gr.mask[1] && gr.mask[2] && gr.mw[0] >= 1 && gr.mw[0] <= 2 &&
                      gr.mw[1] >= 1 && gr.mw[1] <= 2 && gr.mw[2] == gr.mw[1] &&
                      gr.mbase[2] == gr.mbase[1];
    uint64_t mk0[CPL][2], mk1[CPL][2], mk2[CPL][2];
    if (fast) {
        const int mw0 = gr.mw[0], mw1 = gr.mw[1];
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
            for (int w = 0; w < 2; ++w) {
                mk0[k][w] = (slot0[k] >= 0 && w < mw0) ? gr.mask[0][(int64_t)slot0[k] * mw0 + w]
                                                       : 0ull;
                mk1[k][w] = (slot1[k] >= 0 && w < mw1) ? gr.mask[1][(int64_t)slot1[k] * mw1 + w]
                                                       : 0ull;
                mk2[k][w] = (slot1[k] >= 0 && w < mw1) ? gr.mask[2][(int64_t)slot1[k] * mw1 + w]
                                                       : 0ull;
            }
        uint64_t any0[2] = {0ull, 0ull}, any1[2] = {0ull, 0ull};
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
            for (int w = 0; w < 2; ++w) any0[w] |= mk0[k][w], any1[w] |= mk1[k][w] | mk2[k][w];
        const uint64_t u00 = wave_or_u64(any0[0]), u01 = mw0 > 1 ? wave_or_u64(any0[1]) : 0ull;
        const uint64_t u10 = wave_or_u64(any1[0]), u11 = mw1 > 1 ? wave_or_u64(any1[1]) : 0ull;
#pragma unroll
        for (int w = 0; w < 2; ++w)
            for (uint64_t bb = w ? u01 : u00; bb; bb &= bb - 1) {
                const int bit = __builtin_ctzll(bb);
                uint32_t mine = 0;
#pragma unroll
                for (int k = 0; k < CPL; ++k) mine |= (uint32_t)((mk0[k][w] >> bit) & 1ull) << k;
                body0(gr.mbase[0] + 64 * w + bit, mine);
            }
        k3b_finish_pen();
#pragma unroll
        for (int w = 0; w < 2; ++w)
            for (uint64_t bb = w ? u11 : u10; bb; bb &= bb - 1) {
                const int bit = __builtin_ctzll(bb);
                uint32_t a1 = 0, a2 = 0;
#pragma unroll
                for (int k = 0; k < CPL; ++k) {
                    a1 |= (uint32_t)((mk1[k][w] >> bit) & 1ull) << k;
                    a2 |= (uint32_t)((mk2[k][w] >> bit) & 1ull) << k;
                }
                body1(gr.mbase[1] + 64 * w + bit, a1, a2);
            }
    } else {
        wave_walk_cells<0, CPL>(g, slot0, body0);
        k3b_finish_pen();
        wave_walk_obs_cells<CPL>(g, slot1, body1);
    }
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        if (slot[k] == -1) {  // no index slot (no grid, NaN point): eval_path's per-point loops
            R.pen[k] = total_penalty(g, p, x[k], y[k]);
            R.cnt[k] = 0;
            for (int s = 0; s < g.n_obstacles; ++s) {
                const double v = obstacle_psi(g, p, s, x[k], y[k]);
                if (!(v == 0.0)) add_term(k, v);
            }
            R.hit[k] = collides(g, x[k], y[k]);
        }
    }
}

// eval_path's no-fly terms of one point, added in its order (a point K3b could not park)
__device__ __forceinline__ double k3b_psi_chain(const KGeom& g, const KParams& p, double x0,
                                                double x1, double acc) {
    const int slot = g.grid.gx ? grid_slot(g.grid, x0, x1) : -1;
    if (slot >= 0) {
        const int k1 = g.grid.start[1][slot + 1];
        for (int k = g.grid.start[1][slot]; k < k1; ++k) {
            const DevShape& sh = g.shape[g.grid.items[1][k]];
            if ((sh.flags & SHAPE_CULL_PSI) && outside(sh.box_obs, x0, x1)) continue;
            acc = acc + psi(g, sh, x0, x1, p.obstacle_smooth != 0, 0.0);
        }
        return acc;
    }
    for (int s = 0; s < g.n_obstacles; ++s) acc = acc + obstacle_psi(g, p, s, x0, x1);
    return acc;
}

// LDS of K3b (D displacements, segment S): per point Phi (f64), its first psi term (f64), the
// index of its further terms (u16), sorted order (u16), flags (u8); the list of further terms
// (NPT / 2 doubles) and its fill counter; all of it
// overlaid at the end by k_eval_pairs' output staging (64 D x (6 f64 + 3 i32)).  Then the
// histogram, the scan parts, the block's pairs and the segment's unit-arc rows.
__host__ __device__ __forceinline__ int k3b_tcap(int npt) { return npt / 2 > 64 ? npt / 2 : 64; }
__host__ __device__ __forceinline__ size_t k3b_seg_bytes(int D, int S) {
    const size_t npt = (size_t)64 * D * S;
    const size_t seg = npt * (8 + 8 + 2 + 2 + 1) + 16 + (size_t)k3b_tcap((int)npt) * 8;
    const size_t stage = (size_t)64 * D * (6 * 8 + 3 * 4);
    return ((seg > stage ? seg : stage) + 15) & ~(size_t)15;
}
__host__ __device__ __forceinline__ size_t k3b_mid_bytes(int D) {  // histogram + scan parts
    return ((size_t)K3B_BINS * 4 + (size_t)(D + 2) * 4 + 15) & ~(size_t)15;
}
__host__ __device__ __forceinline__ size_t k3b_lds_bytes(int D, int S) {
    return k3b_seg_bytes(D, S) + k3b_mid_bytes(D) + 64 * 32 + (size_t)D * S * 16;
}

template <int S, int CPL>
__global__ __launch_bounds__(1024) void k_eval_pairs_k3b(KGeom g, KParams p,
                                                         const double* __restrict__ pairs,
                                                         int64_t n_pairs,
                                                         const double* __restrict__ utab, int D,
                                                         KOut out, int32_t* __restrict__ best_f,
                                                         int32_t* __restrict__ best_l,
                                                         const int32_t* __restrict__ order) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int BP = 64 * D, NPT = BP * S, TCAP = k3b_tcap(NPT);
    char* base = reinterpret_cast<char*>(smem);
    double* s_phi = reinterpret_cast<double*>(base);
    double* s_psi = s_phi + NPT;
    double* s_term = s_psi + NPT;
    uint16_t* s_tix = reinterpret_cast<uint16_t*>(s_term + TCAP);
    uint16_t* s_ord = s_tix + NPT;
    uint8_t* s_fl = reinterpret_cast<uint8_t*>(s_ord + NPT);
    int32_t* s_tcnt =  // after the flags (k3b_seg_bytes keeps 16 B for it)
        reinterpret_cast<int32_t*>(base + (((size_t)NPT * 21 + (size_t)TCAP * 8 + 3) & ~(size_t)3));
    int32_t* s_hist = reinterpret_cast<int32_t*>(base + k3b_seg_bytes(D, S));
    int32_t* s_part = s_hist + K3B_BINS;
    double4* s_pair = reinterpret_cast<double4*>(base + k3b_seg_bytes(D, S) + k3b_mid_bytes(D));
    double2* s_u = reinterpret_cast<double2*>(s_pair + 64);
    const int d = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const bool ordered = order != nullptr;
    const int64_t q0 = 64 * (ordered ? xcd_chunk(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x);
    const bool in = q0 + lane < n_pairs;
    const int64_t q = (ordered && in) ? (int64_t)order[q0 + lane] : q0 + lane;
    const int N = p.N, W = N + 2;
    const double dN = (double)N;
    PathSrc<true> src;
    src.W = W;
    src.wp = nullptr;
    src.x0 = src.y0 = src.xf = src.yf = 0.0;
    src.za = src.zb = 0.0;
    if (in) {
        const double4 pr = reinterpret_cast<const double4*>(pairs)[q];
        src.x0 = pr.x, src.y0 = pr.y, src.xf = pr.z, src.yf = pr.w;
    }
    if (d == 0) s_pair[lane] = make_double4(src.x0, src.y0, src.xf, src.yf);
    src.u = utab + (int64_t)d * N * 2;
    PathAcc a;
    a.L = a.len = a.ksum = 0.0;
    if (in) path_pass1<true>(p, src, nullptr, a);
    a.cost = (double)(N + 1) * a.L;
    a.nsum = 0.0;
    a.nh = 0;
    a.off = 0;
    a.below = 0;
    a.hmax = -INFINITY;
    a.cmin = INFINITY;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int wave = tid >> 6, nwaves = nt >> 6;
    int j0 = 0;
    // point tt of the segment of path-thread th (block-local pair th & 63, displacement th >> 6)
    auto seg_point = [&](int th, int tt, double& x, double& y) {
        const double4 pr = s_pair[th & 63];
        const int j = j0 + tt;
        if (j == 0) {
            x = pr.x, y = pr.y;
        } else if (j == W - 1) {
            x = pr.z, y = pr.w;
        } else {
            const double2 u = s_u[(th >> 6) * S + tt];
            arc_point(pr.x, pr.y, pr.z, pr.w, u.x, u.y, x, y);
        }
    };
    for (; j0 < W; j0 += S) {
        const int sn = min(S, W - j0);
        for (int i = tid; i < K3B_BINS; i += nt) s_hist[i] = 0;
        if (tid == 0) *s_tcnt = 0;
        for (int i = tid; i < D * S; i += nt) {  // the segment's unit-arc rows (j = 1..N)
            const int dd = i / S, jj = j0 + (i - dd * S);
            if (jj >= 1 && jj <= N) {
                const double* u = utab + ((int64_t)dd * N + (jj - 1)) * 2;
                s_u[i] = make_double2(u[0], u[1]);
            }
        }
        __syncthreads();
        // A: key and in-bin rank of this lane's sn points
        int key[S], rank[S];
#pragma unroll
        for (int t = 0; t < S; ++t) {
            key[t] = -1;
            rank[t] = 0;
            if (in && t < sn) {
                double x, y;
                seg_point(tid, t, x, y);
                const int slot = g.grid.gx ? grid_slot(g.grid, x, y) : -1;
                key[t] = k3b_key(slot, g.grid.gx);
                rank[t] = atomicAdd(&s_hist[key[t]], 1);
            }
        }
        __syncthreads();
        const int npts = block_excl_scan(s_hist, K3B_BINS, s_part);
        int pos[S];  // sorted position of each of this lane's points (rank reused)
#pragma unroll
        for (int t = 0; t < S; ++t) {
            pos[t] = key[t] >= 0 ? s_hist[key[t]] + rank[t] : 0;
            if (key[t] >= 0) s_ord[pos[t]] = (uint16_t)(tid * S + t);
        }
        __syncthreads();
        // B: evaluate 64 CPL consecutive sorted points per wave step (wave-uniform trip count)
        const int npts_b = npts;
        for (int c0 = wave * 64 * CPL; c0 < npts_b; c0 += nwaves * 64 * CPL) {
            double x[CPL], y[CPL];
            int slot[CPL], id[CPL];
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const int pos = c0 + k * 64 + lane;
                x[k] = y[k] = 0.0;
                slot[k] = -2;
                id[k] = -1;
                if (pos < npts) {
                    id[k] = s_ord[pos];
                    const int th = id[k] / S;
                    seg_point(th, id[k] - th * S, x[k], y[k]);
                    slot[k] = g.grid.gx ? grid_slot(g.grid, x[k], y[k]) : -1;
                }
            }
            K3bRes<CPL> R;
            k3b_points<CPL>(g, p, x, y, slot, R);
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                if (id[k] < 0) continue;
                const int ps = c0 + k * 64 + lane;  // results at the sorted position
                int c = R.cnt[k];
                if (c > K3B_KT) {
                    c = K3B_REWALK;
                } else if (c > 1) {  // terms 2..c go to the segment's list
                    const int b = atomicAdd(s_tcnt, c - 1);
                    if (b + c - 1 > TCAP) {
                        c = K3B_REWALK;
                    } else {
                        s_tix[ps] = (uint16_t)b;
#pragma unroll
                        for (int m = 1; m < K3B_KT; ++m)
                            if (m < c) s_term[b + m - 1] = R.tm[k][m];
                    }
                }
                s_psi[ps] = R.tm[k][0];
                s_phi[ps] = R.pen[k];
                s_fl[ps] = (uint8_t)((R.hit[k] ? K3B_HIT : 0) | (c << 1));
            }
        }
        __syncthreads();
        // C: the path's lane adds its points in waypoint order (eval_path's chains)
        if (in) {
#pragma unroll
            for (int t = 0; t < S; ++t) {
                if (t >= sn) break;
                const int id = pos[t];
                a.cost = a.cost + s_phi[id] / dN;
                const uint8_t fl = s_fl[id];
                const int c = (fl >> 1) & 7;
                if (c == K3B_REWALK) {
                    double x, y;
                    seg_point(tid, t, x, y);
                    a.nsum = k3b_psi_chain(g, p, x, y, a.nsum);
                } else if (c) {
                    a.nsum = a.nsum + s_psi[id];
                    if (c > 1) {
                        const int b = s_tix[id];
                        for (int m = 1; m < c; ++m) a.nsum = a.nsum + s_term[b + m - 1];
                    }
                }
                a.nh += (fl & K3B_HIT) ? 1 : 0;
            }
        }
        __syncthreads();
    }
    // outputs staged through LDS exactly as k_eval_pairs does (the segment arrays are dead)
    double* s_cost = smem;
    double* s_L = s_cost + BP;
    double* s_len = s_L + BP;
    double* s_k = s_len + BP;
    double* s_n = s_k + BP;
    double* s_clr = s_n + BP;
    int32_t* s_nh = reinterpret_cast<int32_t*>(s_clr + BP);
    int32_t* s_off = s_nh + BP;
    int32_t* s_bel = s_off + BP;
    const int slot = d * 64 + lane;
    if (in) {
        s_cost[slot] = a.cost;
        s_L[slot] = a.L;
        s_len[slot] = a.len;
        s_k[slot] = a.ksum;
        s_n[slot] = a.nsum;
        s_clr[slot] = clearance(p, UAM_MODE_ANALYTIC, a);
        s_nh[slot] = a.nh;
        s_off[slot] = a.off;
        s_bel[slot] = a.below;
    }
    __syncthreads();
    const int qi = tid / D, di = tid - qi * D;
    if (q0 + qi < n_pairs) {
        const int64_t gp = (ordered ? (int64_t)order[q0 + qi] : q0 + qi) * D + di;
        const int s = di * 64 + qi;
        if (out.cost) out.cost[gp] = s_cost[s];
        if (out.length_q) out.length_q[gp] = s_L[s];
        if (out.length) out.length[gp] = s_len[s];
        if (out.kin_sum) out.kin_sum[gp] = s_k[s];
        if (out.nfz_sum) out.nfz_sum[gp] = s_n[s];
        if (out.min_clearance) out.min_clearance[gp] = s_clr[s];
        if (out.nfz_hits) out.nfz_hits[gp] = s_nh[s];
        if (out.offmap) out.offmap[gp] = s_off[s];
        if (out.below_terrain) out.below_terrain[gp] = s_bel[s];
    }
    if (d == 0 && in) {
        if (best_f) best_f[q] = select_best(s_cost + lane, 64, D, true);
        if (best_l) best_l[q] = select_best(s_len + lane, 64, D, false);
    }
}

// L(z + a dr); want (a = 0): gradient into gr and |gr|^2 into gn2.  Per-waypoint terms and
// gradient accumulation order as oracle refine_L.  The waypoint loop runs a wave-uniform trip
// count (lane j = jb + lane, valid = j < W) so the geometry can be walked by the whole wave.
__device__ __forceinline__ double rf_L(const KGeom& g, const KParams& p, const RfPath& rp,
                                       int lane, double a, double c, bool want, double* fout,
                                       double* gn2) {
    const int N = rp.N, W = rp.W;
    const bool ls = p.length_smooth != 0, ms = p.maxratio_smooth != 0;
    const double hc = 0.5 * c, dN = (double)N, sc = (double)(N + 1);
    const int kend = p.quirk_length ? N : N + 1;
    double sl = 0.0, sphi = 0.0, saug = 0.0, sg = 0.0;
    for (int jb = 0; jb < W; jb += 64) {
        const int j = jb + lane;
        const bool valid = j < W;
        const bool inner = want && valid && j >= 1 && j <= N;
        double xj = 0.0, yj = 0.0;
        if (valid) rp.pt(j, a, xj, yj);
        double ex, ey;
        const double ph = phi_vg_wave(g, p, xj, yj, valid, inner, ex, ey);
        double aj = 0.0, gx = 0.0, gy = 0.0;
        if (valid) {
            double lj = 0.0, vx0 = 0.0, vy0 = 0.0;
            if (j == 0) {
                if (p.quirk_length) {
                    const double ax = p.anchor_mode ? p.anchor_x : xj;
                    const double ay = p.anchor_mode ? p.anchor_y : yj;
                    lj = seg_term(ax, ay, xj, yj, ls, sc, false, vx0, vy0);
                }
            } else if (j <= kend) {
                double px, py;
                rp.pt(j - 1, a, px, py);
                lj = seg_term(px, py, xj, yj, ls, sc, inner, vx0, vy0);
            }
            sl = sl + lj;
            sphi = sphi + ph / dN;
            if (j < N) {
                double q1x, q1y, q2x, q2y, cv[3], dq[3][2];
                rp.pt(j + 1, a, q1x, q1y);
                rp.pt(j + 2, a, q2x, q2y);
                kin_col(xj, yj, q1x, q1y, q2x, q2y, p.r_eff, p.mincos, ms, -1, cv, dq);
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const double tt = cv[t] + rp.yk[3 * j + t] / c;
                    aj = aj + hc * (tt * tt);
                }
            }
            if (inner) {
                if (j <= kend) {
                    gx = gx + vx0;
                    gy = gy + vy0;
                }
                if (j + 1 <= kend) {
                    double qx, qy, vx, vy;
                    rp.pt(j + 1, a, qx, qy);
                    seg_term(xj, yj, qx, qy, ls, sc, true, vx, vy);
                    gx = gx - vx;
                    gy = gy - vy;
                }
                gx = gx + ex / dN;
                gy = gy + ey / dN;
                for (int q = 2; q >= 0; --q) {  // k = j - q ascending
                    const int k = j - q;
                    if (k < 0 || k >= N) continue;
                    double k0x, k0y, k1x, k1y, k2x, k2y, cv[3], dq[3][2];
                    rp.pt(k, a, k0x, k0y);
                    rp.pt(k + 1, a, k1x, k1y);
                    rp.pt(k + 2, a, k2x, k2y);
                    kin_col(k0x, k0y, k1x, k1y, k2x, k2y, p.r_eff, p.mincos, ms, q, cv, dq);
#pragma unroll
                    for (int t = 0; t < 3; ++t) {
                        if (!(cv[t] > 0.0)) continue;
                        const double coef = c * (cv[t] + rp.yk[3 * k + t] / c);
                        gx = gx + coef * dq[t][0];
                        gy = gy + coef * dq[t][1];
                    }
                }
            }
        }
        auto obstacle_row = [&](int s) {  // s wave-uniform
            const DevShape sh = uload(g.shape, s);
            double v = 0.0, ox = 0.0, oy = 0.0;
            if (!((sh.flags & SHAPE_CULL_PSI) && outside(sh.box_obs, xj, yj)))
                v = psi_vg_u(g, sh, xj, yj, 0.0, inner, ox, oy);
            const double tt = v + rp.yo[(int64_t)s * W + j] / c;
            aj = aj + hc * (tt * tt);
            if (inner && v != 0.0) {
                const double coef = c * tt;
                gx = gx + coef * ox;
                gy = gy + coef * oy;
            }
        };
        if (rp.act) {
            // each lane's candidate rows in ascending order; the wave walks their union so
            // the row index (and the shape's records) is wave-uniform
            uint64_t cw[RF_MASKW] = {0ull, 0ull, 0ull, 0ull};
            if (valid) rf_candidates(g, xj, yj, rp.act + (int64_t)j * rp.nmw, rp.nmw, cw);
            const int nw = (g.n_obstacles + 63) >> 6;
#pragma unroll 1
            for (int w = 0; w < nw; ++w) {
                const uint64_t mine = pick_word(cw, w);
                for (uint64_t b = wave_or_u64(mine); b; b &= b - 1) {
                    const int bit = __builtin_ctzll(b);
                    if ((mine >> bit) & 1ull) obstacle_row(64 * w + bit);
                }
            }
        } else if (valid) {
            for (int s = 0; s < g.n_obstacles; ++s) obstacle_row(s);
        }
        if (valid) {
            saug = saug + aj;
            double tg = 0.0;
            if (inner) {
                rp.gr[2 * j] = gx;
                rp.gr[2 * j + 1] = gy;
                tg = gx * gx + gy * gy;
            }
            sg = sg + tg;
        }
    }
    sl = wave_sum(sl);
    sphi = wave_sum(sphi);
    saug = wave_sum(saug);
    const double f = sc * sl + sphi;
    if (want) *gn2 = wave_sum(sg);
    if (fout) *fout = f;
    return f + saug;
}

// L-BFGS two-loop recursion: dr = -H gr over the cnt newest (s, y) pairs of the ring
__device__ __forceinline__ void lbfgs_dir_loops(const double* gr, double* dr, const double* hs,
                                                const double* hy, const double* rho,
                                                double gamma, int m, int cnt, int head, int N,
                                                int W, int lane) {
    double ai[RF_MAXM];
    for (int j = lane; j < W; j += 64) {
        if (j >= 1 && j <= N) {
            dr[2 * j] = gr[2 * j];
            dr[2 * j + 1] = gr[2 * j + 1];
        }
    }
#pragma unroll
    for (int i = 0; i < RF_MAXM; ++i) {
        if (i >= cnt) break;
        const int sl = (head - 1 - i + m) % m;
        const double* sv = hs + (int64_t)sl * 2 * W;
        const double* yv = hy + (int64_t)sl * 2 * W;
        ai[i] = rho[sl] * wdot(sv, dr, N, lane);
        for (int j = lane; j < W; j += 64) {
            if (j >= 1 && j <= N) {
                dr[2 * j] = dr[2 * j] - ai[i] * yv[2 * j];
                dr[2 * j + 1] = dr[2 * j + 1] - ai[i] * yv[2 * j + 1];
            }
        }
    }
    for (int j = lane; j < W; j += 64) {
        if (j >= 1 && j <= N) {
            dr[2 * j] = gamma * dr[2 * j];
            dr[2 * j + 1] = gamma * dr[2 * j + 1];
        }
    }
#pragma unroll
    for (int i = RF_MAXM - 1; i >= 0; --i) {
        if (i >= cnt) continue;
        const int sl = (head - 1 - i + m) % m;
        const double* sv = hs + (int64_t)sl * 2 * W;
        const double* yv = hy + (int64_t)sl * 2 * W;
        const double b = rho[sl] * wdot(yv, dr, N, lane);
        for (int j = lane; j < W; j += 64) {
            if (j >= 1 && j <= N) {
                dr[2 * j] = dr[2 * j] + sv[2 * j] * (ai[i] - b);
                dr[2 * j + 1] = dr[2 * j + 1] + sv[2 * j + 1] * (ai[i] - b);
            }
        }
    }
    for (int j = lane; j < W; j += 64) {
        if (j >= 1 && j <= N) {
            dr[2 * j] = -dr[2 * j];
            dr[2 * j + 1] = -dr[2 * j + 1];
        }
    }
}

// Two waypoint slots per lane (W <= 128): a lane's entries j = lane, lane + 64 of the ring
// vector at ring slot sl
struct RingPair {
    double a0, a1, b0, b1;  // (x, y) of slot 0, (x, y) of slot 1
};

__device__ __forceinline__ RingPair ring_load(const double* base, int sl, int W, int lane) {
    const double* v = base + (int64_t)sl * 2 * W;
    RingPair r{0.0, 0.0, 0.0, 0.0};
    const int j0 = lane, j1 = lane + 64;
    if (j0 < W) r.a0 = v[2 * j0], r.a1 = v[2 * j0 + 1];
    if (j1 < W) r.b0 = v[2 * j1], r.b1 = v[2 * j1 + 1];
    return r;
}

// The same recursion with the direction held in registers and each stage's ring vectors
// loaded one stage ahead (the loads do not depend on the recursion, its dot products do):
// every operation and its order are those of lbfgs_dir_loops, so dr is bit-identical.
__device__ __forceinline__ void lbfgs_dir(const double* gr, double* dr, const double* hs,
                                          const double* hy, const double* rho, double* ai,
                                          double gamma, int m, int cnt, int head, int N, int W,
                                          int lane) {
    if (W > 128 || !UAM_RF_PREFETCH) {
        lbfgs_dir_loops(gr, dr, hs, hy, rho, gamma, m, cnt, head, N, W, lane);
        return;
    }
    const int j0 = lane, j1 = lane + 64;
    const bool v0 = j0 < W, v1 = j1 < W;  // the lane's slots on the path (wdot's loop range)
    const bool in0 = j0 >= 1 && j0 <= N, in1 = j1 >= 1 && j1 <= N;
    double q0x = 0.0, q0y = 0.0, q1x = 0.0, q1y = 0.0;
    if (in0) q0x = gr[2 * j0], q0y = gr[2 * j0 + 1];
    if (in1) q1x = gr[2 * j1], q1y = gr[2 * j1 + 1];
    // lane-sequential dot over the lane's slots, then the xor tree (== wdot)
    auto dot = [&](const RingPair& u) {
        double s = 0.0;
        if (v0) s = s + (in0 ? u.a0 * q0x + u.a1 * q0y : 0.0);
        if (v1) s = s + (in1 ? u.b0 * q1x + u.b1 * q1y : 0.0);
        return wave_sum(s);
    };
    RingPair S{}, Y{};  // ai: the wave's LDS (uniform values, no registers held across loops)
    if (cnt > 0) {
        const int sl = (head - 1 + m) % m;
        S = ring_load(hs, sl, W, lane);
        Y = ring_load(hy, sl, W, lane);
    }
#pragma unroll
    for (int i = 0; i < RF_MAXM; ++i) {
        if (i >= cnt) break;
        const int sl = (head - 1 - i + m) % m;
        RingPair nS{}, nY{};
        if (i + 1 < cnt) {  // next stage's vectors, in flight during this stage's reduction
            const int nsl = (head - 2 - i + 2 * m) % m;
            nS = ring_load(hs, nsl, W, lane);
            nY = ring_load(hy, nsl, W, lane);
        }
        const double a = rho[sl] * dot(S);
        ai[i] = a;  // every lane writes the same value
        if (in0) q0x = q0x - a * Y.a0, q0y = q0y - a * Y.a1;
        if (in1) q1x = q1x - a * Y.b0, q1y = q1y - a * Y.b1;
        if (i + 1 < cnt) S = nS, Y = nY;
    }
    if (in0) q0x = gamma * q0x, q0y = gamma * q0y;
    if (in1) q1x = gamma * q1x, q1y = gamma * q1y;
    // second loop, oldest first: its first stage (i = cnt - 1) reuses the vectors the first
    // loop ended with
#pragma unroll
    for (int i = RF_MAXM - 1; i >= 0; --i) {
        if (i >= cnt) continue;
        const int sl = (head - 1 - i + m) % m;
        RingPair nS{}, nY{};
        if (i > 0) {
            const int nsl = (head - i + m) % m;
            nS = ring_load(hs, nsl, W, lane);
            nY = ring_load(hy, nsl, W, lane);
        }
        const double b = rho[sl] * dot(Y);
        const double d = ai[i] - b;
        if (in0) q0x = q0x + S.a0 * d, q0y = q0y + S.a1 * d;
        if (in1) q1x = q1x + S.b0 * d, q1y = q1y + S.b1 * d;
        if (i > 0) S = nS, Y = nY;
    }
    if (in0) dr[2 * j0] = -q0x, dr[2 * j0 + 1] = -q0y;
    if (in1) dr[2 * j1] = -q1x, dr[2 * j1 + 1] = -q1y;
}

// register budget: <= 128 VGPRs keeps 4 waves per SIMD (rf_L inlined at every call site; an
// out-of-line call spills around s_swappc)
// distance along the unit direction (ux, uy) from a point inside shape sh (every h_i < 0) to
// its boundary: the smallest positive root over its inequalities (oracle exit_dist, op for op)
__device__ double rf_exit_dist(const KGeom& g, const DevShape& sh, double x0, double x1,
                               double ux, double uy) {
    double t = INFINITY;
    for (int i = sh.first; i < sh.first + sh.count; ++i) {
        const DevIneq& q = g.ineq[i];
        const double h = ineq_h(&q, x0, x1);
        double ti = INFINITY;
        if (q.kind == UAM_INEQ_ELLIPSE) {
            const double a0 = (x0 - q.p[0]) / q.p[2], b0 = (x1 - q.p[1]) / q.p[3];
            const double da = ux / q.p[2], db = uy / q.p[3];
            double qa = 0.0, qb = 0.0;
            qa = qa + da * da;
            qa = qa + db * db;
            qb = qb + a0 * da;
            qb = qb + b0 * db;
            qb = 2.0 * qb;
            const double disc = qb * qb - (4.0 * qa) * h;
            if (qa > 0.0 && disc >= 0.0) ti = (sqrt(disc) - qb) / (2.0 * qa);
        } else {
            double gx, gy;
            ineq_grad(&q, x0, x1, gx, gy);
            double rate = 0.0;
            rate = rate + gx * ux;
            rate = rate + gy * uy;
            if (rate > 0.0) ti = -h / rate;
        }
        if (ti >= 0.0 && ti < t) t = ti;
    }
    return t;
}

// Restart of a stalled path (oracle refine_restart): the obstacle holding the most interior
// waypoints (ties: the lowest index) has them moved along the start-goal chord's normal to
// margin past its boundary, to the side their mean offset from its centre leans to.  Returns
// false (wave-uniform) when no interior waypoint lies inside an obstacle.
__device__ bool rf_restart(const KGeom& g, double* z, int N, int lane, double margin) {
    const int W = N + 2, S = g.n_obstacles;
    auto inside = [&](const DevShape& sh, double x, double y) {
        if ((sh.flags & SHAPE_CULL_PSI) && outside(sh.box_obs, x, y)) return false;  // psi +0
        return psi(g, sh, x, y, true, 0.0) > 0.0;
    };
    int best = -1, bestn = 0;
    for (int s = 0; s < S; ++s) {
        const DevShape& sh = g.shape[s];
        int n = 0;
        for (int j = lane; j < W; j += 64)
            if (j >= 1 && j <= N && inside(sh, z[2 * j], z[2 * j + 1])) ++n;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) n += __shfl_xor(n, off, 64);
        if (n > bestn) best = s, bestn = n;
    }
    if (best < 0) return false;
    const double cx = z[2 * (W - 1)] - z[0], cy = z[2 * (W - 1) + 1] - z[1];
    double l2 = 0.0;
    l2 = l2 + cx * cx;
    l2 = l2 + cy * cy;
    const double len = sqrt(l2);
    if (!(len > 0.0)) return false;
    const double nx = -cy / len, ny = cx / len;
    const DevShape& sh = g.shape[best];
    double ox = sh.cx, oy = sh.cy;
    if (isnan(ox) || isnan(oy))
        ox = 0.5 * (z[0] + z[2 * (W - 1)]), oy = 0.5 * (z[1] + z[2 * (W - 1) + 1]);
    double part = 0.0;
    bool mine[8];  // j = lane + 64 k, k < 8 (W <= 512 for the refinement)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int j = lane + 64 * k;
        mine[k] = j >= 1 && j <= N && inside(sh, z[2 * j], z[2 * j + 1]);
        if (j < W) part = part + (mine[k] ? (z[2 * j] - ox) * nx + (z[2 * j + 1] - oy) * ny : 0.0);
    }
    const double lean = wave_sum(part);
    const double sx = lean < 0.0 ? -nx : nx, sy = lean < 0.0 ? -ny : ny;
    wave_sync();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int j = lane + 64 * k;
        if (!mine[k]) continue;
        const double t = rf_exit_dist(g, sh, z[2 * j], z[2 * j + 1], sx, sy);
        if (!(t < INFINITY)) continue;
        const double step = t + margin;
        z[2 * j] = z[2 * j] + step * sx;
        z[2 * j + 1] = z[2 * j + 1] + step * sy;
    }
    wave_sync();
    return true;
}

// Restarts (n_restart > 0, uam_refine): attempt 0 is k_refine<false> (it also saves each path's
// final waypoints to zlast); then per restart k_rf_push moves zlast of every path still above
// delta and k_refine<true> runs the ALM again from it, keeping the better attempt (sum g^2,
// first on ties) in wp / cost / infeas -- oracle orc_refine's restart loop, one launch per
// step, so the plain refinement keeps its register budget.
__global__ __launch_bounds__(256) void k_rf_push(KGeom g, KParams p, KRefine rf, int64_t P,
                                                 double* __restrict__ zlast,
                                                 const double* __restrict__ infeas,
                                                 int32_t* __restrict__ active) {
    extern __shared__ double rp_lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    const int64_t path = (int64_t)blockIdx.x * wpb + wave;
    if (path >= P) return;  // whole wave
    if (!active[path]) return;
    const int N = p.N, W = N + 2;
    if (sqrt(infeas[path]) <= rf.delta) {  // converged: no further attempts
        if (lane == 0) active[path] = 0;
        return;
    }
    double* z = rp_lds + (int64_t)wave * 2 * W;
    double* zg = zlast + path * (int64_t)W * 2;
    for (int k = lane; k < 2 * W; k += 64) z[k] = zg[k];
    wave_sync();
    const bool ok = rf_restart(g, z, N, lane, rf.restart_margin);
    if (!ok) {
        if (lane == 0) active[path] = 0;
        return;
    }
    for (int k = lane; k < 2 * W; k += 64) zg[k] = z[k];
}

template <bool RESTART>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(UAM_RF_WAVES))) void k_refine(
    KGeom g, KParams p, KRefine rf, double* __restrict__ wp, int64_t P, double* __restrict__ ws,
    double* __restrict__ cost, double* __restrict__ infeas, int32_t* __restrict__ iters,
    double* __restrict__ zlast, const int32_t* __restrict__ active) {
    extern __shared__ double rf_lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    const int64_t path = (int64_t)blockIdx.x * wpb + wave;
    if (path >= P) return;  // whole wave
    if (RESTART && !active[path]) return;
    const int N = p.N, W = N + 2, S = g.n_obstacles;
    const int m = rf.memory < 0 ? 0 : (rf.memory > RF_MAXM ? RF_MAXM : rf.memory);
    const int nmw = rf_mask_words(S);
    double* z = rf_lds + (int64_t)wave * (6 * W + 3 * N + 2 * RF_MAXM + nmw * W);
    double* gr = z + 2 * W;
    double* dr = gr + 2 * W;
    double* yk = dr + 2 * W;
    double* rho = yk + 3 * N;
    double* aiv = rho + RF_MAXM;
    uint64_t* act = nmw ? reinterpret_cast<uint64_t*>(aiv + RF_MAXM) : nullptr;
    double* zg = wp + path * (int64_t)W * 2;
    double* yo = ws + path * ((int64_t)S * W + (int64_t)m * 4 * W);
    double* hs = yo + (int64_t)S * W;
    double* hy = hs + (int64_t)m * 2 * W;
    double* zl = zlast ? zlast + path * (int64_t)W * 2 : nullptr;
    for (int k = lane; k < 2 * W; k += 64) {
        z[k] = RESTART ? zl[k] : zg[k];
        gr[k] = 0.0;
        dr[k] = 0.0;
    }
    for (int k = lane; k < 3 * N; k += 64) yk[k] = 0.0;
    if (act)
        for (int k = lane; k < nmw * W; k += 64) act[k] = 0ull;
    for (int s = 0; s < S; ++s)
        for (int j = lane; j < W; j += 64) yo[(int64_t)s * W + j] = 0.0;
    wave_sync();
    RfPath rp{z, gr, dr, yk, yo, act, N, W, nmw};
    const bool ms = p.maxratio_smooth != 0;
    double c = rf.c0, alpha = rf.alpha0, prev = INFINITY, inf = 0.0, f = 0.0;
    int32_t used = 0;
    for (int o = 0; o < rf.n_outer; ++o) {
        int cnt = 0, head = 0;
        double gamma = 1.0, gn2 = 0.0;
        double Lz = rf_L(g, p, rp, lane, 0.0, c, true, nullptr, &gn2);
        wave_sync();
        for (int it = 0; it < rf.n_inner; ++it) {
            if (!(gn2 > 0.0) || !(gn2 < INFINITY)) break;  // wave-uniform
            if (sqrt(gn2) <= rf.inner_tol) break;
            double gd = 0.0, dn2 = gn2;
            if (cnt > 0) {
                lbfgs_dir(gr, dr, hs, hy, rho, aiv, gamma, m, cnt, head, N, W, lane);
                gd = wdot(gr, dr, N, lane);
                if (!(gd < 0.0))
                    cnt = 0;
                else
                    dn2 = wdot(dr, dr, N, lane);
            }
            if (cnt == 0) {
                for (int j = lane; j < W; j += 64) {
                    if (j >= 1 && j <= N) {
                        dr[2 * j] = -gr[2 * j];
                        dr[2 * j + 1] = -gr[2 * j + 1];
                    }
                }
                gd = -gn2;
                dn2 = gn2;
            }
            wave_sync();
            double a = fmin(cnt > 0 ? 1.0 : alpha * 2.0, rf.max_step / sqrt(dn2));
            bool ok = false;
            for (int b = 0; b < rf.max_backtrack; ++b) {
                const double Lt = rf_L(g, p, rp, lane, a, c, false, nullptr, nullptr);
                if (Lt <= Lz + (rf.armijo * a) * gd) {
                    ok = true;
                    break;
                }
                a = a * 0.5;
            }
            if (!ok) {
                if (cnt > 0) {  // retry along -g
                    cnt = 0;
                    continue;
                }
                break;
            }
            wave_sync();
            double* hsl = hs + (int64_t)head * 2 * W;
            double* hyl = hy + (int64_t)head * 2 * W;
            for (int j = lane; j < W; j += 64) {
                if (j >= 1 && j <= N) {
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const double st = a * dr[2 * j + e];
                        if (m > 0) {
                            hsl[2 * j + e] = st;
                            hyl[2 * j + e] = gr[2 * j + e];
                        }
                        z[2 * j + e] = z[2 * j + e] + st;
                    }
                }
            }
            wave_sync();
            alpha = a;
            ++used;
            Lz = rf_L(g, p, rp, lane, 0.0, c, true, nullptr, &gn2);
            wave_sync();
            if (m > 0) {
                for (int j = lane; j < W; j += 64) {
                    if (j >= 1 && j <= N) {
                        hyl[2 * j] = gr[2 * j] - hyl[2 * j];
                        hyl[2 * j + 1] = gr[2 * j + 1] - hyl[2 * j + 1];
                    }
                }
                const double sy = wdot(hsl, hyl, N, lane), yy = wdot(hyl, hyl, N, lane);
                if (sy > 0.0 && yy > 0.0) {
                    rho[head] = 1.0 / sy;  // same value from every lane
                    gamma = sy / yy;
                    head = (head + 1) % m;
                    if (cnt < m) ++cnt;
                }
                wave_sync();
            }
        }
        // outer update: y += c * row, inf = sum row^2 (kinematic rows of j, then obstacles)
        double si = 0.0;
        for (int j = lane; j < W; j += 64) {
            const double xj = z[2 * j], yj = z[2 * j + 1];
            double sj = 0.0;
            if (j < N) {
                double cv[3], dq[3][2];
                kin_col(xj, yj, z[2 * j + 2], z[2 * j + 3], z[2 * j + 4], z[2 * j + 5], p.r_eff,
                        p.mincos, ms, -1, cv, dq);
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    yk[3 * j + t] = yk[3 * j + t] + c * cv[t];
                    sj = sj + cv[t] * cv[t];
                }
            }
            auto update_row = [&](int s) {
                const DevShape& sh = g.shape[s];
                if ((sh.flags & SHAPE_CULL_PSI) && outside(sh.box_obs, xj, yj)) return;  // +0
                const double v = psi(g, sh, xj, yj, true, 0.0);
                double* yi = yo + (int64_t)s * W + j;
                *yi = *yi + c * v;
                sj = sj + v * v;
                if (act && v != 0.0) act[(int64_t)j * nmw + (s >> 6)] |= 1ull << (s & 63);
            };
            if (act) {  // rows with psi = 0 leave y and the sum unchanged
                uint64_t cw[RF_MASKW];
                rf_candidates(g, xj, yj, nullptr, 0, cw);
                const int nw = (S + 63) >> 6;
#pragma unroll 1
                for (int w = 0; w < nw; ++w)
                    for (uint64_t b = pick_word(cw, w); b; b &= b - 1)
                        update_row(64 * w + __builtin_ctzll(b));
            } else {
                for (int s = 0; s < S; ++s) update_row(s);
            }
            si = si + sj;
        }
        inf = wave_sum(si);
        wave_sync();
        if (inf > rf.theta * prev) c = fmin(c * rf.rho, rf.c_max);
        prev = inf;
        if (sqrt(inf) <= rf.delta) break;
    }
    if (zl && !RESTART)
        for (int k = lane; k < 2 * W; k += 64) zl[k] = z[k];
    if (RESTART) {
        for (int k = lane; k < 2 * W; k += 64) zl[k] = z[k];  // the next restart starts here
        const double best = infeas[path];                    // same value in every lane
        const int32_t before = iters[path];
        wave_sync();
        if (!(inf < best)) {  // the earlier attempt stays
            if (lane == 0) iters[path] = before + used;
            return;
        }
        used += before;
    }
    rf_L(g, p, rp, lane, 0.0, c, false, &f, nullptr);
    for (int k = lane; k < 2 * W; k += 64) zg[k] = z[k];
    if (lane == 0) {
        if (cost) cost[path] = f;
        if (infeas) infeas[path] = inf;
        if (iters) iters[path] = used;
    }
}

// ----------------------------------------------------------------------------------------
// K2w: wave-per-path evaluation for small batches (raster / volume modes).  The lane-per-path
// kernels walk a path serially, so a batch of 1k paths is 16 waves on a 256-CU chip and runs
// at the latency of one 256-waypoint walk.  Here lane l owns waypoints l, l+64, ...: points,
// segment norms, kinematic rows and record gathers run across the wave; the per-waypoint terms
// are staged in LDS and lane 0 forms every reference-ordered sum (L, length, kinematic sum,
// cost, no-fly sum) in exactly eval_path's order, so outputs are bit-identical to the
// lane-per-path kernels.  max terrain / min clearance / counts are order-free (shuffles).
__host__ __device__ constexpr int64_t ewave_doubles(int N) {
    return 6 * (int64_t)(N + 2) + 3 * (int64_t)N;
}

__device__ __forceinline__ double wave_fmax(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
    return v;
}
__device__ __forceinline__ double wave_fmin(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmin(v, __shfl_xor(v, off, 64));
    return v;
}
__device__ __forceinline__ int wave_isum(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Stable in-place compaction of a[0..n) (the wave's LDS slice) to its entries that are not
// ±0.0 (NaN is kept); returns their count.  Whole wave active.  Entry i moves to a position
// <= i, and each chunk is read by every lane before any lane writes, so nothing unread is
// overwritten.
__device__ __forceinline__ int wave_compact_nonzero(double* a, int n, int lane) {
    int cnt = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane;
        const double v = i < n ? a[i] : 0.0;
        const bool nz = i < n && !(v == 0.0);
        const uint64_t m = __ballot(nz);
        const int pos = cnt + __popcll(m & ((1ull << lane) - 1ull));
        wave_sync();
        if (nz) a[pos] = v;
        cnt += __popcll(m);
        wave_sync();
    }
    return cnt;
}


template <int MODE, bool GEN>
__global__ __launch_bounds__(256) void k_eval_wave(KGeom g, KParams p, KRaster rs, KVolume vs,
                                                   const uint4* __restrict__ rec,
                                                   const double* __restrict__ wp,
                                                   const double* __restrict__ pairs,
                                                   const double* __restrict__ utab, int D,
                                                   int64_t n_paths, KOut out) {
    extern __shared__ double ew_lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    const int64_t path = (int64_t)blockIdx.x * wpb + wave;
    if (path >= n_paths) return;  // whole wave
    const int N = p.N, W = N + 2;
    const bool ls = p.length_smooth != 0, ms = p.maxratio_smooth != 0;
    double* px = ew_lds + (int64_t)wave * ewave_doubles(N);
    double* py = px + W;
    double* lq = py + W;  // get_cost length term of the segment ending at j (anchor for j=0)
    double* sg = lq + W;  // true segment norm
    double* ph = sg + W;  // Phi_j / N
    double* ps = ph + W;  // no-fly psi_j
    double* kn = ps + W;  // kinematic rows [N][3]
    PathSrc<GEN> src;
    src.W = W;
    src.wp = nullptr;
    src.u = nullptr;
    src.x0 = src.y0 = src.xf = src.yf = 0.0;
    src.za = src.zb = 0.0;
    if (GEN) {
        const int64_t q = path / D;
        const int d = (int)(path - q * D);
        if (MODE == UAM_MODE_VOLUME) {
            const double* pr = pairs + 6 * q;
            src.x0 = pr[0], src.y0 = pr[1], src.za = pr[2];
            src.xf = pr[3], src.yf = pr[4], src.zb = pr[5];
        } else {
            const double4 pr = reinterpret_cast<const double4*>(pairs)[q];
            src.x0 = pr.x, src.y0 = pr.y, src.xf = pr.z, src.yf = pr.w;
        }
        src.u = utab + (int64_t)d * N * 2;
    } else {
        src.wp = wp + path * (int64_t)W * 2;
    }
    for (int j = lane; j < W; j += 64) {
        double x, y;
        src.at(j, x, y);
        px[j] = x;
        py[j] = y;
    }
    wave_sync();
    // geometry terms: lq = get_cost length term of the segment ending at j (anchor segment
    // for j = 0; +0.0 where eval_path adds nothing), sg = true segment norm, kinematic rows
    for (int j = lane; j < W; j += 64) {
        const double x = px[j], y = py[j];
        if (j == 0) {
            double t = 0.0;
            if (p.quirk_length) {
                const double ax = p.anchor_mode ? p.anchor_x : x;
                const double ay = p.anchor_mode ? p.anchor_y : y;
                const double dx = x - ax, dy = y - ay;
                double s = 0.0;
                s = s + dx * dx;
                s = s + dy * dy;
                const double n = sqrt(s);
                t = ls ? n * n : n;
            }
            lq[0] = t;
            sg[0] = 0.0;
        } else {
            const double dx = x - px[j - 1], dy = y - py[j - 1];
            double s = 0.0;
            s = s + dx * dx;
            s = s + dy * dy;
            const double n = sqrt(s);
            sg[j] = n;
            lq[j] = (!p.quirk_length || j <= N) ? (ls ? n * n : n) : 0.0;
            if (j >= 2) {  // kinematic row k = j-2, recomputing the previous segment
                const double pdx = px[j - 1] - px[j - 2], pdy = py[j - 1] - py[j - 2];
                double s2 = 0.0;
                s2 = s2 + pdx * pdx;
                s2 = s2 + pdy * pdy;
                const double n2 = sqrt(s2);
                const double pn = ms ? n2 * n2 : n2, nk = ms ? n * n : n;
                double dt = 0.0;
                dt = dt + pdx * dx;
                dt = dt + pdy * dy;
                double c1, c2, c3;
                kin_row(p, pn, nk, dt, c1, c2, c3);
                kn[3 * (j - 2)] = c1;
                kn[3 * (j - 2) + 1] = c2;
                kn[3 * (j - 2) + 2] = c3;
            }
        }
    }
    wave_sync();
    // eval_path's sequential sums, same order, on four lanes at once.  Every accumulator
    // starts at +0.0 and so is never -0.0, which makes a ±0.0 term an exact no-op: the
    // kinematic, no-fly and Φ/N term lists are compacted (stable, in place) to their nonzero
    // entries first -- an arc within the turn and ratio limits has no nonzero kinematic row.
    // Chains A (lane 0 L over W terms, lane 1 length, lane 3 kinematic sum) need only the
    // geometry terms, so they run while the first batch of record gathers is in flight;
    // chains B (lane 0 cost = (N+1) L + the nonzero Φ/N terms, lane 2 no-fly sum) follow.
    // The serial length is max(gather latency, W) + nnz(Φ) adds instead of max(2W, 3N).
    const int nkn = wave_compact_nonzero(kn, 3 * N, lane);
    double hmax = -INFINITY, cmin = INFINITY;
    int nh = 0, off = 0, below = 0;
    int32_t* cells = out.cells ? out.cells + path * W : nullptr;
    const double dN = (double)N;
    // record gathers, up to 4 per lane in flight; ph / ps = +0.0 for off-grid waypoints
    uint4 r[4];
    bool in[4];
    double zz[4];
    auto issue = [&](int jb) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = jb + 64 * t;
            in[t] = false;
            r[t] = make_uint4(0, 0, 0, 0);
            zz[t] = 0.0;
            if (j >= W) continue;
            const double x = px[j], y = py[j];
            int64_t cell;
            if (MODE == UAM_MODE_VOLUME) {
                const double z = src.alt(j);
                r[t] = vol_fetch(vs, nullptr, x, y, z, in[t], cell);
                zz[t] = z;
            } else {
                const double fx = floor((x - rs.x0) * rs.inv_dx);
                const double fy = floor((rs.y_top - y) * rs.inv_dy);
                in[t] = (fx >= 0.0) && (fx < (double)rs.nx) && (fy >= 0.0) &&
                        (fy < (double)rs.ny);
                cell = in[t] ? (int64_t)fy * rs.nx + (int64_t)fx : (int64_t)0;
                r[t] = rec[cell];
            }
            if (cells) cells[j] = in[t] ? (int32_t)cell : -1;
        }
    };
    auto consume = [&](int jb) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = jb + 64 * t;
            if (j >= W) continue;
            if (MODE == UAM_MODE_VOLUME) {
                if (in[t]) {
                    below += vol_below(vs, zz[t], r[t].z) ? 1 : 0;
                    cmin = fmin(cmin, zz[t] - (double)__uint_as_float(r[t].z));
                }
            } else {
                const double terrain = (!in[t] || (r[t].w & UAM_FLAG_NODATA))
                                           ? 0.0
                                           : (double)__uint_as_float(r[t].z);
                hmax = fmax(hmax, terrain);  // off-raster counts as sea level
            }
            if (in[t]) {
                ph[j] = (double)__uint_as_float(r[t].x) / dN;
                ps[j] = (double)__uint_as_float(r[t].y);
                nh += (r[t].w & UAM_FLAG_NFZ) ? 1 : 0;
            } else {
                ph[j] = 0.0;
                ps[j] = 0.0;
                ++off;
            }
        }
    };
    issue(lane);
    // chains A, beside the gathers
    const double* arr = lane == 0 ? lq : (lane == 1 ? sg : kn);
    const int na = lane < 2 ? W : (lane == 3 ? nkn : 0);
    double acc = 0.0;
#pragma unroll 8
    for (int i = 0; i < na; ++i) acc = acc + arr[i];
    consume(lane);
    for (int jb = lane + 256; jb < W; jb += 256) {
        issue(jb);
        consume(jb);
    }
    hmax = wave_fmax(hmax);
    cmin = wave_fmin(cmin);
    nh = wave_isum(nh);
    off = wave_isum(off);
    below = wave_isum(below);
    wave_sync();
    const int nps = wave_compact_nonzero(ps, W, lane);
    const int nph = wave_compact_nonzero(ph, W, lane);
    // chains B
    double L = acc;
    if (lane == 0) acc = (double)(N + 1) * L;
    const double* brr = lane == 0 ? ph : ps;
    const int nb = lane == 0 ? nph : (lane == 2 ? nps : 0);
#pragma unroll 8
    for (int i = 0; i < nb; ++i) acc = acc + brr[i];
    L = __shfl(L, 0, 64);
    const double len = __shfl(acc, 1, 64), nsum = __shfl(acc, 2, 64);
    const double ksum = __shfl(acc, 3, 64);
    if (lane == 0) {
        const double cost = acc;
        if (out.cost) out.cost[path] = cost;
        if (out.length_q) out.length_q[path] = L;
        if (out.length) out.length[path] = len;
        if (out.kin_sum) out.kin_sum[path] = ksum;
        if (out.nfz_sum) out.nfz_sum[path] = nsum;
        if (out.nfz_hits) out.nfz_hits[path] = nh;
        if (out.offmap) out.offmap[path] = off;
        if (out.min_clearance)
            out.min_clearance[path] = MODE == UAM_MODE_RASTER ? p.altitude - hmax : cmin;
        if (out.below_terrain) out.below_terrain[path] = below;
    }
}

// ----------------------------------------------------------------------------------------
// K7: coordinate reference systems.  Transverse Mercator between
// geographic JGD2000/JGD2011 (lon, lat degrees) and the Japan Plane Rectangular CS (metres),
// the transform pyproj applies at data_manager.py:24-26 / 84-85 and main.py:106-115.  Krueger
// series to n^6, geodetic latitude from conformal latitude by 2 Newton steps; definition and
// coefficient formulas as oracle/uam_oracle.c (tm_prepare / tm_fwd1 / tm_inv1); the host
// computes the coefficients once (KTm) so device and oracle share them.
struct KTm {
    double k0, A, e, e2, xi0, lon0, fe, fn;
    double alpha[6], beta[6];
};

// Krueger series by complex Clenshaw summation: oracle/uam_oracle.c kr_sum, same operations
__device__ __forceinline__ void kr_sum(const double (&c)[6], double xi, double eta, double& sr,
                                       double& si) {
    const double s2 = sin(2.0 * xi), c2 = cos(2.0 * xi);
    const double sh = sinh(2.0 * eta), ch = cosh(2.0 * eta);
    const double ar = 2.0 * (c2 * ch), ai = -2.0 * (s2 * sh);
    double y0r = 0.0, y0i = 0.0, y1r = 0.0, y1i = 0.0;
#pragma unroll
    for (int j = 5; j >= 0; --j) {
        const double tr = (ar * y0r - ai * y0i) - y1r + c[j];
        const double ti = (ar * y0i + ai * y0r) - y1i;
        y1r = y0r;
        y1i = y0i;
        y0r = tr;
        y0i = ti;
    }
    const double zr = s2 * ch, zi = c2 * sh;
    sr = y0r * zr - y0i * zi;
    si = y0r * zi + y0i * zr;
}

// kr_sum with sin/cos(2 xi) and sinh/cosh(2 eta) given (same operations after them)
__device__ __forceinline__ void kr_sum_pre(const double (&c)[6], double s2, double c2, double sh,
                                           double ch, double& sr, double& si) {
    const double ar = 2.0 * (c2 * ch), ai = -2.0 * (s2 * sh);
    double y0r = 0.0, y0i = 0.0, y1r = 0.0, y1i = 0.0;
#pragma unroll
    for (int j = 5; j >= 0; --j) {
        const double tr = (ar * y0r - ai * y0i) - y1r + c[j];
        const double ti = (ar * y0i + ai * y0r) - y1i;
        y1r = y0r;
        y1i = y0i;
        y0r = tr;
        y0i = ti;
    }
    const double zr = s2 * ch, zi = c2 * sh;
    sr = y0r * zr - y0i * zi;
    si = y0r * zi + y0i * zr;
}

__device__ __forceinline__ void tm_fwd(const KTm& k, double lon, double lat, double& x,
                                       double& y) {
    const double phi = lat * (M_PI / 180.0), dl = lon * (M_PI / 180.0) - k.lon0;
    const double s = sin(phi);
    const double tt = sinh(atanh(s) - k.e * atanh(k.e * s));
    const double xp = atan2(tt, cos(dl));
    const double ep = atanh(sin(dl) / sqrt(1.0 + tt * tt));
    double sr, si;
    kr_sum(k.alpha, xp, ep, sr, si);
    const double xi = xp + sr, eta = ep + si;
    x = k.k0 * k.A * eta + k.fe;
    y = k.k0 * k.A * (xi - k.xi0) + k.fn;
}

// the part of tm_inv after the series' trigonometric inputs (shared by both forms below)
__device__ __forceinline__ void tm_inv_tail(const KTm& k, double xi, double eta, double sr,
                                            double si, double& lon, double& lat);

__device__ __forceinline__ void tm_inv(const KTm& k, double x, double y, double& lon,
                                       double& lat) {
    const double kA = k.k0 * k.A;
    const double xi = (y - k.fn) / kA + k.xi0, eta = (x - k.fe) / kA;
    double sr, si;
    kr_sum(k.beta, xi, eta, sr, si);
    tm_inv_tail(k, xi, eta, sr, si, lon, lat);
}

__device__ __forceinline__ void tm_inv_tail(const KTm& k, double xi, double eta, double sr,
                                            double si, double& lon, double& lat) {
    const double xp = xi - sr, ep = eta - si;
    const double se = sinh(ep), cx = cos(xp);
    const double taup = sin(xp) / sqrt(se * se + cx * cx);
    const double lam = atan2(se, cx);
    const double e = k.e, e2m = 1.0 - k.e2;
    double tau = taup / e2m;  // oracle tm_inv1: GeographicLib's start, 2 Newton steps
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const double r = sqrt(1.0 + tau * tau);
        const double sg = sinh(e * atanh(e * tau / r));
        const double tp = tau * sqrt(1.0 + sg * sg) - sg * r;
        tau = tau + (taup - tp) * (1.0 + e2m * tau * tau) / (e2m * sqrt(1.0 + tp * tp) * r);
    }
    lat = atan(tau) * (180.0 / M_PI);
    lon = (lam + k.lon0) * (180.0 / M_PI);
}

__global__ __launch_bounds__(256) void k_tm_points(KTm k, int inverse,
                                                   const double* __restrict__ in, int64_t n,
                                                   double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double2 v = reinterpret_cast<const double2*>(in)[i];
    double a, b;
    if (inverse)
        tm_inv(k, v.x, v.y, a, b);
    else
        tm_fwd(k, v.x, v.y, a, b);
    reinterpret_cast<double2*>(out)[i] = make_double2(a, b);
}

struct KGeoGrid {
    int32_t nx, ny;
    double lon0, lat_top, dlon, dlat;
    float nodata;
};

// The output grid is axis-aligned in the plane, so the series' inputs separate: xi depends on
// the row only and eta on the column only.  k_tm_sep tabulates (xi, sin 2xi, cos 2xi) per row
// and (eta, sinh 2eta, cosh 2eta) per column, with tm_inv's own expressions, so each cell
// skips four transcendentals and the results are the same bits.
__global__ __launch_bounds__(256) void k_tm_sep(KTm k, KRaster r, double unit,
                                                double* __restrict__ rowtab,
                                                double* __restrict__ coltab) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const double kA = k.k0 * k.A;
    if (i < r.ny) {
        const double yc = r.y_top - ((double)i + 0.5) * r.dy;
        const double xi = (yc * unit - k.fn) / kA + k.xi0;
        rowtab[3 * i] = xi;
        rowtab[3 * i + 1] = sin(2.0 * xi);
        rowtab[3 * i + 2] = cos(2.0 * xi);
    } else if (i < (int64_t)r.ny + r.nx) {
        const int64_t ix = i - r.ny;
        const double xc = r.x0 + ((double)ix + 0.5) * r.dx;
        const double eta = (xc * unit - k.fe) / kA;
        coltab[3 * ix] = eta;
        coltab[3 * ix + 1] = sinh(2.0 * eta);
        coltab[3 * ix + 2] = cosh(2.0 * eta);
    }
}

// DEM reprojection (definition: oracle orc_reproject).  One lane per output cell, rows
// contiguous (coalesced 4-B stores); neighbouring cells read neighbouring source pixels.
__global__ __launch_bounds__(256) void k_reproject(KTm k, KGeoGrid g, KRaster r, double unit,
                                                   int resample, const float* __restrict__ src,
                                                   const double* __restrict__ rowtab,
                                                   const double* __restrict__ coltab,
                                                   float* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)r.nx * r.ny) return;
    const int64_t iy = i / r.nx, ix = i - iy * r.nx;
    double lon, lat;
    {
        const double xi = rowtab[3 * iy], eta = coltab[3 * ix];
        double sr, si;
        kr_sum_pre(k.beta, rowtab[3 * iy + 1], rowtab[3 * iy + 2], coltab[3 * ix + 1],
                   coltab[3 * ix + 2], sr, si);
        tm_inv_tail(k, xi, eta, sr, si, lon, lat);
    }
    const double u = (lon - g.lon0) / g.dlon, v = (g.lat_top - lat) / g.dlat;
    float val = g.nodata;
    const double fu = floor(u), fv = floor(v);
    if (fu >= 0.0 && fu < (double)g.nx && fv >= 0.0 && fv < (double)g.ny) {
        val = src[(int64_t)fv * g.nx + (int64_t)fu];
        if (resample == 1) {
            const double uu = u - 0.5, vv = v - 0.5;
            const double bu = floor(uu), bv = floor(vv);
            if (bu >= 0.0 && bu + 1.0 < (double)g.nx && bv >= 0.0 && bv + 1.0 < (double)g.ny) {
                const int64_t i0 = (int64_t)bv * g.nx + (int64_t)bu;
                const float a00 = src[i0], a01 = src[i0 + 1], a10 = src[i0 + g.nx],
                            a11 = src[i0 + g.nx + 1];
                if (a00 != g.nodata && a01 != g.nodata && a10 != g.nodata && a11 != g.nodata) {
                    const double wu = uu - bu, wv = vv - bv;
                    const double top = (double)a00 + wu * ((double)a01 - (double)a00);
                    const double bot = (double)a10 + wu * ((double)a11 - (double)a10);
                    val = (float)(top + wv * (bot - top));
                }
            }
        }
    }
    dst[i] = val;
}

// ----------------------------------------------------------------------------------------
// K8: DEM polygonisation: the connected regions rasterio.features.shapes
// returns for the DEM mask (data_manager.py:11-19, 4-connectivity), as union-find labels.
// L[i] = smallest linear index of i's component (the root), -1 off the mask.  Merging hooks
// the larger root under the smaller with atomicMin (L[x] <= x always holds, so every find
// terminates); labels are flattened afterwards.  A labelling grid may carry "cuts": cells s and
// s+1 of a row (t and t+1 of a column) connect only when colbox[s] == colbox[s+1]
// (rowbox[t] == rowbox[t+1]) -- the split of a large polygon into its box pieces
// (data_processor.py:34-51) as labelling on a grid refined at the box edges.
__device__ __forceinline__ int32_t ccl_find(const int32_t* L, int32_t x) {
    while (true) {
        const int32_t p = __hip_atomic_load(&L[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p == x || p < 0 || p > x) return x;  // L[x] <= x always; never walk out of range
        x = p;
    }
}

__device__ __forceinline__ void ccl_union(int32_t* L, int32_t a, int32_t b) {
    while (true) {
        a = ccl_find(L, a);
        b = ccl_find(L, b);
        if (a == b) return;
        if (a > b) {
            const int32_t t = a;
            a = b;
            b = t;
        }
        const int32_t old = atomicMin(&L[b], a);
        if (old == b) return;  // b was a root: now under a
        b = old;               // somebody re-hooked b meanwhile: retry from its new parent
    }
}

// mask of data_manager.py:14-17: dem == -9999 when threshold == -9999, else dem > threshold.
// Each cell starts labelled with the first cell of its horizontal run inside its wave (ballot
// of run breaks), so k_ccl_merge only has to join runs across waves and rows.
__device__ __forceinline__ int32_t run_start_label(bool m, int64_t i, int32_t nx,
                                                   bool cut_before = false) {
    const int lane = threadIdx.x & 63;
    const int prev = __shfl_up((int)m, 1, 64);  // every lane takes part (no divergence)
    const bool brk = m && (lane == 0 || (i % nx) == 0 || !prev || cut_before);
    const uint64_t b = __ballot(brk) & ((lane == 63) ? ~0ull : ((2ull << lane) - 1ull));
    const int start = 63 - __clzll(b);  // highest break at or below this lane
    return m ? (int32_t)(i - (lane - start)) : -1;
}

__global__ __launch_bounds__(256) void k_ccl_init_dem(const float* __restrict__ dem, int64_t n,
                                                      int32_t nx, float thr,
                                                      int32_t* __restrict__ L) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool m = false;
    if (i < n) {
        const float v = dem[i];
        m = (thr == -9999.0f) ? (v == -9999.0f) : (v > thr);
    }
    const int32_t l = run_start_label(m, i, nx);
    if (i < n) L[i] = l;
}

// refined sub-grid of one component: cell (s, t) <-> source pixel (col_of[s], row_of[t])
__global__ __launch_bounds__(256) void k_ccl_init_sub(const int32_t* __restrict__ Lsrc,
                                                      int32_t src_nx, int32_t root,
                                                      const int32_t* __restrict__ col_of,
                                                      const int32_t* __restrict__ row_of,
                                                      const int32_t* __restrict__ colbox,
                                                      int32_t ws, int32_t hs,
                                                      int32_t* __restrict__ L) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < (int64_t)ws * hs;
    const int32_t t = valid ? (int32_t)(i / ws) : 0, s = valid ? (int32_t)(i - (int64_t)t * ws) : 0;
    const bool m = valid && Lsrc[(int64_t)row_of[t] * src_nx + col_of[s]] == root;
    const bool cut = valid && s > 0 && colbox[s] != colbox[s - 1];
    const int32_t l = run_start_label(m, i, ws, cut);
    if (valid) L[i] = l;
}

// Joins 4-neighbours.  With runs pre-labelled (runs = true) only two kinds of join remain:
// the left neighbour across a wave boundary, and the cell above when the left neighbour does
// not already connect the same two rows (left and above-left both on the mask).
__global__ __launch_bounds__(256) void k_ccl_merge(int32_t nx, int32_t ny,
                                                   const int32_t* __restrict__ colbox,
                                                   const int32_t* __restrict__ rowbox, int runs,
                                                   int32_t* __restrict__ L) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)nx * ny) return;
    if (L[i] < 0) return;
    const int32_t y = (int32_t)(i / nx), x = (int32_t)(i - (int64_t)y * nx);
    if (runs) {
        const bool left = x > 0 && L[i - 1] >= 0 && (!colbox || colbox[x] == colbox[x - 1]);
        if (left && (threadIdx.x & 63) == 0) ccl_union(L, (int32_t)i, (int32_t)(i - 1));
        if (y > 0 && L[i - nx] >= 0 && (!rowbox || rowbox[y] == rowbox[y - 1]) &&
            !(left && L[i - nx - 1] >= 0))
            ccl_union(L, (int32_t)i, (int32_t)(i - nx));
        return;
    }
    if (x + 1 < nx && L[i + 1] >= 0 && (!colbox || colbox[x] == colbox[x + 1]))
        ccl_union(L, (int32_t)i, (int32_t)(i + 1));
    if (y + 1 < ny && L[i + nx] >= 0 && (!rowbox || rowbox[y] == rowbox[y + 1]))
        ccl_union(L, (int32_t)i, (int32_t)(i + nx));
}

__global__ __launch_bounds__(256) void k_ccl_flatten(int64_t n, int32_t* __restrict__ L) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || L[i] < 0) return;
    L[i] = ccl_find(L, (int32_t)i);
}

#include "ccl_tile.inc"

constexpr int CCL_ITEMS = 16;  // cells per thread in the root scan (block = 256 x 16 cells)

__global__ __launch_bounds__(256) void k_ccl_count_roots(const int32_t* __restrict__ L,
                                                         int64_t n, int32_t* __restrict__ cnt) {
    const int64_t base = (int64_t)blockIdx.x * 256 * CCL_ITEMS;
    int c = 0;
    for (int it = 0; it < CCL_ITEMS; ++it) {
        const int64_t i = base + (int64_t)it * 256 + threadIdx.x;
        if (i < n && L[i] == (int32_t)i) ++c;
    }
    c = wave_isum(c);
    __shared__ int part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// component id of every root = rank of the root in raster order (deterministic)
__global__ __launch_bounds__(256) void k_ccl_assign(const int32_t* __restrict__ L, int64_t n,
                                                    const int32_t* __restrict__ off,
                                                    int32_t* __restrict__ cid) {
    const int64_t base = (int64_t)blockIdx.x * 256 * CCL_ITEMS;
    __shared__ int wsum[4];
    int running = off[blockIdx.x];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int it = 0; it < CCL_ITEMS; ++it) {
        const int64_t i = base + (int64_t)it * 256 + threadIdx.x;
        const bool r = i < n && L[i] == (int32_t)i;
        const uint64_t bal = __ballot(r);
        const int before = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wv] = __popcll(bal);
        __syncthreads();
        int woff = 0;
        for (int k = 0; k < wv; ++k) woff += wsum[k];
        if (r) cid[i] = running + woff + before;
        running += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
}

// per component: cell count, bounding box and root.  Each block folds its 256 x CCL_ITEMS
// cells into a small LDS table (open addressing on the component id), then flushes one set
// of global atomics per distinct component: a large region costs O(blocks) global atomics
// instead of O(cells).  Table overflow falls back to direct global atomics.
constexpr int STAT_SLOTS = 32;

__global__ __launch_bounds__(256) void k_ccl_stats(const int32_t* __restrict__ L,
                                                   const int32_t* __restrict__ cid, int32_t nx,
                                                   int64_t n, int32_t* __restrict__ cnt,
                                                   int32_t* __restrict__ bx0,
                                                   int32_t* __restrict__ by0,
                                                   int32_t* __restrict__ bx1,
                                                   int32_t* __restrict__ by1,
                                                   int32_t* __restrict__ croot) {
    __shared__ int32_t key[STAT_SLOTS], sc[STAT_SLOTS], sx0[STAT_SLOTS], sy0[STAT_SLOTS],
        sx1[STAT_SLOTS], sy1[STAT_SLOTS];
    if (threadIdx.x < STAT_SLOTS) {
        key[threadIdx.x] = -1;
        sc[threadIdx.x] = 0;
        sx0[threadIdx.x] = sy0[threadIdx.x] = INT32_MAX;
        sx1[threadIdx.x] = sy1[threadIdx.x] = -1;
    }
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * 256 * CCL_ITEMS;
    for (int it = 0; it < CCL_ITEMS; ++it) {
        const int64_t i = base + (int64_t)it * 256 + threadIdx.x;
        const bool in = i < n && L[i] >= 0;
        const int32_t c = in ? cid[L[i]] : -1;
        if (in && L[i] == (int32_t)i) croot[c] = (int32_t)i;
        const int32_t y = in ? (int32_t)(i / nx) : 0, x = in ? (int32_t)(i - (int64_t)y * nx) : 0;
        // wave-uniform component: reduce in registers first
        const int32_t c0 = __shfl(c, 0, 64);
        const bool uni = __ballot(c != c0) == 0;
        int32_t cc = c, k = 1, xmn = x, xmx = x, ymn = y, ymx = y;
        bool lead = true;
        if (uni) {
            k = wave_isum(1);
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                xmn = min(xmn, __shfl_xor(xmn, o, 64));
                xmx = max(xmx, __shfl_xor(xmx, o, 64));
                ymn = min(ymn, __shfl_xor(ymn, o, 64));
                ymx = max(ymx, __shfl_xor(ymx, o, 64));
            }
            lead = (threadIdx.x & 63) == 0;
        }
        if (cc < 0 || !lead) continue;
        int slot = -1;
        for (int p = 0; p < STAT_SLOTS; ++p) {
            const int h = (int)(((uint32_t)cc * 2654435761u + p) % STAT_SLOTS);
            const int32_t old = atomicCAS(&key[h], -1, cc);
            if (old == -1 || old == cc) {
                slot = h;
                break;
            }
        }
        if (slot >= 0) {
            atomicAdd(&sc[slot], k);
            atomicMin(&sx0[slot], xmn);
            atomicMax(&sx1[slot], xmx);
            atomicMin(&sy0[slot], ymn);
            atomicMax(&sy1[slot], ymx);
        } else {
            atomicAdd(&cnt[cc], k);
            atomicMin(&bx0[cc], xmn);
            atomicMax(&bx1[cc], xmx);
            atomicMin(&by0[cc], ymn);
            atomicMax(&by1[cc], ymx);
        }
    }
    __syncthreads();
    if (threadIdx.x < STAT_SLOTS) {
        const int32_t cc = key[threadIdx.x];
        if (cc >= 0) {
            atomicAdd(&cnt[cc], sc[threadIdx.x]);
            atomicMin(&bx0[cc], sx0[threadIdx.x]);
            atomicMax(&bx1[cc], sx1[threadIdx.x]);
            atomicMin(&by0[cc], sy0[threadIdx.x]);
            atomicMax(&by1[cc], sy1[threadIdx.x]);
        }
    }
}

// per kept component and row: leftmost / rightmost cell (hull input)
__global__ __launch_bounds__(256) void k_ccl_extents(const int32_t* __restrict__ L,
                                                     const int32_t* __restrict__ cid,
                                                     int32_t nx, int64_t n,
                                                     const int64_t* __restrict__ row_off,
                                                     const int32_t* __restrict__ by0,
                                                     int32_t* __restrict__ xmin,
                                                     int32_t* __restrict__ xmax) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = i < n && L[i] >= 0;
    const int32_t c = in ? cid[L[i]] : -1;
    const int64_t ro = c >= 0 ? row_off[c] : -1;
    const int32_t y = in ? (int32_t)(i / nx) : 0, x = in ? (int32_t)(i - (int64_t)y * nx) : 0;
    const int64_t slot = ro >= 0 ? ro + (y - by0[c]) : -1;
    const int64_t s0 = __shfl(slot, 0, 64);
    if (__ballot(slot != s0) == 0) {
        if (s0 < 0) return;
        int xmn = x, xmx = x;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            xmn = min(xmn, __shfl_xor(xmn, o, 64));
            xmx = max(xmx, __shfl_xor(xmx, o, 64));
        }
        if ((threadIdx.x & 63) == 0) {
            atomicMin(&xmin[s0], xmn);
            atomicMax(&xmax[s0], xmx);
        }
        return;
    }
    if (slot < 0) return;
    atomicMin(&xmin[slot], x);
    atomicMax(&xmax[slot], x);
}

// nseg consecutive arrays of n values, array k filled with v[k]: one launch instead of nseg
struct FillSegs {
    int32_t v[6];
};
__global__ __launch_bounds__(256) void k_fill_segs_i32(int32_t* __restrict__ p, int64_t n,
                                                       int32_t nseg, FillSegs fs) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int k = 0; k < nseg; ++k) p[k * n + i] = fs.v[k];
}

// exclusive scan of n int32 (n < 2^31): per-block scan, then the block-total scan; the
// consumers add the scanned block total themselves
constexpr int SCAN_ITEMS = 16;
__global__ __launch_bounds__(256) void k_scan_local(const int32_t* __restrict__ in, int64_t n,
                                                    int32_t* __restrict__ out,
                                                    int32_t* __restrict__ totals) {
    __shared__ int32_t wsum[4];
    const int64_t base = (int64_t)blockIdx.x * 256 * SCAN_ITEMS + (int64_t)threadIdx.x * SCAN_ITEMS;
    int32_t v[SCAN_ITEMS], run = 0;
    const bool full = base + SCAN_ITEMS <= n;  // a whole run: 16-B loads and stores
    if (full) {
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; k += 4) {
            const int4 q = *reinterpret_cast<const int4*>(in + base + k);
            v[k] = q.x, v[k + 1] = q.y, v[k + 2] = q.z, v[k + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k) v[k] = base + k < n ? in[base + k] : 0;
    }
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        const int32_t t = v[k];
        v[k] = run;
        run += t;
    }
    // inclusive scan of the thread totals across the block
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int32_t x = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int32_t woff = 0;
    for (int k = 0; k < wv; ++k) woff += wsum[k];
    const int32_t excl = woff + x - run;
    if (full) {
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; k += 4)
            *reinterpret_cast<int4*>(out + base + k) =
                make_int4(v[k] + excl, v[k + 1] + excl, v[k + 2] + excl, v[k + 3] + excl);
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k)
            if (base + k < n) out[base + k] = v[k] + excl;
    }
    if (threadIdx.x == 255) totals[blockIdx.x] = woff + x;
}

__global__ __launch_bounds__(1024) void k_scan_totals(int32_t* __restrict__ totals, int n) {
    __shared__ int32_t buf[4096];
    __shared__ int32_t part[1024];
    int32_t run = 0;
    for (int k = 0; k < 4; ++k) {
        const int i = threadIdx.x * 4 + k;
        buf[i] = i < n ? totals[i] : 0;
    }
    __syncthreads();
    for (int k = 0; k < 4; ++k) {
        const int i = threadIdx.x * 4 + k;
        const int32_t t = buf[i];
        buf[i] = run;
        run += t;
    }
    part[threadIdx.x] = run;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan of 1024 totals
        const int32_t y = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += y;
        __syncthreads();
    }
    const int32_t excl = part[threadIdx.x] - run;
    for (int k = 0; k < 4; ++k) {
        const int i = threadIdx.x * 4 + k;
        if (i < n) totals[i] = buf[i] + excl;
    }
}

// raster cell of a point (uampath.h convention, exactly issue_chunk's arithmetic)
__device__ __forceinline__ bool raster_cell(const KRaster& rs, double x0, double x1, int& ix,
                                            int& iy) {
    const double fx = floor((x0 - rs.x0) * rs.inv_dx);
    const double fy = floor((rs.y_top - x1) * rs.inv_dy);
    const bool in = (fx >= 0.0) && (fx < (double)rs.nx) && (fy >= 0.0) && (fy < (double)rs.ny);
    ix = in ? (int)fx : 0;
    iy = in ? (int)fy : 0;
    return in;
}

__global__ __launch_bounds__(256) void k_gen_paths(const double* __restrict__ pairs,
                                                   int64_t n_pairs,
                                                   const double* __restrict__ utab, int D,
                                                   int N, double* __restrict__ wp) {
    const int W = N + 2;
    const int64_t total = n_pairs * D * W;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t path = i / W;
        const int j = (int)(i - path * W);
        const int64_t q = path / D;
        const int d = (int)(path - q * D);
        const double4 pr = reinterpret_cast<const double4*>(pairs)[q];
        double px, py;
        if (j == 0) {
            px = pr.x;
            py = pr.y;
        } else if (j == W - 1) {
            px = pr.z;
            py = pr.w;
        } else {
            const double* u = utab + ((int64_t)d * N + (j - 1)) * 2;
            arc_point(pr.x, pr.y, pr.z, pr.w, u[0], u[1], px, py);
        }
        wp[2 * i] = px;
        wp[2 * i + 1] = py;
    }
}

// main.py:175-180 (see uam_argmin)
__global__ __launch_bounds__(256) void k_argmin(const double* __restrict__ v, int64_t groups,
                                                int G, int take_sqrt, int32_t* __restrict__ best) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= groups) return;
    int bi = 0;
    double bv = 0.0;
    for (int d = 0; d < G; ++d) {
        const double x = take_sqrt ? sqrt(v[q * G + d]) : v[q * G + d];
        if (bv == 0.0 || x < bv) {
            bv = x;
            bi = d;
        }
    }
    best[q] = bi;
}

__global__ __launch_bounds__(256) void k_path_length(const double* __restrict__ pts,
                                                     int64_t n_paths, int n_points, int n_seg,
                                                     int smooth, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_paths) return;
    const double* z = pts + i * (int64_t)n_points * 2;
    double acc = 0.0;
    for (int k = 0; k < n_seg; ++k) {
        const double dx = z[2 * k + 2] - z[2 * k], dy = z[2 * k + 3] - z[2 * k + 1];
        double s = 0.0;
        s = s + dx * dx;
        s = s + dy * dy;
        const double n = sqrt(s);
        acc = acc + (smooth ? n * n : n);
    }
    out[i] = acc;
}

// ----------------------------------------------------------------------------------------
// host side

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(UAM_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));        \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int grid_for(int64_t n, int block, int64_t cap = 1 << 20) {
    int64_t b = (n + block - 1) / block;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (int)b;
}

// Conservative axis-aligned box of {x : h_i(x) < e for all inequalities i of a shape},
// padded by 1e-6 km (>> float64 error of h) so that x outside the box has some h_i(x) >= e
// exactly as the kernels compute it.  Returns false when no safe box is known (no culling).
bool shape_box(const DevIneq* q, int n, double e, double box[4]) {
    if (n < 1) return false;
    const int kind = q[0].kind;
    for (int i = 1; i < n; ++i)
        if (q[i].kind != kind) return false;
    double b[4] = {INFINITY, -INFINITY, INFINITY, -INFINITY};
    if (kind == UAM_INEQ_ELLIPSE) {
        if (n != 1) return false;
        const double s = 1.0 + e;
        if (!(s > 0.0)) {  // empty region: every point is outside
            box[0] = INFINITY, box[1] = -INFINITY, box[2] = INFINITY, box[3] = -INFINITY;
            return s <= 0.0;
        }
        const double k = std::sqrt(s), r1 = std::fabs(q[0].p[2]), r2 = std::fabs(q[0].p[3]);
        b[0] = q[0].p[0] - r1 * k, b[1] = q[0].p[0] + r1 * k;
        b[2] = q[0].p[1] - r2 * k, b[3] = q[0].p[1] + r2 * k;
    } else if (kind == UAM_INEQ_AXIS) {
        for (int i = 0; i < n; ++i) {
            const int k = q[i].p[0] == 0.0 ? 0 : 1;
            const double c = q[i].p[1], r = q[i].p[2], sg = q[i].p[3];
            if (sg > 0) b[2 * k + 1] = std::fmin(b[2 * k + 1], c + r + e);  // x_k < c + r + e
            else if (sg < 0) b[2 * k] = std::fmax(b[2 * k], c - r - e);     // x_k > c - r - e
            else return false;
        }
    } else {  // half-planes a x + b y < c, vertices among pairwise intersections
        if (n < 3) return false;
        std::vector<double> A(n), B(n), C(n);
        for (int i = 0; i < n; ++i) {
            const double* p = q[i].p;  // {ax, ay, dx, dy, s}
            A[i] = p[4] * p[3];
            B[i] = -p[4] * p[2];
            C[i] = e + p[4] * (p[3] * p[0] - p[2] * p[1]);
        }
        int found = 0;
        for (int i = 0; i < n; ++i)
            for (int j = i + 1; j < n; ++j) {
                const double det = A[i] * B[j] - A[j] * B[i];
                if (!(std::fabs(det) > 1e-300)) continue;
                const double x = (C[i] * B[j] - C[j] * B[i]) / det;
                const double y = (A[i] * C[j] - A[j] * C[i]) / det;
                bool feas = std::isfinite(x) && std::isfinite(y);
                for (int k = 0; k < n && feas; ++k) {
                    const double tol =
                        1e-9 * (std::fabs(A[k] * x) + std::fabs(B[k] * y) + std::fabs(C[k])) + 1e-12;
                    feas = A[k] * x + B[k] * y <= C[k] + tol;
                }
                if (!feas) continue;
                ++found;
                b[0] = std::fmin(b[0], x), b[1] = std::fmax(b[1], x);
                b[2] = std::fmin(b[2], y), b[3] = std::fmax(b[3], y);
            }
        if (found < 3) return false;
        // sanity for e >= 0: the polygon's own vertices (edge start points) lie inside
        if (e >= 0)
            for (int i = 0; i < n; ++i)
                if (q[i].p[0] < b[0] - 1e-9 || q[i].p[0] > b[1] + 1e-9 ||
                    q[i].p[1] < b[2] - 1e-9 || q[i].p[1] > b[3] + 1e-9)
                    return false;
    }
    for (int k = 0; k < 4; ++k)
        if (!std::isfinite(b[k])) return false;
    const double m = 1e-6 * (1.0 + std::fmax(std::fmax(std::fabs(b[0]), std::fabs(b[1])),
                                             std::fmax(std::fabs(b[2]), std::fabs(b[3]))));
    box[0] = b[0] - m, box[1] = b[1] + m, box[2] = b[2] - m, box[3] = b[3] + m;
    return true;
}


// ----------------------------------------------------------------------------------------
// Pair order for K3 (analytic mode).  K3 runs one lane per path, so a wave's 64 lanes walk 64
// shape-grid lists; pairs in a spatial order (Morton order of (x0, y0, xf, yf), 4 bits per
// coordinate over the pairs' extent) put similar paths in one wave and cut the
// divergence (8.6 -> 4.8 ms per cfg3 launch, tools/probe_analytic_sort.py).  A counting sort
// on the 16-bit key: histogram, one-block scan, scatter.  The order inside a key is whatever
// the atomics give -- results do not depend on it, since each pair is read and written at its
// own index.
// doubles as order-preserving unsigned keys (for atomicMin / atomicMax of the bounds)
__device__ __forceinline__ unsigned long long dkey(double v) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double dkey_inv(unsigned long long k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k));
}

// bounds of the pairs' x and y: bnd[0..1] = min x, min y; bnd[2..3] = max x, max y (keys)
__global__ __launch_bounds__(256) void k_pair_bounds(const double* __restrict__ pairs, int64_t n,
                                                     unsigned long long* __restrict__ bnd) {
    // grid-stride over the pairs (the launch caps the grid at 256 workgroups), then a wave and
    // a workgroup reduction, so only 4 atomics per workgroup hit the bounds' one cache line:
    // one atomic set per wave serialised ~6k atomics on that line at 100k pairs (72 us)
    double v[4] = {INFINITY, INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double4 pr = reinterpret_cast<const double4*>(pairs)[i];
        v[0] = fmin(v[0], fmin(pr.x, pr.z)), v[1] = fmin(v[1], fmin(pr.y, pr.w));
        v[2] = fmax(v[2], fmax(pr.x, pr.z)), v[3] = fmax(v[3], fmax(pr.y, pr.w));
    }
    for (int o = 32; o; o >>= 1) {
        v[0] = fmin(v[0], __shfl_xor(v[0], o, 64));
        v[1] = fmin(v[1], __shfl_xor(v[1], o, 64));
        v[2] = fmax(v[2], __shfl_xor(v[2], o, 64));
        v[3] = fmax(v[3], __shfl_xor(v[3], o, 64));
    }
    __shared__ double wv[4][4];  // [wave][bound], 256 threads = 4 waves
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 4; ++k) wv[wave][k] = v[k];
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) {
            v[0] = fmin(v[0], wv[w][0]), v[1] = fmin(v[1], wv[w][1]);
            v[2] = fmax(v[2], wv[w][2]), v[3] = fmax(v[3], wv[w][3]);
        }
        atomicMin(&bnd[0], dkey(v[0]));
        atomicMin(&bnd[1], dkey(v[1]));
        atomicMax(&bnd[2], dkey(v[2]));
        atomicMax(&bnd[3], dkey(v[3]));
    }
}

__device__ __forceinline__ uint32_t pair_key(const double4 pr, const double* b) {
    auto q4 = [](double v, double lo, double inv) {
        const double t = (v - lo) * inv;
        return (uint32_t)(t > 0.0 ? (t < 15.0 ? t : 15.0) : 0.0);  // NaN -> 0
    };
    const double ix = 16.0 / fmax(b[2] - b[0], 1e-300), iy = 16.0 / fmax(b[3] - b[1], 1e-300);
    const uint32_t c[4] = {q4(pr.x, b[0], ix), q4(pr.y, b[1], iy), q4(pr.z, b[0], ix),
                           q4(pr.w, b[1], iy)};
    uint32_t k = 0;
    // yf, xf, y0, x0 from the most significant bit of each level: measured ~0.17 ms faster on
    // cfg3 than x0 first (tools/probe_analytic_sort.py, "morton16" vs "device16")
    for (int b = 3; b >= 0; --b)
        for (int d = 3; d >= 0; --d) k = (k << 1) | ((c[d] >> b) & 1u);
    return k;
}

__global__ __launch_bounds__(256) void k_pair_keys(const double* __restrict__ pairs, int64_t n,
                                                   const unsigned long long* __restrict__ bnd,
                                                   uint16_t* __restrict__ key,
                                                   int32_t* __restrict__ hist) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double b[4] = {dkey_inv(bnd[0]), dkey_inv(bnd[1]), dkey_inv(bnd[2]), dkey_inv(bnd[3])};
    const uint32_t k = pair_key(reinterpret_cast<const double4*>(pairs)[i], b);
    key[i] = (uint16_t)k;
    atomicAdd(&hist[k], 1);
}

// exclusive scan of the 65536 key counts, one workgroup of 1024 threads x 64 counts
__global__ __launch_bounds__(1024) void k_pair_scan(int32_t* __restrict__ hist) {
    __shared__ int32_t part[1024];
    const int t = threadIdx.x;
    // the thread's 64 counts stay in registers: 16 independent 16-B loads in flight instead of
    // 64 dependent scalar loads, and no reload for the write-back (hist is 256-B aligned)
    int4* h4 = reinterpret_cast<int4*>(hist + t * 64);
    int4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = h4[i];
    int32_t sum = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) sum += v[i].x + v[i].y + v[i].z + v[i].w;
    part[t] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
        const int32_t v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int32_t run = part[t] - sum;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        int4 o;
        o.x = run; run += v[i].x;
        o.y = run; run += v[i].y;
        o.z = run; run += v[i].z;
        o.w = run; run += v[i].w;
        h4[i] = o;
    }
}

__global__ __launch_bounds__(256) void k_pair_scatter(const uint16_t* __restrict__ key, int64_t n,
                                                      int32_t* __restrict__ next,
                                                      int32_t* __restrict__ order) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    order[atomicAdd(&next[key[i]], 1)] = (int32_t)i;
}

// Raster pair order (K2).  Only which pairs share an XCD's L2 (and the dispatch order within
// it) matters, so a coarse key suffices: 2 bits of each of (yf, xf, y0, x0) over the raster
// extent, interleaved from the top bit into an 8-bit key (256 bins).  A counting sort without
// global atomics in two launches over RORD_NB fixed partitions of the pairs: (1) keys and a
// per-partition LDS histogram, stored bin-major; (2) every partition scans the 256 x RORD_NB
// counts (thread t owns bin t across all partitions) and scatters its pairs through LDS cursors.
// cfg3: the order takes the raster kernel from 0.765 to 0.718 ms (profiles/r02).
constexpr int RORD_BITS = UAM_RORD_BITS, RORD_BINS = 1 << (4 * RORD_BITS);
constexpr int RORD_BPT = RORD_BINS / 256;          // bins per thread of the order kernels
constexpr int RORD_NB = RORD_BPT > 1 ? 16 : 64;    // partitions of the pairs
static_assert(RORD_BINS >= 256, "at least one bin per thread");

struct KOrdBox {
    double x0, y0, ix, iy;  // lower corner, 2^RORD_BITS / extent
};

__device__ __forceinline__ uint32_t rorder_key(const double4 pr, const KOrdBox& b) {
    auto q = [](double v, double lo, double inv) {
        const double t = (v - lo) * inv;
        constexpr double m = (double)((1 << RORD_BITS) - 1);
        return (uint32_t)(t > 0.0 ? (t < m ? t : m) : 0.0);  // NaN -> 0
    };
    const uint32_t c[4] = {q(pr.x, b.x0, b.ix), q(pr.y, b.y0, b.iy), q(pr.z, b.x0, b.ix),
                           q(pr.w, b.y0, b.iy)};
    uint32_t k = 0;
    for (int l = RORD_BITS - 1; l >= 0; --l)
        for (int d = 3; d >= 0; --d) k = (k << 1) | ((c[d] >> l) & 1u);
    return k;
}

// pairs [n][4] (x0, y0, xf, yf), or [n][6] (x0, y0, z0, xf, yf, zf) when vol (config 5)
__global__ __launch_bounds__(256) void k_rorder_hist(const double* __restrict__ pairs, int64_t n,
                                                     KOrdBox box, uint16_t* __restrict__ key,
                                                     int32_t* __restrict__ H, int vol) {
    __shared__ int32_t h[RORD_BINS];
    const int t = threadIdx.x, blk = blockIdx.x;
    for (int b = t; b < RORD_BINS; b += 256) h[b] = 0;
    __syncthreads();
    const int64_t lo = n * blk / RORD_NB, hi = n * (blk + 1) / RORD_NB;
    for (int64_t i = lo + t; i < hi; i += 256) {
        const double4 pr =
            vol ? make_double4(pairs[6 * i], pairs[6 * i + 1], pairs[6 * i + 3], pairs[6 * i + 4])
                : reinterpret_cast<const double4*>(pairs)[i];
        const uint32_t k = rorder_key(pr, box);
        key[i] = (uint16_t)k;
        atomicAdd(&h[k], 1);
    }
    __syncthreads();
    for (int b = t; b < RORD_BINS; b += 256) H[b * RORD_NB + blk] = h[b];
}

__global__ __launch_bounds__(256) void k_rorder_scatter(const uint16_t* __restrict__ key, int64_t n,
                                                        const int32_t* __restrict__ H,
                                                        int32_t* __restrict__ order) {
    __shared__ int32_t part[256];
    __shared__ int32_t off[RORD_BINS];
    const int t = threadIdx.x, blk = blockIdx.x;
    // thread t owns bins [t * BPT, (t + 1) * BPT), each across all partitions
    const int4* h4 = reinterpret_cast<const int4*>(H + (int64_t)t * RORD_BPT * RORD_NB);
    int32_t tot = 0;
    int32_t pre[RORD_BPT], mine[RORD_BPT];
#pragma unroll
    for (int bb = 0; bb < RORD_BPT; ++bb) {
        int32_t bt = 0, bm = 0;
#pragma unroll
        for (int k = 0; k < RORD_NB / 4; ++k) {
            const int4 v = h4[bb * (RORD_NB / 4) + k];
            const int b = 4 * k;
            bm += (b < blk ? v.x : 0) + (b + 1 < blk ? v.y : 0) + (b + 2 < blk ? v.z : 0) +
                  (b + 3 < blk ? v.w : 0);
            bt += v.x + v.y + v.z + v.w;
        }
        pre[bb] = tot;
        mine[bb] = bm;
        tot += bt;
    }
    part[t] = tot;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // Hillis-Steele inclusive scan of the thread totals
        const int32_t x = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
#pragma unroll
    for (int bb = 0; bb < RORD_BPT; ++bb)
        off[t * RORD_BPT + bb] = part[t] - tot + pre[bb] + mine[bb];
    __syncthreads();
    const int64_t lo = n * blk / RORD_NB, hi = n * (blk + 1) / RORD_NB;
    for (int64_t i = lo + t; i < hi; i += 256) order[atomicAdd(&off[key[i]], 1)] = (int32_t)i;
}

// ---- K2s: segment-sorted raster evaluation (build-defined; no reference counterpart) --------
// K2 (one lane walks one path's W waypoints) is bound by scattered 128-B record lines: 14% L2
// hits and 6.4x the algorithmic bytes across the fabric (profiles/r02/final).  K2s cuts every
// path into nseg segments of L = ceil(W / nseg) waypoints and evaluates segment k of all paths
// in one launch, the (path, segment) items sorted by the Morton key of the 16 x 16-tile raster
// tile under the segment's middle waypoint, so the workgroups an XCD runs together gather from
// one region of the raster.  Between launches a path's running sums live in a 32-B SegState;
// every waypoint is still added in waypoint order with raster_pass2_skip's arithmetic (the
// order of the items changes which lane does the work, never the operations a path sees), so
// every output is bit-identical to K2's.  Launches: k_seg_hist -> scan -> k_seg_scatter for
// segment 0's order, then segment 0 (k_seg_eval<.., FIRST>: the lane runs the path's pass 1
// too, so its ALU work overlaps the gathers as in K2) while the other segments' orders are
// sorted on the side stream, then segments 1.. (workgroups per CU capped through an LDS
// floor), then k_seg_final (outputs, the main.py:175-180 selection).  K2s is the fast form
// of the reference's sequential order (UAM_OPT_GROUP = 0); K2g (below) is the default.
// Measured on cfg3: DESIGN.md §4 K2s.  Tile grid of the sort key: 16 x 16 tiles over the
// raster (cfg3 K2s ms by tile bits, r02: 6 0.630, 5 0.603, 4 0.595, 3 0.613); 6 gathers per
// chunk (6/6 0.590, 8/8 0.598, 8/4 0.592, 4/4 0.595, 8/16 0.755 ms).
constexpr int SEG_TBITS = 4;                           // 16 x 16 tiles over the raster
constexpr int SEG_BINS = (1 << (2 * SEG_TBITS)) + 1;   // + one bin for off-raster / NaN
constexpr int SEG_NBK = 256;                           // partitions of a segment's items
constexpr int SEG_MAX = 8;                             // segments per path
constexpr int SEG_CH = 6;                              // gathers per chunk

struct SegState {  // 32 B per path
    double cost, nsum, hmax;
    int32_t nh, off;
};

struct KSeg {
    const double* __restrict__ pairs;
    const double* __restrict__ utab;
    int64_t n_pairs;
    int32_t P, D, W, nseg, L, tshift;  // segments of L waypoints
    int32_t g0;                 // sort launches: first group (blockIdx.y = g - g0)
    int64_t obase;              // sort launches: order index of group g0's first item
    SegState* __restrict__ st;  // [P]
    double4* __restrict__ p1;   // [P] pass 1: (L, length, kinematic sum, 0)
    uint16_t* __restrict__ key; // [nseg][P] sort keys
    int32_t* __restrict__ cnt;  // [nseg][SEG_BINS][SEG_NBK] counts -> offsets
    int32_t* __restrict__ tot;  // scan block totals
    int32_t* __restrict__ order;  // [nseg][P] path of each sorted item
    __device__ __forceinline__ void bounds(int s, int& j0, int& j1) const {
        j0 = s * L;
        j1 = min(j0 + L, W);
    }
};

__device__ __forceinline__ PathSrc<true> seg_src(const KSeg& ks, int N, int32_t path) {
    const int32_t q = path / ks.D, d = path - q * ks.D;
    PathSrc<true> src;
    src.W = N + 2;
    src.wp = nullptr;
    const double4 pr = reinterpret_cast<const double4*>(ks.pairs)[q];
    src.x0 = pr.x, src.y0 = pr.y, src.xf = pr.z, src.yf = pr.w;
    src.za = src.zb = 0.0;
    src.u = ks.utab + (int64_t)d * N * 2;
    return src;
}

// sort key of segment s of path i: Morton code of the tile under its middle waypoint
__device__ __forceinline__ uint32_t seg_key(const KSeg& ks, const KRaster& rs, int N, int32_t i,
                                            int s) {
    int j0, j1;
    ks.bounds(s, j0, j1);
    const PathSrc<true> src = seg_src(ks, N, i);
    double x0, x1;
    src.at((j0 + j1 - 1) >> 1, x0, x1);
    const double fx = floor((x0 - rs.x0) * rs.inv_dx);
    const double fy = floor((rs.y_top - x1) * rs.inv_dy);
    if (!((fx >= 0.0) && (fx < (double)rs.nx) && (fy >= 0.0) && (fy < (double)rs.ny)))
        return SEG_BINS - 1;
    const uint32_t tx = (uint32_t)fx >> ks.tshift, ty = (uint32_t)fy >> ks.tshift;
    uint32_t k = 0;
#pragma unroll
    for (int b = SEG_TBITS - 1; b >= 0; --b) k = (k << 2) | (((ty >> b) & 1u) << 1) | ((tx >> b) & 1u);
    return k;
}

// counting sort, launch 1: block (b, g) keys partition b of segment g's items and stores its
// LDS histogram bin-major, so the scan of cnt yields each (segment, bin, partition)'s offset;
// segment g's items land in one contiguous run of order
__device__ __forceinline__ void seg_group(const KSeg& ks, int g, int b, int& s, int32_t& lo,
                                          int32_t& hi) {
    s = g;
    lo = (int32_t)((int64_t)ks.P * b / SEG_NBK);
    hi = (int32_t)((int64_t)ks.P * (b + 1) / SEG_NBK);
}

__global__ __launch_bounds__(256) void k_seg_hist(KParams p, KRaster rs, KSeg ks) {
    __shared__ int32_t h[SEG_BINS];
    const int t = threadIdx.x, b = blockIdx.x, g = blockIdx.y + ks.g0;
    for (int k = t; k < SEG_BINS; k += 256) h[k] = 0;
    __syncthreads();
    int s;
    int32_t lo, hi;
    seg_group(ks, g, b, s, lo, hi);
    uint16_t* key = ks.key + (int64_t)s * ks.P;
    for (int32_t i = lo + t; i < hi; i += 256) {
        const uint32_t k = seg_key(ks, rs, p.N, i, s);
        key[i] = (uint16_t)k;
        atomicAdd(&h[k], 1);
    }
    __syncthreads();
    for (int k = t; k < SEG_BINS; k += 256)
        ks.cnt[((int64_t)blockIdx.y * SEG_BINS + k) * SEG_NBK + b] = h[k];
}

// launch 3 (after k_scan_local / k_scan_totals over cnt): LDS cursors = scanned offset + block
// total, items scattered in partition order
__global__ __launch_bounds__(256) void k_seg_scatter(KSeg ks) {
    __shared__ int32_t cur[SEG_BINS];
    const int t = threadIdx.x, b = blockIdx.x, g = blockIdx.y + ks.g0;
    for (int k = t; k < SEG_BINS; k += 256) {
        const int64_t c = ((int64_t)blockIdx.y * SEG_BINS + k) * SEG_NBK + b;
        cur[k] = ks.cnt[c] + ks.tot[c / (256 * SCAN_ITEMS)];
    }
    __syncthreads();
    int s;
    int32_t lo, hi;
    seg_group(ks, g, b, s, lo, hi);
    const uint16_t* key = ks.key + (int64_t)s * ks.P;
    int32_t* order = ks.order + ks.obase;
    // (loading 8 strides' keys together made the segment-0 scatter 6.5 -> 5.4 us and the side
    // stream's 85 -> 115 us beside segment 0's launch: no net change, not kept)
    for (int32_t i = lo + t; i < hi; i += 256) order[atomicAdd(&cur[key[i]], 1)] = i;
}

// waypoints [j0, j1) of one path: raster_pass2_skip's chunks, cell arithmetic and sums
// (SKIP = false: no bitmap, every in-raster waypoint gathered, as consume_chunk)
template <bool SKIP, int CH>
__device__ __forceinline__ void seg_pass2(const KRaster& rs, const uint4* __restrict__ rec,
                                          const uint32_t* bits, const PathSrc<true>& src,
                                          int j0, int j1, double dN, PathAcc& a) {
    for (int jc = j0; jc < j1; jc += CH) {
        uint4 r[CH];
        uint32_t inb = 0, need = 0;
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            if (jc + t < j1) {
                double x0, x1;
                src.at(jc + t, x0, x1);
                bool sk = false;
                int32_t cl;
                if (SKIP) {
                    cl = raster_cell_skip(rs, bits, x0, x1, sk);
                } else {
                    int ix, iy;
                    cl = raster_cell(rs, x0, x1, ix, iy) ? iy * rs.nx + ix : -1;
                }
                if (cl >= 0) {
                    inb |= 1u << t;
                    if (!sk) {
                        need |= 1u << t;
                        r[t] = rec[cl];
                    }
                }
            }
        }
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            if (jc + t >= j1) break;
            if (!((inb >> t) & 1u)) {
                ++a.off;
                a.hmax = fmax(a.hmax, 0.0);  // off-raster counts as sea level
                continue;
            }
            if (!((need >> t) & 1u)) {  // phi, psi +-0 (exact no-ops), terrain +0.0
                a.hmax = fmax(a.hmax, 0.0);
                continue;
            }
            a.cost = a.cost + (double)__uint_as_float(r[t].x) / dN;
            a.nsum = a.nsum + (double)__uint_as_float(r[t].y);
            a.nh += (r[t].w & UAM_FLAG_NFZ) ? 1 : 0;
            const double terrain =
                (r[t].w & UAM_FLAG_NODATA) ? 0.0 : (double)__uint_as_float(r[t].z);
            a.hmax = fmax(a.hmax, terrain);
        }
    }
}

// waypoints [j0, j1) of one path from the packed raster (KRaster::pmap and planes, the 2-bit
// block codes in LDS): raster_pass2_skip's cell arithmetic, values and sums.  Per waypoint one
// value load (pk_locate: the record, the e8 or p4 entry, or the dummy line) and one terrain load
// (t4 outside code 3), both outside every branch; a code-0 waypoint adds no phi / psi term (exact
// no-ops), a code-1 waypoint no psi term and no hit.
template <int CH>
__device__ __forceinline__ void seg_pass2_pack(const KRaster& rs, const uint4* __restrict__ rec,
                                               const uint32_t* map, const PathSrc<true>& src,
                                               int j0, int j1, double dN, PathAcc& a) {
    const uint4* const vdummy = reinterpret_cast<const uint4*>(rs.p4);
    for (int jc = j0; jc < j1; jc += CH) {
        uint4 r[CH];
        float tv[CH];
        uint32_t inb = 0;
        PkSlots cs;
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            const uint4* vp = vdummy;
            const float* tp = rs.t4;
            if (jc + t < j1) {
                double x0, x1;
                src.at(jc + t, x0, x1);
                const double fx = floor((x0 - rs.x0) * rs.inv_dx);
                const double fy = floor((rs.y_top - x1) * rs.inv_dy);
                if ((fx >= 0.0) && (fx < (double)rs.nx) && (fy >= 0.0) && (fy < (double)rs.ny)) {
                    inb |= 1u << t;
                    cs.set(t, pk_locate(rs, rec, map, (int32_t)fx, (int32_t)fy, vp, tp));
                }
            }
            r[t] = *vp;
            tv[t] = *tp;
        }
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            if (jc + t >= j1) break;
            if (!((inb >> t) & 1u)) {
                ++a.off;
                a.hmax = fmax(a.hmax, 0.0);  // off-raster counts as sea level
                continue;
            }
            const uint32_t code = ((cs.c0 >> t) & 1u) | (((cs.c1 >> t) & 1u) << 1);
            uint32_t phi, psi, hit;
            float rter;
            pk_terms(r[t], cs, t, phi, psi, hit, rter);
            if (code) a.cost = a.cost + (double)__uint_as_float(phi) / dN;
            if (code & 2u) {
                a.nsum = a.nsum + (double)__uint_as_float(psi);
                a.nh += (int)hit;
            }
            a.hmax = fmax(a.hmax, (double)(code == 3u ? rter : tv[t]));
        }
    }
}

// segment s of every path, items in sorted order; workgroup b takes the sorted chunk
// xcd_chunk(b), so an XCD's workgroups cover one contiguous run of tiles.  Dynamic LDS: the
// skip bitmap, padded to a floor that caps the workgroups per CU (later segments).
// FIRST (segment 0): the lane runs the path's pass 1 itself and seeds the state, so pass 1's
// ALU work overlaps the gathers as in K2.
// PACK: the packed raster (seg_pass2_pack; SKIP ignored), its block codes in LDS.
template <bool SKIP, bool FIRST, bool PACK = false>
__global__ __launch_bounds__(256) void k_seg_eval(KParams p, KRaster rs, KSeg ks,
                                                  const uint4* __restrict__ rec, int s,
                                                  int64_t base, int32_t n) {
    extern __shared__ uint32_t s_bits[];
    if (PACK) {
        for (int i = threadIdx.x; i < rs.pwords; i += 256) s_bits[i] = rs.pmap[i];
        __syncthreads();
    } else if (SKIP) {
        for (int i = threadIdx.x; i < rs.swords; i += 256) s_bits[i] = rs.sum[i];
        __syncthreads();
    }
    const int64_t i = xcd_chunk(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
    if (i >= n) return;
    const int32_t path = ks.order[base + i];
    const PathSrc<true> src = seg_src(ks, p.N, path);
    PathAcc a;
    if (FIRST) {
        path_pass1<true>(p, src, nullptr, a);
        ks.p1[path] = make_double4(a.L, a.len, a.ksum, 0.0);
        a.cost = (double)(p.N + 1) * a.L;
        a.nsum = 0.0;
        a.hmax = -INFINITY;
        a.nh = 0;
        a.off = 0;
    } else {
        const SegState st = ks.st[path];
        a.cost = st.cost;
        a.nsum = st.nsum;
        a.hmax = st.hmax;
        a.nh = st.nh;
        a.off = st.off;
    }
    int j0, j1;
    ks.bounds(s, j0, j1);
    // gathers in flight per lane: the capped later segments (2 waves per SIMD) have the
    // registers for more
    if (PACK)
        seg_pass2_pack<SEG_CH>(rs, rec, s_bits, src, j0, j1, (double)p.N, a);
    else
        seg_pass2<SKIP, SEG_CH>(rs, rec, s_bits, src, j0, j1, (double)p.N, a);
    SegState o;
    o.cost = a.cost;
    o.nsum = a.nsum;
    o.hmax = a.hmax;
    o.nh = a.nh;
    o.off = a.off;
    ks.st[path] = o;
}

// outputs of every path (block = 64 pairs x D, k_eval_pairs's store layout) and the selection
// over each pair's D paths
__global__ __launch_bounds__(1024) void k_seg_final(KParams p, KSeg ks, KOut out,
                                                    int32_t* __restrict__ best_f,
                                                    int32_t* __restrict__ best_l) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int D = ks.D, t = threadIdx.x;
    double* s_cost = smem;
    double* s_len = smem + 64 * D;

    const int64_t q0 = (int64_t)blockIdx.x * 64;
    const int qi = t / D, di = t - qi * D;
    if (q0 + qi < ks.n_pairs) {
        const int64_t gp = (q0 + qi) * D + di;
        const double4 q1 = ks.p1[gp];
        const SegState st = ks.st[gp];
        const double cost = st.cost, nsum = st.nsum, clr = p.altitude - st.hmax;
        const int32_t nh = st.nh, off = st.off, below = 0;
        if (out.cost) out.cost[gp] = cost;
        if (out.length_q) out.length_q[gp] = q1.x;
        if (out.length) out.length[gp] = q1.y;
        if (out.kin_sum) out.kin_sum[gp] = q1.z;
        if (out.nfz_sum) out.nfz_sum[gp] = nsum;
        if (out.min_clearance) out.min_clearance[gp] = clr;
        if (out.nfz_hits) out.nfz_hits[gp] = nh;
        if (out.offmap) out.offmap[gp] = off;
        if (out.below_terrain) out.below_terrain[gp] = below;
        s_cost[di * 64 + qi] = cost;
        s_len[di * 64 + qi] = q1.y;
    }
    __syncthreads();
    if (t < 64 && q0 + t < ks.n_pairs) {
        if (best_f) best_f[q0 + t] = select_best(s_cost + t, 64, D, true);
        if (best_l) best_l[q0 + t] = select_best(s_len + t, 64, D, false);
    }
}

// ---- K2g: segment-grouped raster evaluation (build-defined; no reference counterpart) -------
// K2s keeps each path's sums in waypoint order, so its segments run one launch after another
// and stay long (41 waypoints, ~13 km): its gathers reach 46% L2 hits and move 4.5x the
// algorithmic bytes (profiles/r02/pack_final).  K2g restates the per-path sums in a grouped
// order (oracle/uam_oracle.c orc_eval_paths_g): the waypoints are cut into groups of G, each
// group's Phi/N and psi partial sums are formed from +0.0 in waypoint order, and the partials
// are added to cost = (N+1) L and nsum = 0 in group order; the terrain maximum, hits and
// off-raster counts are order-free.  Every (path, group) item is then independent, so ONE
// counting sort on the Morton key of the raster tile under the item's middle waypoint and ONE
// launch evaluate all of them in the XCD-placed sorted order: the items an XCD runs together
// cover a few tiles, whose lines stay in its L2.  The partials go to a 48-B slot per item;
// k_g_final combines them in group order with pass 1 and runs the main.py:175-180 selection.
// Every per-path sum is grouped the same way -- each term attached to a waypoint (Phi/N, psi
// of waypoint j; the length terms of segment p_{j-1} -> p_j; kinematic row k to k + 1) -- so
// an item also forms its group's share of pass 1 (get_cost's L, the true length, the
// kinematic rows): that f64 work runs in the memory-bound evaluation launch, whose waves wait
// on gathers with the VALU mostly idle (profiles/r03/k2g_order: pass 1 as its own launch beside
// the evaluation cost ~90 us of its 130-150).  Against the sequential reference the grouped
// sums differ by rounding only (<= 1e-12 relative, tests/test_oracle_golden.py); against the
// grouped oracle they are bit-exact.
constexpr int G_TBITS_MAX = 6;                          // up to 64 x 64 tiles over the raster
// tile bins twice over (a ragged last group's items have their own) + one for off-raster / NaN
constexpr int G_BINS_MAX = (2 << (2 * G_TBITS_MAX)) + 1;
constexpr int G_NBK = UAM_G_NBK;                        // partitions of the counting sort
constexpr int G_HIST_DYN_MAX = 119 * 1024;  // k_g_hist's dynamic LDS (K2h seeds) beside its 40 KiB
constexpr int G_MAXLEN = 64;                            // longest group
constexpr int G_UTAB_LDS = 48 * 1024;                   // K2g: unit-arc table (in LDS) up to this

struct alignas(16) GSlot {  // 48 B per (path, group), written by one lane
    double cost;     // partial sums from +0.0 in waypoint order: Phi/N,
    double psi;      //   the no-fly psi,
    double L;        //   get_cost's length term (problem.py:130-146 with the quirk),
    double len;      //   the true length (solver.py:49),
    double ksum;     //   the kinematic rows (problem.py:100-107)
    float hmax;      // max terrain of the group's waypoints as consume_chunk reads it
    uint32_t cnt;    // nfz hits | off-raster << 8
};

// K2h: the unit polyline's sums of one displacement row (oracle orc_unit_geo)
struct UGeo {
    double s1n, s2n, s1a, s2a, e12, e3;
};

// the unit polyline's sums of one table row u[N] (oracle unit_geo: the same operations)
__device__ void unit_geo_row(const KParams& p, const double2* __restrict__ u, UGeo* out) {
    const int N = p.N;
    const double mincos = p.mincos, r = p.r_eff;
    double s1n = 0.0, s2n = 0.0, s1a = 0.0, s2a = 0.0, e12 = 0.0, e3 = 0.0;
    double qx = 1.0, qy = 0.0, pdx = 0.0, pdy = 0.0, pb = 0.0;
    for (int k = 1; k <= N + 1; ++k) {
        double cx = -1.0, cy = 0.0;
        if (k <= N) {
            const double2 c = u[k - 1];
            cx = c.x, cy = c.y;
        }
        const double dx = cx - qx, dy = cy - qy;
        const double b = sqrt(dx * dx + dy * dy);
        if (k <= N) {
            s1n = s1n + b;
            s2n = s2n + b * b;
        }
        s1a = s1a + b;
        s2a = s2a + b * b;
        if (k >= 2) {  // row k - 2: chords k - 1 and k
            e12 = e12 + fmax(0.0, b - r * pb);
            e12 = e12 + fmax(0.0, pb / r - b);
            const double dt = pdx * dx + pdy * dy;
            e3 = e3 + fmax(0.0, mincos - dt / (pb * b));
        }
        qx = cx, qy = cy, pdx = dx, pdy = dy, pb = b;
    }
    out->s1n = s1n, out->s2n = s2n, out->s1a = s1a, out->s2a = s2a, out->e12 = e12, out->e3 = e3;
}

struct KGrp {
    const double* __restrict__ pairs;
    const double* __restrict__ utab;
    int64_t n_pairs;
    int32_t P, D, W, G, nseg, tshift, tbits, bins;
    int32_t last_bin;              // key offset of the last group's items (0: groups all G long)
    const uint16_t* __restrict__ tkey;  // [2^tbits][2^tbits] tile -> position on the curve
    uint64_t m_nseg, m_d;          // div_magic multipliers and shifts for / nseg and / D
    int32_t sh_nseg, sh_d;
    double inv_n;                  // RN(1 / N) for Phi / N (0: divide; N > 4096)
    int64_t n_items;               // P * nseg; item i = path * nseg + group
    uint16_t* __restrict__ key;    // [n_items]
    int32_t* __restrict__ cnt;     // [bins][G_NBK] counts -> offsets
    int32_t* __restrict__ tot;     // scan block totals
    int32_t nsb_raw;               // > 0: tot holds nsb_raw (<= 1024) unscanned block totals,
                                   // which k_g_scatter scans itself (no k_scan_totals launch)
    int32_t* __restrict__ order;   // [n_items] item of each sorted position
    GSlot* __restrict__ slot;      // [nseg][P]: group-major, so the output launch's lanes read
                                   // a group's slots of consecutive paths contiguously
    int32_t* __restrict__ cells;   // [P][W] waypoint cells (k_cells), or null
    double cx0, cy_top, cinv_dx, cinv_dy;  // the raster's cell grid (gen_cell) for k_cells
    int32_t cnx, cny;
    UGeo* __restrict__ ugeo;       // K2h / K4h: [D] unit sums, formed by k_g_scatter's block 0
    int32_t lb_stride;             // K2h: the path lower bound's sample stride (>= 1)
    float* __restrict__ lbp;       // K2h: [P] each path's terrain seed (h_path_seed, formed by
                                   // the histogram launch), or null
    int32_t seed_lds;              // K2h: the histogram launch stages header + unit arcs in LDS
    double* __restrict__ ubp;      // K4h: [P] each path's clearance seed (v_path_seed), likewise
    int32_t* __restrict__ err;     // the sort's check word: zeroed by the histogram launch, set
                                   // by the scatter on a position outside the order (keys of the
                                   // two launches disagreeing); the output launch then writes
                                   // NaN / -1 in every output of the whole batch
    int32_t* herr;                 // page-locked host word the output launch sets on err
                                   // (uam_device_status), or null
    int32_t test_fault;            // UAM_OPT_TEST_SORT_FAULT: the scatter flags err (tests)
};

// a path's outputs from the output launches (k_g_final / k_h_final / k_v_final); with the
// sort's check word set (bad), NaN in every f64 output and -1 in every count
__device__ __forceinline__ void put_outputs(const KOut& out, int64_t gp, bool bad, double cost,
                                            double L, double len, double ksum, double nsum,
                                            double clear, int32_t nh, int32_t off, int32_t bel) {
    const double nan = __builtin_nan("");
    if (out.cost) out.cost[gp] = bad ? nan : cost;
    if (out.length_q) out.length_q[gp] = bad ? nan : L;
    if (out.length) out.length[gp] = bad ? nan : len;
    if (out.kin_sum) out.kin_sum[gp] = bad ? nan : ksum;
    if (out.nfz_sum) out.nfz_sum[gp] = bad ? nan : nsum;
    if (out.min_clearance) out.min_clearance[gp] = bad ? nan : clear;
    if (out.nfz_hits) out.nfz_hits[gp] = bad ? -1 : nh;
    if (out.offmap) out.offmap[gp] = bad ? -1 : off;
    if (out.below_terrain) out.below_terrain[gp] = bad ? -1 : bel;
}

// the output launches' selections and, on a failed sort check, the host word (one lane)
__device__ __forceinline__ void put_selection(const KGrp& kg, bool bad, int64_t q0, int t,
                                              const double* s_cost, const double* s_len,
                                              int32_t* best_f, int32_t* best_l) {
    if (bad && blockIdx.x == 0 && t == 0 && kg.herr) *kg.herr = 1;
    if (t < 64 && q0 + t < kg.n_pairs) {
        if (best_f) best_f[q0 + t] = bad ? -1 : select_best(s_cost + t, 64, kg.D, true);
        if (best_l) best_l[q0 + t] = bad ? -1 : select_best(s_len + t, 64, kg.D, false);
    }
}

// K2h / K4h: the D rows' unit sums by one block (block 0 of the scatter launch, one more than
// its partitions, so the step has no launch for them).
// The terms are independent, the sums are not: every (row, chord) term first, one thread each
// (unit_geo_row's operations), into LDS; then one thread per (row, sum) adds its terms in
// unit_geo_row's order, so the bits are unit_geo_row's.  (One thread per row walking its 81
// chords took ~30 us, the term-parallel form ~5 us: hidden beside the scatter's 10.)
// su: the calling kernel's histogram LDS, cap bytes; a table or term set that does not fit is
// done by unit_geo_row per row.
__device__ __forceinline__ void unit_geo_block(const KParams& p, const KGrp& kg, double2* su,
                                               int cap) {
    const int N = p.N, D = kg.D, nk = N + 1;  // chords k = 1..N+1 (index k - 1)
    const int nu = D * N;
    const size_t need = (size_t)nu * 16 + (size_t)D * nk * 5 * 8;
    const double2* u = reinterpret_cast<const double2*>(kg.utab);
    if (need > (size_t)cap) {
        if ((int)threadIdx.x < D) unit_geo_row(p, u + threadIdx.x * N, kg.ugeo + threadIdx.x);
        return;
    }
    for (int i = threadIdx.x; i < nu; i += blockDim.x) su[i] = u[i];
    __syncthreads();
    double* tb = reinterpret_cast<double*>(su + nu);  // [D][nk] b_k
    double* tb2 = tb + D * nk;                        // b_k^2
    double* tc1 = tb2 + D * nk;                       // row terms at their later chord
    double* tc2 = tc1 + D * nk;
    double* tc3 = tc2 + D * nk;
    const double mincos = p.mincos, r = p.r_eff;
    for (int i = threadIdx.x; i < D * nk; i += blockDim.x) {
        const int d = i / nk, k = i - d * nk + 1;
        const double2* ur = su + d * N;
        auto pt = [&](int m, double& x, double& y) {  // u_0 = (1, 0), u_{N+1} = (-1, 0)
            if (m == 0) {
                x = 1.0, y = 0.0;
            } else if (m == N + 1) {
                x = -1.0, y = 0.0;
            } else {
                x = ur[m - 1].x, y = ur[m - 1].y;
            }
        };
        double qx, qy, cx, cy;
        pt(k - 1, qx, qy);
        pt(k, cx, cy);
        const double dx = cx - qx, dy = cy - qy;
        const double b = sqrt(dx * dx + dy * dy);
        tb[i] = b;
        tb2[i] = b * b;
        double c1 = 0.0, c2 = 0.0, c3 = 0.0;
        if (k >= 2) {
            double px, py;
            pt(k - 2, px, py);
            const double pdx = qx - px, pdy = qy - py;
            const double pb = sqrt(pdx * pdx + pdy * pdy);
            c1 = fmax(0.0, b - r * pb);
            c2 = fmax(0.0, pb / r - b);
            const double dt = pdx * dx + pdy * dy;
            c3 = fmax(0.0, mincos - dt / (pb * b));
        }
        tc1[i] = c1, tc2[i] = c2, tc3[i] = c3;
    }
    __syncthreads();
    if ((int)threadIdx.x < D * 5) {
        const int d = threadIdx.x / 5, w = threadIdx.x - d * 5;
        const double* b = tb + d * nk;
        const double* b2 = tb2 + d * nk;
        UGeo* g = kg.ugeo + d;
        double acc = 0.0, acc2 = 0.0;
        if (w == 0) {  // s1n, then s1a continues the same chain over k = N+1
#pragma unroll 8
            for (int k = 0; k < N; ++k) acc = acc + b[k];
            g->s1n = acc;
        } else if (w == 1) {
#pragma unroll 8
            for (int k = 0; k < N; ++k) acc = acc + b2[k];
            g->s2n = acc;
        } else if (w == 2) {
#pragma unroll 8
            for (int k = 0; k < nk; ++k) acc = acc + b[k];
            g->s1a = acc;
        } else if (w == 3) {
#pragma unroll 8
            for (int k = 0; k < nk; ++k) acc = acc + b2[k];
            g->s2a = acc;
        } else {  // the ratio rows, then the turn rows
            const double* c1 = tc1 + d * nk;
            const double* c2 = tc2 + d * nk;
            const double* c3 = tc3 + d * nk;
#pragma unroll 8
            for (int k = 1; k < nk; ++k) {
                acc = acc + c1[k];
                acc = acc + c2[k];
                acc2 = acc2 + c3[k];
            }
            g->e12 = acc;
            g->e3 = acc2;
        }
    }
}

// a / D for a < 2^31 by one 64-bit multiply (Granlund-Montgomery): sh = 32 + ceil(log2 D),
// m = ceil(2^sh / D) <= 2^33, so a m < 2^64 and the error a (m D - 2^sh) / (D 2^sh) < a / 2^sh
// stays below 1 / D (host: magic_div)
__device__ __forceinline__ uint32_t div_magic(uint32_t a, uint64_t m, int sh) {
    return (uint32_t)(((uint64_t)a * m) >> sh);
}

// K2h: a path's terrain seed E0 (h_item): the exact terrain (t4; +0.0 off the raster) of the
// sampled waypoint with the largest decoded lb, over j = 0, s, 2s, ... (s = kg.lb_stride) and
// j = W - 1, each at its own cell by the evaluation's operations (the pair's points,
// arc_point's); -inf when no sample has a bound.  E0 is an exact terrain value of the path, so
// it is at most the path's maximum M, and every item of the path may start its running maximum
// E (and its lower bound Lb) there.  hdr / u: the packed header and the unit-arc table (LDS
// copies when the launch staged them).
__device__ __forceinline__ float h_path_seed(const KParams& p, const KRaster& rs, const KGrp& kg,
                                            int32_t path, const uint32_t* __restrict__ hdr,
                                            const double2* __restrict__ utab) {
    if (!rs.pmap) return -INFINITY;
    const int32_t q = (int32_t)div_magic((uint32_t)path, kg.m_d, kg.sh_d);
    const int32_t d = path - q * kg.D;
    const double4 pr = reinterpret_cast<const double4*>(kg.pairs)[q];
    const double2* u = utab + d * p.N - 1;
    const int W = kg.W;
    constexpr uint32_t NONE = 0xffffffffu, OFF = 0xfffffffeu;
    float Lb = -INFINITY;
    uint32_t best = NONE;  // the t4 index of the sample holding Lb (OFF: off the raster)
    auto take = [&](bool in, int32_t ix, int32_t iy, uint32_t e, float2 sb) {
        float ub, lb;
        pk_bound_decode(e, sb, ub, lb);
        const float v = in ? lb : 0.0f;
        const bool up = v > Lb;  // (a NaN bound: no)
        Lb = up ? v : Lb;
        best = up ? (in ? (uint32_t)p4_addr(rs, ix, iy) : OFF) : best;
    };
    {
        int32_t ix, iy;
        uint32_t e;
        float2 sb;
        bool in = gen_cell(rs, pr.x, pr.y, ix, iy);
        pk_bound_raw(rs, hdr, ix, iy, e, sb);
        take(in, ix, iy, e, sb);
        in = gen_cell(rs, pr.z, pr.w, ix, iy);
        pk_bound_raw(rs, hdr, ix, iy, e, sb);
        take(in, ix, iy, e, sb);
    }
    // four samples at a time, every load of the four issued together (a sample past the last
    // interior waypoint repeats it)
    constexpr int K = 4;
    for (int j0 = kg.lb_stride; j0 < W - 1; j0 += K * kg.lb_stride) {
        double2 uu[K];
#pragma unroll
        for (int k = 0; k < K; ++k) uu[k] = u[min(j0 + k * kg.lb_stride, W - 2)];
        uint32_t e[K];
        float2 sb[K];
        int32_t ix[K], iy[K];
        bool in[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double x0, x1;
            arc_point(pr.x, pr.y, pr.z, pr.w, uu[k].x, uu[k].y, x0, x1);
            in[k] = gen_cell(rs, x0, x1, ix[k], iy[k]);
            pk_bound_raw(rs, hdr, ix[k], iy[k], e[k], sb[k]);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) take(in[k], ix[k], iy[k], e[k], sb[k]);
    }
    return best == NONE ? -INFINITY : best == OFF ? 0.0f : rs.t4[best];
}

// counting sort, launch 1: partition b = paths [P b / NBK, P (b+1) / NBK); keys of all their
// groups (the tile under the group's middle waypoint) and the partition's histogram, stored
// bin-major so the scan yields each (bin, partition)'s offset
__global__ __launch_bounds__(1024) void k_g_hist(KParams p, KRaster rs, KGrp kg) {
    __shared__ __attribute__((aligned(16))) int32_t h[G_BINS_MAX];
    __shared__ uint16_t tk[1 << (2 * G_TBITS_MAX)];  // the tile-key table (curve order)
    // K2h with kg.seed_lds: the packed header and the unit-arc table staged for the seeds
    extern __shared__ __attribute__((aligned(16))) uint32_t s_hist_dyn[];
    const int t = threadIdx.x, b = blockIdx.x;
    if (b == 0 && t == 0) *kg.err = 0;
    for (int k = t; k < kg.bins; k += 1024) h[k] = 0;
    for (int k = t; k < (1 << (2 * kg.tbits)); k += 1024) tk[k] = kg.tkey[k];
    const uint32_t* s_hdr = rs.pmap;
    const double2* s_ut = reinterpret_cast<const double2*>(kg.utab);
    if (kg.lbp && kg.seed_lds) {
        uint4* dh = reinterpret_cast<uint4*>(s_hist_dyn);
        const uint4* gh = reinterpret_cast<const uint4*>(rs.pmap);
        for (int k = t; k < (rs.hwords >> 2); k += 1024) dh[k] = gh[k];
        double2* du = reinterpret_cast<double2*>(s_hist_dyn + rs.hwords);
        for (int k = t; k < kg.D * p.N; k += 1024) du[k] = s_ut[k];
        s_hdr = s_hist_dyn;
        s_ut = du;
    }
    __syncthreads();
    // thread = item (consecutive threads: the groups of one path, then the next path's), so
    // the key stores are coalesced and a path's pair is one broadcast load; U items per thread
    // with all their loads issued first (indices clamped into the partition)
    const int64_t lo = ((int64_t)kg.P * b / G_NBK) * kg.nseg;
    const int64_t hi = ((int64_t)kg.P * (b + 1) / G_NBK) * kg.nseg;
    const int N = p.N, W = kg.W;
    constexpr int U = 4;
    for (int64_t i0 = lo + t; i0 < hi; i0 += 1024 * U) {
        double4 pr[U];
        double2 u[U];
        int jm[U], sg[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int32_t i = (int32_t)min(i0 + k * 1024, hi - 1);
            const int32_t path = (int32_t)div_magic((uint32_t)i, kg.m_nseg, kg.sh_nseg);
            sg[k] = i - path * kg.nseg;
            const int32_t q = (int32_t)div_magic((uint32_t)path, kg.m_d, kg.sh_d);
            const int32_t d = path - q * kg.D;
            const int j0 = sg[k] * kg.G, j1 = min(j0 + kg.G, W);
            jm[k] = (j0 + j1 - 1) >> 1;  // the group's middle waypoint
            pr[k] = reinterpret_cast<const double4*>(kg.pairs)[q];
            u[k] = reinterpret_cast<const double2*>(kg.utab)[d * N + min(max(jm[k] - 1, 0), N - 1)];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int64_t i = i0 + k * 1024;
            if (i >= hi) break;
            double x0, x1;  // PathSrc::at's point
            if (jm[k] == 0) {
                x0 = pr[k].x, x1 = pr[k].y;
            } else if (jm[k] == W - 1) {
                x0 = pr[k].z, x1 = pr[k].w;
            } else {
                arc_point(pr[k].x, pr[k].y, pr[k].z, pr[k].w, u[k].x, u[k].y, x0, x1);
            }
            // the key: the position of the point's tile of the 2^tbits x 2^tbits grid on the
            // tile curve (Hilbert by default: consecutive tiles always adjacent), bins - 1 off
            // the raster or NaN
            const double fx = floor((x0 - rs.x0) * rs.inv_dx);
            const double fy = floor((rs.y_top - x1) * rs.inv_dy);
            uint32_t key = kg.bins - 1;
            if ((fx >= 0.0) && (fx < (double)rs.nx) && (fy >= 0.0) && (fy < (double)rs.ny)) {
                const uint32_t tx = (uint32_t)fx >> kg.tshift, ty = (uint32_t)fy >> kg.tshift;
                key = tk[(ty << kg.tbits) | tx];
                // a ragged last group's items in their own bins: the waves then rarely mix
                // group lengths, so k_g_eval's straight-line chunks stay wave-uniform
                if (sg[k] == kg.nseg - 1) key += kg.last_bin;
            }
            kg.key[i] = (uint16_t)key;
            atomicAdd(&h[key], 1);
        }
    }
    if (kg.lbp) {  // K2h: the partition's paths' terrain seeds, one thread per path
        const int64_t plo = (int64_t)kg.P * b / G_NBK, phi = (int64_t)kg.P * (b + 1) / G_NBK;
        for (int64_t pth = plo + t; pth < phi; pth += 1024)
            kg.lbp[pth] = h_path_seed(p, rs, kg, (int32_t)pth, s_hdr, s_ut);
    }
    __syncthreads();
    // the partition's count per bin, bin-major ([bin][partition]): k_scan_local's exclusive
    // scan of it is each (bin, partition)'s place, up to its scan block's total
    for (int k = t; k < kg.bins; k += 1024) kg.cnt[(int64_t)k * G_NBK + b] = h[k];
}

// launch 3 (after k_scan_local over cnt; the scan blocks' totals are scanned here, or by
// k_scan_totals beyond 1024 of them): LDS cursors, items scattered; U keys per thread loaded
// before the first cursor update.  The order of the items inside a (bin, partition) run follows
// the LDS atomics: it only decides which lane evaluates an item, never what the item computes.
// (A two-launch form -- device-scope
// atomics on the bin totals in the histogram launch, their scan in this one -- ran the
// histogram 11 -> 34 us at cfg3: 256 partitions' atomics on each bin address serialise
// across the XCDs; profiles/r04/prof1.)
__global__ __launch_bounds__(1024) void k_g_scatter(KParams p, KGrp kg) {
    __shared__ __attribute__((aligned(16))) int32_t cur[G_BINS_MAX];
    __shared__ int32_t stot[1024];
    __shared__ int32_t wsum[16];
    const int t = threadIdx.x;
    // K2h / K4h: block 0 forms the unit rows through its LDS (dispatched first, so hidden under
    // the scatter); the partitions are the other blocks
    if (kg.ugeo && blockIdx.x == 0) {
        unit_geo_block(p, kg, reinterpret_cast<double2*>(cur), (int)sizeof(cur));
        return;
    }
    const int b = blockIdx.x - (kg.ugeo ? 1 : 0);
    if (kg.test_fault && b == 0 && t == 0) atomicOr(kg.err, 1);  // (UAM_OPT_TEST_SORT_FAULT)
    const int nsb = kg.nsb_raw;
    if (nsb > 0) {  // the scan's block totals, scanned here (replaces k_scan_totals' launch)
        const int32_t v = t < nsb ? kg.tot[t] : 0;
        const int lane = t & 63, wv = t >> 6;
        int32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wv] = x;
        __syncthreads();
        int32_t woff = 0;
        for (int k = 0; k < wv; ++k) woff += wsum[k];
        stot[t] = woff + x - v;
        __syncthreads();
    }
    for (int k = t; k < kg.bins; k += 1024) {
        const int64_t c = (int64_t)k * G_NBK + b;
        const int sb = (int)(c / (256 * SCAN_ITEMS));
        cur[k] = kg.cnt[c] + (nsb > 0 ? stot[sb] : kg.tot[sb]);
    }
    __syncthreads();
    const int64_t lo = ((int64_t)kg.P * b / G_NBK) * kg.nseg;
    const int64_t hi = ((int64_t)kg.P * (b + 1) / G_NBK) * kg.nseg;
    constexpr int U = 8;
    for (int64_t i0 = lo + t; i0 < hi; i0 += 1024 * U) {
        uint16_t kk[U];
#pragma unroll
        for (int k = 0; k < U; ++k) kk[k] = kg.key[min(i0 + k * 1024, hi - 1)];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int64_t i = i0 + k * 1024;
            if (i < hi) {
                const int32_t at = atomicAdd(&cur[kk[k]], 1);
                if ((uint32_t)at < (uint32_t)kg.n_items)
                    kg.order[at] = (int32_t)i;
                else
                    atomicOr(kg.err, 1);  // never in a consistent sort: poisons the outputs
            }
        }
    }
}

// sqrt(x) for x in [2^-767, 2^1000]: the gfx9 lowering of sqrt(double) (rsq, then two
// Goldschmidt / Newton corrections) without its scaling and special-value steps, which are
// identities in that range -- so bit-equal to sqrt() there.  Callers check the range.
__device__ __forceinline__ double sqrt_mid(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    double g = x * r, h = r * 0.5;
    const double e = fma(-h, g, 0.5);
    g = fma(g, e, g);
    h = fma(h, e, h);
    const double d0 = fma(-g, g, x);
    g = fma(d0, h, g);
    const double d1 = fma(-g, g, x);
    return fma(d1, h, g);
}

// every (path, group) item in sorted order (workgroup b takes the sorted chunk xcd_chunk(b));
// the group's waypoints from the packed raster exactly as seg_pass2_pack reads them (block
// codes in LDS), CH gathers issued before the first of them is consumed; the unit-arc rows in
// LDS (the items of a wave come from different groups and displacements: per-lane rows); the
// partials go to the item's slot.  Dynamic LDS: the block codes, the unit-arc table, padded
// to a floor that caps the workgroups per CU (UAM_OPT_K2G_LDS) so an XCD's resident items
// cover a narrow range of the sorted order.
// LS / MS: get_cost's length term and the ratio rows on squared norms (length_smooth,
// maxratio_smooth), compile-time so the waypoint loop carries no select for them.
// The group's waypoints go through in chunks of CH.  A chunk in which every lane of the wave
// has CH waypoints, none of them the goal p_{W-1} (the key puts a ragged last group's items in
// their own bins, so waves rarely mix group lengths), runs the straight-line form: each point
// generated by the arc formula, every segment term and kinematic row added (the first chunk
// only skips the rows that belong to the previous group), the segment norm through sqrt_mid
// when the whole wave's squared norms are in its range.  Any other chunk runs the general form
// with the endpoint, range and row tests per waypoint.  Both add exactly the same terms in the
// same order.
// (The waypoint cells, when requested, come from k_cells beside this launch.)
template <int CH, bool LS, bool MS>
__global__ __launch_bounds__(256, CH > 11 ? 2 : 4) void k_g_eval(KParams p, KRaster rs, KGrp kg,
                                                const uint4* __restrict__ rec) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    uint32_t* s_map = s_dyn;
    const int mapw = (rs.pwords + 3) & ~3;
    double2* s_u = reinterpret_cast<double2*>(s_dyn + mapw);
    // staging: every load of a thread issued before its first LDS store (one round trip per
    // workgroup instead of one per 256 words)
    {
        constexpr int U = 4;
        const int nv = rs.pwords >> 2, nu = kg.D * p.N;
        const uint4* src = reinterpret_cast<const uint4*>(rs.pmap);
        uint4* dst = reinterpret_cast<uint4*>(s_map);
        const uint4* gu = reinterpret_cast<const uint4*>(kg.utab);
        uint4* du = reinterpret_cast<uint4*>(s_u);
        for (int i0 = threadIdx.x; i0 < nv + nu; i0 += 256 * U) {
            uint4 v[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {  // unconditional loads (past the end: the first word)
                const int i = i0 + k * 256;
                v[k] = *(i < nv ? src + i : i < nv + nu ? gu + (i - nv) : src);
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {  // unconditional stores (past the end: a junk slot)
                const int i = i0 + k * 256;
                *(i < nv ? dst + i : du + min(i - nv, nu)) = v[k];
            }
        }
        for (int i = (nv << 2) + threadIdx.x; i < rs.pwords; i += 256) s_map[i] = rs.pmap[i];
    }
    __syncthreads();
    const int64_t pos = xcd_chunk(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
    if (pos >= kg.n_items) return;
    const int32_t item = kg.order[pos];
    const int32_t path = (int32_t)div_magic((uint32_t)item, kg.m_nseg, kg.sh_nseg);
    const int s = item - path * kg.nseg;
    const int32_t q = (int32_t)div_magic((uint32_t)path, kg.m_d, kg.sh_d), d = path - q * kg.D;
    const double4 pr = reinterpret_cast<const double4*>(kg.pairs)[q];
    const int N = p.N, W = kg.W;
    const double2* urow = s_u + d * N;
    const int j0 = s * kg.G, j1 = min(j0 + kg.G, W);
    // arc_point's arithmetic with the pair's terms hoisted (the same operations in the same
    // order: v = x0 - xf, C = (xf + x0) / 2, p = C + 0.5 (R(v) u))
    const double vx = pr.x - pr.z, vy = pr.y - pr.w;
    const double cx = (pr.z + pr.x) * 0.5, cy = (pr.w + pr.y) * 0.5;
    auto arc = [&](int j, double& x0, double& x1) {  // 1 <= j <= N
        const double2 u = urow[j - 1];
        x0 = cx + 0.5 * (vx * u.x - vy * u.y);
        x1 = cy + 0.5 * (vy * u.x + vx * u.y);
    };
    auto point = [&](int j, double& x0, double& x1) {
        if (j == 0) {
            x0 = pr.x, x1 = pr.y;
        } else if (j == W - 1) {
            x0 = pr.z, x1 = pr.w;
        } else {
            arc(j, x0, x1);
        }
    };
    // this group's share of pass 1 (path_pass1's arithmetic), formed while the waypoints are
    // generated for the gathers, each point once: segment p_{j-1} -> p_j for j in
    // [max(j0, 1), j1) adds to L and the length; kinematic row k (segments k + 1 and k + 2)
    // belongs to the group of waypoint k + 1, so the point after the group closes its last row
    double gL = 0.0, glen = 0.0, gk = 0.0;
    double px, py, pdx = 0.0, pdy = 0.0, pn = 0.0;
    point(j0 == 0 ? 0 : j0 - 1, px, py);
    if (j0 == 0 && p.quirk_length) {  // get_cost's anchor term (y_0 = anchor, y_1 = p_0)
        const double ax = p.anchor_mode ? p.anchor_x : px;
        const double ay = p.anchor_mode ? p.anchor_y : py;
        const double dx = px - ax, dy = py - ay;
        const double n = sqrt(dx * dx + dy * dy);  // = (0 + dx dx) + dy dy: dx dx is never -0
        gL = gL + (LS ? n * n : n);
    }
    auto row = [&](double nk, double dx, double dy) {  // kinematic row: segments (pd, d)
        double dt = 0.0;
        dt = dt + pdx * dx;
        dt = dt + pdy * dy;
        double c1, c2, c3;
        kin_row(p, pn, nk, dt, c1, c2, c3);
        gk = gk + c1;
        gk = gk + c2;
        gk = gk + c3;
    };
    // general form: segment p_{j-1} -> (qx, qy) = p_j with every test of the reference's loop
    auto segment = [&](int j, double qx, double qy) {
        const double dx = qx - px, dy = qy - py;
        const double n = sqrt(dx * dx + dy * dy);  // norm_2 = sqrt(dot) (casadi_norm_2)
        if (j < j1) {
            glen = glen + n;
            if (!p.quirk_length || j <= N) gL = gL + (LS ? n * n : n);
        }
        const double nk = MS ? n * n : n;
        if (j >= j0 + 1 && j >= 2) row(nk, dx, dy);  // row k = j - 2 (problem.py:100-107)
        pdx = dx, pdy = dy, pn = nk, px = qx, py = qy;
    };
    // straight-line form: j0 < j < j1, 2 <= j <= N (RV: the row is added; false only for the
    // first chunk's waypoints j0 and, in group 0, j0 + 1 -- decided per lane)
    // The empty asm statements pin the running sums to their waypoint: without them the
    // scheduler defers the dependent adds to the chunk's end and keeps every waypoint's terms
    // live (the kernel then spills at 4 waves per SIMD).
    auto pin = [](double& v) { asm volatile("" : "+v"(v)); };
    auto segment_fast = [&](double qx, double qy, bool rv) {
        const double dx = qx - px, dy = qy - py;
        const double ss = dx * dx + dy * dy;
        double n = sqrt_mid(ss);
        const bool ok = (ss >= 0x1p-767) && (ss <= 0x1p1000);  // NaN: not ok
        if (__builtin_expect(__any(!ok), 0)) {  // wave-uniform: sqrt() where out of range
            if (!ok) n = sqrt(ss);
        }
        glen = glen + n;
        gL = gL + (LS ? n * n : n);
        const double nk = MS ? n * n : n;
        if (rv) row(nk, dx, dy);
        pin(glen), pin(gL), pin(gk);
        pdx = dx, pdy = dy, pn = nk, px = qx, py = qy;
    };
    // Phi / N: q0 = a (1/N) and one residual step (Markstein), correctly rounded for every
    // finite float a and 1 <= N <= 4096 (all 2^23 significands checked; the power-of-two
    // scaling is exact in double: tests/test_host_cpu.py), so bit-equal to the division.
    // kg.inv_n = 0 (larger N): the division itself.
    const double dN = (double)N, yN = kg.inv_n;
    auto over_n = [&](double a) {
        if (yN == 0.0) return a / dN;
        const double q0 = a * yN;
        const double q1 = fma(fma(-q0, dN, a), yN, q0);
        return __builtin_isinf(a) ? q0 : q1;  // -0 / N comes out +0: both add to gc alike
    };
    // the gathers of point (x0, x1): one value load and one terrain load per waypoint
    // (pk_locate), issued outside every branch so the compiler's wait counts stay exact and CH
    // gathers are really in flight; a waypoint with nothing to read (code 0's value, code 3's
    // terrain, off the raster) reads the planes' first line, one line per wave, unused.
    const uint4* const vdummy = reinterpret_cast<const uint4*>(rs.p4);
    auto locate = [&](double x0, double x1, int t, uint32_t& inb, auto& cs,
                      const float*& tp) -> const uint4* {
        // the cell: floor(t) in [0, n) <=> t in [0, n) for integer n, and the truncating
        // conversion equals floor for t >= 0 (NaN fails both tests)
        const double tx = (x0 - rs.x0) * rs.inv_dx;
        const double ty = (rs.y_top - x1) * rs.inv_dy;
        const uint4* vp = vdummy;
        tp = rs.t4;
        if ((tx >= 0.0) && (tx < (double)rs.nx) && (ty >= 0.0) && (ty < (double)rs.ny)) {
            inb |= 1u << t;
            const int32_t ix = (int32_t)tx, iy = (int32_t)ty;
            cs.set(t, pk_locate(rs, rec, s_map, ix, iy, vp, tp));
        }
        return vp;
    };
    // the consume step, branch-free: a lane with nothing gathered adds +0.0 (an exact no-op on
    // accumulators that are never -0) and takes fmax(hmax, +0.0) off the raster, exactly what
    // the branches of raster_pass2_skip do
    double gc = 0.0, gn = 0.0;
    float hmax = -INFINITY;
    uint32_t nh = 0, off = 0;
    auto consume1 = [&](const uint4& r, float tv, bool in, const PkSlots& cs, int t) {
        const uint32_t c = ((cs.c0 >> t) & 1u) | (((cs.c1 >> t) & 1u) << 1);
        uint32_t phi, psi, hit;
        float rter;
        pk_terms(r, cs, t, phi, psi, hit, rter);
        nh += hit;
        off += in ? 0u : 1u;
        gc = gc + over_n((double)__uint_as_float(phi));
        gn = gn + (double)__uint_as_float(psi);
        hmax = fmaxf(hmax, !in ? 0.0f : (c & 3u) == 3u ? rter : tv);
    };
    for (int jc = j0, it = 0; jc < j1; jc += CH, ++it) {
        const int je = min(jc + CH, j1);
        if (__all(je - jc == CH && je < W)) {  // wave-uniform: the straight-line form
            const bool first = it == 0;
            uint4 r[CH];
            float tv[CH];
            uint32_t inb = 0;
            PkSlots cs;
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int j = jc + t;
                double x0, x1;
                if (t == 0 && first && __any(j == 0)) {
                    point(j, x0, x1);
                } else {
                    arc(j, x0, x1);
                }
                // the rows of waypoints j0 and (group 0) j0 + 1 belong elsewhere / do not exist
                const bool rv = !(first && (t == 0 || (t == 1 && j0 == 0)));
                if (t == 0 && first && j == 0) {
                    // p_0 of group 0: no segment ends here (the anchor term stands for it)
                    px = x0, py = x1;
                } else {
                    segment_fast(x0, x1, rv);
                }
                const float* tp;
                r[t] = *locate(x0, x1, t, inb, cs, tp);
                tv[t] = *tp;
            }
#pragma unroll
            for (int t = 0; t < CH; ++t)
                consume1(r[t], tv[t], (inb >> t) & 1u, cs, t);
        } else {  // the general form, one waypoint at a time (the ragged and last chunks)
#pragma unroll 1
            for (int j = jc; j < je; ++j) {
                double x0 = px, x1 = py;  // j = 0: p_0, generated above
                if (j > 0) {
                    point(j, x0, x1);
                    segment(j, x0, x1);
                }
                uint32_t inb = 0;
                PkSlots cs;
                const float* tp;
                const uint4 r = *locate(x0, x1, 0, inb, cs, tp);
                consume1(r, *tp, inb & 1u, cs, 0);
            }
        }
    }
    if (j1 <= W - 1) {  // the point after the group: its last kinematic row only
        double x0, x1;
        point(j1, x0, x1);
        segment(j1, x0, x1);
    }
    GSlot o;
    o.cost = gc;
    o.psi = gn;
    o.L = gL;
    o.len = glen;
    o.ksum = gk;
    o.hmax = hmax;
    o.cnt = nh | (off << 8);
    kg.slot[(int64_t)s * kg.P + path] = o;
}

// outputs of every path (block = 64 pairs x D, k_eval_pairs's store layout): the partials
// combined in group order (cost = (N+1) L + the Phi/N partials), and the selection over each
// pair's D paths
template <int NR>  // slots per path held in registers (0: a loop for long paths)
__global__ __launch_bounds__(1024) void k_g_final(KParams p, KGrp kg, KOut out,
                                                  int32_t* __restrict__ best_f,
                                                  int32_t* __restrict__ best_l) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int D = kg.D, t = threadIdx.x;
    double* s_cost = smem;
    double* s_len = smem + 64 * D;
    const int64_t q0 = (int64_t)blockIdx.x * 64;
    const int qi = t / D, di = t - qi * D;
    const bool bad = *kg.err != 0;  // an inconsistent sort (k_g_scatter / k_v_hist)
    if (q0 + qi < kg.n_pairs) {
        const int64_t gp = (q0 + qi) * D + di;
        double L = 0.0, len = 0.0, ksum = 0.0, nsum = 0.0, hmax = -INFINITY;
        int32_t nh = 0, off = 0;
        double cost;
        if (NR > 0) {
            // every slot loaded before the first is used (clamped indices: unconditional
            // loads, one round trip); the Phi/N partials wait in registers for L
            GSlot g[NR > 0 ? NR : 1];
#pragma unroll
            for (int s = 0; s < NR; ++s)
                g[s] = kg.slot[(int64_t)min(s, kg.nseg - 1) * kg.P + gp];
#pragma unroll
            for (int s = 0; s < NR; ++s) {
                if (s >= kg.nseg) break;
                L = L + g[s].L;
                len = len + g[s].len;
                ksum = ksum + g[s].ksum;
                nsum = nsum + g[s].psi;
                hmax = fmax(hmax, (double)g[s].hmax);
                nh += (int32_t)(g[s].cnt & 255u);
                off += (int32_t)((g[s].cnt >> 8) & 255u);
            }
            cost = (double)(p.N + 1) * L;
#pragma unroll
            for (int s = 0; s < NR; ++s) {
                if (s >= kg.nseg) break;
                cost = cost + g[s].cost;
            }
        } else {
            for (int s = 0; s < kg.nseg; ++s) {
                const GSlot g = kg.slot[(int64_t)s * kg.P + gp];
                L = L + g.L;
                len = len + g.len;
                ksum = ksum + g.ksum;
                nsum = nsum + g.psi;
                hmax = fmax(hmax, (double)g.hmax);
                nh += (int32_t)(g.cnt & 255u);
                off += (int32_t)((g.cnt >> 8) & 255u);
            }
            cost = (double)(p.N + 1) * L;
            for (int s = 0; s < kg.nseg; ++s) cost = cost + kg.slot[(int64_t)s * kg.P + gp].cost;
        }
        put_outputs(out, gp, bad, cost, L, len, ksum, nsum, p.altitude - hmax, nh, off, 0);
        s_cost[di * 64 + qi] = cost;
        s_len[di * 64 + qi] = len;
    }
    __syncthreads();
    put_selection(kg, bad, q0, t, s_cost, s_len, best_f, best_l);
}

// ---- K2h: generated candidates in the similarity form (oracle orc_eval_generated_h) --------
// The candidate arcs are p_k = C + (1/2) R(v) u_k (u_0 = (1, 0), u_{N+1} = (-1, 0)): the unit
// polyline of the displacement's table row under a similarity of scale h = |v| / 2.  Every
// term that depends on the geometry only -- get_cost's L (problem.py:130-146, with the quirk's
// anchor term), the true length (solver.py:49), the kinematic rows (problem.py:100-107, their
// ratio rows scale with h, their turn rows are the unit polyline's) -- is a per-displacement
// sum of the unit polyline times h (maxratio_smooth = 0), formed once per launch (UGeo) and
// scaled per path in the output launch.  What stays per waypoint is what the raster decides:
// the point, its cell and its record (Phi / N, psi, terrain, no-fly hit), with K2g's sort,
// staging and grouped partial sums; so an item carries no f64 geometry (no segment norms, no
// square roots, no kinematic rows) and its slot is 24 B.  Exact in real arithmetic; in float64
// the geometry terms differ from per-segment sums by rounding only (bench.py
// parity.vs_sequential_order on the whole cfg3 batch).

struct alignas(8) HSlot {  // 24 B per (path, group), written by one lane
    double cost;   // Phi / N of the group's waypoints, from +0.0 in waypoint order
    double psi;    // the no-fly psi, likewise
    float hmax;    // max terrain of the group's waypoints as consume reads it
    uint32_t cnt;  // nfz hits | off-raster << 8
};

// every (path, group) item in K2g's sorted order: the group's points, cells and packed entries
// only.  Every chunk is straight-line, in three phases so the LDS and memory round trips of its
// CH slots overlap: the CH cells (the arc formula; p_0 / p_{W-1} from the pair's cells), the CH
// header reads (code word, bound entry, superblock), then per slot the decisions and two
// unconditional loads -- the code's entry (a slot with nothing to read takes the first p4 line)
// and the terrain (the first t4 word unless fetched) -- by 32-bit offsets from the packed
// copy's base; then the branch-free consume.
//
// The terrain maximum by bounds (build-defined; the outputs are exactly the per-waypoint
// maximum's): min_clearance needs only the path's maximum terrain M, an order-free maximum, so
// a waypoint's exact terrain is fetched (t4) only when it could still be M.  Every in-raster
// waypoint w has decoded bounds lb_w <= terrain_w <= ub_w (pk_bound_raw + pk_bound_decode).  The item keeps
//   Lb: a lower bound of M: the path's seed (below), raised by its own waypoints' lb as it
//       goes; off-raster waypoints count +0.0, their exact value;
//   E:  the maximum of exact terrain values of the path: the seed E0 (h_path_seed, formed once
//       per path by the histogram launch: the exact terrain of the sampled waypoint with the
//       largest lb) and those the item takes (fetched, code-3 records, off-raster +0.0, blocks
//       whose bounds coincide).
// It fetches w iff !(ub_w <= E) && !(ub_w < Lb) (NaN bounds: "no bound", always fetched).
// Exactness: let w* hold M, in this item's group.  If w* was not taken exactly, then either
// ub_w* <= E, so M <= E and E -- an exact terrain value of the path -- is M; or ub_w* < Lb <= M,
// impossible since M <= ub_w*.  So the group holding M reports M, every group reports at most
// its own maximum (E holds exact values), and the output launch's maximum over the groups is M.
// (A group without M may report less than its own maximum: only the path's is an output.)
// The slot's hmax is that E.  (Measured, cfg3: 0.19 fetches per waypoint with the sampled lb
// alone and chunks issued one ahead, tools/k2h_counts.py.)
// K2h workgroup: 256 items (cfg3 0.297 ms against 0.306 at 512, profiles/r05/k2h12)
constexpr int H_BS = UAM_K2H_BS;
template <int CH, bool TE>  // TE: the terrain in the entry (UAM_OPT_K2H_TERRAIN 1)
__device__ __forceinline__ void h_item(const KParams& p, const KRaster& rs, const KGrp& kg,
                                       const uint32_t* __restrict__ s_hdr,
                                       const double2* __restrict__ s_u, bool live, int32_t item,
                                       int32_t path, int32_t q, const double4& pr,
                                       float seed) {
    // a lane past the last item evaluates nothing and writes nothing
    const int s = item - path * kg.nseg;
    const int32_t d = path - q * kg.D;
    const int N = p.N, W = kg.W;
    // waypoint j's unit vector is urow[j] (j = 1..N); the slots past a row's ends read the
    // neighbouring rows or the staged padding (LDS either way), and their cells are replaced
    const double2* urow = s_u + d * N - 1;
    const int j0 = s * kg.G, j1 = live ? min(j0 + kg.G, W) : j0;
    // chunks: the wave's most, so the loop is wave-uniform
    int nch = (j1 - j0 + CH - 1) / CH;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nch = max(nch, __shfl_xor(nch, o));
    const double vx = pr.x - pr.z, vy = pr.y - pr.w;
    const double cx = (pr.z + pr.x) * 0.5, cy = (pr.w + pr.y) * 0.5;
    const double dN = (double)N, yN = kg.inv_n;
    auto over_n = [&](double a) {  // Phi / N exactly as k_g_eval forms it (K2h: N <= 4096)
        const double q0 = a * yN;
        const double q1 = fma(fma(-q0, dN, a), yN, q0);
        return __builtin_isinf(a) ? q0 : q1;
    };
    // the end points' cells, formed once
    int32_t ixF, iyF, ixL, iyL;
    const bool inF = gen_cell(rs, pr.x, pr.y, ixF, iyF);
    const bool inL = gen_cell(rs, pr.z, pr.w, ixL, iyL);
    const uint16_t* const bnd = reinterpret_cast<const uint16_t*>(s_hdr + rs.bnd_off);
    const float2* const sbt = reinterpret_cast<const float2*>(s_hdr + rs.sbt_off);
    const char* const pk = rs.pk;
    // the plane offsets as values (a select between the struct's fields otherwise becomes a
    // select of their addresses and a memory read per slot)
    const uint32_t o4 = __builtin_amdgcn_readfirstlane(rs.o4);
    const uint32_t o8 = __builtin_amdgcn_readfirstlane(rs.o8);
    const uint32_t o16 = __builtin_amdgcn_readfirstlane(rs.o16);
    const uint32_t ot4 = __builtin_amdgcn_readfirstlane(rs.ot4);
    const uint32_t op8 = __builtin_amdgcn_readfirstlane(rs.op8);
    double gc = 0.0, gn = 0.0;
    float Lb = seed, E = seed;  // the path's seed: an exact terrain value of the path
    uint32_t nh = 0, off = 0;
    // one chunk ahead: chunk c + 1's loads are issued before chunk c is consumed (the fetch
    // rule then sees E without chunk c's fetched values: valid, E only holds exact values).
    // Iteration c issues chunk c + 1 into the B arrays and consumes chunk c from the A arrays.
    uint4 rA[CH];
    float tvA[CH];
    uint32_t kcA[CH], vinA = 0, tkA = 0;
    int nvA = 0;
    // (ahead: chunk c + 1 issued before chunk c is consumed -- the same at cfg3 with 256-item
    // workgroups, profiles/r05/k2h12)
    constexpr bool ahead = false;
    for (int c = ahead ? -1 : 0; c < nch; ++c) {  // (nch wave-uniform)
        const int ci = ahead ? c + 1 : c;  // the chunk issued by this iteration
        uint4 rB[CH];
        float tvB[CH];
        uint32_t kcB[CH], vinB = 0, tkB = 0;
        int nvB = 0;
        if (ci < nch) {
            const int jc = j0 + ci * CH;
            const double2* uc = urow + jc;
            // phase 1: the cells (in-raster and in-group bits per slot)
            int32_t ix[CH], iy[CH];
            uint32_t vjb = 0;
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int j = jc + t;
                const double2 u = uc[t];
                int32_t x, y;
                bool in = gen_cell(rs, cx + 0.5 * (vx * u.x - vy * u.y),
                                   cy + 0.5 * (vy * u.x + vx * u.y), x, y);
                if (t == 0) {  // (j == 0 only in a chunk's first slot)
                    const bool f = jc == 0;
                    x = f ? ixF : x;
                    y = f ? iyF : y;
                    in = f ? inF : in;
                }
                const bool l = j == W - 1;
                ix[t] = l ? ixL : x;
                iy[t] = l ? iyL : y;
                in = l ? inL : in;
                const bool vj = j < j1;
                vjb |= (uint32_t)vj << t;
                vinB |= (uint32_t)(in & vj) << t;
            }
            // phase 2: the header reads (cell (0, 0) for a slot off the raster: valid reads)
            uint32_t cw[CH], be[CH];
            float2 sb[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int32_t b = pk_block(rs, ix[t], iy[t]);
                cw[t] = s_hdr[b >> 4] >> ((b & 15) * 2);
                if constexpr (!TE) {
                    const uint32_t bx = (uint32_t)(ix[t] >> rs.bshift);
                    const uint32_t by = (uint32_t)(iy[t] >> rs.bshift);
                    be[t] = bnd[__umul24(by, (uint32_t)rs.bnbx) + bx];
                    sb[t] = sbt[__umul24(by >> 2, (uint32_t)rs.sbnbx) + (bx >> 2)];
                }
            }
            // phase 3: the decisions and the loads
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const bool vin = (vinB >> t) & 1u, vj = (vjb >> t) & 1u;
                const uint32_t code = cw[t] & (vin ? 3u : 0u);
                if constexpr (TE) {
                    // code 1: the 8-B {phi, terrain} entry; 2 / 3: the 16-B record (both carry
                    // the exact terrain); code 0: nothing to read (phi, psi +-0, terrain +0.0)
                    const bool rec = code & 2u;
                    const uint32_t a4 = (uint32_t)p4_addr(rs, ix[t], iy[t]);
                    const uint32_t ab = (uint32_t)p44_addr(rs, ix[t], iy[t]) << 3;
                    const uint32_t voff = rec ? o16 + (a4 << 4) : code ? op8 + (ab & ~15u) : o4;
                    kcB[t] = code | (rec ? 0u : (ab & 8u));
                    rB[t] = *reinterpret_cast<const uint4*>(pk + voff);
                    (void)vj;
                    continue;
                }
                float ub, lb;
                pk_bound_decode(be[t], sb[t], ub, lb);
                // off the raster or code 0: +0.0, an exact value and a lower bound; a block
                // of one value: ub
                const bool zero = !vin | (code == 0u);
                Lb = fmaxf(Lb, vj ? (zero ? 0.0f : lb) : -INFINITY);
                E = fmaxf(E, vj ? (zero ? 0.0f : lb == ub ? ub : -INFINITY) : -INFINITY);
                const bool fetch = !zero & (code != 3u) & !(ub <= E) & !(ub < Lb);
                const uint32_t a4 = (uint32_t)p4_addr(rs, ix[t], iy[t]);
                // the entry's byte offset in its plane: a4 * 4 / 8 / 16 for codes 1 / 2 / 3;
                // its aligned 16 B and the cell's word in them
                const uint32_t ab = a4 << (code + 1u);
                const uint32_t base = (code & 2u) ? ((code & 1u) ? o16 : o8) : o4;
                const uint32_t voff = base + (code ? (ab & ~15u) : 0u);
                kcB[t] = code | (ab & 12u);
                rB[t] = *reinterpret_cast<const uint4*>(pk + voff);
                tvB[t] = *reinterpret_cast<const float*>(pk + (ot4 + (fetch ? a4 * 4u : 0u)));
                tkB |= (uint32_t)fetch << t;
            }
            nvB = max(0, min(CH, j1 - jc));  // slots past the group's end: no waypoint
        }
        if (!ahead) {
#pragma unroll
            for (int t = 0; t < CH; ++t) rA[t] = rB[t], tvA[t] = tvB[t], kcA[t] = kcB[t];
            vinA = vinB, tkA = tkB, nvA = nvB;
        }
        if (c >= 0) {
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const bool vl = t < nvA;
                const bool in = (vinA >> t) & 1u;
                if constexpr (TE) {
                    const uint4 r = rA[t];
                    const uint32_t code = kcA[t] & 3u;  // (0 off the raster)
                    const bool rec = code & 2u, s1 = kcA[t] & 8u;
                    const uint32_t lo = s1 ? r.z : r.x, hi = s1 ? r.w : r.y;
                    const uint32_t phi = code ? (rec ? r.x : lo) : 0u;
                    const uint32_t tb = rec ? ((r.w & UAM_FLAG_NODATA) ? 0u : r.z) : hi;
                    nh += (rec && (r.w & UAM_FLAG_NFZ)) ? 1u : 0u;
                    off += (vl && !in) ? 1u : 0u;
                    gc = gc + over_n((double)__uint_as_float(phi));
                    gn = gn + (rec ? (double)__uint_as_float(r.y) : 0.0);
                    // (off the raster, or code 0: +0.0 exactly)
                    E = fmaxf(E, code ? __uint_as_float(tb) : vl ? 0.0f : -INFINITY);
                    continue;
                }
                uint32_t phi, psi, hit;
                float rter;
                pk_terms_k(rA[t], kcA[t], phi, psi, hit, rter);
                nh += hit;
                off += (vl && !in) ? 1u : 0u;
                gc = gc + over_n((double)__uint_as_float(phi));
                gn = gn + (double)__uint_as_float(psi);
                const float ter = (kcA[t] & 3u) == 3u ? rter : ((tkA >> t) & 1u) ? tvA[t] : -INFINITY;
                E = fmaxf(E, ter);
            }
        }
        if (ahead) {
#pragma unroll
            for (int t = 0; t < CH; ++t) rA[t] = rB[t], tvA[t] = tvB[t], kcA[t] = kcB[t];
            vinA = vinB, tkA = tkB, nvA = nvB;
        }
    }
    HSlot o;
    o.cost = gc;
    o.psi = gn;
    o.hmax = E;
    o.cnt = nh | (off << 8);
    if (live) reinterpret_cast<HSlot*>(kg.slot)[(int64_t)s * kg.P + path] = o;
}

// K2h evaluation: workgroups of H_BS items (xcd_chunk), the packed raster's header (codes,
// bounds, superblocks) and the unit-arc rows (+ G + CH padding slots) staged in LDS, then one item
// per lane (h_item)
template <int CH, bool TE>
__global__ __launch_bounds__(H_BS, UAM_K2H_MINW) void k_h_eval(KParams p, KRaster rs, KGrp kg) {
    PK_CODES_CHECK(CH);
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    uint32_t* s_hdr = s_dyn;
    // the header in LDS: codes, bounds and superblocks; the code map alone with TE
    const int hw = TE ? rs.bnd_off : rs.hwords;
    double2* s_u = reinterpret_cast<double2*>(s_dyn + hw);
    // the item's order entry, pair and path bound first: their dependent round trips overlap
    // the staging below instead of following it
    const int64_t pos = xcd_chunk(blockIdx.x, gridDim.x) * H_BS + threadIdx.x;
    const bool live = pos < kg.n_items;
    const int32_t item = live ? kg.order[pos] : 0;
    const int32_t path = (int32_t)div_magic((uint32_t)item, kg.m_nseg, kg.sh_nseg);
    const int32_t q = (int32_t)div_magic((uint32_t)path, kg.m_d, kg.sh_d);
    const double4 pr = reinterpret_cast<const double4*>(kg.pairs)[q];
    const float seed = kg.lbp ? kg.lbp[path] : -INFINITY;
    const int nu = kg.D * p.N;
    {  // staging: every load of a thread issued before its first LDS store (hw % 4 == 0)
        constexpr int U = 4;
        const int nv = hw >> 2;
        const uint4* src = reinterpret_cast<const uint4*>(rs.pmap);
        uint4* dst = reinterpret_cast<uint4*>(s_hdr);
        const uint4* gu = reinterpret_cast<const uint4*>(kg.utab);
        uint4* du = reinterpret_cast<uint4*>(s_u);
        for (int i0 = threadIdx.x; i0 < nv + nu; i0 += H_BS * U) {
            uint4 v[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {  // unconditional loads (past the end: the first word)
                const int i = i0 + k * H_BS;
                v[k] = *(i < nv ? src + i : i < nv + nu ? gu + (i - nv) : src);
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {  // unconditional stores (past the end: a pad slot)
                const int i = i0 + k * H_BS;
                *(i < nv ? dst + i : du + min(i - nv, nu)) = v[k];
            }
        }
    }
    __syncthreads();
    // the padding: a lane's slots reach index nu + G + CH - 2 at most (a last group of one
    // waypoint in a wave of full ones)
    if ((int)threadIdx.x < kg.G + CH) s_u[nu + threadIdx.x] = make_double2(0.0, 0.0);
    __syncthreads();
    h_item<CH, TE>(p, rs, kg, s_hdr, s_u, live, item, path, q, pr, seed);
}

// The waypoint cells (the reference's returned waypoints as raster cells, solver.py:49,
// main.py:186-190) of the sorted forms: cells[path][j] = iy nx + ix (-1 off the raster) by the
// evaluations' own point and cell arithmetic (gen_cell), one thread per (path, j), so
// consecutive threads write consecutive cells -- whole lines, no gathers.  (Written by the
// evaluation's lanes through LDS instead, the 21-cell runs of scattered items cost K2h ~120 us
// of partial-line writes per cfg3 step: 402 MB of WRITE_SIZE for 164 MB of cells,
// profiles/r04/final2/cells.)
// The waypoint cells of paths [path0, path0 + np) by one workgroup of nt threads (np <= 1024):
// each path's chord terms (cx, cy, vx, vy: arc_point's) and end-point cells go to s_cv / s_e
// once, then work item w = (path lp = w / R, run k = w % R) forms the run's 4 cells
// j = 4k ... 4k + 3 of one path (R = ceil(W / 4) runs a path; cells past W are not stored),
// so a lane reads its path's terms once and selects nothing per cell; items advance by nt a
// step (nt = lstep R + kstep, one conditional subtraction).  Every thread of the workgroup
// calls it (it synchronises).  u_rows: the unit-arc rows (LDS when staged).
__device__ __forceinline__ void cells_rows(const KParams& p, const KGrp& kg, int64_t path0,
                                           int np, double4* s_cv, int4* s_e,
                                           const double2* __restrict__ u_rows, int t, int nt) {
    const int W = kg.W, N = p.N;
    __syncthreads();  // (a previous block's reads of s_cv / s_e are done)
    for (int i = t; i < np; i += nt) {
        const int32_t path = (int32_t)(path0 + i);
        const int32_t q = (int32_t)div_magic((uint32_t)path, kg.m_d, kg.sh_d);
        const double4 pr = reinterpret_cast<const double4*>(kg.pairs)[q];
        s_cv[i] = make_double4((pr.z + pr.x) * 0.5, (pr.w + pr.y) * 0.5, pr.x - pr.z,
                               pr.y - pr.w);
        int32_t ix, iy;  // the end points: the pair's own coordinates
        const int32_t c0 = gen_cell_g(kg.cx0, kg.cy_top, kg.cinv_dx, kg.cinv_dy, kg.cnx, kg.cny,
                                      pr.x, pr.y, ix, iy) ? iy * kg.cnx + ix : -1;
        const int32_t c1 = gen_cell_g(kg.cx0, kg.cy_top, kg.cinv_dx, kg.cinv_dy, kg.cnx, kg.cny,
                                      pr.z, pr.w, ix, iy) ? iy * kg.cnx + ix : -1;
        s_e[i] = make_int4((path - q * kg.D) * N, c0, c1, 0);
    }
    __syncthreads();
    int32_t* out = kg.cells + path0 * W;
    const int R = (W + 3) >> 2, items = np * R;
    int lp = t / R, k = t - lp * R;
    const int lstep = nt / R, kstep = nt - lstep * R;
    for (int w = t; w < items; w += nt) {
        const double4 cv = s_cv[lp];
        const int4 e = s_e[lp];
        const int j0 = 4 * k;
        int32_t v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int jj = j0 + c;
            const double2 u = u_rows[e.x + min(max(jj - 1, 0), N - 1)];
            const double x0 = cv.x + 0.5 * (cv.z * u.x - cv.w * u.y);  // arc_point's ops
            const double x1 = cv.y + 0.5 * (cv.w * u.x + cv.z * u.y);
            int32_t ix, iy;
            const bool in = gen_cell_g(kg.cx0, kg.cy_top, kg.cinv_dx, kg.cinv_dy, kg.cnx, kg.cny,
                                       x0, x1, ix, iy);
            v[c] = jj == 0 ? e.y : jj == W - 1 ? e.z : in ? iy * kg.cnx + ix : -1;
        }
        // streaming stores: the 164 MB of cfg3's cells do not stay in L2 / the Infinity Cache
        // as dirty lines whose write-back the next step's gathers would meet (plain stores:
        // cfg3 with cells 0.399 against 0.374 ms, profiles/r05/cc6); a wave's runs cover ~3
        // paths' contiguous rows
        int32_t* o = out + (int64_t)lp * W + j0;
        if (j0 + 3 < W && !(((uintptr_t)o) & 7)) {
            typedef int32_t v2i __attribute__((ext_vector_type(2)));
            const v2i w0 = {v[0], v[1]}, w1 = {v[2], v[3]};
            __builtin_nontemporal_store(w0, reinterpret_cast<v2i*>(o));
            __builtin_nontemporal_store(w1, reinterpret_cast<v2i*>(o) + 1);
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (j0 + c < W) o[c] = v[c];
        }
        lp += lstep, k += kstep;
        if (k >= R) k -= R, ++lp;
    }
}

// The waypoint cells (the reference's returned waypoints as raster cells, solver.py:49,
// main.py:186-190) of the sorted forms that do not write them in their output launch (K2g):
// cells[path][j] = iy nx + ix (-1 off the raster) by the evaluations' own point and cell
// arithmetic, workgroups of 64 consecutive paths (cells_rows) looping over the path blocks.
// (Written by the evaluation's lanes through LDS instead, the 21-cell runs of scattered items
// cost K2h ~120 us of partial-line writes per cfg3 step: 402 MB of WRITE_SIZE for 164 MB of
// cells, profiles/r04/final2/cells.)
template <bool ULDS>  // the unit-arc rows staged in LDS (D N <= 1024) or read from global
__global__ __launch_bounds__(256) void k_cells(KParams p, KGrp kg) {
    constexpr int kUtabLds = 1024;  // (16 KiB)
    __shared__ double4 s_cv[64];
    __shared__ int4 s_e[64];
    __shared__ double2 s_u[ULDS ? kUtabLds : 1];
    const int t = threadIdx.x;
    const double2* __restrict__ gu = reinterpret_cast<const double2*>(kg.utab);
    if (ULDS)
        for (int k = t; k < kg.D * p.N; k += 256) s_u[k] = gu[k];
    const int64_t nblk = ((int64_t)kg.P + 63) / 64;
    // (a grid smaller than nblk loops over the blocks: the side-stream launch's share of CUs)
    for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const int64_t path0 = blk * 64;
        const int np = (int)min((int64_t)64, (int64_t)kg.P - path0);
        cells_rows(p, kg, path0, np, s_cv, s_e, ULDS ? s_u : gu, t, 256);
    }
}

// outputs of every path (block = 64 pairs x D, k_g_final's layout): the geometry terms from
// the pair's scale and the displacement's unit sums (oracle sim_geo), cost = (N+1) L + the
// Phi / N partials in group order, and the main.py:175-180 selection
template <int NR>  // slots per path held in registers (0: a loop for long paths)
__global__ __launch_bounds__(1024) void k_h_final(KParams p, KGrp kg, KOut out,
                                                  int32_t* __restrict__ best_f,
                                                  int32_t* __restrict__ best_l) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int D = kg.D, t = threadIdx.x;
    double* s_cost = smem;
    double* s_len = smem + 64 * D;
    const int64_t q0 = (int64_t)blockIdx.x * 64;
    const int qi = t / D, di = t - qi * D;
    const bool bad = *kg.err != 0;  // an inconsistent sort (k_g_scatter / k_v_hist)
    const HSlot* slot = reinterpret_cast<const HSlot*>(kg.slot);
    if (q0 + qi < kg.n_pairs) {
        const int64_t gp = (q0 + qi) * D + di;
        HSlot g[NR > 0 ? NR : 1];
        if (NR > 0) {
#pragma unroll
            for (int s = 0; s < NR; ++s) g[s] = slot[(int64_t)min(s, kg.nseg - 1) * kg.P + gp];
        }
        const double4 pr = reinterpret_cast<const double4*>(kg.pairs)[q0 + qi];
        const UGeo u = kg.ugeo[di];
        // sim_geo (oracle): h = |v| / 2, h^2 = |v|^2 / 4
        const double vx = pr.x - pr.z, vy = pr.y - pr.w;
        const double sv = vx * vx + vy * vy;
        const double h = sqrt(sv) * 0.5, h2 = sv * 0.25;
        const bool ls = p.length_smooth != 0;
        double L;
        if (p.quirk_length) {
            const double ax = p.anchor_mode ? p.anchor_x : pr.x;
            const double ay = p.anchor_mode ? p.anchor_y : pr.y;
            const double dx = pr.x - ax, dy = pr.y - ay;
            const double n = sqrt(dx * dx + dy * dy);
            L = (ls ? n * n : n) + (ls ? h2 * u.s2n : h * u.s1n);
        } else {
            L = ls ? h2 * u.s2a : h * u.s1a;
        }
        const double len = h * u.s1a;
        const double ksum = (h > 0.0 && h < INFINITY) ? h * u.e12 + u.e3 : 0.0;
        double nsum = 0.0, hmax = -INFINITY;
        int32_t nh = 0, off = 0;
        double cost = (double)(p.N + 1) * L;
        if (NR > 0) {
#pragma unroll
            for (int s = 0; s < NR; ++s) {
                if (s >= kg.nseg) break;
                cost = cost + g[s].cost;
                nsum = nsum + g[s].psi;
                hmax = fmax(hmax, (double)g[s].hmax);
                nh += (int32_t)(g[s].cnt & 255u);
                off += (int32_t)((g[s].cnt >> 8) & 255u);
            }
        } else {
            for (int s = 0; s < kg.nseg; ++s) {
                const HSlot gs = slot[(int64_t)s * kg.P + gp];
                cost = cost + gs.cost;
                nsum = nsum + gs.psi;
                hmax = fmax(hmax, (double)gs.hmax);
                nh += (int32_t)(gs.cnt & 255u);
                off += (int32_t)((gs.cnt >> 8) & 255u);
            }
        }
        put_outputs(out, gp, bad, cost, L, len, ksum, nsum, p.altitude - hmax, nh, off, 0);
        s_cost[di * 64 + qi] = cost;
        s_len[di * 64 + qi] = len;
    }
    __syncthreads();
    put_selection(kg, bad, q0, t, s_cost, s_len, best_f, best_l);
}

// ---- K4h: the volume (config 5) in K2h's form -------------------------------------------------
// The packed volume (uam_volume_pack; layout: VpkDims).  Planes in K2h's 4 x 8-column blocks,
// one per layer (layer-major), all at one index i4: r4 {risk}, e8 {risk, |psi| | nfz << 31} and
// v16, the whole voxel {risk, psi_nfz, terrain, flags} (the column's terrain and flags beside
// the layer's pair); t4 the column terrain (one layer, the same column index).  A header
// (staged in LDS) holds a 2-bit code per 8 x 8-column block -- 0: every voxel of its columns has
// risk == +-0, psi == +-0 and no no-fly flag (nothing to read but the terrain); 1: psi == +-0 and
// no flag (r4); 2: no psi below zero (e8); 3: v16 -- then the column terrain's bounds (the
// raster's scheme: u16 codes per bound block of columns, float2 {base, step} per 4 x 4 bound
// blocks).  The (path, group) items are sorted on the altitude band and the Hilbert tile of the
// middle waypoint (band-major, so the items an XCD runs together share a band's lines),
// evaluated with K2h's grouped partial sums, and the output launch adds the similarity-form
// geometry.  Definition: oracle orc_eval_generated_h, mode 2.

struct alignas(16) VSlot {  // 32 B per (path, group)
    double cost;   // risk / N of the group's waypoints, from +0.0 in waypoint order
    double psi;    // psi_nfz likewise
    double cm;     // min over the group's waypoints of z_j - terrain (+inf: none)
    uint32_t cnt;  // nfz hits | off-volume << 8 | below-terrain << 16
    uint32_t pad;
};

struct KVol4 {
    int32_t nx, ny, nz;
    double x0, y_top, z0, dz, inv_dx, inv_dy, inv_dz;
    int32_t zshift, nbands;
    const uint32_t* __restrict__ hdr;   // codes | bounds | superblocks
    int32_t hwords, cnbx, bnd_off, sbt_off, bshift, bnbx, sbnbx;
    int32_t nb8, lnby4;
    uint32_t layer;                     // i4 entries per layer (lnby4 nb8 32)
    // the planes from the packed base by 32-bit byte offsets (o4: r4, o8: e8, o16: v16, ot4:
    // t4); null when the copy is 4 GiB or larger or a layer holds 2^24 entries (K4h stands aside)
    const char* __restrict__ pk;
    uint32_t o4, o8, o16, ot4;
    // the terrain-in-entry form's plane q8 {risk, column terrain} in 4 x 4-column blocks per
    // layer (nb4 blocks a row, layer44 entries a layer) at byte offset oq8
    uint32_t oq8, layer44;
    int32_t nb4;
    // v16 in 4 x 2-column blocks per layer (8 entries, one 128-B line): nbx4 blocks a row,
    // layer42 entries a layer
    uint32_t layer42;
    int32_t nbx4;
};

constexpr int VPK_CSHIFT = 3;           // code blocks of 8 x 8 columns
constexpr int VPK_HDR_LDS = 64 * 1024;  // the header in LDS up to this

// the column (ix, iy)'s index in the 4 x 8-column blocks (t4; i4 = it + iz layer)
__device__ __forceinline__ uint32_t vt4_index(const KVol4& v, int32_t ix, int32_t iy) {
    return ((__umul24((uint32_t)(iy >> 2), (uint32_t)v.nb8) + (uint32_t)(ix >> 3)) << 5) |
           (((uint32_t)iy & 3u) << 3) | ((uint32_t)ix & 7u);
}

// v16's in-layer index of column (ix, iy): 4 x 2-column blocks (8 entries of 16 B, one line)
__device__ __forceinline__ uint32_t vv16_index(const KVol4& v, int32_t ix, int32_t iy) {
    return ((__umul24((uint32_t)(iy >> 1), (uint32_t)v.nbx4) + (uint32_t)(ix >> 2)) << 3) |
           (((uint32_t)iy & 1u) << 2) | ((uint32_t)ix & 3u);
}

// q8's in-layer index of column (ix, iy): 4 x 4-column blocks (16 entries of 8 B, one line)
__device__ __forceinline__ uint32_t vq8_index(const KVol4& v, int32_t ix, int32_t iy) {
    return ((__umul24((uint32_t)(iy >> 2), (uint32_t)v.nb4) + (uint32_t)(ix >> 2)) << 4) |
           (((uint32_t)iy & 3u) << 2) | ((uint32_t)ix & 3u);
}

// the layer planes r4, e8, v16 and q8: one thread per i4 entry (r4 / e8 at i4, v16 and q8 at
// their own block indices), which writes all four (padding: zero)
__global__ __launch_bounds__(256) void k_volume_pack_planes(const uint2* __restrict__ vox,
                                                            const uint2* __restrict__ col,
                                                            KVol4 v, uint32_t* __restrict__ r4,
                                                            uint2* __restrict__ e8,
                                                            uint4* __restrict__ v16,
                                                            uint2* __restrict__ q8) {
    const int64_t total = (int64_t)v.nz * v.layer;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t w = (int32_t)(i & 31);
        const int64_t blk = i >> 5;
        const int32_t bx = (int32_t)(blk % v.nb8);
        const int64_t r = blk / v.nb8;
        const int32_t by = (int32_t)(r % v.lnby4), iz = (int32_t)(r / v.lnby4);
        const int32_t ix = bx * 8 + (w & 7), iy = by * 4 + (w >> 3);
        uint2 a = make_uint2(0u, 0u), cl = make_uint2(0u, 0u);
        if (ix < v.nx && iy < v.ny) {
            const int64_t c = (int64_t)iy * v.nx + ix;
            a = vox[c * v.nz + iz];
            cl = col[c];
        }
        r4[i] = a.x;
        e8[i] = make_uint2(a.x, (a.y & 0x7fffffffu) | ((cl.y & UAM_FLAG_NFZ) ? 0x80000000u : 0u));
        if (ix < v.nbx4 * 4 && iy < ((v.ny + 1) >> 1) * 2)  // (v16's padded extent)
            v16[(int64_t)iz * v.layer42 + vv16_index(v, ix, iy)] = make_uint4(a.x, a.y, cl.x, cl.y);
        if (ix < v.nb4 * 4 && iy < v.lnby4 * 4)  // (q8 is narrower: nb4 4-column blocks)
            q8[(int64_t)iz * v.layer44 + vq8_index(v, ix, iy)] = make_uint2(a.x, cl.x);
    }
}

// the column terrain plane (one thread per entry; padding: zero)
__global__ __launch_bounds__(256) void k_volume_pack_t4(const uint2* __restrict__ col, KVol4 v,
                                                        float* __restrict__ t4) {
    const int64_t total = (int64_t)v.lnby4 * v.nb8 * 32;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int32_t w = (int32_t)(i & 31);
    const int64_t blk = i >> 5;
    const int32_t bx = (int32_t)(blk % v.nb8), by = (int32_t)(blk / v.nb8);
    const int32_t ix = bx * 8 + (w & 7), iy = by * 4 + (w >> 3);
    t4[i] = (ix < v.nx && iy < v.ny) ? __uint_as_float(col[(int64_t)iy * v.nx + ix].x) : 0.0f;
}

// the code map: one thread per 32-bit word (16 blocks of 8 x 8 columns)
__global__ __launch_bounds__(256) void k_volume_codes(const uint2* __restrict__ vox,
                                                      const uint2* __restrict__ col, int nx,
                                                      int ny, int nz, int cnbx, int nblocks,
                                                      int cwords, uint32_t* __restrict__ cmap) {
    const int wd = blockIdx.x * blockDim.x + threadIdx.x;
    if (wd >= cwords) return;
    uint32_t word = 0;
    for (int k = 0; k < 16; ++k) {
        const int b = wd * 16 + k;
        if (b >= nblocks) break;
        const int by = b / cnbx, bx = b - by * cnbx;
        bool need = false, neg = false, nz_r = false;
        for (int y = by << VPK_CSHIFT; y < min(ny, (by + 1) << VPK_CSHIFT); ++y)
            for (int x = bx << VPK_CSHIFT; x < min(nx, (bx + 1) << VPK_CSHIFT); ++x) {
                const int64_t c = (int64_t)y * nx + x;
                if (col[c].y & UAM_FLAG_NFZ) need = true;
                for (int iz = 0; iz < nz; ++iz) {  // every layer's own psi and risk
                    const uint2 a = vox[c * nz + iz];
                    if (a.y & 0x7fffffffu) need = true;
                    if ((a.y >> 31) && a.y != 0x80000000u) neg = true;
                    if (a.x & 0x7fffffffu) nz_r = true;
                }
            }
        const uint32_t code = need ? (neg ? 3u : 2u) : nz_r ? 1u : 0u;
        word |= code << (2 * k);
    }
    cmap[wd] = word;
}

// the altitude of waypoint j (uam_eval_generated3d: z0 + (zf - z0) (j / (N+1)))
__device__ __forceinline__ double vz_at(double za, double zb, double jw) {
    return za + (zb - za) * jw;
}

// the voxel of a generated point (false outside the volume or NaN, with (0, 0, 0) then: valid
// header and plane indices)
__device__ __forceinline__ bool vol_voxel(const KVol4& vs, double x0, double x1, double z,
                                          int32_t& ix, int32_t& iy, int32_t& iz) {
    const double tx = (x0 - vs.x0) * vs.inv_dx, ty = (vs.y_top - x1) * vs.inv_dy;
    const double tz = (z - vs.z0) * vs.inv_dz;
    const bool in = (tx >= 0.0) & (tx < (double)vs.nx) & (ty >= 0.0) & (ty < (double)vs.ny) &
                    (tz >= 0.0) & (tz < (double)vs.nz);
    ix = in ? (int32_t)tx : 0;
    iy = in ? (int32_t)ty : 0;
    iz = in ? (int32_t)tz : 0;
    return in;
}

// K4h: a path's clearance seed (k_v_eval's E and Ub): the exact clearance z - T (T the column's
// terrain, t4) of the in-volume sampled waypoint with the smallest z - lb, over j = 0, s, 2s,
// ... (s = kg.lb_stride) and j = W - 1, at their own voxels and altitudes by the evaluation's
// operations (+inf: none).  It is an exact clearance of the path, so at least the path's
// minimum M.  hdr / u: the packed header and the unit-arc table (LDS copies when staged).
__device__ __forceinline__ double v_path_seed(const KParams& p, const KVol4& vs, const KGrp& kg,
                                             int32_t path, const uint32_t* __restrict__ hdr,
                                             const double2* __restrict__ utab) {
    const int32_t q = (int32_t)div_magic((uint32_t)path, kg.m_d, kg.sh_d), d = path - q * kg.D;
    const double* pr = kg.pairs + (int64_t)q * 6;
    const double ax = pr[0], ay = pr[1], za = pr[2], bx = pr[3], by = pr[4], zb = pr[5];
    const double2* u = utab + d * p.N - 1;
    const int W = kg.W;
    constexpr uint32_t NONE = 0xffffffffu;
    double Ub = INFINITY, zbest = 0.0;
    uint32_t best = NONE;  // the t4 index of the sample holding Ub
    auto take = [&](double x0, double x1, double z) {
        int32_t ix, iy, iz;
        const bool in = vol_voxel(vs, x0, x1, z, ix, iy, iz);
        const uint32_t bx2 = (uint32_t)(ix >> vs.bshift), by2 = (uint32_t)(iy >> vs.bshift);
        const uint32_t e = reinterpret_cast<const uint16_t*>(hdr + vs.bnd_off)[by2 * vs.bnbx + bx2];
        const float2 sb =
            reinterpret_cast<const float2*>(hdr + vs.sbt_off)[(by2 >> 2) * vs.sbnbx + (bx2 >> 2)];
        float ub, lb;
        pk_bound_decode(e, sb, ub, lb);
        const double v = z - (double)lb;
        const bool dn = in && v < Ub;  // (a NaN bound: no)
        Ub = dn ? v : Ub;
        zbest = dn ? z : zbest;
        best = dn ? vt4_index(vs, ix, iy) : best;
    };
    take(ax, ay, vz_at(za, zb, 0.0 / (double)(W - 1)));
    take(bx, by, vz_at(za, zb, (double)(W - 1) / (double)(W - 1)));
    // four samples at a time, every load of the four issued together (a sample past the last
    // interior waypoint repeats it)
    constexpr int K = 4;
    for (int j0 = kg.lb_stride; j0 < W - 1; j0 += K * kg.lb_stride) {
        double2 uu[K];
        int jj[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            jj[k] = min(j0 + k * kg.lb_stride, W - 2);
            uu[k] = u[jj[k]];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double x0, x1;
            arc_point(ax, ay, bx, by, uu[k].x, uu[k].y, x0, x1);
            take(x0, x1, vz_at(za, zb, (double)jj[k] / (double)(W - 1)));
        }
    }
    return best == NONE ? INFINITY
                        : zbest - (double)reinterpret_cast<const float*>(vs.pk + vs.ot4)[best];
}

// sort, launch 1 (K4h): keys on (altitude band, tile) of each item's middle waypoint
__global__ __launch_bounds__(1024) void k_v_hist(KParams p, KVol4 vs, KGrp kg) {
    __shared__ __attribute__((aligned(16))) int32_t h[G_BINS_MAX];
    __shared__ uint16_t tk[1 << (2 * G_TBITS_MAX)];
    // with kg.seed_lds: the packed header and the unit-arc table staged for the seeds
    extern __shared__ __attribute__((aligned(16))) uint32_t s_vhist_dyn[];
    const int t = threadIdx.x, b = blockIdx.x;
    if (b == 0 && t == 0) *kg.err = 0;
    for (int k = t; k < kg.bins; k += 1024) h[k] = 0;
    for (int k = t; k < (1 << (2 * kg.tbits)); k += 1024) tk[k] = kg.tkey[k];
    const uint32_t* s_hdr = vs.hdr;
    const double2* s_ut = reinterpret_cast<const double2*>(kg.utab);
    if (kg.ubp && kg.seed_lds) {
        uint4* dh = reinterpret_cast<uint4*>(s_vhist_dyn);
        const uint4* gh = reinterpret_cast<const uint4*>(vs.hdr);
        for (int k = t; k < (vs.hwords >> 2); k += 1024) dh[k] = gh[k];
        double2* du = reinterpret_cast<double2*>(s_vhist_dyn + vs.hwords);
        for (int k = t; k < kg.D * p.N; k += 1024) du[k] = s_ut[k];
        s_hdr = s_vhist_dyn;
        s_ut = du;
    }
    __syncthreads();
    const int64_t lo = ((int64_t)kg.P * b / G_NBK) * kg.nseg;
    const int64_t hi = ((int64_t)kg.P * (b + 1) / G_NBK) * kg.nseg;
    const int N = p.N, W = kg.W;
    const int tiles = 1 << (2 * kg.tbits);
    const double inv_w1 = 1.0 / (double)(W - 1);
    // U items per thread with all their loads issued first (k_g_hist's batching)
    constexpr int U = 4;
    for (int64_t i0 = lo + t; i0 < hi; i0 += 1024 * U) {
        double pr[U][6];
        double2 u[U];
        int jm[U], sg[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int32_t i = (int32_t)min(i0 + k * 1024, hi - 1);
            const int32_t path = (int32_t)div_magic((uint32_t)i, kg.m_nseg, kg.sh_nseg);
            sg[k] = (int)(i - (int64_t)path * kg.nseg);
            const int32_t q = (int32_t)div_magic((uint32_t)path, kg.m_d, kg.sh_d);
            const int32_t d = path - q * kg.D;
            const int j0 = sg[k] * kg.G, j1 = min(j0 + kg.G, W);
            jm[k] = (j0 + j1 - 1) >> 1;
            const double2* pp = reinterpret_cast<const double2*>(kg.pairs + (int64_t)q * 6);
            const double2 a = pp[0], b2 = pp[1], c = pp[2];
            pr[k][0] = a.x, pr[k][1] = a.y, pr[k][2] = b2.x, pr[k][3] = b2.y, pr[k][4] = c.x,
            pr[k][5] = c.y;
            u[k] = reinterpret_cast<const double2*>(kg.utab)[d * N + min(max(jm[k] - 1, 0), N - 1)];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int64_t i = i0 + k * 1024;
            if (i >= hi) break;
            double x0, x1;
            if (jm[k] == 0) {
                x0 = pr[k][0], x1 = pr[k][1];
            } else if (jm[k] == W - 1) {
                x0 = pr[k][3], x1 = pr[k][4];
            } else {
                arc_point(pr[k][0], pr[k][1], pr[k][3], pr[k][4], u[k].x, u[k].y, x0, x1);
            }
            // (the key only orders the items: j / (W-1) by a reciprocal is exact enough)
            const double z = vz_at(pr[k][2], pr[k][5], (double)jm[k] * inv_w1);
            const double tx = (x0 - vs.x0) * vs.inv_dx, ty = (vs.y_top - x1) * vs.inv_dy;
            const double tz = (z - vs.z0) * vs.inv_dz;
            uint32_t key = kg.bins - 1;
            if ((tx >= 0.0) && (tx < (double)vs.nx) && (ty >= 0.0) && (ty < (double)vs.ny) &&
                (tz >= 0.0) && (tz < (double)vs.nz)) {
                const uint32_t cx = (uint32_t)tx >> kg.tshift, cy = (uint32_t)ty >> kg.tshift;
                key = ((uint32_t)tz >> vs.zshift) * tiles + tk[(cy << kg.tbits) | cx];
                if (sg[k] == kg.nseg - 1) key += kg.last_bin;
            }
            kg.key[i] = (uint16_t)key;
            atomicAdd(&h[key], 1);
        }
    }
    if (kg.ubp) {  // the partition's paths' clearance seeds, one thread per path
        const int64_t plo = (int64_t)kg.P * b / G_NBK, phi = (int64_t)kg.P * (b + 1) / G_NBK;
        for (int64_t pth = plo + t; pth < phi; pth += 1024)
            kg.ubp[pth] = v_path_seed(p, vs, kg, (int32_t)pth, s_hdr, s_ut);
    }
    __syncthreads();
    for (int k = t; k < kg.bins; k += 1024) kg.cnt[(int64_t)k * G_NBK + b] = h[k];
}

// every (path, group) item in sorted order (h_item's phases): the CH waypoints' voxels (x, y by
// the arc formula or the pair's end points, z on the linear climb), the header reads, then per
// slot the decisions and two unconditional loads -- the code's entry (r4 / e8 / v16, the dummy
// line in code 0 or outside the volume) and the terrain (the first t4 word unless fetched) -- by
// 32-bit offsets from the packed base; then the branch-free consume.
//
// The terrain by bounds (as K2h's; the outputs are exactly the per-waypoint ones).  Waypoint j
// in the volume has lb_j <= T_j <= ub_j (the column grid's bounds) and
//   below_j = zc_j < T_j (zc_j its layer centre): decided when zc_j < lb_j (1) or zc_j >= ub_j
//       (0), else its terrain is fetched;
//   c_j = z_j - T_j, whose path minimum is min_clearance: z_j - ub_j <= c_j <= z_j - lb_j (the
//       float64 subtraction is monotone).  The item keeps Ub, an upper bound of the path minimum
//       M (the path's seed, then its own waypoints' z - lb), and E, the minimum of exact c_j of
//       the path: the seed (v_path_seed: the exact clearance of the sampled waypoint with the
//       smallest z - lb, formed once per path by the histogram launch) and those it takes
//       (fetched, v16's, one-value blocks); it fetches w iff it is undecided or
//       !(z_w - ub_w >= E) && !(z_w - ub_w > Ub).  If w* holds M and is not taken: z - ub >= E
//       gives M >= E >= M, and z - ub > Ub >= M is impossible.  NaN bounds (no bound) always
//       fetch.
template <int CH, bool TE>  // TE: the terrain in the entry (UAM_OPT_K2H_TERRAIN 1)
__global__ __launch_bounds__(256, CH >= 11 ? 2 : CH >= 7 ? 3 : 4) void k_v_eval(KParams p, KVol4 vs,
                                                                              KGrp kg) {
    PK_CODES_CHECK(CH);
    // unit-arc rows + padding, then j / (W-1) (+ padding), then the header
    extern __shared__ __attribute__((aligned(16))) double2 s_u[];
    const int N = p.N, W = kg.W;
    const int nu = kg.D * N, npad = kg.G + 16;  // a lane's slots reach j <= W + G + CH - 3
    double* s_jw = reinterpret_cast<double*>(s_u + nu + npad);
    const int njw = W + npad;
    uint32_t* s_hdr = reinterpret_cast<uint32_t*>(s_jw + ((njw + 1) & ~1));
    // the item's order entry, pair and path bound before the staging (their round trips
    // overlap it)
    const int64_t pos = xcd_chunk(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
    const bool live = pos < kg.n_items;
    const int32_t item = live ? kg.order[pos] : 0;
    const int32_t path = (int32_t)div_magic((uint32_t)item, kg.m_nseg, kg.sh_nseg);
    const int s = item - path * kg.nseg;
    const int32_t q = (int32_t)div_magic((uint32_t)path, kg.m_d, kg.sh_d), d = path - q * kg.D;
    const double* prp = kg.pairs + (int64_t)q * 6;
    const double2 pa = *reinterpret_cast<const double2*>(prp);
    const double2 pb = *reinterpret_cast<const double2*>(prp + 2);
    const double2 pc = *reinterpret_cast<const double2*>(prp + 4);
    const double seed = kg.ubp ? kg.ubp[path] : INFINITY;  // an exact clearance of the path
    double Ub = seed;
    for (int i = threadIdx.x; i < nu + npad; i += 256)
        s_u[i] = i < nu ? reinterpret_cast<const double2*>(kg.utab)[i] : make_double2(0.0, 0.0);
    for (int j = threadIdx.x; j < njw; j += 256)
        s_jw[j] = j < W ? (double)j / (double)(W - 1) : 0.0;
    {
        const uint4* src = reinterpret_cast<const uint4*>(vs.hdr);
        uint4* dst = reinterpret_cast<uint4*>(s_hdr);
        const int hw = TE ? vs.bnd_off : vs.hwords;  // (TE: the code map alone)
        for (int i = threadIdx.x; i < (hw >> 2); i += 256) dst[i] = src[i];
    }
    __syncthreads();
    const double ax = pa.x, ay = pa.y, za = pb.x, bx = pb.y, by = pc.x, zb = pc.y;
    const double2* urow = s_u + d * N - 1;  // waypoint j's unit vector: urow[j]
    const int j0 = s * kg.G, j1 = live ? min(j0 + kg.G, W) : j0;
    int nch = (j1 - j0 + CH - 1) / CH;  // the wave's most: a wave-uniform loop
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nch = max(nch, __shfl_xor(nch, o));
    const double vx = ax - bx, vy = ay - by;
    const double cx = (bx + ax) * 0.5, cy = (by + ay) * 0.5;
    const double dN = (double)N, yN = kg.inv_n;
    auto over_n = [&](double a) {  // (K4h: N <= 4096)
        const double q0 = a * yN;
        const double q1 = fma(fma(-q0, dN, a), yN, q0);
        return __builtin_isinf(a) ? q0 : q1;
    };
    // the layer centre of layer iz (the below-terrain test)
    auto zc_of = [&](int32_t iz) { return vs.z0 + ((double)iz + 0.5) * vs.dz; };
    // the end points' voxels, formed once
    int32_t ixF, iyF, izF, ixL, iyL, izL;
    const double zF = vz_at(za, zb, s_jw[0]), zL = vz_at(za, zb, s_jw[W - 1]);
    const bool inF = vol_voxel(vs, ax, ay, zF, ixF, iyF, izF);
    const bool inL = vol_voxel(vs, bx, by, zL, ixL, iyL, izL);
    const uint16_t* const bnd = reinterpret_cast<const uint16_t*>(s_hdr + vs.bnd_off);
    const float2* const sbt = reinterpret_cast<const float2*>(s_hdr + vs.sbt_off);
    const char* const pk = vs.pk;
    const uint32_t o4 = __builtin_amdgcn_readfirstlane(vs.o4);
    const uint32_t o8 = __builtin_amdgcn_readfirstlane(vs.o8);
    const uint32_t o16 = __builtin_amdgcn_readfirstlane(vs.o16);
    const uint32_t ot4 = __builtin_amdgcn_readfirstlane(vs.ot4);
    const uint32_t layer = __builtin_amdgcn_readfirstlane(vs.layer);
    const uint32_t oq8 = __builtin_amdgcn_readfirstlane(vs.oq8);
    const uint32_t layer44 = __builtin_amdgcn_readfirstlane(vs.layer44);
    const uint32_t layer42 = __builtin_amdgcn_readfirstlane(vs.layer42);
    double gc = 0.0, gn = 0.0, E = seed;
    uint32_t nh = 0, off = 0, bel = 0;
    // one chunk ahead, as h_item: iteration c issues chunk c + 1 (B arrays) and consumes chunk
    // c (A arrays)
    // (the slot's layer rides in its kind word's high bits; consume recomputes its altitude)
    uint4 rA[CH];
    float tvA[CH];
    uint32_t kcA[CH], vinA = 0, tkA = 0, bvA = 0;
    int nvA = 0, jcA = 0;
    constexpr bool ahead = false;  // (h_item's)
    for (int c = ahead ? -1 : 0; c < nch; ++c) {  // (nch wave-uniform)
        const int ci = ahead ? c + 1 : c;  // the chunk issued by this iteration
        uint4 rB[CH];
        float tvB[CH];
        uint32_t kcB[CH], vinB = 0, tkB = 0, bvB = 0;
        int nvB = 0;
        const int jc = j0 + ci * CH;
        if (ci < nch) {
            double zB[CH];
            int32_t izB[CH];
            const double2* uc = urow + jc;
            // phase 1: the voxels
            int32_t ix[CH], iy[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int j = jc + t;
                const double2 u = uc[t];
                const double z = vz_at(za, zb, s_jw[j]);
                int32_t x, y, zz;
                bool in = vol_voxel(vs, cx + 0.5 * (vx * u.x - vy * u.y),
                                    cy + 0.5 * (vy * u.x + vx * u.y), z, x, y, zz);
                if (t == 0) {  // (j == 0 only in a chunk's first slot)
                    const bool f = jc == 0;
                    x = f ? ixF : x;
                    y = f ? iyF : y;
                    zz = f ? izF : zz;
                    in = f ? inF : in;
                }
                const bool l = j == W - 1;
                ix[t] = l ? ixL : x;
                iy[t] = l ? iyL : y;
                izB[t] = l ? izL : zz;
                in = l ? inL : in;
                zB[t] = z;  // (the end points' z by the same formula)
                vinB |= (uint32_t)(in & (j < j1)) << t;
            }
            // phase 2: the header reads (column (0, 0) outside the volume: valid reads)
            uint32_t cw[CH], be[CH];
            float2 sb[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const uint32_t b = __umul24((uint32_t)(iy[t] >> VPK_CSHIFT), (uint32_t)vs.cnbx) +
                                   (uint32_t)(ix[t] >> VPK_CSHIFT);
                cw[t] = s_hdr[b >> 4] >> ((b & 15u) * 2u);
                if constexpr (!TE) {
                    const uint32_t bx2 = (uint32_t)(ix[t] >> vs.bshift);
                    const uint32_t by2 = (uint32_t)(iy[t] >> vs.bshift);
                    be[t] = bnd[__umul24(by2, (uint32_t)vs.bnbx) + bx2];
                    sb[t] = sbt[__umul24(by2 >> 2, (uint32_t)vs.sbnbx) + (bx2 >> 2)];
                }
            }
            // phase 3: the decisions and the loads
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const bool vin = (vinB >> t) & 1u;
                const uint32_t code = cw[t] & (vin ? 3u : 0u);
                if constexpr (TE) {
                    // codes 0 / 1: the 8-B {risk, column terrain} entry (q8); 2 / 3: v16
                    const bool rec = code & 2u;
                    const uint32_t iz = (uint32_t)izB[t];
                    const uint32_t a16 = vv16_index(vs, ix[t], iy[t]) + __umul24(iz, layer42);
                    const uint32_t ab = (vq8_index(vs, ix[t], iy[t]) + __umul24(iz, layer44)) << 3;
                    const uint32_t voff = rec ? o16 + (a16 << 4) : oq8 + (ab & ~15u);
                    kcB[t] = code | (rec ? 0u : (ab & 8u)) | (iz << 8);
                    rB[t] = *reinterpret_cast<const uint4*>(pk + voff);
                    continue;
                }
                float ub, lb;
                pk_bound_decode(be[t], sb[t], ub, lb);
                const double z = zB[t], zc = zc_of(izB[t]);
                const bool k1 = zc < (double)lb, k0 = zc >= (double)ub;
                // a one-value block: the exact term; every in-volume waypoint's z - lb bounds M
                E = (vin & (lb == ub)) ? fmin(E, z - (double)ub) : E;
                Ub = vin ? fmin(Ub, z - (double)lb) : Ub;
                const double clo = z - (double)ub;
                const bool fetch =
                    vin & (code != 3u) & (!(k1 | k0) | (!(clo >= E) & !(clo > Ub)));
                const uint32_t it = vt4_index(vs, ix[t], iy[t]);
                const uint32_t a4 = it + __umul24((uint32_t)izB[t], layer);
                // codes 1 / 2: the r4 / e8 entry's aligned 16 B and word; 3: v16 (its own index)
                const uint32_t ab = a4 << (code + 1u);
                const uint32_t a16 = vv16_index(vs, ix[t], iy[t]) + __umul24((uint32_t)izB[t], layer42);
                const uint32_t voff = code == 3u ? o16 + (a16 << 4)
                                                 : (code == 2u ? o8 : o4) + (code ? (ab & ~15u) : 0u);
                kcB[t] = code | (code == 3u ? 0u : (ab & 12u)) | ((uint32_t)izB[t] << 8);
                rB[t] = *reinterpret_cast<const uint4*>(pk + voff);
                tvB[t] = *reinterpret_cast<const float*>(pk + (ot4 + (fetch ? it * 4u : 0u)));
                tkB |= (uint32_t)fetch << t;
                bvB |= (uint32_t)k1 << t;
            }
            nvB = max(0, min(CH, j1 - jc));  // slots past the group's end: no waypoint
        }
        if (!ahead) {
#pragma unroll
            for (int t = 0; t < CH; ++t) rA[t] = rB[t], tvA[t] = tvB[t], kcA[t] = kcB[t];
            vinA = vinB, tkA = tkB, bvA = bvB, nvA = nvB, jcA = jc;
        }
        if (c >= 0) {
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const bool vl = t < nvA, in = (vinA >> t) & 1u;
                if constexpr (TE) {
                    const uint4 r = rA[t];
                    const bool rec = kcA[t] & 2u, s1 = kcA[t] & 8u;
                    const uint32_t lo = s1 ? r.z : r.x, hi = s1 ? r.w : r.y;
                    const uint32_t risk = in ? (rec ? r.x : lo) : 0u;
                    const float ter = __uint_as_float(rec ? r.z : hi);  // (+0 on nodata)
                    nh += (rec && (r.w & UAM_FLAG_NFZ)) ? 1u : 0u;
                    off += (vl && !in) ? 1u : 0u;
                    gc = gc + over_n((double)__uint_as_float(risk));
                    gn = gn + (rec ? (double)__uint_as_float(r.y) : 0.0);
                    const double z = vz_at(za, zb, s_jw[jcA + t]);
                    bel += (in && zc_of((int32_t)(kcA[t] >> 8)) < (double)ter) ? 1u : 0u;
                    E = in ? fmin(E, z - (double)ter) : E;
                    continue;
                }
                uint32_t risk, psi, hit;
                float rter;
                pk_terms_k(rA[t], kcA[t], risk, psi, hit, rter);
                const bool c3 = (kcA[t] & 3u) == 3u;
                gc = gc + over_n((double)__uint_as_float(risk));
                gn = gn + (double)__uint_as_float(psi);
                nh += hit;
                off += (vl && !in) ? 1u : 0u;
                // the exact terrain, where taken: v16's (code 3) or the fetched one
                const bool ex = in & (c3 | ((tkA >> t) & 1u));
                const float ter = c3 ? rter : tvA[t];
                const double z = vz_at(za, zb, s_jw[jcA + t]);
                const uint32_t below =
                    ex ? (zc_of((int32_t)(kcA[t] >> 8)) < (double)ter ? 1u : 0u) : ((bvA >> t) & 1u);
                bel += in ? below : 0u;
                E = ex ? fmin(E, z - (double)ter) : E;
            }
        }
        if (ahead) {
#pragma unroll
            for (int t = 0; t < CH; ++t) rA[t] = rB[t], tvA[t] = tvB[t], kcA[t] = kcB[t];
            vinA = vinB, tkA = tkB, bvA = bvB, nvA = nvB, jcA = jc;
        }
    }
    VSlot o;
    o.cost = gc;
    o.psi = gn;
    o.cm = E;
    o.cnt = nh | (off << 8) | (bel << 16);
    o.pad = 0;
    if (live) reinterpret_cast<VSlot*>(kg.slot)[(int64_t)s * kg.P + path] = o;
}

// outputs of every path (block = 64 pairs x D): the similarity-form geometry (oracle sim_geo on
// the pair's x/y), cost = (N+1) L + the risk / N partials in group order, min clearance, the
// counts, and the main.py:175-180 selection
__global__ __launch_bounds__(1024) void k_v_final(KParams p, KGrp kg, KOut out,
                                                  int32_t* __restrict__ best_f,
                                                  int32_t* __restrict__ best_l) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int D = kg.D, t = threadIdx.x;
    double* s_cost = smem;
    double* s_len = smem + 64 * D;
    const int64_t q0 = (int64_t)blockIdx.x * 64;
    const int qi = t / D, di = t - qi * D;
    const bool bad = *kg.err != 0;  // an inconsistent sort (k_g_scatter / k_v_hist)
    const VSlot* slot = reinterpret_cast<const VSlot*>(kg.slot);
    if (q0 + qi < kg.n_pairs) {
        const int64_t gp = (q0 + qi) * D + di;
        const double* pr = kg.pairs + (q0 + qi) * 6;
        const double x0 = pr[0], y0 = pr[1], xf = pr[3], yf = pr[4];
        const UGeo u = kg.ugeo[di];
        const double vx = x0 - xf, vy = y0 - yf;
        const double sv = vx * vx + vy * vy;
        const double h = sqrt(sv) * 0.5, h2 = sv * 0.25;
        const bool ls = p.length_smooth != 0;
        double L;
        if (p.quirk_length) {
            const double axx = p.anchor_mode ? p.anchor_x : x0;
            const double ayy = p.anchor_mode ? p.anchor_y : y0;
            const double dx = x0 - axx, dy = y0 - ayy;
            const double n = sqrt(dx * dx + dy * dy);
            L = (ls ? n * n : n) + (ls ? h2 * u.s2n : h * u.s1n);
        } else {
            L = ls ? h2 * u.s2a : h * u.s1a;
        }
        const double len = h * u.s1a;
        const double ksum = (h > 0.0 && h < INFINITY) ? h * u.e12 + u.e3 : 0.0;
        double cost = (double)(p.N + 1) * L, nsum = 0.0, cm = INFINITY;
        int32_t nh = 0, off = 0, bel = 0;
        for (int s = 0; s < kg.nseg; ++s) {
            const VSlot g = slot[(int64_t)s * kg.P + gp];
            cost = cost + g.cost;
            nsum = nsum + g.psi;
            cm = fmin(cm, g.cm);
            nh += (int32_t)(g.cnt & 255u);
            off += (int32_t)((g.cnt >> 8) & 255u);
            bel += (int32_t)((g.cnt >> 16) & 255u);
        }
        put_outputs(out, gp, bad, cost, L, len, ksum, nsum, cm, nh, off, bel);
        s_cost[di * 64 + qi] = cost;
        s_len[di * 64 + qi] = len;
    }
    __syncthreads();
    put_selection(kg, bad, q0, t, s_cost, s_len, best_f, best_l);
}

}  // namespace

namespace {
void pinned_arena_free(void* a);  // K8 host arena (defined with PinnedArena)
void dev_arena_free(void* a);     // K8 device arena (defined with DevArena)
}  // namespace

struct uam_ctx {
    int device = 0;
    DevIneq* d_ineq = nullptr;
    DevShape* d_shape = nullptr;
    int n_ineq = 0, n_shapes = 0;
    KGeom kg{};
    KParams kp{};
    bool have_geom = false, have_params = false;
    std::vector<DevIneq> h_ineq;
    std::vector<DevShape> h_shape;
    int32_t* d_grid = nullptr;  // shape-grid index (KShapeGrid), rebuilt by uam_set_params
    // kernel timing (uam_kernel_timing): HIP event pairs around the dominant path kernel
    bool ktime_on = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ktime_ev;
    size_t ktime_n = 0;
    double ktime_acc_ms = 0.0;  // folded pairs (uam_kernel_time reports these + the pending)
    int64_t ktime_acc_n = 0;
    int k1_cpl = 2;             // K1 cells (rows) per lane: 1 = single-cell kernel, 2, 4, 8
                                // (UAM_OPT_K1_ROWS)
    hipStream_t s2 = nullptr;   // side stream (K2s: the later segments' sorts beside segment 0)
    hipStream_t s_lo = nullptr; // low-priority side stream (the waypoint cells beside K2h)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    void* pinned = nullptr;     // K8 page-locked host arena (PinnedArena), created on first use
    // uam_load_tiles: two page-locked chunk buffers, each reused once its copy has completed
    char* tring[2] = {nullptr, nullptr};
    size_t tring_bytes = 0;
    hipEvent_t tring_ev[2] = {nullptr, nullptr};
    bool tring_used[2] = {false, false};
    void* devarena = nullptr;   // K8 device scratch arena (DevArena), created on first use
    double* d_tmtab = nullptr;  // K7 reprojection row / column tables (grow-only)
    size_t tmtab_n = 0;
    bool k8_tiled = true;       // K8 tile labelling (UAM_OPT_K8_TILED = 0: cell-parallel merge)
    int k8_nstreams = 4;        // K8 large regions: streams they are spread over
                                // (UAM_OPT_K8_STREAMS)
    bool pair_order = true;     // K2 / K3 / K4: pairs in a spatial order (UAM_OPT_PAIR_ORDER)
    int k3b_seg = 8;            // K3b segment (waypoints sorted together; UAM_OPT_K3B_SEGMENT:
                                // 2/4/6/8/16, 0 = the lane-per-path K3)
    int k3b_cpl = 1;            // K3b points per lane in the evaluation phase
                                // (UAM_OPT_K3B_POINTS_PER_LANE: 1, 2)
    bool k3b_attrs = false;     // K3b dynamic-LDS attributes raised on this context's device
    int64_t wave_max = 16384;   // K2w / K4w for batches of up to this many paths
                                // (UAM_OPT_WAVE_MAX_PATHS; tools/probe_wave.py crossover)
    int k2s_segs = 2;           // K2s segments per path (UAM_OPT_K2S_SEGMENTS: 2..8)
    int64_t k2s_min = 65536;    // K2g / K2s: smallest batch in paths (UAM_OPT_SORTED_MIN_PATHS)
    bool k2s_attrs = false;     // K2s dynamic-LDS attributes raised on this context's device
    bool k2h_attrs = false;     // K2h's dynamic-LDS attributes raised on this context's device
    bool k4h_hist_attr = false;  // k_v_hist's, likewise
    bool k2g_attrs = false;     // K2g dynamic-LDS attributes raised on this context's device
    bool k4h_attrs = false;     // the same for K4h
    void* d_ord = nullptr;      // pair_order scratch (grow-only)
    uint16_t* d_tkey = nullptr; // K2g: sort key of each tile (curve order), for tkey_bits/curve
    int tkey_bits = -1, tkey_curve = -1;
    size_t ord_bytes = 0;
    hipEvent_t ev_ord = nullptr;  // recorded after the last launch that read d_ord: a call on
                                  // another stream waits for it before rewriting the scratch
    bool ord_pending = false;
    hipStream_t ord_stream = nullptr;  // the stream of the last launch that read the scratch
    hipStream_t k8s[7] = {};    // K8 side streams (created on first use)
    void* comm = nullptr;       // RCCL communicator of uam_comm_init / uam_bcast_raster_group
    const char* last_kernel = "";  // uam_last_kernel: the path evaluation the last call ran
    int32_t last_group = 0;     // uam_last_group: waypoint-group length of the last call's sums
    int k2g_group = 21;         // K2g waypoints per group (UAM_OPT_GROUP; 0 = K2s).  cfg3 ms
                                // (profiles/r03/k2g13, tile bits 4, Hilbert, 8 in flight): 14
                                // 0.387, 16 0.405, 18 0.365, 21 0.329, 24 0.356
    int k2g_tbits = 0;          // K2g sort key: 2^tbits x 2^tbits tiles (UAM_OPT_K2G_TILE_BITS;
                                // 0 = tiles of ~256^2 cells: cfg3 (4096^2) Hilbert 4 0.329,
                                // 5 0.343, 6 0.381 ms (k2g13); cfg4 (8192^2) 4 1.062, 5 0.996,
                                // 6 1.043 ms (cfg4_tbits))
    int k2g_lds = 0;            // K2g / K2h / K4h evaluation: dynamic-LDS floor per workgroup,
                                // which caps the workgroups resident per CU
                                // (UAM_OPT_K2G_LDS_FLOOR; K2g cfg3: 45 / 54 / 80 KiB 0.43 / 0.54
                                // / 0.52 ms against 0.39, k2g7; 0 = the launchers' defaults)
    int k2g_curve = 1;          // K2g tile order: 1 Hilbert, 0 Morton (UAM_OPT_K2G_CURVE)
    int k4h_band = 0;           // K4h sort key: layers per altitude band (UAM_OPT_K4H_BAND;
                                // 0 = the fewest giving <= 16 bands)
    int k2h_te = 1;             // K2h: terrain in the entry (UAM_OPT_K2H_TERRAIN)
    int k4h_te = 0;             // K4h: likewise (UAM_OPT_K4H_TERRAIN)
    int k2h_lbs = 16;           // K2h / K4h: the path seed's sample stride (UAM_OPT_K2H_LB_STRIDE;
                                // tools/sim_terrain_bound.py at cfg3: fetches per waypoint 0.17
                                // at 8, 0.15 at 4, 0.37 without the path bound; cfg5 K4h step
                                // 0.392 / 0.385 / 0.382 / 0.382 / 0.383 / 0.392 ms at 4 / 8 / 16
                                // / 32 / 81 / none, profiles/r06/c7: the histogram launch's seeds
                                // 35 -> 30 us at 16, the evaluation unchanged)
    int k2g_sim = 1;            // K2g: the similarity form K2h (UAM_OPT_K2G_SIM; 0 = per-waypoint
                                // geometry, K2g proper; maxratio_smooth always runs K2g)
    int k2g_chunk = 0;          // K2g / K2h / K4h gathers in flight per lane (UAM_OPT_K2G_CHUNK:
                                // 6, 7, 8, 11, 16, 21; 0 = the launchers' defaults)
    int32_t* h_err = nullptr;   // page-locked, device-mapped word the sorted forms' output
    int32_t* d_err = nullptr;   // launches set on a failed sort check (uam_device_status)
    int test_sort_fault = 0;    // UAM_OPT_TEST_SORT_FAULT (tests only)

};

namespace {

int check_ctx(uam_ctx* ctx, bool need_params) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    if (!ctx->have_geom) return fail(UAM_E_STATE, "uam_set_geometry has not been called");
    if (need_params && !ctx->have_params)
        return fail(UAM_E_STATE, "uam_set_params has not been called");
    return UAM_OK;
}

// Kernel timing (uam_kernel_timing): an event pair recorded on the launch stream around the
// dominant path kernel; pairs are pooled and reused after uam_kernel_time / a reset.
// the pending event pairs' times added to the running total (waits for the last of them)
int ktime_fold(uam_ctx* ctx) {
    for (size_t i = 0; i < ctx->ktime_n; ++i) {
        HIP_TRY(hipEventSynchronize(ctx->ktime_ev[i].second));
        float ms = 0.0f;
        HIP_TRY(hipEventElapsedTime(&ms, ctx->ktime_ev[i].first, ctx->ktime_ev[i].second));
        ctx->ktime_acc_ms += ms;
    }
    ctx->ktime_acc_n += (int64_t)ctx->ktime_n;
    ctx->ktime_n = 0;
    return UAM_OK;
}

int ktime_begin(uam_ctx* ctx, hipStream_t s) {
    if (!ctx->ktime_on) return UAM_OK;
    if (ctx->ktime_n >= 4096) {  // fold the pending pairs into the running total (one wait)
        const int st = ktime_fold(ctx);
        if (st) return st;
    }
    if (ctx->ktime_n == ctx->ktime_ev.size()) {
        hipEvent_t a, b;
        HIP_TRY(hipEventCreate(&a));
        if (hipEventCreate(&b) != hipSuccess) {
            (void)hipEventDestroy(a);
            return fail(UAM_E_HIP, "hipEventCreate failed");
        }
        ctx->ktime_ev.emplace_back(a, b);
    }
    HIP_TRY(hipEventRecord(ctx->ktime_ev[ctx->ktime_n].first, s));
    return UAM_OK;
}

int ktime_end(uam_ctx* ctx, hipStream_t s) {
    if (!ctx->ktime_on) return UAM_OK;
    HIP_TRY(hipEventRecord(ctx->ktime_ev[ctx->ktime_n].second, s));
    ++ctx->ktime_n;
    return UAM_OK;
}

// the device-error word (uam_device_status), created on the first sorted call; the output
// launches write it only when the sort check fails, so a good call issues no copy for it
int err_word(uam_ctx* ctx, KGrp* kg) {
    if (!ctx->h_err) {
        HIP_TRY(hipHostMalloc((void**)&ctx->h_err, 64, hipHostMallocMapped));
        *ctx->h_err = 0;
        void* d = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&d, ctx->h_err, 0));
        ctx->d_err = (int32_t*)d;
    }
    kg->herr = ctx->d_err;
    kg->test_fault = ctx->test_sort_fault;
    return UAM_OK;
}

int device_status(uam_ctx* ctx) {
    if (!ctx->h_err || !*(volatile int32_t*)ctx->h_err) return UAM_OK;
    *(volatile int32_t*)ctx->h_err = 0;
    return fail(UAM_E_DEVICE,
                "a sorted evaluation (K2h / K2g / K4h) found its counting sort inconsistent on "
                "the device; that call wrote NaN / -1 to every output of its batch");
}

int make_kraster(const uam_raster_desc* d, KRaster* k) {
    if (!d) return fail(UAM_E_INVALID, "raster mode needs a raster descriptor");
    if (d->nx <= 0 || d->ny <= 0) return fail(UAM_E_INVALID, "raster size %dx%d", d->nx, d->ny);
    if ((int64_t)d->nx * d->ny >= ((int64_t)1 << 31))
        return fail(UAM_E_INVALID, "raster has more than 2^31 cells");
    if (!(d->dx > 0.0) || !(d->dy > 0.0)) return fail(UAM_E_INVALID, "dx, dy must be > 0");
    k->nx = d->nx;
    k->ny = d->ny;
    k->x0 = d->x0;
    k->y_top = d->y_top;
    k->dx = d->dx;
    k->dy = d->dy;
    k->inv_dx = 1.0 / d->dx;
    k->inv_dy = 1.0 / d->dy;
    return UAM_OK;
}

KOut make_kout(const uam_path_outputs* o) {
    KOut k{};
    if (!o) return k;
    k.cost = o->cost;
    k.length_q = o->length_q;
    k.length = o->length;
    k.kin_sum = o->kin_sum;
    k.nfz_sum = o->nfz_sum;
    k.nfz_hits = o->nfz_hits;
    k.min_clearance = o->min_clearance;
    k.offmap = o->offmap;
    k.cells = o->cells;
    k.g_rows = o->g_rows;
    k.below_terrain = o->below_terrain;
    return k;
}

}  // namespace

// error reporting for the host-only translation units (polyproc.cpp)
int uam_fail_(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

extern "C" {

int uam_abi_version(void) { return UAM_ABI_VERSION; }

const char* uam_last_error(void) { return g_last_error.c_str(); }

int uam_device_count(int* n) {
    if (!n) return fail(UAM_E_INVALID, "n is NULL");
    HIP_TRY(hipGetDeviceCount(n));
    return UAM_OK;
}

int uam_ctx_create(int device, uam_ctx** out) {
    if (!out) return fail(UAM_E_INVALID, "out is NULL");
    *out = nullptr;
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device < 0 || device >= n)
        return fail(UAM_E_INVALID, "device %d out of range (%d devices)", device, n);
    uam_ctx* c = new (std::nothrow) uam_ctx();
    if (!c) return fail(UAM_E_NOMEM, "ctx allocation failed");
    c->device = device;
    *out = c;
    return UAM_OK;
}

static void comm_release(uam_ctx* ctx);

void uam_ctx_destroy(uam_ctx* ctx) {
    if (!ctx) return;
    DeviceGuard dg(ctx->device);
    comm_release(ctx);
    if (ctx->d_ineq) (void)hipFree(ctx->d_ineq);
    if (ctx->d_shape) (void)hipFree(ctx->d_shape);
    if (ctx->d_grid) (void)hipFree(ctx->d_grid);
    if (ctx->ev_ord) (void)hipEventSynchronize(ctx->ev_ord);
    if (ctx->d_ord) (void)hipFree(ctx->d_ord);
    if (ctx->d_tkey) (void)hipFree(ctx->d_tkey);
    if (ctx->ev_ord) (void)hipEventDestroy(ctx->ev_ord);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    for (auto& e : ctx->ktime_ev) {
        (void)hipEventSynchronize(e.second);
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    if (ctx->s2) (void)hipStreamDestroy(ctx->s2);
    if (ctx->s_lo) (void)hipStreamDestroy(ctx->s_lo);
    for (hipStream_t k : ctx->k8s)
        if (k) (void)hipStreamDestroy(k);
    if (ctx->pinned) pinned_arena_free(ctx->pinned);
    for (int b = 0; b < 2; ++b) {
        if (ctx->tring_ev[b]) {
            (void)hipEventSynchronize(ctx->tring_ev[b]);
            (void)hipEventDestroy(ctx->tring_ev[b]);
        }
        if (ctx->tring[b]) (void)hipHostFree(ctx->tring[b]);
    }
    if (ctx->devarena) dev_arena_free(ctx->devarena);
    if (ctx->d_tmtab) (void)hipFree(ctx->d_tmtab);
    if (ctx->h_err) (void)hipHostFree(ctx->h_err);
    delete ctx;
}

int uam_set_geometry(uam_ctx* ctx, const uam_geometry* geom) {
    if (!ctx || !geom) return fail(UAM_E_INVALID, "ctx/geom is NULL");
    if (geom->abi_version != UAM_ABI_VERSION)
        return fail(UAM_E_VERSION, "geometry abi_version %u != %d", geom->abi_version,
                    UAM_ABI_VERSION);
    const int ni = geom->n_ineq, ns = geom->n_shapes, nr = geom->n_regions;
    if (ni < 0 || ns < 0 || geom->n_obstacles < 0 || geom->n_obstacles > ns)
        return fail(UAM_E_INVALID, "bad counts n_ineq=%d n_shapes=%d n_obstacles=%d", ni, ns,
                    geom->n_obstacles);
    if (nr < 0 || nr > UAM_MAX_REGIONS)
        return fail(UAM_E_INVALID, "n_regions %d exceeds %d", nr, UAM_MAX_REGIONS);
    if (ns > 0 && (!geom->shape_first || !geom->shape_count || !geom->shape_center))
        return fail(UAM_E_INVALID, "shape arrays are NULL");
    if (ni > 0 && (!geom->ineq_kind || !geom->ineq_par))
        return fail(UAM_E_INVALID, "inequality arrays are NULL");
    if (!geom->region_first) return fail(UAM_E_INVALID, "region_first is NULL");
    if (geom->region_first[0] != geom->n_obstacles || geom->region_first[nr] != ns)
        return fail(UAM_E_INVALID, "region_first must run from n_obstacles to n_shapes");
    for (int r = 0; r < nr; ++r)
        if (geom->region_first[r + 1] < geom->region_first[r])
            return fail(UAM_E_INVALID, "region_first not monotonic at %d", r);
    for (int s = 0; s < ns; ++s)
        if (geom->shape_count[s] < 1 || geom->shape_first[s] < 0 ||
            geom->shape_first[s] + geom->shape_count[s] > ni)
            return fail(UAM_E_INVALID, "shape %d inequality range out of bounds", s);
    for (int i = 0; i < ni; ++i)
        if (geom->ineq_kind[i] < UAM_INEQ_HALFPLANE || geom->ineq_kind[i] > UAM_INEQ_AXIS)
            return fail(UAM_E_INVALID, "inequality %d has unknown kind %d", i,
                        geom->ineq_kind[i]);

    DeviceGuard dg(ctx->device);
    if (!dg.ok) return fail(UAM_E_HIP, "hipSetDevice(%d) failed", ctx->device);
    std::string hi(sizeof(DevIneq) * (ni > 0 ? ni : 1), '\0');
    std::string hs(sizeof(DevShape) * (ns > 0 ? ns : 1), '\0');
    DevIneq* ti = reinterpret_cast<DevIneq*>(&hi[0]);
    DevShape* ts = reinterpret_cast<DevShape*>(&hs[0]);
    for (int i = 0; i < ni; ++i) {
        for (int k = 0; k < 6; ++k) ti[i].p[k] = geom->ineq_par[6 * i + k];
        ti[i].kind = geom->ineq_kind[i];
    }
    for (int s = 0; s < ns; ++s) {
        ts[s].first = geom->shape_first[s];
        ts[s].count = geom->shape_count[s];
        ts[s].cx = geom->shape_center[2 * s];
        ts[s].cy = geom->shape_center[2 * s + 1];
        ts[s].region = -1;
    }
    for (int r = 0; r < nr; ++r)
        for (int s = geom->region_first[r]; s < geom->region_first[r + 1]; ++s) ts[s].region = r;
    if (ctx->d_ineq) (void)hipFree(ctx->d_ineq);
    if (ctx->d_shape) (void)hipFree(ctx->d_shape);
    ctx->d_ineq = nullptr;
    ctx->d_shape = nullptr;
    ctx->have_geom = ctx->have_params = false;
    if (ctx->d_grid) (void)hipFree(ctx->d_grid);
    ctx->d_grid = nullptr;
    ctx->kg.grid = KShapeGrid{};
    HIP_TRY(hipMalloc(&ctx->d_ineq, hi.size()));
    HIP_TRY(hipMalloc(&ctx->d_shape, hs.size()));
    HIP_TRY(hipMemcpy(ctx->d_ineq, hi.data(), hi.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(ctx->d_shape, hs.data(), hs.size(), hipMemcpyHostToDevice));
    ctx->n_ineq = ni;
    ctx->n_shapes = ns;
    ctx->h_ineq.assign(ti, ti + ni);
    ctx->h_shape.assign(ts, ts + ns);
    KGeom& kg = ctx->kg;
    kg.ineq = ctx->d_ineq;
    kg.shape = ctx->d_shape;
    kg.n_obstacles = geom->n_obstacles;
    kg.n_regions = nr;
    for (int r = 0; r <= UAM_MAX_REGIONS; ++r)
        kg.region_first[r] = r <= nr ? geom->region_first[r] : ns;
    ctx->have_geom = true;
    return UAM_OK;
}

// Shape-grid index (KShapeGrid).  Lists: 0 = region shapes by box_pen (SHAPE_CULL_PEN),
// 1 = obstacles by box_obs for psi (SHAPE_CULL_PSI), 2 = obstacles by box_obs for contains
// (SHAPE_CULL_HIT); a shape without its cull flag is listed in every cell and in the off-grid
// slot.  The grid spans the union of the flagged boxes.
static constexpr int kShapeGridN = UAM_SHAPE_GRID_N;

// true when inequality q's h exceeds thr over the whole rectangle [rx0, rx1] x [ry0, ry1] by a
// margin far above any evaluation's rounding (h affine in a half-plane or square side: its
// minimum is at a corner; an ellipse's at the rectangle's point nearest its centre), so every
// point a kernel places there computes h > thr: the shape's psi has a zero factor (h >= e in
// the smooth forms) and contains() is false (h > 1e-14)
static bool ineq_above(const DevIneq& q, double rx0, double rx1, double ry0, double ry1,
                       double thr) {
    const double* p = q.p;
    double hmin, mag;
    if (q.kind == UAM_INEQ_HALFPLANE) {
        auto h = [&](double x, double y) { return p[4] * (p[3] * (x - p[0]) - p[2] * (y - p[1])); };
        hmin = std::min(std::min(h(rx0, ry0), h(rx0, ry1)), std::min(h(rx1, ry0), h(rx1, ry1)));
        mag = std::fabs(p[4]) * (std::fabs(p[3]) * (std::max(std::fabs(rx0), std::fabs(rx1)) +
                                                    std::fabs(p[0])) +
                                 std::fabs(p[2]) * (std::max(std::fabs(ry0), std::fabs(ry1)) +
                                                    std::fabs(p[1])));
    } else if (q.kind == UAM_INEQ_ELLIPSE) {
        const double xs = std::min(std::max(p[0], rx0), rx1), ys = std::min(std::max(p[1], ry0), ry1);
        const double a = (xs - p[0]) / p[2], b = (ys - p[1]) / p[3];
        hmin = a * a + b * b - 1.0;
        mag = a * a + b * b + 1.0;
    } else {
        const bool onx = p[0] == 0.0;
        const double v0 = onx ? rx0 : ry0, v1 = onx ? rx1 : ry1;
        hmin = std::min(p[3] * (v0 - p[1]) - p[2], p[3] * (v1 - p[1]) - p[2]);
        mag = std::fabs(p[3]) * (std::max(std::fabs(v0), std::fabs(v1)) + std::fabs(p[1])) +
              std::fabs(p[2]);
    }
    const double need = thr + 1e-9 * (mag + std::fabs(thr)) + 1e-300;
    return std::isfinite(hmin) && std::isfinite(mag) && hmin > need;
}

static int build_shape_grid(uam_ctx* ctx) {
    if (ctx->d_grid) (void)hipFree(ctx->d_grid);
    ctx->d_grid = nullptr;
    ctx->kg.grid = KShapeGrid{};
    const int ns = ctx->n_shapes, nobs = ctx->kg.n_obstacles;
    const int first_reg = ctx->kg.region_first[0], last_reg = ctx->kg.region_first[ctx->kg.n_regions];
    struct Src {
        int lo, hi, flag;
        bool pen;
    } src[3] = {{first_reg, last_reg, SHAPE_CULL_PEN, true},
                {0, nobs, SHAPE_CULL_PSI, false},
                {0, nobs, SHAPE_CULL_HIT, false}};
    double x0 = 1e300, y0 = 1e300, x1 = -1e300, y1 = -1e300;
    int flagged = 0;
    for (int l = 0; l < 3; ++l)
        for (int sh = src[l].lo; sh < src[l].hi; ++sh) {
            const DevShape& d = ctx->h_shape[sh];
            if (!(d.flags & src[l].flag)) continue;
            const double* b = src[l].pen ? d.box_pen : d.box_obs;
            if (!(std::isfinite(b[0]) && std::isfinite(b[1]) && std::isfinite(b[2]) &&
                  std::isfinite(b[3])))
                continue;
            x0 = std::min(x0, b[0]), x1 = std::max(x1, b[1]);
            y0 = std::min(y0, b[2]), y1 = std::max(y1, b[3]);
            ++flagged;
        }
    if (flagged == 0 || ns == 0 || !(x1 > x0) || !(y1 > y0)) return UAM_OK;  // no index
    const int G = kShapeGridN, cells = G * G;
    KShapeGrid gr{};
    gr.x0 = x0, gr.x1 = x1, gr.y0 = y0, gr.y1 = y1;
    gr.inv_dx = G / (x1 - x0), gr.inv_dy = G / (y1 - y0);
    gr.gx = gr.gy = G;
    auto cell_of = [&](double v, double o, double inv) {
        const double f = std::floor((v - o) * inv);
        return (int)std::max(0.0, std::min((double)(G - 1), f));
    };
    std::vector<int32_t> all;
    size_t offs[3][2];
    for (int l = 0; l < 3; ++l) {
        std::vector<std::vector<int32_t>> lists(cells + 1);
        for (int sh = src[l].lo; sh < src[l].hi; ++sh) {
            const DevShape& d = ctx->h_shape[sh];
            const double* b = src[l].pen ? d.box_pen : d.box_obs;
            const bool finite = std::isfinite(b[0]) && std::isfinite(b[1]) &&
                                std::isfinite(b[2]) && std::isfinite(b[3]);
            if (!(d.flags & src[l].flag) || !finite) {  // never culled: everywhere
                for (int c = 0; c <= cells; ++c) lists[c].push_back(sh);
                continue;
            }
            if (b[1] < x0 || b[0] > x1 || b[3] < y0 || b[2] > y1) continue;
            const int cx0 = cell_of(b[0], x0, gr.inv_dx), cx1 = cell_of(b[1], x0, gr.inv_dx);
            const int cy0 = cell_of(b[2], y0, gr.inv_dy), cy1 = cell_of(b[3], y0, gr.inv_dy);
            // a grid cell the shape's support misses entirely (one of its inequalities above
            // the threshold over the whole cell, grown by a relative 1e-6 for the kernels'
            // rounding of the slot index) does not list it: the per-point box test would have
            // let its points through to an exact +0 (or a false contains)
            const double thr = l == 0 ? ctx->kp.enlargement : l == 1 ? 0.0 : 1e-14;
            const DevIneq* qi = ctx->h_ineq.data() + d.first;
            const double cw = (x1 - x0) / G, chh = (y1 - y0) / G;
            for (int cy = cy0; cy <= cy1; ++cy)
                for (int cx = cx0; cx <= cx1; ++cx) {
                    const double rx0 = x0 + cx * cw - 1e-6 * cw, rx1 = x0 + (cx + 1) * cw + 1e-6 * cw;
                    const double ry0 = y0 + cy * chh - 1e-6 * chh;
                    const double ry1 = y0 + (cy + 1) * chh + 1e-6 * chh;
                    bool out = false;
                    for (int k = 0; UAM_GRID_REFINE && k < d.count && !out; ++k)
                        out = ineq_above(qi[k], rx0, rx1, ry0, ry1, thr);
                    if (!out) lists[cy * G + cx].push_back(sh);
                }
        }
        offs[l][0] = all.size();
        int32_t run = 0;
        all.push_back(0);
        for (int c = 0; c <= cells; ++c) {
            run += (int32_t)lists[c].size();
            all.push_back(run);
        }
        offs[l][1] = all.size();
        for (int c = 0; c <= cells; ++c) all.insert(all.end(), lists[c].begin(), lists[c].end());
    }
    // bitmask form of the lists (<= 256 shapes), appended as int32 pairs after the lists
    size_t moff[3] = {0, 0, 0};
    for (int l = 0; l < 3; ++l) {
        const int span = src[l].hi - src[l].lo;
        gr.mbase[l] = src[l].lo;
        gr.mw[l] = (span > 0 && span <= 256) ? (span + 63) >> 6 : 0;
        if (!gr.mw[l]) continue;
        while (all.size() % 2) all.push_back(0);  // 8-B alignment of the words
        moff[l] = all.size();
        std::vector<uint64_t> words((size_t)(cells + 1) * gr.mw[l], 0ull);
        const int32_t* st0 = all.data() + offs[l][0];
        const int32_t* it0 = all.data() + offs[l][1];
        for (int c = 0; c <= cells; ++c)
            for (int32_t k = st0[c]; k < st0[c + 1]; ++k) {
                const int b = it0[k] - src[l].lo;
                words[(size_t)c * gr.mw[l] + (b >> 6)] |= 1ull << (b & 63);
            }
        const int32_t* w32 = reinterpret_cast<const int32_t*>(words.data());
        all.insert(all.end(), w32, w32 + 2 * words.size());
    }
    HIP_TRY(hipMalloc(&ctx->d_grid, all.size() * sizeof(int32_t)));
    HIP_TRY(hipMemcpy(ctx->d_grid, all.data(), all.size() * sizeof(int32_t),
                      hipMemcpyHostToDevice));
    for (int l = 0; l < 3; ++l) {
        gr.start[l] = ctx->d_grid + offs[l][0];
        gr.items[l] = ctx->d_grid + offs[l][1];
    }
    for (int l = 0; l < 3; ++l)
        gr.mask[l] = gr.mw[l] ? reinterpret_cast<const uint64_t*>(ctx->d_grid + moff[l]) : nullptr;
    ctx->kg.grid = gr;
    return UAM_OK;
}

int uam_set_params(uam_ctx* ctx, const uam_params* prm, uam_stream stream) {
    int st = check_ctx(ctx, false);
    if (st) return st;
    if (!prm) return fail(UAM_E_INVALID, "params is NULL");
    if (prm->abi_version != UAM_ABI_VERSION)
        return fail(UAM_E_VERSION, "params abi_version %u != %d", prm->abi_version,
                    UAM_ABI_VERSION);
    if (prm->N < 1) return fail(UAM_E_INVALID, "N must be >= 1 (got %d)", prm->N);
    KParams& k = ctx->kp;
    k.N = prm->N;
    k.length_smooth = prm->length_smooth != 0;
    k.penalty_smooth = prm->penalty_smooth != 0;
    k.obstacle_smooth = prm->obstacle_smooth != 0;
    k.maxratio_smooth = prm->maxratio_smooth != 0;
    k.quirk_length = prm->quirk_length != 0;
    k.anchor_mode = prm->anchor_mode != 0;
    k.anchor_x = prm->anchor_x;
    k.anchor_y = prm->anchor_y;
    k.r_eff = prm->maxratio_smooth ? prm->maxratio * prm->maxratio : prm->maxratio;
    k.mincos = std::cos(prm->maxalpha);
    k.enlargement = prm->enlargement;
    k.altitude = prm->altitude;
    for (int r = 0; r < UAM_MAX_REGIONS; ++r) k.weights[r] = prm->weights[r];
    DeviceGuard dg(ctx->device);
    for (int sh = 0; sh < ctx->n_shapes; ++sh) {
        DevShape& d = ctx->h_shape[sh];
        const DevIneq* q = ctx->h_ineq.data() + d.first;
        d.flags = 0;
        if (shape_box(q, d.count, prm->enlargement, d.box_pen)) d.flags |= SHAPE_BOX_PEN_OK;
        if (shape_box(q, d.count, 1e-14, d.box_obs)) d.flags |= SHAPE_BOX_OBS_OK;
    }
    if (ctx->n_shapes > 0) {
        HIP_TRY(hipMemcpy(ctx->d_shape, ctx->h_shape.data(), sizeof(DevShape) * ctx->n_shapes,
                          hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_prepare, dim3(grid_for(ctx->n_shapes, 64)), dim3(64), 0,
                           (hipStream_t)stream, ctx->kg, k, ctx->d_shape, ctx->n_shapes);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
        HIP_TRY(hipMemcpy(ctx->h_shape.data(), ctx->d_shape, sizeof(DevShape) * ctx->n_shapes,
                          hipMemcpyDeviceToHost));
        // each region shape carries its region's weight (p.weights[region], bit for bit)
        for (DevShape& d : ctx->h_shape) d.wreg = d.region >= 0 ? k.weights[d.region] : 0.0;
        HIP_TRY(hipMemcpy(ctx->d_shape, ctx->h_shape.data(), sizeof(DevShape) * ctx->n_shapes,
                          hipMemcpyHostToDevice));
    }
    st = build_shape_grid(ctx);
    if (st) return st;
    ctx->have_params = true;
    return UAM_OK;
}

int uam_eval_points(uam_ctx* ctx, const double* pts, int64_t n, double* phi,
                    double* phi_regions, double* obs_norm, double* psi_raw, int32_t* collide,
                    uam_stream stream) {
    int st = check_ctx(ctx, true);
    if (st) return st;
    if (n < 0) return fail(UAM_E_INVALID, "n < 0");
    if (n == 0) return UAM_OK;
    if (!pts) return fail(UAM_E_INVALID, "pts is NULL");
    DeviceGuard dg(ctx->device);
    hipLaunchKernelGGL(k_eval_points, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                       ctx->kg, ctx->kp, pts, n, phi, phi_regions, obs_norm, psi_raw, collide);
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}

int uam_raster_build(uam_ctx* ctx, const uam_raster_desc* desc, const float* dem, void* rec,
                     uam_stream stream) {
    int st = check_ctx(ctx, true);
    if (st) return st;
    KRaster kr;
    st = make_kraster(desc, &kr);
    if (st) return st;
    if (!rec) return fail(UAM_E_INVALID, "rec is NULL");
    DeviceGuard dg(ctx->device);
    const int64_t cells = (int64_t)kr.nx * kr.ny;
    const hipStream_t s = (hipStream_t)stream;
    const int cpl = ctx->k1_cpl;  // cells (rows) per lane
    const int sny = (kr.ny + cpl - 1) / cpl, spt = UAM_K1_TILE_ROWS / cpl;
    const int64_t strips = (int64_t)((kr.nx + 63) / 64) *
                           (spt > 0 ? (int64_t)((sny + spt - 1) / spt) * spt : sny);
    // (the column order's XCD mapping wants a multiple of 8 workgroups; a capped grid loops,
    // each wave prefetching its next strip's DEM)
    const dim3 gs((grid_for(strips * 64, 256, UAM_K1_GRID_CAP) + 7) & ~7);
    switch (cpl) {
        case 1:  // the single-cell kernel
            hipLaunchKernelGGL(k_raster_build, dim3(grid_for(cells, 256)), dim3(256), 0, s,
                               ctx->kg, ctx->kp, kr, dem, desc->nodata, desc->dem_threshold,
                               (uint4*)rec);
            break;
        case 2:
            hipLaunchKernelGGL(k_raster_build_cells<2>, gs, dim3(256), 0, s, ctx->kg, ctx->kp,
                               kr, dem, desc->nodata, desc->dem_threshold, (uint4*)rec);
            break;
        case 8:
            hipLaunchKernelGGL(k_raster_build_cells<8>, gs, dim3(256), 0, s, ctx->kg, ctx->kp,
                               kr, dem, desc->nodata, desc->dem_threshold, (uint4*)rec);
            break;
        default:
            hipLaunchKernelGGL(k_raster_build_cells<4>, gs, dim3(256), 0, s, ctx->kg, ctx->kp,
                               kr, dem, desc->nodata, desc->dem_threshold, (uint4*)rec);
            break;
    }
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}

int uam_dem_mosaic(uam_ctx* ctx, const float* tiles, int32_t n_tiles, int32_t th, int32_t tw,
                   const int32_t* xoff, const int32_t* yoff, float* dem, int32_t nx, int32_t ny,
                   uam_stream stream) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    if (n_tiles < 0 || th <= 0 || tw <= 0 || nx <= 0 || ny <= 0)
        return fail(UAM_E_INVALID, "bad mosaic sizes");
    if (n_tiles == 0) return UAM_OK;
    if (!tiles || !xoff || !yoff || !dem) return fail(UAM_E_INVALID, "mosaic pointer is NULL");
    DeviceGuard dg(ctx->device);
    const int64_t total = (int64_t)n_tiles * th * tw;
    hipLaunchKernelGGL(k_dem_mosaic, dim3(grid_for(total, 256)), dim3(256), 0,
                       (hipStream_t)stream, tiles, n_tiles, th, tw, xoff, yoff, dem, nx, ny);
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}

int uam_load_tiles(uam_ctx* ctx, const char* const* paths, int32_t n_tiles, int32_t th,
                   int32_t tw, float* tiles_dev, int32_t n_threads, uam_stream stream) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    if (n_tiles < 0 || th <= 0 || tw <= 0 || (n_tiles > 0 && (!paths || !tiles_dev)))
        return fail(UAM_E_INVALID, "uam_load_tiles: bad arguments");
    if (n_tiles == 0) return UAM_OK;
    DeviceGuard dg(ctx->device);
    const size_t tile_bytes = (size_t)th * tw * 4;
    constexpr size_t CHUNK = (size_t)32 << 20;  // per buffer: ~230 of mergeLL.vrt's tiles
    const int32_t per = (int32_t)std::max<size_t>(1, CHUNK / tile_bytes);
    const size_t need = (size_t)per * tile_bytes;
    if (ctx->tring_bytes < need) {  // grow: wait for the old buffers' copies, then replace
        for (int b = 0; b < 2; ++b) {
            if (ctx->tring_used[b]) HIP_TRY(hipEventSynchronize(ctx->tring_ev[b]));
            ctx->tring_used[b] = false;
            if (ctx->tring[b]) HIP_TRY(hipHostFree(ctx->tring[b]));
            ctx->tring[b] = nullptr;
        }
        ctx->tring_bytes = 0;
        for (int b = 0; b < 2; ++b) {
            HIP_TRY(hipHostMalloc((void**)&ctx->tring[b], need));
            if (!ctx->tring_ev[b])
                HIP_TRY(hipEventCreateWithFlags(&ctx->tring_ev[b], hipEventDisableTiming));
        }
        ctx->tring_bytes = need;
    }
    const hipStream_t s = (hipStream_t)stream;
    // chunk c is read into buffer c % 2 while chunk c - 1's copy runs
    return tiles_stream(
        paths, n_tiles, th, tw, n_threads, per,
        [&](int32_t c) -> float* {
            const int b = c & 1;
            if (ctx->tring_used[b] && hipEventSynchronize(ctx->tring_ev[b]) != hipSuccess) {
                fail(UAM_E_HIP, "uam_load_tiles: chunk copy failed");
                return nullptr;
            }
            ctx->tring_used[b] = false;
            return reinterpret_cast<float*>(ctx->tring[b]);
        },
        [&](int32_t c, int32_t i0, int32_t i1) -> int {
            const int b = c & 1;
            HIP_TRY(hipMemcpyAsync(reinterpret_cast<char*>(tiles_dev) + (size_t)i0 * tile_bytes,
                                   ctx->tring[b], (size_t)(i1 - i0) * tile_bytes,
                                   hipMemcpyHostToDevice, s));
            HIP_TRY(hipEventRecord(ctx->tring_ev[b], s));
            ctx->tring_used[b] = true;
            return UAM_OK;
        });
}

int uam_gen_paths(uam_ctx* ctx, const double* pairs, int64_t n_pairs, const double* utab,
                  int32_t D, double* wp, uam_stream stream) {
    int st = check_ctx(ctx, true);
    if (st) return st;
    if (n_pairs < 0 || D < 1) return fail(UAM_E_INVALID, "n_pairs < 0 or D < 1");
    if (n_pairs == 0) return UAM_OK;
    if (!pairs || !utab || !wp) return fail(UAM_E_INVALID, "pointer is NULL");
    DeviceGuard dg(ctx->device);
    const int64_t total = n_pairs * D * (ctx->kp.N + 2);
    hipLaunchKernelGGL(k_gen_paths, dim3(grid_for(total, 256)), dim3(256), 0,
                       (hipStream_t)stream, pairs, n_pairs, utab, D, ctx->kp.N, wp);
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}

// K2w launch (raster / volume, explicit or generated); returns 1 if launched, 0 if the
// shape does not fit (caller falls back to the lane-per-path kernels), <0 on error.
static int launch_wave(uam_ctx* ctx, int mode, bool gen, const KRaster& kr, const KVolume& kv,
                       const void* rec, const double* wp, const double* pairs,
                       const double* utab, int D, int64_t n_paths, const KOut& ko,
                       int32_t* best_f, int32_t* best_l, hipStream_t s) {
    const int64_t per_wave = ewave_doubles(ctx->kp.N) * (int64_t)sizeof(double);
    if (per_wave > 65536) return 0;
    if ((best_f && !ko.cost) || (best_l && !ko.length)) return 0;
    const int wpb = (int)std::min<int64_t>(4, 65536 / per_wave);
    const int64_t blocks = (n_paths + wpb - 1) / wpb;
    if (blocks > INT32_MAX) return 0;
    const dim3 grid((unsigned)blocks), block(64 * wpb);
    const size_t lds = (size_t)(wpb * per_wave);
    const uint4* r = (const uint4*)rec;
    int st = ktime_begin(ctx, s);
    if (st) return st;
    if (mode == UAM_MODE_VOLUME)
        hipLaunchKernelGGL((k_eval_wave<UAM_MODE_VOLUME, true>), grid, block, lds, s, ctx->kg,
                           ctx->kp, kr, kv, r, wp, pairs, utab, D, n_paths, ko);
    else if (gen)
        hipLaunchKernelGGL((k_eval_wave<UAM_MODE_RASTER, true>), grid, block, lds, s, ctx->kg,
                           ctx->kp, kr, kv, r, wp, pairs, utab, D, n_paths, ko);
    else
        hipLaunchKernelGGL((k_eval_wave<UAM_MODE_RASTER, false>), grid, block, lds, s, ctx->kg,
                           ctx->kp, kr, kv, r, wp, pairs, utab, D, n_paths, ko);
    if (hipGetLastError() != hipSuccess) return fail(UAM_E_HIP, "k_eval_wave launch failed");
    st = ktime_end(ctx, s);
    if (st) return st;
    if (gen && (best_f || best_l)) {
        const int64_t n_pairs = n_paths / D;
        const dim3 g2(grid_for(n_pairs, 256, INT32_MAX));
        if (best_f) hipLaunchKernelGGL(k_argmin, g2, dim3(256), 0, s, ko.cost, n_pairs, D, 1, best_f);
        if (best_l)
            hipLaunchKernelGGL(k_argmin, g2, dim3(256), 0, s, ko.length, n_pairs, D, 0, best_l);
        if (hipGetLastError() != hipSuccess) return fail(UAM_E_HIP, "k_argmin launch failed");
    }
    return 1;
}

static bool want_wave(const uam_ctx* ctx, int64_t n_paths) { return n_paths <= ctx->wave_max; }

int uam_eval_waypoints(uam_ctx* ctx, int32_t mode, const uam_raster_desc* desc,
                       const void* rec, const double* wp, int64_t n_paths,
                       const uam_path_outputs* out, uam_stream stream) {
    int st = check_ctx(ctx, true);
    if (st) return st;
    if (n_paths < 0) return fail(UAM_E_INVALID, "n_paths < 0");
    if (n_paths == 0) return UAM_OK;
    if (!wp) return fail(UAM_E_INVALID, "wp is NULL");
    KRaster kr{};
    if (mode == UAM_MODE_RASTER) {
        st = make_kraster(desc, &kr);
        if (st) return st;
        if (!rec) return fail(UAM_E_INVALID, "raster mode needs rec");
    } else if (mode != UAM_MODE_ANALYTIC) {
        return fail(UAM_E_INVALID, "unknown mode %d", mode);
    }
    const KOut ko = make_kout(out);
    DeviceGuard dg(ctx->device);
    if (mode == UAM_MODE_RASTER && want_wave(ctx, n_paths)) {
        const KVolume kv{};
        st = launch_wave(ctx, mode, false, kr, kv, rec, wp, nullptr, nullptr, 1, n_paths, ko,
                         nullptr, nullptr, (hipStream_t)stream);
        if (st < 0) return st;
        if (st == 1) return UAM_OK;
    }
    const dim3 grid(grid_for(n_paths, 256, INT32_MAX)), block(256);
    if (mode == UAM_MODE_RASTER)
        hipLaunchKernelGGL(k_eval_waypoints<UAM_MODE_RASTER>, grid, block, 0, (hipStream_t)stream,
                           ctx->kg, ctx->kp, kr, (const uint4*)rec, wp, n_paths, ko);
    else
        hipLaunchKernelGGL(k_eval_waypoints<UAM_MODE_ANALYTIC>, grid, block, 0,
                           (hipStream_t)stream, ctx->kg, ctx->kp, kr, (const uint4*)rec, wp,
                           n_paths, ko);
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}


int uam_kernel_timing(uam_ctx* ctx, int32_t enable) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    ctx->ktime_on = enable != 0;
    ctx->ktime_n = 0;
    ctx->ktime_acc_ms = 0.0;
    ctx->ktime_acc_n = 0;
    return UAM_OK;
}

const char* uam_last_kernel(const uam_ctx* ctx) { return ctx ? ctx->last_kernel : ""; }

int32_t uam_last_group(const uam_ctx* ctx) { return ctx ? ctx->last_group : 0; }

int uam_set_option(uam_ctx* ctx, int32_t option, int64_t value) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    switch (option) {
        case UAM_OPT_GROUP:
            if (value < 0 || value > G_MAXLEN)
                return fail(UAM_E_INVALID, "UAM_OPT_GROUP %lld outside [0, %d]", (long long)value,
                            G_MAXLEN);
            ctx->k2g_group = (int)value;
            return UAM_OK;
        case UAM_OPT_SORTED_MIN_PATHS:
            if (value < 0) return fail(UAM_E_INVALID, "UAM_OPT_SORTED_MIN_PATHS < 0");
            ctx->k2s_min = value;
            return UAM_OK;
        case UAM_OPT_K2S_SEGMENTS:
            if (value < 2 || value > SEG_MAX)
                return fail(UAM_E_INVALID, "UAM_OPT_K2S_SEGMENTS %lld outside [2, %d]",
                            (long long)value, SEG_MAX);
            ctx->k2s_segs = (int)value;
            return UAM_OK;
        case UAM_OPT_WAVE_MAX_PATHS:
            if (value < 0) return fail(UAM_E_INVALID, "UAM_OPT_WAVE_MAX_PATHS < 0");
            ctx->wave_max = value;
            return UAM_OK;
        case UAM_OPT_PAIR_ORDER:
            ctx->pair_order = value != 0;
            return UAM_OK;
        case UAM_OPT_K1_ROWS:
            if (value != 1 && value != 2 && value != 4 && value != 8)
                return fail(UAM_E_INVALID, "UAM_OPT_K1_ROWS %lld not 1, 2, 4 or 8",
                            (long long)value);
            ctx->k1_cpl = (int)value;
            return UAM_OK;
        case UAM_OPT_K3B_SEGMENT:
            if (value != 0 && value != 2 && value != 4 && value != 6 && value != 8 && value != 16)
                return fail(UAM_E_INVALID, "UAM_OPT_K3B_SEGMENT %lld not 0, 2, 4, 6, 8 or 16",
                            (long long)value);
            ctx->k3b_seg = (int)value;
            return UAM_OK;
        case UAM_OPT_K3B_POINTS_PER_LANE:
            if (value != 1 && value != 2)
                return fail(UAM_E_INVALID, "UAM_OPT_K3B_POINTS_PER_LANE %lld not 1 or 2",
                            (long long)value);
            ctx->k3b_cpl = (int)value;
            return UAM_OK;
        case UAM_OPT_K8_TILED:
            ctx->k8_tiled = value != 0;
            return UAM_OK;
        case UAM_OPT_K2G_TILE_BITS:
            if (value != 0 && (value < 3 || value > G_TBITS_MAX))
                return fail(UAM_E_INVALID, "UAM_OPT_K2G_TILE_BITS %lld not 0 or in [3, %d]",
                            (long long)value, G_TBITS_MAX);
            ctx->k2g_tbits = (int)value;
            return UAM_OK;
        case UAM_OPT_K2G_LDS_FLOOR:
            if (value < 0 || value > 160 * 1024)
                return fail(UAM_E_INVALID, "UAM_OPT_K2G_LDS_FLOOR outside [0, 163840]");
            ctx->k2g_lds = (int)value;
            return UAM_OK;
        case UAM_OPT_K2G_CURVE:
            if (value != 0 && value != 1)
                return fail(UAM_E_INVALID, "UAM_OPT_K2G_CURVE %lld not 0 or 1", (long long)value);
            ctx->k2g_curve = (int)value;
            return UAM_OK;
        case UAM_OPT_K2G_CHUNK:
            if (value != 0 && value != 6 && value != 7 && value != 8 && value != 11 &&
                value != 16 && value != 21)
                return fail(UAM_E_INVALID, "UAM_OPT_K2G_CHUNK %lld not 0, 6, 7, 8, 11, 16 or 21",
                            (long long)value);
            ctx->k2g_chunk = (int)value;
            return UAM_OK;
        case UAM_OPT_K4H_BAND:
            if (value < 0 || value > 64 || (value & (value - 1)))
                return fail(UAM_E_INVALID, "UAM_OPT_K4H_BAND %lld not 0 or a power of two <= 64",
                            (long long)value);
            ctx->k4h_band = (int)value;
            return UAM_OK;
        case UAM_OPT_K2H_TERRAIN:
        case UAM_OPT_K4H_TERRAIN:
            if (value != 0 && value != 1)
                return fail(UAM_E_INVALID, "UAM_OPT_K%cH_TERRAIN %lld is not 0 or 1",
                            option == UAM_OPT_K2H_TERRAIN ? '2' : '4', (long long)value);
            (option == UAM_OPT_K2H_TERRAIN ? ctx->k2h_te : ctx->k4h_te) = (int)value;
            return UAM_OK;
        case UAM_OPT_TEST_SORT_FAULT:
            if (value != 0 && value != 1)
                return fail(UAM_E_INVALID, "UAM_OPT_TEST_SORT_FAULT %lld is not 0 or 1",
                            (long long)value);
            ctx->test_sort_fault = (int)value;
            return UAM_OK;
        case UAM_OPT_K2H_LB_STRIDE:
            if (value < 0 || value > 1024)
                return fail(UAM_E_INVALID, "UAM_OPT_K2H_LB_STRIDE %lld outside [0, 1024]",
                            (long long)value);
            ctx->k2h_lbs = (int)value;
            return UAM_OK;
        case UAM_OPT_K2G_SIM:
            if (value != 0 && value != 1)
                return fail(UAM_E_INVALID, "UAM_OPT_K2G_SIM %lld not 0 or 1", (long long)value);
            ctx->k2g_sim = (int)value;
            return UAM_OK;
        case UAM_OPT_K8_STREAMS:
            if (value < 1 || value > 8)
                return fail(UAM_E_INVALID, "UAM_OPT_K8_STREAMS %lld outside [1, 8]",
                            (long long)value);
            ctx->k8_nstreams = (int)value;
            return UAM_OK;
        default:
            return fail(UAM_E_INVALID, "unknown option %d", option);
    }
}

int uam_get_option(const uam_ctx* ctx, int32_t option, int64_t* value) {
    if (!ctx || !value) return fail(UAM_E_INVALID, "NULL argument");
    switch (option) {
        case UAM_OPT_GROUP: *value = ctx->k2g_group; return UAM_OK;
        case UAM_OPT_SORTED_MIN_PATHS: *value = ctx->k2s_min; return UAM_OK;
        case UAM_OPT_K2S_SEGMENTS: *value = ctx->k2s_segs; return UAM_OK;
        case UAM_OPT_WAVE_MAX_PATHS: *value = ctx->wave_max; return UAM_OK;
        case UAM_OPT_PAIR_ORDER: *value = ctx->pair_order ? 1 : 0; return UAM_OK;
        case UAM_OPT_K1_ROWS: *value = ctx->k1_cpl; return UAM_OK;
        case UAM_OPT_K3B_SEGMENT: *value = ctx->k3b_seg; return UAM_OK;
        case UAM_OPT_K3B_POINTS_PER_LANE: *value = ctx->k3b_cpl; return UAM_OK;
        case UAM_OPT_K8_TILED: *value = ctx->k8_tiled ? 1 : 0; return UAM_OK;
        case UAM_OPT_K8_STREAMS: *value = ctx->k8_nstreams; return UAM_OK;
        case UAM_OPT_K2G_TILE_BITS: *value = ctx->k2g_tbits; return UAM_OK;
        case UAM_OPT_K2G_LDS_FLOOR: *value = ctx->k2g_lds; return UAM_OK;
        case UAM_OPT_K2G_CHUNK: *value = ctx->k2g_chunk; return UAM_OK;
        case UAM_OPT_K2G_SIM: *value = ctx->k2g_sim; return UAM_OK;
        case UAM_OPT_K2H_LB_STRIDE: *value = ctx->k2h_lbs; return UAM_OK;
        case UAM_OPT_K2H_TERRAIN: *value = ctx->k2h_te; return UAM_OK;
        case UAM_OPT_K4H_TERRAIN: *value = ctx->k4h_te; return UAM_OK;
        case UAM_OPT_TEST_SORT_FAULT: *value = ctx->test_sort_fault; return UAM_OK;
        case UAM_OPT_K4H_BAND: *value = ctx->k4h_band; return UAM_OK;
        case UAM_OPT_K2G_CURVE: *value = ctx->k2g_curve; return UAM_OK;

        default: return fail(UAM_E_INVALID, "unknown option %d", option);
    }
}

int uam_kernel_time(uam_ctx* ctx, double* ms_total, int64_t* launches) {
    if (!ctx || !ms_total || !launches) return fail(UAM_E_INVALID, "NULL argument");
    DeviceGuard dg(ctx->device);
    const int st = ktime_fold(ctx);
    if (st) return st;
    *ms_total = ctx->ktime_acc_ms;
    *launches = ctx->ktime_acc_n;
    ctx->ktime_acc_ms = 0.0;
    ctx->ktime_acc_n = 0;
    return UAM_OK;
}

// K3 pair order (k_pair_keys / k_pair_scan / k_pair_scatter) into the context's scratch; *order
// stays null when the geometry has no shape grid (nothing to gain)
// The pair-order scratch (ctx->d_ord, grow-only) on stream s: waits for the last launch that
// read it (possibly on another stream), so two streams sharing a context cannot overwrite each
// other's order; the caller records ctx->ev_ord after the launch that reads the order.
// the context's side stream and its fork / join events (created on first use)
static int side_stream(uam_ctx* ctx) {
    if (ctx->s2) return UAM_OK;
    HIP_TRY(hipStreamCreateWithFlags(&ctx->s2, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
    return UAM_OK;
}

// the side stream at the device's lowest priority (created on first use; the fork / join
// events are side_stream's)
static int side_stream_lo(uam_ctx* ctx) {
    int st = side_stream(ctx);
    if (st || ctx->s_lo) return st;
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_TRY(hipStreamCreateWithPriority(&ctx->s_lo, hipStreamNonBlocking, least));
    return UAM_OK;
}

static int order_scratch(uam_ctx* ctx, size_t need, hipStream_t s, char** w) {
    if (!ctx->ev_ord) HIP_TRY(hipEventCreateWithFlags(&ctx->ev_ord, hipEventDisableTiming));
    // another stream's launches that read the scratch must finish first (the caller's own
    // stream is ordered already: no wait packet on the common path)
    if (ctx->ord_pending && ctx->ord_stream != s) HIP_TRY(hipStreamWaitEvent(s, ctx->ev_ord, 0));
    if (need > ctx->ord_bytes) {
        if (ctx->d_ord) {
            HIP_TRY(hipEventSynchronize(ctx->ev_ord));
            (void)hipFree(ctx->d_ord);
        }
        ctx->d_ord = nullptr;
        ctx->ord_bytes = 0;
        if (hipMalloc(&ctx->d_ord, need) != hipSuccess) return fail(UAM_E_NOMEM, "pair order");
        ctx->ord_bytes = need;
    }
    *w = (char*)ctx->d_ord;
    return UAM_OK;
}

static int order_done(uam_ctx* ctx, hipStream_t s) {
    HIP_TRY(hipEventRecord(ctx->ev_ord, s));
    ctx->ord_pending = true;
    ctx->ord_stream = s;
    return UAM_OK;
}

static int pair_order(uam_ctx* ctx, const double* pairs, int64_t n, hipStream_t s,
                      const int32_t** order) {
    *order = nullptr;
    const KShapeGrid& g = ctx->kg.grid;
    if (g.gx == 0 || !(g.x1 > g.x0) || !(g.y1 > g.y0)) return UAM_OK;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    // [hist 65536 | max bounds 2 x u64] zeroed together, then min bounds 2 x u64 (all ones)
    const size_t b_hist = al(65536 * 4 + 16 + 16), b_key = al((size_t)n * 2),
                 b_ord = al((size_t)n * 4);
    char* w = nullptr;
    const int st = order_scratch(ctx, b_hist + b_key + b_ord, s, &w);
    if (st) return st;
    int32_t* hist = (int32_t*)w;
    uint16_t* key = (uint16_t*)(w + b_hist);
    int32_t* ord = (int32_t*)(w + b_hist + b_key);
    unsigned long long* bnd = (unsigned long long*)(w + 65536 * 4);  // min x, min y, max x, max y
    HIP_TRY(hipMemsetAsync(hist, 0, 65536 * 4 + 32, s));
    HIP_TRY(hipMemsetAsync(bnd, 0xff, 16, s));
    const dim3 gr(grid_for(n, 256, INT32_MAX)), b(256);
    hipLaunchKernelGGL(k_pair_bounds, dim3(gr.x < 256 ? gr.x : 256), b, 0, s, pairs, n, bnd);
    hipLaunchKernelGGL(k_pair_keys, gr, b, 0, s, pairs, n, (const unsigned long long*)bnd, key,
                       hist);
    hipLaunchKernelGGL(k_pair_scan, dim3(1), dim3(1024), 0, s, hist);
    hipLaunchKernelGGL(k_pair_scatter, gr, b, 0, s, (const uint16_t*)key, n, hist, ord);
    HIP_TRY(hipGetLastError());
    *order = ord;
    return UAM_OK;
}

// K2 pair order over the raster extent (k_rorder_hist / k_rorder_scatter)
static size_t raster_pair_order_bytes(int64_t n) {
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    return al((size_t)RORD_BINS * RORD_NB * 4) + al((size_t)n * 2) + al((size_t)n * 4);
}

// w_in: caller-owned scratch of raster_pair_order_bytes(n) (null: the context's order scratch)
static int raster_pair_order(uam_ctx* ctx, const KRaster& kr, const double* pairs, int64_t n,
                             hipStream_t s, const int32_t** order, int vol = 0,
                             char* w_in = nullptr) {
    *order = nullptr;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t b_h = al((size_t)RORD_BINS * RORD_NB * 4), b_key = al((size_t)n * 2);
    char* w = w_in;
    if (!w) {
        const int st = order_scratch(ctx, raster_pair_order_bytes(n), s, &w);
        if (st) return st;
    }
    int32_t* H = (int32_t*)w;
    uint16_t* key = (uint16_t*)(w + b_h);
    int32_t* ord = (int32_t*)(w + b_h + b_key);
    const double ex = kr.nx * kr.dx, ey = kr.ny * kr.dy;
    const KOrdBox box{kr.x0, kr.y_top - ey, (double)(1 << RORD_BITS) / ex,
                      (double)(1 << RORD_BITS) / ey};
    hipLaunchKernelGGL(k_rorder_hist, dim3(RORD_NB), dim3(256), 0, s, pairs, n, box, key, H, vol);
    hipLaunchKernelGGL(k_rorder_scatter, dim3(RORD_NB), dim3(256), 0, s, (const uint16_t*)key, n,
                       (const int32_t*)H, ord);
    HIP_TRY(hipGetLastError());
    *order = ord;
    return UAM_OK;
}

// K2s launch (segment-sorted raster evaluation, the reference's sequential sums); returns 1 if
// launched, 0 if the batch is not one it takes (the caller runs K2).  Scratch: the pair-order
// scratch (order_scratch), so two streams sharing the context serialise on it.
static int launch_segmented(uam_ctx* ctx, const KRaster& kr, const void* rec, const double* pairs,
                            int64_t n_pairs, const double* utab, int32_t D, const KOut& ko,
                            int32_t* best_f, int32_t* best_l, hipStream_t s) {
    const int64_t W = ctx->kp.N + 2;
    const int want = std::min(ctx->k2s_segs, SEG_MAX);
    if (want < 2 || ko.cells || ko.g_rows || D > 16) return 0;
    const int L = (int)((W + want - 1) / want);
    const int nseg = (int)((W + L - 1) / L);  // e.g. W = 10 in 4: 3, 3, 3, 1
    if (nseg < 2) return 0;
    if (n_pairs > (INT32_MAX / SEG_MAX) / D) return 0;
    const int64_t P = n_pairs * D;
    if (P < ctx->k2s_min) return 0;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const int64_t ncnt = (int64_t)nseg * SEG_BINS * SEG_NBK;
    const int64_t nsb = (ncnt + 256 * SCAN_ITEMS - 1) / (256 * SCAN_ITEMS);
    if (nsb > 4096) return 0;
    const size_t b_st = al((size_t)P * sizeof(SegState)), b_len = al((size_t)P * 32),
                 b_key = al((size_t)nseg * P * 2), b_cnt = al((size_t)ncnt * 4),
                 b_tot = al(4096 * 4), b_ord = al((size_t)nseg * P * 4);
    char* w = nullptr;
    int st = order_scratch(ctx, b_st + b_len + b_key + b_cnt + b_tot + b_ord, s, &w);
    if (st) return st;
    KSeg ks{};
    ks.pairs = pairs;
    ks.utab = utab;
    ks.n_pairs = n_pairs;
    ks.P = (int32_t)P;
    ks.D = D;
    ks.W = (int32_t)W;
    ks.nseg = nseg;
    ks.L = L;
    int tshift = 0;
    while (((std::max(kr.nx, kr.ny) - 1) >> tshift) >= (1 << SEG_TBITS)) ++tshift;
    ks.tshift = tshift;
    ks.st = (SegState*)w;
    ks.p1 = (double4*)(w + b_st);
    ks.key = (uint16_t*)(w + b_st + b_len);
    ks.cnt = (int32_t*)(w + b_st + b_len + b_key);
    ks.tot = (int32_t*)(w + b_st + b_len + b_key + b_cnt);
    ks.order = (int32_t*)(w + b_st + b_len + b_key + b_cnt + b_tot);
    // the later segments' launches pad their dynamic LDS to a floor that caps the workgroups
    // resident per CU, so an XCD's resident items cover a narrow range of the sorted order
    // (cfg3 kernel ms by floor, packed: 40 KiB 0.541, 48 0.542-0.545, 56-80 0.555; 16-B
    // records: 80 KiB); segment 0 carries pass 1 and needs its occupancy (no floor)
    const size_t lds_min = kr.pmap ? (size_t)kr.pwords * 4 : kr.sum ? (size_t)kr.swords * 4 : 0;
    const size_t lds = std::max(lds_min, (size_t)(kr.pmap ? 40 : 80) * 1024);
    const size_t lds0 = lds_min;
    if (!ctx->k2s_attrs) {  // per context = per device (the caller's DeviceGuard is active)
        const void* fns[] = {(const void*)k_seg_eval<true, false>,
                             (const void*)k_seg_eval<false, false>,
                             (const void*)k_seg_eval<true, true>,
                             (const void*)k_seg_eval<false, true>,
                             (const void*)k_seg_eval<false, true, true>,
                             (const void*)k_seg_eval<false, false, true>};
        for (const void* f : fns)
            HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        160 * 1024));
        ctx->k2s_attrs = true;
    }
    st = side_stream(ctx);
    if (st) return st;
    // kernel timing brackets the whole sequence (sorts included)
    st = ktime_begin(ctx, s);
    if (st) return st;
    // counting sort of the segments [g0, g0 + ng) on stream q (cnt / tot: its own count and
    // block-total scratch); order positions start at segment g0's (g0 * P)
    auto sort_groups = [&](int g0, int ng, hipStream_t q, int32_t* cnt, int32_t* tot) {
        KSeg kq = ks;
        kq.g0 = g0;
        kq.obase = (int64_t)g0 * P;
        kq.cnt = cnt;
        kq.tot = tot;
        const int64_t nc = (int64_t)ng * SEG_BINS * SEG_NBK;
        const int64_t nb = (nc + 256 * SCAN_ITEMS - 1) / (256 * SCAN_ITEMS);
        hipLaunchKernelGGL(k_seg_hist, dim3(SEG_NBK, ng), dim3(256), 0, q, ctx->kp, kr, kq);
        hipLaunchKernelGGL(k_scan_local, dim3((unsigned)nb), dim3(256), 0, q, cnt, nc, cnt, tot);
        hipLaunchKernelGGL(k_scan_totals, dim3(1), dim3(1024), 0, q, tot, (int)nb);
        hipLaunchKernelGGL(k_seg_scatter, dim3(SEG_NBK, ng), dim3(256), 0, q, kq);
    };
    // segment 0's order first on s, the other segments' orders on the side stream beside
    // segment 0's launch (joined before segment 1)
    HIP_TRY(hipEventRecord(ctx->ev_fork, s));
    HIP_TRY(hipStreamWaitEvent(ctx->s2, ctx->ev_fork, 0));
    sort_groups(0, 1, s, ks.cnt, ks.tot);
    sort_groups(1, nseg - 1, ctx->s2, ks.cnt + (int64_t)SEG_BINS * SEG_NBK, ks.tot + 2048);
    HIP_TRY(hipEventRecord(ctx->ev_join, ctx->s2));
    for (int k = 0; k < nseg; ++k) {
        const int64_t base = (int64_t)k * P;
        if (k == 1) HIP_TRY(hipStreamWaitEvent(s, ctx->ev_join, 0));
        const dim3 ge((unsigned)((P + 255) / 256));
#define UAM_LAUNCH_SEG(SK_, F_, LDS_, PK_)                                                     \
    hipLaunchKernelGGL((k_seg_eval<SK_, F_, PK_>), ge, dim3(256), LDS_, s, ctx->kp, kr, ks,    \
                       (const uint4*)rec, k, base, (int32_t)P)
        if (kr.pmap) {
            if (k == 0) UAM_LAUNCH_SEG(false, true, lds0, true);
            else UAM_LAUNCH_SEG(false, false, lds, true);
        } else if (k == 0) {
            if (kr.sum) UAM_LAUNCH_SEG(true, true, lds0, false);
            else UAM_LAUNCH_SEG(false, true, lds0, false);
        } else {
            if (kr.sum) UAM_LAUNCH_SEG(true, false, lds, false);
            else UAM_LAUNCH_SEG(false, false, lds, false);
        }
#undef UAM_LAUNCH_SEG
    }
    const dim3 gf((unsigned)((n_pairs + 63) / 64));
    const size_t lf = (size_t)2 * 64 * D * sizeof(double);
    hipLaunchKernelGGL(k_seg_final, gf, dim3(64 * D), lf, s, ctx->kp, ks, ko, best_f, best_l);
    if (hipGetLastError() != hipSuccess) return fail(UAM_E_HIP, "segmented evaluation launch");
    st = ktime_end(ctx, s);
    if (st) return st;
    st = order_done(ctx, s);
    return st ? st : 1;
}

// position of tile (x, y) on the Hilbert curve of a 2^bits x 2^bits grid
static uint32_t hilbert_d(int bits, uint32_t x, uint32_t y) {
    uint32_t d = 0;
    for (uint32_t s = 1u << (bits - 1); s > 0; s >>= 1) {
        const uint32_t rx = (x & s) ? 1u : 0u, ry = (y & s) ? 1u : 0u;
        d += s * s * ((3u * rx) ^ ry);
        if (ry == 0) {
            if (rx == 1) {
                x = s - 1 - x;
                y = s - 1 - y;
            }
            const uint32_t t = x;
            x = y;
            y = t;
        }
    }
    return d;
}

// the K2g tile-key table for (bits, curve), uploaded once per setting
static int tile_keys(uam_ctx* ctx, int bits, int curve, hipStream_t s) {
    if (ctx->d_tkey && ctx->tkey_bits == bits && ctx->tkey_curve == curve) return UAM_OK;
    const uint32_t n = 1u << bits;
    std::vector<uint16_t> h((size_t)n * n);
    for (uint32_t y = 0; y < n; ++y)
        for (uint32_t x = 0; x < n; ++x) {
            uint32_t k = 0;
            if (curve) {
                k = hilbert_d(bits, x, y);
            } else {
                for (int b = bits - 1; b >= 0; --b)
                    k = (k << 2) | (((y >> b) & 1u) << 1) | ((x >> b) & 1u);
            }
            h[(size_t)y * n + x] = (uint16_t)k;
        }
    h.resize((size_t)2 * n * n);  // then the inverse: curve position -> tile y n + x
    for (uint32_t i = 0; i < n * n; ++i) h[(size_t)n * n + h[i]] = (uint16_t)i;
    if (!ctx->d_tkey) {
        const size_t cap = (2 * sizeof(uint16_t)) << (2 * G_TBITS_MAX);
        if (hipMalloc(&ctx->d_tkey, cap) != hipSuccess) return fail(UAM_E_NOMEM, "tile keys");
    }
    // stream-ordered: the launches that read the table follow on s
    HIP_TRY(hipMemcpyAsync(ctx->d_tkey, h.data(), h.size() * sizeof(uint16_t),
                           hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));  // h is freed on return
    ctx->tkey_bits = bits;
    ctx->tkey_curve = curve;
    return UAM_OK;
}

// div_magic's multiplier and shift for divisor D >= 1: sh = 32 + ceil(log2 D), m = ceil(2^sh / D)
static void magic_div(uint32_t D, uint64_t* m, int32_t* sh) {
    int k = 0;
    while ((1u << k) < D) ++k;
    *sh = 32 + k;
    const unsigned __int128 one = 1;
    *m = (uint64_t)(((one << *sh) + D - 1) / D);
}

// One K2g / K2h launch sequence (segment-grouped raster evaluation): what grouped_plan decides
// for a batch, then its scratch carved by grouped_carve, then the launches (grouped_sort: the
// counting sort's histogram, scan and scatter; grouped_eval; grouped_final: the output launch)
using GEvalFn = void (*)(KParams, KRaster, KGrp, const uint4*);
using HEvalFn = void (*)(KParams, KRaster, KGrp);
using GFinalFn = void (*)(KParams, KGrp, KOut, int32_t*, int32_t*);
struct GPlan {
    KGrp kg;
    bool sim;                 // K2h (the similarity form); K2g otherwise
    int64_t ncnt, nsb;        // counts ([bins][G_NBK]) and scan blocks
    size_t lds, hist_dyn, ubytes, bytes;  // eval / histogram dynamic LDS, arc rows, scratch
    size_t b_key, b_cnt, b_tot, b_ord, b_slot, b_ug, b_err, b_lbp;
    int bs;                   // evaluation workgroup
    GEvalFn ev;
    HEvalFn hev;
    GFinalFn fin;
};

// the sequence a batch takes: 1 (pl filled, scratch not yet carved), 0 when the batch is not
// one K2g / K2h takes, < 0 on error
static int grouped_plan(uam_ctx* ctx, const KRaster& kr, const double* pairs, int64_t n_pairs,
                        const double* utab, int32_t D, const KOut& ko, GPlan* pl) {
    const int G = ctx->k2g_group;
    if (G < 1 || G > G_MAXLEN || !kr.pmap || ko.g_rows || D > 16) return 0;
    const int64_t W = ctx->kp.N + 2, P = n_pairs * D;
    if (P < ctx->k2s_min || n_pairs > INT32_MAX / D) return 0;
    const size_t ubytes = (size_t)D * ctx->kp.N * 16;  // the unit-arc rows, staged in LDS
    if (ubytes > (size_t)G_UTAB_LDS) return 0;
    const int nseg = (int)((W + G - 1) / G);
    const int64_t n_items = P * nseg;
    if (n_items >= INT32_MAX) return 0;
    int tbits = ctx->k2g_tbits;
    if (tbits == 0) {  // tiles of ~256 x 256 cells ...
        tbits = 3;
        while (tbits < G_TBITS_MAX && (std::max(kr.nx, kr.ny) >> tbits) > 256) ++tbits;
        // ... but coarser for a small batch, so the sort's counts (bins x partitions) stay
        // within half its items (cfg4's rank share of 8, 500k items at 8192^2: tiles of 512^2
        // 0.175 ms against 0.178-0.181 at 256^2; the whole 1M-path job keeps 256^2: 0.900
        // against 0.958 ms; profiles/r06/c10)
        while (tbits > 3 && ((int64_t)(2 << (2 * tbits)) + 1) * G_NBK > n_items / 2) --tbits;
    }
    const int tiles = 1 << (2 * tbits);
    const int last_bin = (W % G) ? tiles : 0;  // a ragged last group gets its own bins
    const int bins = tiles + last_bin + 1;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    pl->ncnt = (int64_t)bins * G_NBK;
    pl->nsb = (pl->ncnt + 256 * SCAN_ITEMS - 1) / (256 * SCAN_ITEMS);
    if (pl->nsb > 4096) return 0;
    // K2h (the similarity form) unless disabled or maxratio_smooth (its turn rows are not
    // scale-free): 24-B slots, the geometry in the output launch
    // and its 32-bit offsets reach the whole packed copy; N <= 4096 (Phi / N by the reciprocal)
    const bool sim = ctx->k2g_sim && !ctx->kp.maxratio_smooth && kr.pk && ctx->kp.N <= 4096;
    pl->sim = sim;
    pl->ubytes = ubytes;
    pl->b_key = al((size_t)n_items * 2), pl->b_cnt = al((size_t)pl->ncnt * 4);
    pl->b_tot = al(4096 * 4), pl->b_ord = al((size_t)n_items * 4);
    pl->b_slot = al((size_t)n_items * (sim ? sizeof(HSlot) : sizeof(GSlot)));
    pl->b_ug = al((size_t)D * sizeof(UGeo)), pl->b_err = 256;
    pl->b_lbp = sim ? al((size_t)P * 4) : 0;
    pl->bytes = pl->b_key + pl->b_cnt + pl->b_tot + pl->b_ord + pl->b_slot + pl->b_ug +
                pl->b_err + pl->b_lbp;
    KGrp& kg = pl->kg;
    kg = KGrp{};
    kg.pairs = pairs;
    kg.utab = utab;
    kg.n_pairs = n_pairs;
    kg.P = (int32_t)P;
    kg.D = D;
    kg.W = (int32_t)W;
    kg.G = G;
    kg.nseg = nseg;
    int tshift = 0;
    while (((std::max(kr.nx, kr.ny) - 1) >> tshift) >= (1 << tbits)) ++tshift;
    kg.tshift = tshift;
    kg.tbits = tbits;
    kg.bins = bins;
    kg.last_bin = last_bin;
    magic_div((uint32_t)nseg, &kg.m_nseg, &kg.sh_nseg);
    magic_div((uint32_t)D, &kg.m_d, &kg.sh_d);
    kg.inv_n = ctx->kp.N <= 4096 ? 1.0 / (double)ctx->kp.N : 0.0;
    kg.n_items = n_items;
    kg.lb_stride = ctx->k2h_lbs;
    kg.nsb_raw = pl->nsb <= 1024 ? (int32_t)pl->nsb : 0;  // up to 1024 totals: scanned by the
                                                          // scatter
    // gathers in flight per lane (K2g, profiles/r03/k2g9, cfg3: 8 at G = 21 0.337 ms, 11 0.350,
    // 10 0.369, 6 0.351; K2h: 7, groups of 21 = three full chunks).  A raster far beyond the
    // L2s (over 2^25 cells: cfg4's 8192^2) misses more: fewer items resident per XCD (3
    // workgroups per CU through an LDS floor of 54 000 B) with 11 gathers in flight (cfg4
    // 0.886 against 0.936 ms, profiles/r04/sweep7)
    const bool big = sim && (int64_t)kr.nx * kr.ny > ((int64_t)1 << 25);
    const int chl = ctx->k2g_chunk ? ctx->k2g_chunk : big ? 11 : sim ? 7 : 8;
    pl->ev = nullptr;
    pl->hev = nullptr;
    const bool lbp = sim && !ctx->k2h_te && ctx->k2h_lbs > 0;
    // the seeds' header and unit-arc reads from LDS when both fit beside the histogram's own
    pl->hist_dyn = lbp ? (size_t)kr.hwords * 4 + ubytes : 0;
    if (sim) {  // K2h: H_BS-item workgroups, the packed header in LDS
        static const HEvalFn hevals[8] = {k_h_eval<6, false>, k_h_eval<7, false>,
                                          k_h_eval<8, false>, k_h_eval<11, false>,
                                          k_h_eval<6, true>,  k_h_eval<7, true>,
                                          k_h_eval<8, true>,  k_h_eval<11, true>};
        pl->hev = hevals[(chl <= 6 ? 0 : chl == 7 ? 1 : chl == 8 ? 2 : 3) + (ctx->k2h_te ? 4 : 0)];
        pl->bs = H_BS;
        const size_t hw = ctx->k2h_te ? (size_t)kr.bnd_off : (size_t)kr.hwords;
        const size_t need = hw * 4 + ubytes + (size_t)16 * (G + 16);  // + padding
        const int floor_lds = ctx->k2g_lds ? ctx->k2g_lds : big ? 54000 : 0;
        pl->lds = std::max(need, (size_t)std::min(floor_lds, 160 * 1024));
        if (pl->lds > 160 * 1024) return 0;
        if (!ctx->k2h_attrs) {  // per context = per device (DeviceGuard active)
            for (HEvalFn f : hevals)
                HIP_TRY(hipFuncSetAttribute((const void*)f,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            HIP_TRY(hipFuncSetAttribute((const void*)k_g_hist,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, G_HIST_DYN_MAX));
            ctx->k2h_attrs = true;
        }
    } else {  // K2g: 256-item workgroups, the code map in LDS
#define UAM_G_EVALS(CH) k_g_eval<CH, false, false>, k_g_eval<CH, false, true>, \
                        k_g_eval<CH, true, false>, k_g_eval<CH, true, true>
        static const GEvalFn evals[16] = {UAM_G_EVALS(6), UAM_G_EVALS(8), UAM_G_EVALS(11),
                                          UAM_G_EVALS(16)};
#undef UAM_G_EVALS
        const int ch = (chl == 6 || chl == 7 ? 0 : chl == 8 ? 1 : chl == 11 ? 2 : 3) * 4 +
                       (ctx->kp.length_smooth ? 2 : 0) + (ctx->kp.maxratio_smooth ? 1 : 0);
        pl->ev = evals[ch];
        pl->bs = 256;
        const size_t need = (size_t)((kr.pwords + 3) & ~3) * 4 + ubytes + 16;
        pl->lds = std::max(need, (size_t)std::min(ctx->k2g_lds, 160 * 1024));
        if (pl->lds > 64 * 1024 && !ctx->k2g_attrs) {
            for (GEvalFn f : evals)
                HIP_TRY(hipFuncSetAttribute((const void*)f,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            ctx->k2g_attrs = true;
        }
    }
    // the output launch holds a path's slots in registers up to 8 groups
    pl->fin = sim ? (nseg <= 4 ? k_h_final<4> : nseg <= 8 ? k_h_final<8> : k_h_final<0>)
                  : nseg <= 4 ? k_g_final<4> : nseg <= 8 ? k_g_final<8> : k_g_final<0>;
    const int st = err_word(ctx, &kg);  // (kg.tkey: the launchers, after tile_keys)
    return st ? st : 1;
}

// the plan's scratch at w (pl->bytes, 256-B aligned)
static void grouped_carve(uam_ctx* ctx, GPlan* pl, char* w) {
    KGrp& kg = pl->kg;
    size_t o = 0;
    kg.slot = (GSlot*)(w + o), o += pl->b_slot;  // 256-B aligned slots first (HSlot for K2h)
    kg.ugeo = pl->sim ? (UGeo*)(w + o) : nullptr, o += pl->b_ug;
    kg.order = (int32_t*)(w + o), o += pl->b_ord;
    kg.cnt = (int32_t*)(w + o), o += pl->b_cnt;
    kg.tot = (int32_t*)(w + o), o += pl->b_tot;
    kg.err = (int32_t*)(w + o), o += pl->b_err;
    kg.lbp = pl->sim && !ctx->k2h_te && ctx->k2h_lbs > 0 ? (float*)(w + o) : nullptr;
    o += pl->b_lbp;
    kg.seed_lds = kg.lbp && pl->hist_dyn <= (size_t)G_HIST_DYN_MAX;
    kg.key = (uint16_t*)(w + o);
}

static void grouped_sort(uam_ctx* ctx, const GPlan& pl, const KRaster& kr, hipStream_t s) {
    const KGrp& kg = pl.kg;
    hipLaunchKernelGGL(k_g_hist, dim3(G_NBK), dim3(1024), kg.seed_lds ? pl.hist_dyn : 0, s,
                       ctx->kp, kr, kg);
    hipLaunchKernelGGL(k_scan_local, dim3((unsigned)pl.nsb), dim3(256), 0, s, kg.cnt, pl.ncnt,
                       kg.cnt, kg.tot);
    if (!kg.nsb_raw)
        hipLaunchKernelGGL(k_scan_totals, dim3(1), dim3(1024), 0, s, kg.tot, (int)pl.nsb);
    hipLaunchKernelGGL(k_g_scatter, dim3(G_NBK + (kg.ugeo ? 1 : 0)), dim3(1024), 0, s, ctx->kp,
                       kg);
}

static void grouped_eval(uam_ctx* ctx, const GPlan& pl, const KRaster& kr, const void* rec,
                         hipStream_t s) {
    const dim3 grid((unsigned)((pl.kg.n_items + pl.bs - 1) / pl.bs));
    if (pl.hev)
        hipLaunchKernelGGL(pl.hev, grid, dim3(pl.bs), pl.lds, s, ctx->kp, kr, pl.kg);
    else
        hipLaunchKernelGGL(pl.ev, grid, dim3(pl.bs), pl.lds, s, ctx->kp, kr, pl.kg,
                           (const uint4*)rec);
}

static void grouped_final(uam_ctx* ctx, const GPlan& pl, const KOut& ko, int32_t* best_f,
                          int32_t* best_l, hipStream_t s) {
    const int D = pl.kg.D;
    hipLaunchKernelGGL(pl.fin, dim3((unsigned)((pl.kg.n_pairs + 63) / 64)), dim3(64 * D),
                       (size_t)2 * 64 * D * sizeof(double), s, ctx->kp, pl.kg, ko, best_f,
                       best_l);
}

// K2g launch (segment-grouped raster evaluation); returns 1 if launched, 0 if the batch is not
// one it takes (the caller runs K2s / K2).  Needs the packed raster.  Scratch: the pair-order
// scratch (order_scratch), so two streams sharing the context serialise on it.
static int launch_grouped(uam_ctx* ctx, const KRaster& kr, const void* rec, const double* pairs,
                          int64_t n_pairs, const double* utab, int32_t D, const KOut& ko,
                          int32_t* best_f, int32_t* best_l, hipStream_t s) {
    GPlan pl;
    int st = grouped_plan(ctx, kr, pairs, n_pairs, utab, D, ko, &pl);
    if (st <= 0) return st;
    char* w = nullptr;
    st = order_scratch(ctx, pl.bytes, s, &w);
    if (st) return st;
    st = tile_keys(ctx, pl.kg.tbits, ctx->k2g_curve, s);  // (enqueued only when they change)
    if (st) return st;
    pl.kg.tkey = ctx->d_tkey;
    grouped_carve(ctx, &pl, w);
    KGrp& kg = pl.kg;
    kg.cells = ko.cells;
    // the waypoint cells depend on the pairs and arc rows only: k_cells (VALU and store bound)
    // runs beside the sort and the gathers (miss bound) on a side stream of the device's lowest
    // priority, so their workgroups dispatch first and the cells fill what they leave, on a
    // grid capped at 512 workgroups looping over the 64-path blocks; joined before the call
    // returns.  cfg3 with cells (profiles/r05/cc9, cc10, cc20): 0.350-0.353 ms; at normal
    // priority 0.355-0.358; forked after the scatter 0.363; inline after the evaluation 0.362;
    // uncapped 0.372; the arc rows from global memory instead of LDS 0.005-0.02 ms more
    kg.cx0 = kr.x0, kg.cy_top = kr.y_top, kg.cinv_dx = kr.inv_dx, kg.cinv_dy = kr.inv_dy;
    kg.cnx = kr.nx, kg.cny = kr.ny;
    // (the cells written by K2h's output launch instead, the block's 320 paths each: that
    // launch 80.6 us against 15.1 + k_cells' 57.7, cfg3 with cells 0.365 against 0.350 ms;
    // profiles/r06/final1)
    const bool cells_side = ko.cells != nullptr;
    if (cells_side) {
        st = side_stream_lo(ctx);
        if (st) return st;
    }
    st = ktime_begin(ctx, s);
    if (st) return st;
    const int64_t P = kg.P;
    const unsigned cells_wg = (unsigned)std::min<int64_t>((P + 63) / 64, 512);
    void (*const cells_fn)(KParams, KGrp) =
        (int64_t)D * ctx->kp.N <= 1024 ? k_cells<true> : k_cells<false>;
    // once the cells are forked, every exit makes the caller's stream wait for them (an error
    // return must not leave k_cells writing the caller's buffer behind the call)
    bool forked = false;
    auto join = [&](int r) -> int {
        if (forked) {
            forked = false;
            const hipError_t e = hipStreamWaitEvent(s, ctx->ev_join, 0);
            if (e != hipSuccess && r >= 0) return fail(UAM_E_HIP, "cells join: %s", hipGetErrorString(e));
        }
        return r;
    };
    if (cells_side) {
        HIP_TRY(hipEventRecord(ctx->ev_fork, s));
        HIP_TRY(hipStreamWaitEvent(ctx->s_lo, ctx->ev_fork, 0));
        hipLaunchKernelGGL(cells_fn, dim3(cells_wg), dim3(256), 0, ctx->s_lo, ctx->kp, kg);
        HIP_TRY(hipEventRecord(ctx->ev_join, ctx->s_lo));
        forked = true;
    }
    grouped_sort(ctx, pl, kr, s);
    grouped_eval(ctx, pl, kr, rec, s);
    grouped_final(ctx, pl, ko, best_f, best_l, s);
    if (hipGetLastError() != hipSuccess) return join(fail(UAM_E_HIP, "grouped evaluation launch"));
    st = join(UAM_OK);
    if (st) return st;
    st = ktime_end(ctx, s);
    if (st) return st;
    ctx->last_group = pl.kg.G;
    ctx->last_kernel = pl.sim ? "K2h+pack" : "K2g+pack";
    st = order_done(ctx, s);
    return st ? st : 1;
}

// K4h launch (the packed volume in K2h's form); returns 1 if launched, 0 if the batch is not
// one it takes (the caller runs K4).  Scratch: the pair-order scratch (order_scratch).
static int launch_grouped3d(uam_ctx* ctx, const KVol4& kv, const double* pairs6, int64_t n_pairs,
                            const double* utab, int32_t D, const KOut& ko, int32_t* best_f,
                            int32_t* best_l, hipStream_t s) {
    const int G = ctx->k2g_group;
    if (G < 1 || G > G_MAXLEN || ko.cells || ko.g_rows || D > 16 || ctx->kp.maxratio_smooth ||
        !ctx->k2g_sim || !kv.pk || ctx->kp.N > 4096)
        return 0;
    const int64_t W = ctx->kp.N + 2, P = n_pairs * D;
    if (P < ctx->k2s_min || n_pairs > INT32_MAX / D) return 0;
    if ((size_t)D * ctx->kp.N * 16 > (size_t)G_UTAB_LDS) return 0;
    if ((size_t)kv.hwords * 4 > (size_t)VPK_HDR_LDS) return 0;
    // workgroups per CU: 3 by default through an LDS floor of 40 000 B (UAM_OPT_K2G_LDS_FLOOR
    // sets another): fewer items resident per XCD, so fewer of their lines miss L2 -- round 5's
    // bound form, cfg5: 0.394 ms at 3 with 7 in flight, 0.397 at 5 (28 000 B), 0.428 at 2
    // (60 000 B), 0.448 at 2 with 11 (profiles/r05/k4h2, cc)
    const int64_t npad = G + 16;  // k_v_eval's padding slots
    const size_t lds = std::max((size_t)(D * ctx->kp.N + npad) * 16 +
                                    (size_t)((W + npad + 1) & ~1) * 8 +
                                    (size_t)(ctx->k4h_te ? kv.bnd_off : kv.hwords) * 4,
                                (size_t)std::min(ctx->k2g_lds ? ctx->k2g_lds : 40000, 160 * 1024));
    const int nseg = (int)((W + G - 1) / G);
    const int64_t n_items = P * nseg;
    if (n_items >= INT32_MAX) return 0;
    // tiles: 8 x 8 by default (128^2 columns at 1024^2: cfg5 0.461 vs 0.491 ms at 16 x 16,
    // profiles/r04/vol2), UAM_OPT_K2G_TILE_BITS otherwise
    // (a tile-bits setting made for 2-D rasters may give more (tile, band) bins than the sort
    // holds: the key then takes the finest tiles that fit, which moves no bit of the outputs)
    int tbits = ctx->k2g_tbits ? ctx->k2g_tbits : 3;
    while (tbits > 1 && (2 << (2 * tbits)) * kv.nbands + 1 > G_BINS_MAX) --tbits;
    const int tiles = 1 << (2 * tbits);
    if (tiles * kv.nbands * 2 + 1 > G_BINS_MAX) return 0;  // (more bands than bins: K4)
    const int last_bin = (W % G) ? tiles * kv.nbands : 0;
    const int bins = tiles * kv.nbands + last_bin + 1;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const int64_t ncnt = (int64_t)bins * G_NBK;
    const int64_t nsb = (ncnt + 256 * SCAN_ITEMS - 1) / (256 * SCAN_ITEMS);
    if (nsb > 4096) return 0;
    const size_t b_key = al((size_t)n_items * 2), b_cnt = al((size_t)ncnt * 4),
                 b_ord = al((size_t)n_items * 4), b_slot = al((size_t)n_items * sizeof(VSlot)),
                 b_ug = al((size_t)D * sizeof(UGeo)), b_tot = al(4096 * 4), b_err = 256,
                 b_ubp = al((size_t)P * 8);
    char* w = nullptr;
    int st = order_scratch(ctx, b_key + b_cnt + b_ord + b_slot + b_ug + b_tot + b_err + b_ubp, s,
                           &w);
    if (st) return st;
    KGrp kg{};
    kg.pairs = pairs6;
    kg.utab = utab;
    kg.n_pairs = n_pairs;
    kg.P = (int32_t)P;
    kg.D = D;
    kg.W = (int32_t)W;
    kg.G = G;
    kg.nseg = nseg;
    int tshift = 0;
    while (((std::max(kv.nx, kv.ny) - 1) >> tshift) >= (1 << tbits)) ++tshift;
    kg.tshift = tshift;
    kg.tbits = tbits;
    kg.bins = bins;
    kg.last_bin = last_bin;
    st = tile_keys(ctx, tbits, ctx->k2g_curve, s);
    if (st) return st;
    kg.tkey = ctx->d_tkey;
    magic_div((uint32_t)nseg, &kg.m_nseg, &kg.sh_nseg);
    magic_div((uint32_t)D, &kg.m_d, &kg.sh_d);
    kg.inv_n = ctx->kp.N <= 4096 ? 1.0 / (double)ctx->kp.N : 0.0;
    kg.lb_stride = ctx->k2h_lbs;
    kg.n_items = n_items;
    size_t o = 0;
    kg.slot = (GSlot*)(w + o), o += b_slot;  // VSlot
    kg.ugeo = (UGeo*)(w + o), o += b_ug;
    kg.order = (int32_t*)(w + o), o += b_ord;
    kg.cnt = (int32_t*)(w + o), o += b_cnt;
    kg.tot = (int32_t*)(w + o), o += b_tot;
    kg.err = (int32_t*)(w + o), o += b_err;
    st = err_word(ctx, &kg);
    if (st) return st;
    kg.ubp = ctx->k2h_lbs > 0 && !ctx->k4h_te ? (double*)(w + o) : nullptr, o += b_ubp;
    const size_t hist_dyn = (size_t)kv.hwords * 4 + (size_t)D * ctx->kp.N * 16;
    kg.seed_lds = kg.ubp && hist_dyn <= (size_t)G_HIST_DYN_MAX;
    kg.key = (uint16_t*)(w + o);
    st = ktime_begin(ctx, s);
    if (st) return st;
    if (kg.seed_lds && !ctx->k4h_hist_attr) {
        HIP_TRY(hipFuncSetAttribute((const void*)k_v_hist,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, G_HIST_DYN_MAX));
        ctx->k4h_hist_attr = true;
    }
    hipLaunchKernelGGL(k_v_hist, dim3(G_NBK), dim3(1024), kg.seed_lds ? hist_dyn : 0, s,
                       ctx->kp, kv, kg);
    hipLaunchKernelGGL(k_scan_local, dim3((unsigned)nsb), dim3(256), 0, s, kg.cnt, ncnt, kg.cnt,
                       kg.tot);
    kg.nsb_raw = nsb <= 1024 ? (int32_t)nsb : 0;  // up to 1024 totals: scanned by the scatter
    if (!kg.nsb_raw)
        hipLaunchKernelGGL(k_scan_totals, dim3(1), dim3(1024), 0, s, kg.tot, (int)nsb);
    hipLaunchKernelGGL(k_g_scatter, dim3(G_NBK + (kg.ugeo ? 1 : 0)), dim3(1024), 0, s, ctx->kp, kg);
    const dim3 ge((unsigned)((n_items + 255) / 256));
    using VEvalFn = void (*)(KParams, KVol4, KGrp);
    // gathers in flight per lane: 7 by default (the bound form at 3 workgroups per CU; 8 and 11
    // are built for 3 / 2 waves per SIMD)
    const int chl = ctx->k2g_chunk ? ctx->k2g_chunk : 7;
    // (21 runs as 16: a chunk's per-slot codes take 4 bits each of 64)
    static const VEvalFn vevals[10] = {k_v_eval<6, false>, k_v_eval<7, false>,
                                       k_v_eval<8, false>,  k_v_eval<11, false>,
                                       k_v_eval<16, false>, k_v_eval<6, true>,
                                       k_v_eval<7, true>,   k_v_eval<8, true>,
                                       k_v_eval<11, true>,  k_v_eval<16, true>};
    const VEvalFn ev = vevals[(chl <= 6 ? 0 : chl == 7 ? 1 : chl <= 8 ? 2 : chl == 11 ? 3 : 4) +
                              (ctx->k4h_te ? 5 : 0)];
    if (lds > 64 * 1024 && !ctx->k4h_attrs) {
        for (VEvalFn f : vevals)
            HIP_TRY(hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        160 * 1024));
        ctx->k4h_attrs = true;
    }
    hipLaunchKernelGGL(ev, ge, dim3(256), lds, s, ctx->kp, kv, kg);
    hipLaunchKernelGGL(k_v_final, dim3((unsigned)((n_pairs + 63) / 64)), dim3(64 * D),
                       (size_t)2 * 64 * D * sizeof(double), s, ctx->kp, kg, ko, best_f, best_l);
    if (hipGetLastError() != hipSuccess) return fail(UAM_E_HIP, "grouped volume evaluation launch");
    st = ktime_end(ctx, s);
    if (st) return st;
    ctx->last_group = G;
    ctx->last_kernel = "K4h+pack";
    st = order_done(ctx, s);
    return st ? st : 1;
}

} // extern "C"

static int summary_dims(const uam_raster_desc* desc, int32_t block, int32_t* shift,
                        int32_t* nbx, int32_t* nby) {
    if (!desc || desc->nx <= 0 || desc->ny <= 0) return fail(UAM_E_INVALID, "bad raster desc");
    auto nblocks = [&](int64_t b) { return ((desc->nx + b - 1) / b) * ((desc->ny + b - 1) / b); };
    if (block == 0) {  // automatic: 8, doubled until the bitmap fits its 8 KiB of LDS
        block = 8;
        while (nblocks(block) > SKIP_MAX_BITS && block < 1024) block *= 2;
    }
    int sh = 0;
    while ((1 << sh) < block) ++sh;
    if ((1 << sh) != block || block < 1 || block > 1024)
        return fail(UAM_E_INVALID, "summary block %d is not a power of two in [1, 1024]", block);
    if (nblocks(block) > SKIP_MAX_BITS)
        return fail(UAM_E_INVALID, "summary block %d: %lld blocks exceed the %d-bit LDS bitmap",
                    block, (long long)nblocks(block), SKIP_MAX_BITS);
    *shift = sh;
    *nbx = (desc->nx + block - 1) / block;
    *nby = (desc->ny + block - 1) / block;
    return UAM_OK;
}

// packed-raster layout (uam_raster_pack), 256-B aligned sections:
//   header (hwords words, the part K2h stages in LDS): the code map (words, 2 bits per summary
//   block, padded to 16 B), the bound table (nbb u16, padded to 16 B; bound blocks of 2^bsh
//   cells square, the smallest with at most PK_BOUND_MAX of them and at least 8 cells wide), the
//   superblock table (nsb float2, 4 x 4 bound blocks each);
//   scratch (nbb float2: the bound blocks' {min, max} while packing);
//   p4 (4-B phi), t4 (4-B terrain), e8 (8 B) and r16 (the 16-B records) in 4 x 8-cell blocks,
//   all at one index; p8 ({phi, terrain}) in 4 x 4-cell blocks (p44_addr).
struct PackDims {
    int32_t sh, nbx, nby, words;           // summary blocks, code-map words
    int32_t bsh, bnbx, bnby, nbb;          // bound blocks
    int32_t sbnbx, sbnby, nsb;             // superblocks
    int32_t hwords, bnd_off, sbt_off;      // header words, word offsets
    int32_t nb8, lnby;                     // 4 x 8-cell blocks per row, block rows
    int32_t nb4;                           // p8's 4 x 4-cell blocks per row
    int64_t off_scr, off_p4, off_t4, off_e8, off_r16, off_p8, bytes;
};

static int pack_dims(const uam_raster_desc* desc, int32_t block, PackDims* d) {
    int st = summary_dims(desc, block, &d->sh, &d->nbx, &d->nby);
    if (st) return st;
    d->words = (int32_t)(((int64_t)d->nbx * d->nby * 2 + 31) / 32);
    d->bsh = 3;
    auto nblk = [&](int s) {
        return (int64_t)((desc->nx + (1 << s) - 1) >> s) * ((desc->ny + (1 << s) - 1) >> s);
    };
    while (nblk(d->bsh) > PK_BOUND_MAX) ++d->bsh;
    d->bnbx = (desc->nx + (1 << d->bsh) - 1) >> d->bsh;
    d->bnby = (desc->ny + (1 << d->bsh) - 1) >> d->bsh;
    d->nbb = d->bnbx * d->bnby;
    d->sbnbx = (d->bnbx + 3) >> 2;
    d->sbnby = (d->bnby + 3) >> 2;
    d->nsb = d->sbnbx * d->sbnby;
    auto w16 = [](int64_t bytes) { return (int32_t)(((bytes + 15) & ~(int64_t)15) / 4); };
    d->bnd_off = w16((int64_t)d->words * 4);
    d->sbt_off = d->bnd_off + w16((int64_t)d->nbb * 2);
    d->hwords = d->sbt_off + w16((int64_t)d->nsb * 8);
    d->nb8 = (desc->nx + 7) >> 3;
    d->lnby = (desc->ny + 3) >> 2;
    const int64_t c4 = (int64_t)d->lnby * d->nb8 * 32;
    if (c4 >= ((int64_t)1 << 31) || desc->nx >= (1 << 24) || desc->ny >= (1 << 24))
        return fail(UAM_E_INVALID, "packed raster too large");
    auto a256 = [](int64_t v) { return (v + 255) & ~(int64_t)255; };
    d->off_scr = a256((int64_t)d->hwords * 4);
    d->off_p4 = d->off_scr + a256((int64_t)d->nbb * 8);
    d->off_t4 = d->off_p4 + a256(c4 * 4);
    d->off_e8 = d->off_t4 + a256(c4 * 4);
    d->off_r16 = d->off_e8 + a256(c4 * 8);
    d->off_p8 = d->off_r16 + a256(c4 * 16);
    d->nb4 = (desc->nx + 3) >> 2;
    d->bytes = d->off_p8 + a256((int64_t)d->lnby * d->nb4 * 16 * 8);
    return UAM_OK;
}

static void set_kpack(KRaster* kr, const PackDims& d, const void* packed) {
    const char* b = (const char*)packed;
    kr->pmap = (const uint32_t*)b;
    kr->pwords = d.words;
    kr->hwords = d.hwords;
    kr->bnd_off = d.bnd_off;
    kr->sbt_off = d.sbt_off;
    kr->bshift = d.bsh;
    kr->bnbx = d.bnbx;
    kr->sbnbx = d.sbnbx;
    kr->nb8 = d.nb8;
    kr->nb4 = d.nb4;
    kr->p4 = (const uint32_t*)(b + d.off_p4);
    kr->t4 = (const float*)(b + d.off_t4);
    kr->e8 = (const uint2*)(b + d.off_e8);
    const bool o32 = d.bytes <= (int64_t)UINT32_MAX;  // K2h's 32-bit offsets reach every byte
    kr->pk = o32 ? b : nullptr;
    kr->o4 = (uint32_t)d.off_p4;
    kr->o8 = (uint32_t)d.off_e8;
    kr->o16 = (uint32_t)d.off_r16;
    kr->ot4 = (uint32_t)d.off_t4;
    kr->op8 = (uint32_t)d.off_p8;
}

// the raster's descriptor and its derived copies as the evaluations read them
static int raster_inputs(const uam_raster_desc* desc, const void* rec, const uint32_t* summary,
                         int32_t sblock, const void* packed, KRaster* kr) {
    int st = make_kraster(desc, kr);
    if (st) return st;
    if (!rec) return fail(UAM_E_INVALID, "raster mode needs rec");
    if (summary) {
        int32_t sh, nbx, nby;
        st = summary_dims(desc, sblock, &sh, &nbx, &nby);
        if (st) return st;
        kr->sum = summary;
        kr->sshift = sh;
        kr->snbx = nbx;
        kr->swords = (nbx * nby + 31) / 32;
    }
    if (packed) {
        PackDims pd;
        st = pack_dims(desc, sblock, &pd);
        if (st) return st;
        kr->sshift = pd.sh;  // the block codes use the summary's block grid
        kr->snbx = pd.nbx;
        set_kpack(kr, pd, packed);
    }
    return UAM_OK;
}

static int eval_generated(uam_ctx* ctx, int32_t mode, const uam_raster_desc* desc,
                          const void* rec, const uint32_t* summary, int32_t sblock,
                          const double* pairs, int64_t n_pairs, const double* utab, int32_t D,
                          const uam_path_outputs* out, uam_stream stream,
                          const void* packed = nullptr) {
    int st = check_ctx(ctx, true);
    if (st) return st;
    if (n_pairs < 0 || D < 1) return fail(UAM_E_INVALID, "n_pairs < 0 or D < 1");
    if (n_pairs == 0) return UAM_OK;
    if (!pairs || !utab) return fail(UAM_E_INVALID, "pairs/utab is NULL");
    KRaster kr{};
    if (mode == UAM_MODE_RASTER) {
        st = raster_inputs(desc, rec, summary, sblock, packed, &kr);
        if (st) return st;
    } else if (mode != UAM_MODE_ANALYTIC) {
        return fail(UAM_E_INVALID, "unknown mode %d", mode);
    }
    const KOut ko = make_kout(out);
    int32_t* best_f = out ? out->best_fval_idx : nullptr;
    int32_t* best_l = out ? out->best_length_idx : nullptr;
    DeviceGuard dg(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    ctx->last_group = 0;  // sequential sums unless K2g runs
    if (mode == UAM_MODE_RASTER && n_pairs <= INT64_MAX / D && want_wave(ctx, n_pairs * D)) {
        const KVolume kv{};
        st = launch_wave(ctx, mode, true, kr, kv, rec, nullptr, pairs, utab, D, n_pairs * D, ko,
                         best_f, best_l, s);
        if (st < 0) return st;
        if (st == 1) {
            ctx->last_kernel = "K2w";
            return UAM_OK;
        }
    }
    if (mode == UAM_MODE_RASTER && ctx->k2g_group > 0) {
        st = launch_grouped(ctx, kr, rec, pairs, n_pairs, utab, D, ko, best_f, best_l, s);
        if (st < 0) return st;
        if (st == 1) return UAM_OK;  // last_kernel: "K2h+pack" / "K2g+pack"
    }
    if (mode == UAM_MODE_RASTER) {
        st = launch_segmented(ctx, kr, rec, pairs, n_pairs, utab, D, ko, best_f, best_l, s);
        if (st < 0) return st;
        if (st == 1) {
            ctx->last_kernel = kr.pmap ? "K2s+pack" : kr.sum ? "K2s+skip" : "K2s";
            return UAM_OK;
        }
    }
    if (D > 16) {  // the block-of-pairs kernels hold all D waves in one workgroup
        ctx->last_kernel = mode == UAM_MODE_RASTER ? "K2d" : "K3d";
        const int64_t n_waves = ((n_pairs + 63) / 64) * D;
        const int64_t blocks = (n_waves + 3) / 4;
        if (blocks > INT32_MAX) return fail(UAM_E_INVALID, "batch too large");
        const dim3 grid((unsigned)blocks), block(256);
        if (mode == UAM_MODE_RASTER)
            hipLaunchKernelGGL(k_eval_generated<UAM_MODE_RASTER>, grid, block, 0, s, ctx->kg,
                               ctx->kp, kr, (const uint4*)rec, pairs, n_pairs, utab, D, n_waves,
                               ko);
        else
            hipLaunchKernelGGL(k_eval_generated<UAM_MODE_ANALYTIC>, grid, block, 0, s, ctx->kg,
                               ctx->kp, kr, (const uint4*)rec, pairs, n_pairs, utab, D, n_waves,
                               ko);
        HIP_TRY(hipGetLastError());
        if (best_f || best_l) {  // selection needs the costs/lengths even if not requested
            if ((best_f && !ko.cost) || (best_l && !ko.length))
                return fail(UAM_E_INVALID, "best_*_idx needs cost/length outputs (D > 16)");
            const dim3 g2(grid_for(n_pairs, 256, INT32_MAX));
            if (best_f) hipLaunchKernelGGL(k_argmin, g2, dim3(256), 0, s, ko.cost, n_pairs, D, 1, best_f);
            if (best_l) hipLaunchKernelGGL(k_argmin, g2, dim3(256), 0, s, ko.length, n_pairs, D, 0, best_l);
            HIP_TRY(hipGetLastError());
        }
        return UAM_OK;
    }
    const int64_t blocks = (n_pairs + 63) / 64;
    if (blocks > INT32_MAX) return fail(UAM_E_INVALID, "batch too large");
    const dim3 grid((unsigned)blocks), block(64 * D);
    const size_t lds = (size_t)64 * D * (6 * sizeof(double) + 3 * sizeof(int32_t)) +
                       (kr.sum ? (size_t)kr.swords * 4 : 0);
    const KVolume kv{};
    const int32_t* order = nullptr;
    if (ctx->pair_order && n_pairs >= 4096 && n_pairs < INT32_MAX) {
        st = mode == UAM_MODE_ANALYTIC ? pair_order(ctx, pairs, n_pairs, s, &order)
                                       : raster_pair_order(ctx, kr, pairs, n_pairs, s, &order);
        if (st) return st;
    }
#define UAM_LAUNCH_PAIRS(MODE_, MINW_)                                                     \
    hipLaunchKernelGGL((k_eval_pairs<MODE_, MINW_>), grid, block, lds, s, ctx->kg, ctx->kp,   \
                       kr, kv, (const uint4*)rec, pairs, n_pairs, utab, D, ko, best_f, best_l, \
                       order)
    st = ktime_begin(ctx, s);
    if (st) return st;
    if (mode == UAM_MODE_ANALYTIC && !ko.g_rows && ctx->k3b_seg > 0) {
        int S = ctx->k3b_seg >= 16 ? 16
                : ctx->k3b_seg >= 8 ? 8 : ctx->k3b_seg >= 6 ? 6 : ctx->k3b_seg >= 4 ? 4 : 2;
        while (S > 2 && k3b_lds_bytes(D, S) > 160 * 1024) S = S == 6 ? 4 : S / 2;
        const int CPL = ctx->k3b_cpl >= 2 ? 2 : 1;
        const size_t l3 = k3b_lds_bytes(D, S);
        if (!ctx->k3b_attrs) {  // per context = per device (DeviceGuard active)
            const void* fns[] = {(const void*)k_eval_pairs_k3b<2, 1>,
                                 (const void*)k_eval_pairs_k3b<4, 1>,
                                 (const void*)k_eval_pairs_k3b<8, 1>,
                                 (const void*)k_eval_pairs_k3b<16, 1>,
                                 (const void*)k_eval_pairs_k3b<6, 1>,
                                 (const void*)k_eval_pairs_k3b<6, 2>,
                                 (const void*)k_eval_pairs_k3b<2, 2>,
                                 (const void*)k_eval_pairs_k3b<4, 2>,
                                 (const void*)k_eval_pairs_k3b<8, 2>,
                                 (const void*)k_eval_pairs_k3b<16, 2>};
            for (const void* f : fns)
                HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            160 * 1024));
            ctx->k3b_attrs = true;
        }
#define UAM_LAUNCH_K3B(S_, C_)                                                                 \
    hipLaunchKernelGGL((k_eval_pairs_k3b<S_, C_>), grid, block, l3, s, ctx->kg, ctx->kp, pairs,   \
                       n_pairs, utab, D, ko, best_f, best_l, order)
        ctx->last_kernel = "K3b";
        switch (S * 4 + CPL) {
            case 16 * 4 + 2: UAM_LAUNCH_K3B(16, 2); break;
            case 8 * 4 + 2: UAM_LAUNCH_K3B(8, 2); break;
            case 6 * 4 + 2: UAM_LAUNCH_K3B(6, 2); break;
            case 6 * 4 + 1: UAM_LAUNCH_K3B(6, 1); break;
            case 4 * 4 + 2: UAM_LAUNCH_K3B(4, 2); break;
            case 2 * 4 + 2: UAM_LAUNCH_K3B(2, 2); break;
            case 16 * 4 + 1: UAM_LAUNCH_K3B(16, 1); break;
            case 8 * 4 + 1: UAM_LAUNCH_K3B(8, 1); break;
            case 4 * 4 + 1: UAM_LAUNCH_K3B(4, 1); break;
            default: UAM_LAUNCH_K3B(2, 1); break;
        }
#undef UAM_LAUNCH_K3B
    } else if (mode == UAM_MODE_ANALYTIC) {
        ctx->last_kernel = "K3";
        UAM_LAUNCH_PAIRS(UAM_MODE_ANALYTIC, 1);
    } else {
        // (r01: chunks of 2-8 gathers, software pipelining and 5-8 waves per SIMD measured within
        // +-1% of each other on cfg3 -- the kernel sits at the random-gather ceiling)
        ctx->last_kernel = kr.sum ? "K2+skip" : "K2";
        if (kr.sum) UAM_LAUNCH_PAIRS(MODE_RASTER_SKIP, SKIP_MINW);
        else UAM_LAUNCH_PAIRS(UAM_MODE_RASTER, 1);
    }
#undef UAM_LAUNCH_PAIRS
    HIP_TRY(hipGetLastError());
    st = ktime_end(ctx, s);
    if (st) return st;
    if (order) return order_done(ctx, s);
    return UAM_OK;
}

extern "C" {

int uam_eval_generated(uam_ctx* ctx, int32_t mode, const uam_raster_desc* desc,
                       const void* rec, const uint32_t* summary, int32_t block,
                       const void* packed, const double* pairs, int64_t n_pairs,
                       const double* utab, int32_t D, const uam_path_outputs* out,
                       uam_stream stream) {
    if (ctx) {  // an earlier call's failed device check, reported once (uam_device_status)
        const int st = device_status(ctx);
        if (st) return st;
    }
    return eval_generated(ctx, mode, desc, rec, summary, block, pairs, n_pairs, utab, D, out,
                          stream, packed);
}

int uam_raster_pack_shape(const uam_raster_desc* desc, int32_t block, int32_t* block_out,
                          int64_t* bytes) {
    PackDims d;
    const int st = pack_dims(desc, block, &d);
    if (st) return st;
    if (block_out) *block_out = 1 << d.sh;
    if (bytes) *bytes = d.bytes;
    return UAM_OK;
}

int uam_raster_pack(uam_ctx* ctx, const uam_raster_desc* desc, const void* rec, int32_t block,
                    void* packed, uam_stream stream) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    KRaster kr{};
    int st = make_kraster(desc, &kr);
    if (st) return st;
    if (!rec || !packed) return fail(UAM_E_INVALID, "rec/packed is NULL");
    if ((uintptr_t)packed & 255) return fail(UAM_E_INVALID, "packed must be 256-B aligned");
    PackDims d;
    st = pack_dims(desc, block, &d);
    if (st) return st;
    set_kpack(&kr, d, packed);
    DeviceGuard dg(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    char* b = (char*)packed;
    const uint4* r4 = (const uint4*)rec;
    // header padding and the planes' padding cells: zero (never addressed, but defined bytes)
    HIP_TRY(hipMemsetAsync(b, 0, (size_t)d.off_scr, s));
    HIP_TRY(hipMemsetAsync(b + d.off_p4, 0, (size_t)(d.bytes - d.off_p4), s));
    const int32_t nb = d.nbx * d.nby;
    if (d.sh >= 3)  // (the map words were zeroed above)
        hipLaunchKernelGGL(k_raster_pack_map_w, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, s,
                           r4, kr.nx, kr.ny, d.sh, d.nbx, nb, (uint32_t*)b);
    else
        hipLaunchKernelGGL(k_raster_pack_map, dim3(grid_for(nb, 256)), dim3(256), 0, s, r4,
                           kr.nx, kr.ny, d.sh, d.nbx, nb, (uint32_t*)b);
    const int64_t cells = (int64_t)kr.nx * kr.ny;
    hipLaunchKernelGGL(k_raster_pack, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, s, r4,
                       kr, (uint32_t*)(b + d.off_p4), (float*)(b + d.off_t4),
                       (uint2*)(b + d.off_e8), (uint4*)(b + d.off_r16),
                       (uint2*)(b + d.off_p8));
    hipLaunchKernelGGL(k_t4_bminmax, dim3((unsigned)((d.nbb + 3) / 4)), dim3(256), 0, s,
                       (const float*)(b + d.off_t4), kr.nx, kr.ny, d.nb8, d.bsh, d.bnbx, d.nbb,
                       (float2*)(b + d.off_scr));
    hipLaunchKernelGGL(k_raster_bounds, dim3((unsigned)((d.nbb + 255) / 256)), dim3(256), 0, s,
                       (const float2*)(b + d.off_scr), d.bnbx, d.bnby, d.sbnbx,
                       (uint16_t*)(b + (size_t)d.bnd_off * 4), (float2*)(b + (size_t)d.sbt_off * 4));
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}

int uam_raster_summary_shape(const uam_raster_desc* desc, int32_t block, int32_t* block_out,
                             int32_t* nbx, int32_t* nby) {
    int32_t sh, bx, by;
    const int st = summary_dims(desc, block, &sh, &bx, &by);
    if (st) return st;
    if (block_out) *block_out = 1 << sh;
    if (nbx) *nbx = bx;
    if (nby) *nby = by;
    return UAM_OK;
}

int uam_raster_summary(uam_ctx* ctx, const uam_raster_desc* desc, const void* rec,
                       int32_t block, uint32_t* summary, uam_stream stream) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    KRaster kr{};
    int st = make_kraster(desc, &kr);
    if (st) return st;
    if (!rec || !summary) return fail(UAM_E_INVALID, "rec/summary is NULL");
    int32_t sh, nbx, nby;
    st = summary_dims(desc, block, &sh, &nbx, &nby);
    if (st) return st;
    DeviceGuard dg(ctx->device);
    const int32_t nb = nbx * nby;
    if (sh >= 3) {
        HIP_TRY(hipMemsetAsync(summary, 0, (size_t)((nb + 31) / 32) * 4, (hipStream_t)stream));
        hipLaunchKernelGGL(k_raster_summary_w, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0,
                           (hipStream_t)stream, (const uint4*)rec, kr.nx, kr.ny, sh, nbx, nb,
                           summary);
    } else {
        hipLaunchKernelGGL(k_raster_summary, dim3(grid_for(nb, 256)), dim3(256), 0,
                           (hipStream_t)stream, (const uint4*)rec, kr.nx, kr.ny, sh, nbx, nb,
                           summary);
    }
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}

namespace {
int make_kvolume(const uam_volume_desc* d, KVolume* k) {
    if (!d) return fail(UAM_E_INVALID, "volume descriptor is NULL");
    if (d->nx <= 0 || d->ny <= 0 || d->nz <= 0)
        return fail(UAM_E_INVALID, "volume size %dx%dx%d", d->nx, d->ny, d->nz);
    if ((int64_t)d->nx * d->ny * d->nz >= ((int64_t)1 << 31))
        return fail(UAM_E_INVALID, "volume has more than 2^31 voxels");
    if (!(d->dx > 0.0) || !(d->dy > 0.0) || !(d->dz > 0.0))
        return fail(UAM_E_INVALID, "dx, dy, dz must be > 0");
    k->nx = d->nx, k->ny = d->ny, k->nz = d->nz;
    k->x0 = d->x0, k->y_top = d->y_top, k->z0 = d->z0, k->dz = d->dz;
    k->inv_dx = 1.0 / d->dx, k->inv_dy = 1.0 / d->dy, k->inv_dz = 1.0 / d->dz;
    k->vox = nullptr, k->col = nullptr;
    return UAM_OK;
}

// the volume buffer: voxels [ny][nx][nz] 8 B, then (256-B aligned) the column plane 8 B, then
// (256-B aligned) the column bitmap, blocks of 8 x 8 columns doubled until it fits 8 KiB
constexpr int VOL_CBITS_MAX = 8 * 1024 * 8;
int64_t al256(int64_t v) { return (v + 255) & ~(int64_t)255; }
int64_t vol_col_offset(const uam_volume_desc* d) {
    return al256((int64_t)d->nx * d->ny * d->nz * 8);
}
int64_t vol_bits_offset(const uam_volume_desc* d) {
    return vol_col_offset(d) + al256((int64_t)d->nx * d->ny * 8);
}
void vol_bits_dims(const uam_volume_desc* d, KVolume* k) {
    int sh = 3;
    auto nb = [&](int s) {
        return (int64_t)((d->nx + (1 << s) - 1) >> s) * ((d->ny + (1 << s) - 1) >> s);
    };
    while (nb(sh) > VOL_CBITS_MAX) ++sh;
    k->cshift = sh;
    k->cnbx = (d->nx + (1 << sh) - 1) >> sh;
    k->cwords = (int32_t)((nb(sh) + 63) / 64 * 2);  // whole waves of the bitmap kernel
}
}  // namespace

int uam_volume_shape(const uam_volume_desc* vd, int64_t* bytes, int64_t* col_offset) {
    KVolume kv;
    int st = make_kvolume(vd, &kv);
    if (st) return st;
    vol_bits_dims(vd, &kv);
    if (bytes) *bytes = vol_bits_offset(vd) + al256((int64_t)kv.cwords * 4);
    if (col_offset) *col_offset = vol_col_offset(vd);
    return UAM_OK;
}

int uam_volume_build(uam_ctx* ctx, const uam_volume_desc* vd, const void* rec2d,
                     const double* layer_w, void* vol, uam_stream stream) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    KVolume kv;
    int st = make_kvolume(vd, &kv);
    if (st) return st;
    if (!rec2d || !layer_w || !vol) return fail(UAM_E_INVALID, "volume build pointer is NULL");
    DeviceGuard dg(ctx->device);
    if ((uintptr_t)vol & 255) return fail(UAM_E_INVALID, "volume buffer not 256-B aligned");
    const int64_t total = (int64_t)vd->nx * vd->ny * vd->nz;
    hipLaunchKernelGGL(k_volume_build, dim3(grid_for(total, 256)), dim3(256), 0,
                       (hipStream_t)stream, (const uint4*)rec2d, vd->nx, vd->ny, vd->nz,
                       layer_w, (uint2*)vol, (uint2*)((char*)vol + vol_col_offset(vd)));
    vol_bits_dims(vd, &kv);
    const int nblk = kv.cwords * 32;  // whole waves; blocks past the last one are clear
    const int nreal = kv.cnbx * ((vd->ny + (1 << kv.cshift) - 1) >> kv.cshift);
    hipLaunchKernelGGL(k_volume_colbits, dim3(grid_for(nblk, 256)), dim3(256), 0,
                       (hipStream_t)stream, (const uint2*)((char*)vol + vol_col_offset(vd)),
                       vd->nx, vd->ny, kv.cshift, kv.cnbx, nreal, kv.cwords,
                       (uint32_t*)((char*)vol + vol_bits_offset(vd)));
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}

namespace {
// the packed volume's dimensions (uam_volume_pack): 4 x 2-cell blocks, nz layer planes
// [16-B table | 8-B table | code map], 256-B aligned sections
// packed-volume layout (uam_volume_pack), 256-B aligned sections: header (the code map, cwords
// words padded to 16 B; the column terrain's bound table, u16 per bound block of 2^bsh columns,
// at most PK_BOUND_MAX, padded to 16 B; the superblock table, float2 per 4 x 4 bound blocks) |
// scratch (float2 per bound block) | 16-B voxels in 4 x 2-column blocks | 4-B risk in 4 x 8-
// column blocks | 8-B {risk, |psi| | nfz} in the same blocks | the 4-B column terrain in
// 4 x 8-column blocks (one plane)
struct VpkDims {
    int32_t cnbx, cnby, cwords;
    int32_t bsh, bnbx, bnby, nbb, sbnbx, sbnby;
    int32_t hwords, bnd_off, sbt_off;
    int32_t nb8, lnby4;
    int64_t layer;  // i4 entries per layer plane
    int32_t nb4;    // q8: 4 x 4-column blocks per row
    int64_t layer44;
    int32_t nbx4;   // v16: 4 x 2-column blocks per row
    int64_t layer42;
    int64_t off_scr, off_r4, off_t4, off_e8, off_v16, off_q8, bytes;
};
void vpk_dims(const uam_volume_desc* d, VpkDims* v) {
    v->cnbx = (d->nx + (1 << VPK_CSHIFT) - 1) >> VPK_CSHIFT;
    v->cnby = (d->ny + (1 << VPK_CSHIFT) - 1) >> VPK_CSHIFT;
    v->cwords = (v->cnbx * v->cnby + 15) / 16;
    v->bsh = 3;
    auto nblk = [&](int s) {
        return (int64_t)((d->nx + (1 << s) - 1) >> s) * ((d->ny + (1 << s) - 1) >> s);
    };
    while (nblk(v->bsh) > PK_BOUND_MAX) ++v->bsh;
    v->bnbx = (d->nx + (1 << v->bsh) - 1) >> v->bsh;
    v->bnby = (d->ny + (1 << v->bsh) - 1) >> v->bsh;
    v->nbb = v->bnbx * v->bnby;
    v->sbnbx = (v->bnbx + 3) >> 2;
    v->sbnby = (v->bnby + 3) >> 2;
    auto w16 = [](int64_t bytes) { return (int32_t)(((bytes + 15) & ~(int64_t)15) / 4); };
    v->bnd_off = w16((int64_t)v->cwords * 4);
    v->sbt_off = v->bnd_off + w16((int64_t)v->nbb * 2);
    v->hwords = v->sbt_off + w16((int64_t)v->sbnbx * v->sbnby * 8);
    v->nb8 = (d->nx + 7) >> 3;
    v->lnby4 = (d->ny + 3) >> 2;
    v->layer = (int64_t)v->lnby4 * v->nb8 * 32;
    v->off_scr = al256((int64_t)v->hwords * 4);
    v->off_r4 = v->off_scr + al256((int64_t)v->nbb * 8);
    v->off_t4 = v->off_r4 + al256(v->layer * d->nz * 4);
    v->off_e8 = v->off_t4 + al256(v->layer * 4);
    v->off_v16 = v->off_e8 + al256(v->layer * d->nz * 8);
    v->nb4 = (d->nx + 3) >> 2;
    v->layer44 = (int64_t)v->lnby4 * v->nb4 * 16;
    v->nbx4 = (d->nx + 3) >> 2;
    v->layer42 = (int64_t)((d->ny + 1) >> 1) * v->nbx4 * 8;
    v->off_q8 = v->off_v16 + al256(v->layer42 * d->nz * 16);
    v->bytes = v->off_q8 + al256(v->layer44 * d->nz * 8);
}
// the packed volume's view for K4h
void vpk_kvol(const uam_volume_desc* vd, const VpkDims& v, const void* packed, KVol4* kv) {
    const char* b = (const char*)packed;
    kv->nx = vd->nx, kv->ny = vd->ny, kv->nz = vd->nz;
    kv->x0 = vd->x0, kv->y_top = vd->y_top, kv->z0 = vd->z0, kv->dz = vd->dz;
    kv->inv_dx = 1.0 / vd->dx, kv->inv_dy = 1.0 / vd->dy, kv->inv_dz = 1.0 / vd->dz;
    kv->hdr = (const uint32_t*)b;
    kv->hwords = v.hwords, kv->cnbx = v.cnbx, kv->bnd_off = v.bnd_off, kv->sbt_off = v.sbt_off;
    kv->bshift = v.bsh, kv->bnbx = v.bnbx, kv->sbnbx = v.sbnbx;
    kv->nb8 = v.nb8, kv->lnby4 = v.lnby4;
    kv->layer = (uint32_t)std::min(v.layer, (int64_t)UINT32_MAX);
    // K4h's 32-bit offsets and 24-bit products: a copy under 4 GiB, layers under 2^24 entries,
    // columns under 2^24 a side
    const bool o32 = v.bytes <= (int64_t)UINT32_MAX && v.layer < ((int64_t)1 << 24) &&
                     v.layer44 < ((int64_t)1 << 24) && v.layer42 < ((int64_t)1 << 24) &&
                     vd->nx < (1 << 24) && vd->ny < (1 << 24) && vd->nz < (1 << 24);
    kv->pk = o32 ? b : nullptr;
    kv->o4 = (uint32_t)v.off_r4;
    kv->o8 = (uint32_t)v.off_e8;
    kv->o16 = (uint32_t)v.off_v16;
    kv->ot4 = (uint32_t)v.off_t4;
    kv->oq8 = (uint32_t)v.off_q8;
    kv->nbx4 = v.nbx4;
    kv->layer42 = (uint32_t)std::min(v.layer42, (int64_t)UINT32_MAX);
    kv->nb4 = v.nb4;
    kv->layer44 = (uint32_t)std::min(v.layer44, (int64_t)UINT32_MAX);
}
}  // namespace

int uam_volume_packed_bytes(const uam_volume_desc* vd, int64_t* bytes) {
    KVolume kv;
    int st = make_kvolume(vd, &kv);
    if (st) return st;
    if (!bytes) return fail(UAM_E_INVALID, "bytes is NULL");
    VpkDims v;
    vpk_dims(vd, &v);
    *bytes = v.bytes;
    return UAM_OK;
}

int uam_volume_pack(uam_ctx* ctx, const uam_volume_desc* vd, const void* vol, void* packed,
                    uam_stream stream) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    KVolume kv0;
    int st = make_kvolume(vd, &kv0);
    if (st) return st;
    if (!vol || !packed) return fail(UAM_E_INVALID, "volume pack pointer is NULL");
    if (((uintptr_t)vol & 255) || ((uintptr_t)packed & 255))
        return fail(UAM_E_INVALID, "volume buffers not 256-B aligned");
    DeviceGuard dg(ctx->device);
    VpkDims v;
    vpk_dims(vd, &v);
    KVol4 kv{};
    vpk_kvol(vd, v, packed, &kv);
    const uint2* vx = (const uint2*)vol;
    const uint2* cl = (const uint2*)((const char*)vol + vol_col_offset(vd));
    hipStream_t s = (hipStream_t)stream;
    char* b = (char*)packed;
    HIP_TRY(hipMemsetAsync(b, 0, (size_t)v.off_scr, s));  // header padding
    hipLaunchKernelGGL(k_volume_pack_planes, dim3(grid_for(v.layer * vd->nz, 256)), dim3(256), 0,
                       s, vx, cl, kv, (uint32_t*)(b + v.off_r4), (uint2*)(b + v.off_e8),
                       (uint4*)(b + v.off_v16), (uint2*)(b + v.off_q8));
    const int64_t nt4 = (int64_t)v.lnby4 * v.nb8 * 32;
    hipLaunchKernelGGL(k_volume_pack_t4, dim3((unsigned)((nt4 + 255) / 256)), dim3(256), 0, s, cl,
                       kv, (float*)(b + v.off_t4));
    hipLaunchKernelGGL(k_volume_codes, dim3(grid_for(v.cwords, 256)), dim3(256), 0, s, vx, cl,
                       vd->nx, vd->ny, vd->nz, v.cnbx, v.cnbx * v.cnby, v.cwords, (uint32_t*)b);
    hipLaunchKernelGGL(k_t4_bminmax, dim3((unsigned)((v.nbb + 3) / 4)), dim3(256), 0, s,
                       (const float*)(b + v.off_t4), vd->nx, vd->ny, v.nb8, v.bsh, v.bnbx, v.nbb,
                       (float2*)(b + v.off_scr));
    hipLaunchKernelGGL(k_raster_bounds, dim3((unsigned)((v.nbb + 255) / 256)), dim3(256), 0, s,
                       (const float2*)(b + v.off_scr), v.bnbx, v.bnby, v.sbnbx,
                       (uint16_t*)(b + (size_t)v.bnd_off * 4), (float2*)(b + (size_t)v.sbt_off * 4));
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}

static int eval_generated3d_vol(uam_ctx* ctx, const uam_volume_desc* vd, const void* vol,
                                const double* pairs6, int64_t n_pairs, const double* utab,
                                int32_t D, const uam_path_outputs* out, uam_stream stream);

int uam_eval_generated3d(uam_ctx* ctx, const uam_volume_desc* vd, const void* vol,
                         const void* packed, const double* pairs6, int64_t n_pairs,
                         const double* utab, int32_t D, const uam_path_outputs* out,
                         uam_stream stream) {
    if (ctx) {  // an earlier call's failed device check, reported once (uam_device_status)
        const int st = device_status(ctx);
        if (st) return st;
    }
    if (packed) {
        int st = check_ctx(ctx, true);
        if (st) return st;
        if (n_pairs < 0 || D < 1 || D > 16)
            return fail(UAM_E_INVALID, "n_pairs < 0 or D outside [1, 16]");
        if (n_pairs == 0) return UAM_OK;
        KVolume kv0;
        st = make_kvolume(vd, &kv0);
        if (st) return st;
        if (!pairs6 || !utab) return fail(UAM_E_INVALID, "pointer is NULL");
        if ((uintptr_t)packed & 255) return fail(UAM_E_INVALID, "packed volume not 256-B aligned");
        KVol4 kv{};
        VpkDims v;
        vpk_dims(vd, &v);
        vpk_kvol(vd, v, packed, &kv);
        int zs = 0;  // altitude bands: at most 16, or UAM_OPT_K4H_BAND layers each
        if (ctx->k4h_band > 0) {
            while ((1 << zs) < ctx->k4h_band) ++zs;
        }
        while ((vd->nz - 1) >> zs >= 16) ++zs;
        kv.zshift = zs;
        kv.nbands = ((vd->nz - 1) >> zs) + 1;
        const KOut ko = make_kout(out);
        DeviceGuard dg(ctx->device);
        if (!want_wave(ctx, n_pairs * D)) {
            st = launch_grouped3d(ctx, kv, pairs6, n_pairs, utab, D, ko,
                                  out ? out->best_fval_idx : nullptr,
                                  out ? out->best_length_idx : nullptr, (hipStream_t)stream);
            if (st < 0) return st;
            if (st == 1) return UAM_OK;
        }
    }
    return eval_generated3d_vol(ctx, vd, vol, pairs6, n_pairs, utab, D, out, stream);
}

static int eval_generated3d_vol(uam_ctx* ctx, const uam_volume_desc* vd, const void* vol,
                                const double* pairs6, int64_t n_pairs, const double* utab,
                                int32_t D, const uam_path_outputs* out, uam_stream stream) {
    int st = check_ctx(ctx, true);
    if (st) return st;
    if (n_pairs < 0 || D < 1 || D > 16)
        return fail(UAM_E_INVALID, "n_pairs < 0 or D outside [1, 16]");
    if (n_pairs == 0) return UAM_OK;
    KVolume kv;
    st = make_kvolume(vd, &kv);
    if (st) return st;
    if (!vol || !pairs6 || !utab) return fail(UAM_E_INVALID, "pointer is NULL");
    if ((uintptr_t)vol & 255) return fail(UAM_E_INVALID, "volume buffer not 256-B aligned");
    kv.vox = (const uint2*)vol;
    kv.col = (const uint2*)((const char*)vol + vol_col_offset(vd));
    kv.cbits = (const uint32_t*)((const char*)vol + vol_bits_offset(vd));
    vol_bits_dims(vd, &kv);
    const KOut ko = make_kout(out);
    int32_t* best_f = out ? out->best_fval_idx : nullptr;
    int32_t* best_l = out ? out->best_length_idx : nullptr;
    DeviceGuard dg(ctx->device);
    const KRaster kr{};
    ctx->last_kernel = "K4";
    ctx->last_group = 0;
    if (want_wave(ctx, n_pairs * D)) {
        ctx->last_kernel = "K4w";
        st = launch_wave(ctx, UAM_MODE_VOLUME, true, kr, kv, nullptr, nullptr, pairs6, utab, D,
                         n_pairs * D, ko, best_f, best_l, (hipStream_t)stream);
        if (st < 0) return st;
        if (st == 1) return UAM_OK;
    }
    const int64_t blocks = (n_pairs + 63) / 64;
    if (blocks > INT32_MAX) return fail(UAM_E_INVALID, "batch too large");
    const size_t lds = (size_t)64 * D * (6 * sizeof(double) + 3 * sizeof(int32_t)) +
                       (size_t)kv.cwords * 4;
    // the raster pair order over the volume's x/y extent (results do not depend on it)
    const int32_t* order = nullptr;
    if (ctx->pair_order && n_pairs >= 4096 && n_pairs < INT32_MAX) {
        KRaster kxy{};
        kxy.nx = kv.nx, kxy.ny = kv.ny, kxy.x0 = kv.x0, kxy.y_top = kv.y_top;
        kxy.dx = vd->dx, kxy.dy = vd->dy;
        st = raster_pair_order(ctx, kxy, pairs6, n_pairs, (hipStream_t)stream, &order, 1);
        if (st) return st;
    }
    st = ktime_begin(ctx, (hipStream_t)stream);
    if (st) return st;
    hipLaunchKernelGGL((k_eval_pairs<UAM_MODE_VOLUME, 1>), dim3((unsigned)blocks),
                       dim3(64 * D), lds, (hipStream_t)stream, ctx->kg, ctx->kp, kr, kv,
                       nullptr, pairs6, n_pairs, utab, D, ko, best_f, best_l, order);
    HIP_TRY(hipGetLastError());
    st = ktime_end(ctx, (hipStream_t)stream);
    if (st) return st;
    if (order) return order_done(ctx, (hipStream_t)stream);
    return UAM_OK;
}

static int refine_memory(const uam_refine_params* rp) {
    return rp->memory < 0 ? 0 : (rp->memory > RF_MAXM ? RF_MAXM : rp->memory);
}

int64_t uam_refine_workspace_bytes(uam_ctx* ctx, int64_t n_paths,
                                   const uam_refine_params* params) {
    if (!ctx || !ctx->have_params || n_paths < 0 || !params) return -1;
    const int64_t W = ctx->kp.N + 2, m = refine_memory(params);
    // restarts: each path's last waypoints (2W f64) and its still-active flag
    const int64_t rs = params->n_restart > 0 ? 2 * W * (int64_t)sizeof(double) + 4 : 0;
    return ((int64_t)ctx->kg.n_obstacles * W + m * 4 * W) * n_paths * (int64_t)sizeof(double) +
           rs * n_paths;
}

int uam_refine(uam_ctx* ctx, double* wp, int64_t n_paths, const uam_refine_params* rp,
               void* workspace, int64_t workspace_bytes, double* cost, double* infeas,
               int32_t* iters, uam_stream stream) {
    int st = check_ctx(ctx, true);
    if (st) return st;
    if (!rp) return fail(UAM_E_INVALID, "refine params are NULL");
    if (!ctx->kp.penalty_smooth || !ctx->kp.obstacle_smooth)
        return fail(UAM_E_INVALID, "refinement needs penalty_smooth and obstacle_smooth");
    if (n_paths < 0) return fail(UAM_E_INVALID, "n_paths < 0");
    if (rp->n_outer < 0 || rp->n_inner < 0 || rp->max_backtrack < 1 || !(rp->c0 > 0.0) ||
        !(rp->max_step > 0.0) || rp->memory < 0 || rp->memory > RF_MAXM)
        return fail(UAM_E_INVALID, "bad refine params (memory must be 0..%d)", RF_MAXM);
    const int64_t N = ctx->kp.N, W = N + 2;
    if (rp->n_restart < 0 || (rp->n_restart > 0 && (W > 512 || !(rp->restart_margin >= 0.0))))
        return fail(UAM_E_INVALID, "bad restart settings (n_restart >= 0, margin >= 0, W <= 512)");
    const int64_t per_wave =
        (6 * W + 3 * N + 2 * RF_MAXM + rf_mask_words(ctx->kg.n_obstacles) * W) *
        (int64_t)sizeof(double);
    if (per_wave > 65536)
        return fail(UAM_E_INVALID, "N = %lld too large for refinement (LDS)", (long long)N);
    if (n_paths == 0) return UAM_OK;
    const int64_t need = uam_refine_workspace_bytes(ctx, n_paths, rp);
    if (!wp || (need > 0 && !workspace)) return fail(UAM_E_INVALID, "wp/workspace is NULL");
    if (workspace_bytes < need)
        return fail(UAM_E_INVALID, "workspace %lld bytes < %lld", (long long)workspace_bytes,
                    (long long)need);
    const int wpb = (int)std::min<int64_t>(4, 65536 / per_wave);
    const int64_t blocks = (n_paths + wpb - 1) / wpb;
    if (blocks > INT32_MAX) return fail(UAM_E_INVALID, "too many paths");
    KRefine kr{rp->n_outer,  rp->n_inner,   rp->max_backtrack, rp->memory,    rp->c0,
               rp->rho,      rp->c_max,     rp->alpha0,        rp->armijo,    rp->theta,
               rp->max_step, rp->inner_tol, rp->delta,         rp->n_restart, rp->restart_margin};
    DeviceGuard dg(ctx->device);
    const hipStream_t s = (hipStream_t)stream;
    double* zlast = nullptr;
    int32_t* active = nullptr;
    double* cbuf = cost;
    double* ibuf = infeas;
    int32_t* tbuf = iters;
    if (rp->n_restart > 0) {  // restart scratch after the multipliers / L-BFGS rings
        const int64_t base = ((int64_t)ctx->kg.n_obstacles * W + refine_memory(rp) * 4 * W) *
                             n_paths;
        zlast = (double*)workspace + base;
        active = (int32_t*)(zlast + 2 * W * n_paths);
        if (!cbuf || !ibuf || !tbuf)
            return fail(UAM_E_INVALID, "n_restart > 0 needs the cost, infeas and iters outputs");
        HIP_TRY(hipMemsetAsync(active, 0xff, (size_t)n_paths * 4, s));  // all active (-1)
    }
    hipLaunchKernelGGL(k_refine<false>, dim3((unsigned)blocks), dim3(64 * wpb),
                       (size_t)(wpb * per_wave), s, ctx->kg, ctx->kp, kr, wp, n_paths,
                       (double*)workspace, cbuf, ibuf, tbuf, zlast, (const int32_t*)nullptr);
    HIP_TRY(hipGetLastError());
    for (int r = 0; r < rp->n_restart; ++r) {
        hipLaunchKernelGGL(k_rf_push, dim3((unsigned)blocks), dim3(64 * wpb),
                           (size_t)wpb * 2 * W * sizeof(double), s, ctx->kg, ctx->kp, kr,
                           n_paths, zlast, (const double*)ibuf, active);
        hipLaunchKernelGGL(k_refine<true>, dim3((unsigned)blocks), dim3(64 * wpb),
                           (size_t)(wpb * per_wave), s, ctx->kg, ctx->kp, kr, wp, n_paths,
                           (double*)workspace, cbuf, ibuf, tbuf, zlast, (const int32_t*)active);
        HIP_TRY(hipGetLastError());
    }
    return UAM_OK;
}

// ---- CRS (K7) ----------------------------------------------------------------------------
static const double kJprcsOrigin[19][2] = {
    {33.0, 129.5}, {33.0, 131.0}, {36.0, 132.0 + 10.0 / 60}, {33.0, 133.5},
    {36.0, 134.0 + 20.0 / 60}, {36.0, 136.0}, {36.0, 137.0 + 10.0 / 60}, {36.0, 138.5},
    {36.0, 139.0 + 50.0 / 60}, {40.0, 140.0 + 50.0 / 60}, {44.0, 140.25}, {44.0, 142.25},
    {44.0, 144.25}, {26.0, 142.0}, {26.0, 127.5}, {26.0, 124.0}, {26.0, 131.0}, {20.0, 136.0},
    {26.0, 154.0}};

int uam_tm_jprcs(int32_t zone, uam_tm_params* out) {
    if (!out) return fail(UAM_E_INVALID, "out is NULL");
    if (zone < 1 || zone > 19) return fail(UAM_E_INVALID, "JPRCS zone %d outside [1, 19]", zone);
    *out = uam_tm_params{6378137.0, 1.0 / 298.257222101, 0.9999, kJprcsOrigin[zone - 1][0],
                         kJprcsOrigin[zone - 1][1], 0.0, 0.0};
    return UAM_OK;
}

static int make_ktm(const uam_tm_params* t, KTm* k) {
    if (!t) return fail(UAM_E_INVALID, "tm params are NULL");
    if (!(t->a > 0.0) || !(t->f >= 0.0 && t->f < 1.0) || !(t->k0 > 0.0))
        return fail(UAM_E_INVALID, "bad ellipsoid / scale");
    const double n = t->f / (2.0 - t->f), n2 = n * n, n3 = n2 * n, n4 = n3 * n, n5 = n4 * n,
                 n6 = n5 * n;
    k->e2 = t->f * (2.0 - t->f);
    k->e = sqrt(k->e2);
    k->A = t->a / (1.0 + n) * (1.0 + n2 / 4.0 + n4 / 64.0 + n6 / 256.0);
    k->alpha[0] = n / 2 - 2 * n2 / 3 + 5 * n3 / 16 + 41 * n4 / 180 - 127 * n5 / 288 +
                  7891 * n6 / 37800;
    k->alpha[1] = 13 * n2 / 48 - 3 * n3 / 5 + 557 * n4 / 1440 + 281 * n5 / 630 -
                  1983433 * n6 / 1935360;
    k->alpha[2] = 61 * n3 / 240 - 103 * n4 / 140 + 15061 * n5 / 26880 + 167603 * n6 / 181440;
    k->alpha[3] = 49561 * n4 / 161280 - 179 * n5 / 168 + 6601661 * n6 / 7257600;
    k->alpha[4] = 34729 * n5 / 80640 - 3418889 * n6 / 1995840;
    k->alpha[5] = 212378941 * n6 / 319334400;
    k->beta[0] = n / 2 - 2 * n2 / 3 + 37 * n3 / 96 - n4 / 360 - 81 * n5 / 512 +
                 96199 * n6 / 604800;
    k->beta[1] = n2 / 48 + n3 / 15 - 437 * n4 / 1440 + 46 * n5 / 105 - 1118711 * n6 / 3870720;
    k->beta[2] = 17 * n3 / 480 - 37 * n4 / 840 - 209 * n5 / 4480 + 5569 * n6 / 90720;
    k->beta[3] = 4397 * n4 / 161280 - 11 * n5 / 504 - 830251 * n6 / 7257600;
    k->beta[4] = 4583 * n5 / 161280 - 108847 * n6 / 3991680;
    k->beta[5] = 20648693 * n6 / 638668800;
    k->lon0 = t->lon0_deg * (M_PI / 180.0);
    k->k0 = t->k0;
    k->fe = t->false_easting;
    k->fn = t->false_northing;
    const double phi0 = t->lat0_deg * (M_PI / 180.0), s0 = sin(phi0);
    const double tt = sinh(atanh(s0) - k->e * atanh(k->e * s0));
    const double xp = atan2(tt, 1.0);
    double xi = xp;
    for (int j = 0; j < 6; ++j) xi = xi + k->alpha[j] * sin(2.0 * (j + 1) * xp);
    k->xi0 = xi;
    return UAM_OK;
}

static int tm_points(uam_ctx* ctx, const uam_tm_params* t, int inverse, const double* in,
                     int64_t n, double* out, uam_stream stream) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    int st;
    KTm k;
    st = make_ktm(t, &k);
    if (st) return st;
    if (n < 0) return fail(UAM_E_INVALID, "n < 0");
    if (n == 0) return UAM_OK;
    if (!in || !out) return fail(UAM_E_INVALID, "in/out is NULL");
    DeviceGuard dg(ctx->device);
    hipLaunchKernelGGL(k_tm_points, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0,
                       (hipStream_t)stream, k, inverse, in, n, out);
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}

int uam_geo_to_plane(uam_ctx* ctx, const uam_tm_params* t, const double* lonlat, int64_t n,
                     double* xy, uam_stream stream) {
    return tm_points(ctx, t, 0, lonlat, n, xy, stream);
}

int uam_plane_to_geo(uam_ctx* ctx, const uam_tm_params* t, const double* xy, int64_t n,
                     double* lonlat, uam_stream stream) {
    return tm_points(ctx, t, 1, xy, n, lonlat, stream);
}

int uam_reproject_dem(uam_ctx* ctx, const uam_tm_params* t, const float* src,
                      const uam_geo_grid_desc* sg, const uam_raster_desc* dst, double unit_m,
                      int32_t resample, float* out, uam_stream stream) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    int st;
    KTm k;
    st = make_ktm(t, &k);
    if (st) return st;
    if (!sg || !src || !out) return fail(UAM_E_INVALID, "src/grid/out is NULL");
    if (sg->nx < 1 || sg->ny < 1 || !(sg->dlon > 0.0) || !(sg->dlat > 0.0))
        return fail(UAM_E_INVALID, "bad source grid");
    if (resample != 0 && resample != 1) return fail(UAM_E_INVALID, "resample must be 0 or 1");
    if (!(unit_m > 0.0)) return fail(UAM_E_INVALID, "unit_m must be > 0");
    KRaster kr;
    st = make_kraster(dst, &kr);
    if (st) return st;
    const KGeoGrid g{sg->nx, sg->ny, sg->lon0, sg->lat_top, sg->dlon, sg->dlat, sg->nodata};
    const int64_t cells = (int64_t)kr.nx * kr.ny;
    DeviceGuard dg(ctx->device);
    const size_t tab = (size_t)3 * ((size_t)kr.nx + kr.ny);
    if (tab > ctx->tmtab_n) {  // grow-only row / column tables (k_tm_sep)
        if (ctx->d_tmtab) (void)hipFree(ctx->d_tmtab);
        ctx->d_tmtab = nullptr;
        ctx->tmtab_n = 0;
        HIP_TRY(hipMalloc(&ctx->d_tmtab, tab * sizeof(double)));
        ctx->tmtab_n = tab;
    }
    double* rowtab = ctx->d_tmtab;
    double* coltab = rowtab + 3 * (size_t)kr.ny;
    hipLaunchKernelGGL(k_tm_sep, dim3(grid_for((int64_t)kr.nx + kr.ny, 256, INT32_MAX)),
                       dim3(256), 0, (hipStream_t)stream, k, kr, unit_m, rowtab, coltab);
    hipLaunchKernelGGL(k_reproject, dim3(grid_for(cells, 256, INT32_MAX)), dim3(256), 0,
                       (hipStream_t)stream, k, g, kr, unit_m, resample, src,
                       (const double*)rowtab, (const double*)coltab, out);
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}

// ---- DEM polygons (K8) -------------------------------------------------------------------
}  // extern "C"

namespace {

// Device scratch of uam_dem_polygons, served from a grow-only arena the context keeps and
// reset at the start of each call (every use is complete before the call returns).  Freeing
// ~30 stream-ordered buffers per call cost ~2.4 ms at 8192^2; the arena costs nothing.
struct DevArena {
    std::vector<std::pair<char*, size_t>> chunks;
    size_t chunk = 0, used = 0;
    void reset() { chunk = 0, used = 0; }
    void* get(size_t bytes) {
        bytes = (bytes + 255) & ~(size_t)255;
        while (chunk < chunks.size() && used + bytes > chunks[chunk].second) ++chunk, used = 0;
        if (chunk == chunks.size()) {
            const size_t sz = std::max(bytes, (size_t)64 << 20);
            void* p = nullptr;
            if (hipMalloc(&p, sz) != hipSuccess) return nullptr;
            chunks.emplace_back((char*)p, sz);
            used = 0;
        }
        void* p = chunks[chunk].first + used;
        used += bytes;
        return p;
    }
    ~DevArena() {
        for (auto& c : chunks) (void)hipFree(c.first);
    }
};
thread_local DevArena* g_devarena = nullptr;  // the calling context's arena

template <typename T>
struct DevBuf {
    T* p = nullptr;
    int64_t n = 0;
    hipError_t alloc(int64_t count) {
        n = count;
        p = (T*)g_devarena->get((size_t)std::max<int64_t>(count, 1) * sizeof(T));
        return p ? hipSuccess : hipErrorOutOfMemory;
    }
};

#define HIP_TRY2(expr)                                                                    \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(UAM_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));        \
    } while (0)

struct CompStats {
    std::vector<int32_t> cnt, x0, y0, x1, y1, root;
};

// Page-locked host memory for the device -> host copies (so they stay asynchronous), served
// from a grow-only arena the context keeps: pinning and unpinning pages costs milliseconds, so
// chunks are allocated once and reused by later calls.
struct PinnedArena {
    std::vector<std::pair<char*, size_t>> chunks;
    size_t chunk = 0, used = 0;
    void reset() { chunk = 0, used = 0; }
    void* get(size_t bytes) {
        bytes = (bytes + 255) & ~(size_t)255;
        while (chunk < chunks.size() && used + bytes > chunks[chunk].second) ++chunk, used = 0;
        if (chunk == chunks.size()) {
            const size_t sz = std::max(bytes, (size_t)8 << 20);
            void* p = nullptr;
            if (hipHostMalloc(&p, sz) != hipSuccess) return nullptr;
            chunks.emplace_back((char*)p, sz);
            used = 0;
        }
        void* p = chunks[chunk].first + used;
        used += bytes;
        return p;
    }
    ~PinnedArena() {
        for (auto& c : chunks) (void)hipHostFree(c.first);
    }
};
thread_local PinnedArena* g_pinned = nullptr;  // the calling context's arena
void pinned_arena_free(void* a) { delete static_cast<PinnedArena*>(a); }
void dev_arena_free(void* a) { delete static_cast<DevArena*>(a); }

template <typename T>
struct PinnedBuf {
    T* p = nullptr;
    hipError_t alloc(int64_t count) {
        p = (T*)g_pinned->get((size_t)std::max<int64_t>(count, 1) * sizeof(T));
        return p ? hipSuccess : hipErrorOutOfMemory;
    }
};

// Labelling of one grid in three stages, so that several grids can be in flight between two
// host synchronisations (uam_dem_polygons labels all large regions together).
//   1: merge, flatten, per-block root counts (copied to the host)     -- then synchronise
//   2: root ranks from the host prefix, component stats (to the host) -- then synchronise
//   3: unpack the stats
struct GridJob {
    int32_t nx = 0, ny = 0;
    int64_t n = 0, nblk = 0;
    int32_t* L = nullptr;
    int32_t ncomp = 0;
    bool tiled = false;  // tile labelling and the row-segment stats
    uint32_t* rootbits = nullptr;  // tiled: tile-local root bits written by k_ccl_tile
    DevBuf<uint32_t> groots;       // with rootbits: raster-order bitmap of component roots
    DevBuf<int32_t> cnt, off, cid, a;
    PinnedBuf<int32_t> hcnt, hall, hoff;
    CompStats st;
};

// tiled: L holds k_ccl_tile's output (tile-local roots), so only the tile edges are joined
int lg_stage1(GridJob& j, const int32_t* colbox, const int32_t* rowbox, bool runs,
              hipStream_t s, bool tiled = false) {
    j.n = (int64_t)j.nx * j.ny;
    j.tiled = tiled;
    const dim3 g(grid_for(j.n, 256, INT32_MAX)), b(256);
    if (tiled) {
        const int32_t tx = (j.nx + CT_W - 1) / CT_W, ty = (j.ny + CT_H - 1) / CT_H;
        const int64_t nb = (int64_t)(ty - 1) * j.nx + (int64_t)(tx - 1) * j.ny;
        if (nb > 0)
            hipLaunchKernelGGL(k_ccl_bmerge, dim3(grid_for(nb, 256, INT32_MAX)), b, 0, s, j.nx,
                               j.ny, tx, ty, colbox, rowbox, j.L);
        if (j.rootbits) {
            const int64_t nw = (int64_t)tx * ty * (CT_W * CT_H / 32), ngw = (j.n + 31) / 32;
            HIP_TRY2(j.groots.alloc(ngw));
            HIP_TRY2(hipMemsetAsync(j.groots.p, 0, ngw * sizeof(uint32_t), s));
            hipLaunchKernelGGL(k_ccl_flatten_roots, dim3(grid_for(nw, 256, INT32_MAX)), b, 0, s,
                               (const uint32_t*)j.rootbits, nw, j.nx, tx, j.L, j.groots.p);
            hipLaunchKernelGGL(k_ccl_flatten_cells, g, b, 0, s, j.n, j.L);
            j.nblk = (ngw + 255) / 256;
            HIP_TRY2(j.cnt.alloc(j.nblk));
            HIP_TRY2(j.off.alloc(j.nblk));
            HIP_TRY2(j.hcnt.alloc(j.nblk));
            hipLaunchKernelGGL(k_ccl_count_rootbits, dim3((unsigned)j.nblk), b, 0, s,
                               (const uint32_t*)j.groots.p, ngw, j.cnt.p);
            HIP_TRY2(hipGetLastError());
            HIP_TRY2(hipMemcpyAsync(j.hcnt.p, j.cnt.p, j.nblk * sizeof(int32_t),
                                    hipMemcpyDeviceToHost, s));
            return UAM_OK;
        } else {
            hipLaunchKernelGGL(k_ccl_flatten, g, b, 0, s, j.n, j.L);
        }
    } else {
        hipLaunchKernelGGL(k_ccl_merge, g, b, 0, s, j.nx, j.ny, colbox, rowbox, runs ? 1 : 0,
                           j.L);
        hipLaunchKernelGGL(k_ccl_flatten, g, b, 0, s, j.n, j.L);
    }
    j.nblk = (j.n + 256 * CCL_ITEMS - 1) / (256 * CCL_ITEMS);
    HIP_TRY2(j.cnt.alloc(j.nblk));
    HIP_TRY2(j.off.alloc(j.nblk));
    HIP_TRY2(j.hcnt.alloc(j.nblk));
    hipLaunchKernelGGL(k_ccl_count_roots, dim3((unsigned)j.nblk), b, 0, s, j.L, j.n, j.cnt.p);
    HIP_TRY2(hipGetLastError());
    HIP_TRY2(hipMemcpyAsync(j.hcnt.p, j.cnt.p, j.nblk * sizeof(int32_t), hipMemcpyDeviceToHost,
                            s));
    return UAM_OK;
}

int lg_stage2(GridJob& j, hipStream_t s) {
    HIP_TRY2(j.hoff.alloc(j.nblk));
    int64_t acc = 0;
    for (int64_t i = 0; i < j.nblk; ++i) {
        j.hoff.p[i] = (int32_t)acc;
        acc += j.hcnt.p[i];
    }
    j.ncomp = (int32_t)acc;
    const int32_t nc = j.ncomp;
    const dim3 b(256);
    HIP_TRY2(hipMemcpyAsync(j.off.p, j.hoff.p, j.nblk * sizeof(int32_t),
                            hipMemcpyHostToDevice, s));
    HIP_TRY2(j.cid.alloc(j.n));
    if (j.groots.p)
        hipLaunchKernelGGL(k_ccl_assign_rootbits, dim3((unsigned)j.nblk), b, 0, s,
                           (const uint32_t*)j.groots.p, (j.n + 31) / 32, j.off.p, j.cid.p);
    else
        hipLaunchKernelGGL(k_ccl_assign, dim3((unsigned)j.nblk), b, 0, s, j.L, j.n, j.off.p,
                           j.cid.p);
    HIP_TRY2(j.a.alloc(6 * (int64_t)std::max(nc, 1)));
    HIP_TRY2(j.hall.alloc(6 * (int64_t)std::max(nc, 1)));
    if (nc > 0) {
        const dim3 gc(grid_for(nc, 256, INT32_MAX));
        int32_t* p = j.a.p;
        // count 0, x0 / y0 INT32_MAX, x1 / y1 -1 (the root column is written by the stats)
        hipLaunchKernelGGL(k_fill_segs_i32, gc, b, 0, s, p, (int64_t)nc, 5,
                           FillSegs{{0, INT32_MAX, INT32_MAX, -1, -1, 0}});
        if (j.tiled)
            hipLaunchKernelGGL(k_ccl_stats_rows,
                               dim3((unsigned)((j.nx + CS_SEG - 1) / CS_SEG),
                                    (unsigned)((j.ny + CS_ROWS - 1) / CS_ROWS)),
                               b, 0, s, j.L, j.cid.p, j.nx, j.ny, p, p + nc, p + 2 * (int64_t)nc,
                               p + 3 * (int64_t)nc, p + 4 * (int64_t)nc, p + 5 * (int64_t)nc);
        else
            hipLaunchKernelGGL(k_ccl_stats, dim3((unsigned)j.nblk), b, 0, s, j.L, j.cid.p, j.nx,
                               j.n, p, p + nc, p + 2 * (int64_t)nc, p + 3 * (int64_t)nc,
                               p + 4 * (int64_t)nc, p + 5 * (int64_t)nc);
        HIP_TRY2(hipGetLastError());
        HIP_TRY2(hipMemcpyAsync(j.hall.p, j.a.p, 6 * (int64_t)nc * sizeof(int32_t),
                                hipMemcpyDeviceToHost, s));
    }
    return UAM_OK;
}

void lg_stage3(GridJob& j) {
    const int64_t nc = j.ncomp;
    auto col = [&](int k) {
        return std::vector<int32_t>(j.hall.p + k * nc, j.hall.p + (k + 1) * nc);
    };
    j.st.cnt = col(0), j.st.x0 = col(1), j.st.y0 = col(2), j.st.x1 = col(3), j.st.y1 = col(4);
    j.st.root = col(5);
}

// label a grid and return its component stats (synchronises twice)
int label_grid(GridJob& j, const int32_t* colbox, const int32_t* rowbox, bool runs,
               hipStream_t s, bool tiled = false) {
    int rc = lg_stage1(j, colbox, rowbox, runs, s, tiled);
    if (rc) return rc;
    HIP_TRY2(hipStreamSynchronize(s));
    rc = lg_stage2(j, s);
    if (rc) return rc;
    HIP_TRY2(hipStreamSynchronize(s));
    lg_stage3(j);
    return UAM_OK;
}

// per-row [xmin, xmax] of the selected components (sel[c] true), row tables concatenated:
// stage 1 launches and queues the copy back, stage 2 (after a synchronisation) unpacks
struct ExtJob {
    std::vector<int64_t> off;
    int64_t rows = 0;
    DevBuf<int32_t> dtab, dmn;  // dtab: int64 row offsets [ncomp], int32 first rows [ncomp]
    PinnedBuf<int32_t> htab, hmn;
    std::vector<int32_t> xmin, xmax;
};

int ext_stage1(ExtJob& e, int32_t nx, int32_t ny, const int32_t* L, const int32_t* cid,
               const CompStats& st, const std::vector<char>& sel, hipStream_t s,
               bool tiled = false) {
    const int32_t ncomp = (int32_t)st.cnt.size();
    e.off.assign(ncomp, -1);
    e.rows = 0;
    for (int32_t c = 0; c < ncomp; ++c)
        if (sel[c]) {
            e.off[c] = e.rows;
            e.rows += st.y1[c] - st.y0[c] + 1;
        }
    if (e.rows == 0) return UAM_OK;
    // row offsets (int64) then first rows (int32), staged in pinned memory: one upload
    HIP_TRY2(e.dtab.alloc(3 * (int64_t)ncomp));
    HIP_TRY2(e.htab.alloc(3 * (int64_t)ncomp));
    std::memcpy(e.htab.p, e.off.data(), ncomp * sizeof(int64_t));
    std::memcpy(e.htab.p + 2 * (int64_t)ncomp, st.y0.data(), ncomp * sizeof(int32_t));
    HIP_TRY2(e.dmn.alloc(2 * e.rows));
    HIP_TRY2(e.hmn.alloc(2 * e.rows));
    HIP_TRY2(hipMemcpyAsync(e.dtab.p, e.htab.p, 3 * (int64_t)ncomp * sizeof(int32_t),
                            hipMemcpyHostToDevice, s));
    const int64_t* doff = reinterpret_cast<const int64_t*>(e.dtab.p);
    const int32_t* dy0 = e.dtab.p + 2 * (int64_t)ncomp;
    const dim3 gr(grid_for(e.rows, 256, INT32_MAX)), b(256);
    hipLaunchKernelGGL(k_fill_segs_i32, gr, b, 0, s, e.dmn.p, e.rows, 2,
                       FillSegs{{INT32_MAX, -1, 0, 0, 0, 0}});
    const int64_t n = (int64_t)nx * ny;
    if (tiled && ny <= 65535)
        hipLaunchKernelGGL(k_ccl_extents_rows,
                           dim3((unsigned)((nx + CS_SEG - 1) / CS_SEG), (unsigned)ny), b, 0, s, L,
                           cid, nx, doff, dy0, e.dmn.p, e.dmn.p + e.rows);
    else
        hipLaunchKernelGGL(k_ccl_extents, dim3(grid_for(n, 256, INT32_MAX)), b, 0, s, L, cid, nx,
                           n, doff, dy0, e.dmn.p, e.dmn.p + e.rows);
    HIP_TRY2(hipGetLastError());
    HIP_TRY2(hipMemcpyAsync(e.hmn.p, e.dmn.p, 2 * e.rows * sizeof(int32_t),
                            hipMemcpyDeviceToHost, s));
    return UAM_OK;
}

void ext_stage2(ExtJob& e) {
    e.xmin.assign(e.hmn.p, e.hmn.p + e.rows);
    e.xmax.assign(e.hmn.p + e.rows, e.hmn.p + 2 * e.rows);
}

// hull input of one labelled region: each row's [xmin, xmax] run contributes its four pixel
// corners (column c spans [xlo[c], xhi[c]], row r spans [ylo[r], yhi[r]]).  Of the corners at
// one float32 y only the smallest and largest x can be hull vertices, and of those only the
// convex left / right chains; the hull's orientation test is exact on these float32
// coordinates, so this O(rows) filter leaves the hull -- and cv2.minAreaRect -- unchanged
// while the sort inside it sees a few dozen points instead of 4 per row
void region_corners(int32_t ry0, int32_t ry1, const int32_t* xmin, const int32_t* xmax,
                    const std::vector<double>& xlo, const std::vector<double>& xhi,
                    const std::vector<double>& ylo, const std::vector<double>& yhi,
                    std::vector<uampoly::Pt>& pts) {
    struct Lvl {
        float y, lo, hi;
    };
    thread_local std::vector<Lvl> lv;
    thread_local std::vector<uampoly::Pt> ch;
    lv.clear();
    auto add = [&](double y, double lo, double hi) {
        const float fy = (float)y, fl = (float)lo, fh = (float)hi;
        if (!lv.empty() && lv.back().y == fy) {
            lv.back().lo = std::min(lv.back().lo, fl);
            lv.back().hi = std::max(lv.back().hi, fh);
        } else {
            lv.push_back({fy, fl, fh});
        }
    };
    for (int32_t r = ry0; r <= ry1; ++r) {
        const int32_t a = xmin[r - ry0], b = xmax[r - ry0];
        if (a > b) continue;
        add(yhi[r], xlo[a], xhi[b]);
        add(ylo[r], xlo[a], xhi[b]);
    }
    // same predicate as the hull's: double arithmetic on float32 inputs
    auto cross = [](const uampoly::Pt& o, const uampoly::Pt& a, const uampoly::Pt& b) {
        return (a.x - o.x) * (b.y - o.y) - (a.y - o.y) * (b.x - o.x);
    };
    auto chain = [&](bool left) {
        ch.clear();
        const int64_t m = (int64_t)lv.size();
        for (int64_t i = 0; i < m; ++i) {
            const Lvl& e = lv[left ? i : m - 1 - i];  // left: top -> bottom, right: bottom -> top
            const uampoly::Pt p{(double)(left ? e.lo : e.hi), (double)e.y};
            while (ch.size() >= 2 && cross(ch[ch.size() - 2], ch.back(), p) <= 0) ch.pop_back();
            ch.push_back(p);
        }
        pts.insert(pts.end(), ch.begin(), ch.end());
    };
    pts.clear();
    chain(true);
    chain(false);
}

void emit_rect(const std::vector<uampoly::Pt>& pts, double min_approx,
               std::vector<int64_t>& out) {
    int64_t box[8];
    if (!uampoly::min_area_rect_box(pts, box)) return;
    if (!(uampoly::box_area(box) > min_approx)) return;
    out.insert(out.end(), box, box + 8);
}

}  // namespace

extern "C" {

int uam_dem_polygons(uam_ctx* ctx, const float* dem, const uam_raster_desc* rd, float threshold,
                     double unit_m, const uam_polyproc_params* prm, int64_t* rect_xy,
                     int32_t max_rects, int32_t* n_rects, uam_stream stream) {
    if (!ctx || !dem || !rd || !prm || !n_rects) return fail(UAM_E_INVALID, "NULL argument");
    if (rd->nx <= 0 || rd->ny <= 0) return fail(UAM_E_INVALID, "raster size %dx%d", rd->nx, rd->ny);
    if (!(unit_m > 0.0) || prm->divisions < 1) return fail(UAM_E_INVALID, "bad unit / divisions");
    const int32_t nx = rd->nx, ny = rd->ny;
    const int64_t n = (int64_t)nx * ny;
    if (n >= INT32_MAX) return fail(UAM_E_INVALID, "raster too large for int32 labels");
    // plane metres of pixel corners, as an affine geotransform in metres gives them
    const double X0 = rd->x0 * unit_m, DX = rd->dx * unit_m, Y0 = rd->y_top * unit_m,
                 DY = rd->dy * unit_m;
    DeviceGuard dg(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    if (!ctx->pinned) ctx->pinned = new (std::nothrow) PinnedArena();
    if (!ctx->devarena) ctx->devarena = new (std::nothrow) DevArena();
    if (!ctx->pinned || !ctx->devarena) return fail(UAM_E_NOMEM, "K8 arenas");
    g_pinned = (PinnedArena*)ctx->pinned;
    g_pinned->reset();
    g_devarena = (DevArena*)ctx->devarena;
    g_devarena->reset();
    DevBuf<int32_t> L;
    HIP_TRY2(L.alloc(n));
    const bool tiled = ctx->k8_tiled;
    auto tiles = [](int32_t w, int32_t h) {
        return dim3((unsigned)((w + CT_W - 1) / CT_W), (unsigned)((h + CT_H - 1) / CT_H));
    };
    GridJob mj;
    DevBuf<uint32_t> mbits;
    if (tiled) {
        const dim3 tg = tiles(nx, ny);
        HIP_TRY2(mbits.alloc((int64_t)tg.x * tg.y * (CT_W * CT_H / 32)));
        mj.rootbits = mbits.p;
        hipLaunchKernelGGL(k_ccl_tile<CclMaskDem>, tiles(nx, ny), dim3(256), 0, s,
                           CclMaskDem{dem, threshold, nx}, nx, ny, nullptr, nullptr, L.p,
                           mbits.p);
    } else
        hipLaunchKernelGGL(k_ccl_init_dem, dim3(grid_for(n, 256, INT32_MAX)), dim3(256), 0, s,
                           dem, n, nx, threshold, L.p);
    mj.nx = nx, mj.ny = ny, mj.L = L.p;
    int rc = label_grid(mj, nullptr, nullptr, true, s, tiled);
    if (rc) return rc;
    const CompStats& st = mj.st;
    const int32_t ncomp = (int32_t)st.cnt.size();
    const double cell = std::fabs(DX * DY);
    std::vector<char> small(ncomp, 0), large(ncomp, 0);
    for (int32_t c = 0; c < ncomp; ++c) {
        const double area = st.cnt[c] * cell;
        if (!(area > prm->min_area)) continue;
        (area > prm->large_area ? large : small)[c] = 1;
    }
    ExtJob me;
    rc = ext_stage1(me, nx, ny, L.p, mj.cid.p, st, small, s, tiled);
    if (rc) return rc;
    std::vector<double> xlo(nx), xhi(nx), ylo(ny), yhi(ny);
    for (int32_t i = 0; i < nx; ++i) xlo[i] = X0 + i * DX, xhi[i] = X0 + (i + 1) * DX;
    for (int32_t j = 0; j < ny; ++j) yhi[j] = Y0 - j * DY, ylo[j] = Y0 - (j + 1) * DY;
    // Large regions (data_processor.py:34-51: D x D boxes over polygon.bounds; a piece =
    // connected part of polygon n box = component of the region's grid refined at the box
    // edges, cut there).  All of them are labelled together, three synchronisations in all.
    struct Region {
        int32_t c = 0, ws = 0, hs = 0;
        std::vector<int32_t> col_of, colbox, row_of, rowbox;
        std::vector<double> sxlo, sxhi, sylo, syhi;
        DevBuf<int32_t> tab, L2;  // col_of, colbox [ws]; row_of, rowbox [hs]
        PinnedBuf<int32_t> htab;
        const int32_t *dco = nullptr, *dcb = nullptr, *dro = nullptr, *drb = nullptr;
        DevBuf<uint32_t> bits;
        GridJob job;
        ExtJob ext;
    };
    std::vector<Region> regs;  // reserved: a Region's buffers must never be copied
    regs.reserve(std::count(large.begin(), large.end(), (char)1));
    for (int32_t c = 0; c < ncomp; ++c)
        if (large[c]) {
            regs.emplace_back();
            regs.back().c = c;
        }
    const int D = prm->divisions;
    // the regions are independent: region k runs on stream k mod NS (the caller's stream and
    // NS - 1 side streams), so their small launches and tails overlap.  The main labels they
    // read are complete (label_grid synchronised s).
    const int NS = std::max(1, std::min<int>(ctx->k8_nstreams, (int)regs.size()));
    for (int k = 0; k + 1 < NS; ++k)
        if (!ctx->k8s[k]) HIP_TRY2(hipStreamCreateWithFlags(&ctx->k8s[k], hipStreamNonBlocking));
    auto rstream = [&](size_t k) { return k % NS == 0 ? s : ctx->k8s[k % NS - 1]; };
    auto sync_all = [&]() -> hipError_t {
        for (int k = 0; k < NS; ++k) {
            const hipError_t e = hipStreamSynchronize(k == 0 ? s : ctx->k8s[k - 1]);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    };
    // an early error return must not leave side-stream work reading the arenas, which the
    // next call reuses: drain every stream on the way out (idle streams return at once)
    struct Drain {
        std::function<hipError_t()> f;
        ~Drain() { (void)f(); }
    } drain{sync_all};
    for (size_t ri = 0; ri < regs.size(); ++ri) {
        Region& r = regs[ri];
        const hipStream_t rs = rstream(ri);
        const int32_t c = r.c;
        const double minx = X0 + st.x0[c] * DX, maxx = X0 + (st.x1[c] + 1) * DX;
        const double maxy = Y0 - st.y0[c] * DY, miny = Y0 - (st.y1[c] + 1) * DY;
        const double ddx = (maxx - minx) / D, ddy = (maxy - miny) / D;
        for (int32_t col = st.x0[c]; col <= st.x1[c]; ++col)
            for (int j = 0; j < D; ++j) {
                const double lo = std::max(xlo[col], minx + j * ddx);
                const double hi = std::min(xhi[col], minx + (j + 1) * ddx);
                if (hi > lo) {
                    r.col_of.push_back(col), r.colbox.push_back(j);
                    r.sxlo.push_back(lo), r.sxhi.push_back(hi);
                }
            }
        for (int32_t row = st.y0[c]; row <= st.y1[c]; ++row)
            for (int k = D - 1; k >= 0; --k) {
                const double lo = std::max(ylo[row], miny + k * ddy);
                const double hi = std::min(yhi[row], miny + (k + 1) * ddy);
                if (hi > lo) {
                    r.row_of.push_back(row), r.rowbox.push_back(k);
                    r.sylo.push_back(lo), r.syhi.push_back(hi);
                }
            }
        r.ws = (int32_t)r.col_of.size(), r.hs = (int32_t)r.row_of.size();
        const int64_t sn = (int64_t)r.ws * r.hs;
        const int64_t nt = 2 * (int64_t)r.ws + 2 * (int64_t)r.hs;
        HIP_TRY2(r.tab.alloc(nt));
        HIP_TRY2(r.htab.alloc(nt));
        HIP_TRY2(r.L2.alloc(sn));
        int32_t* h = r.htab.p;
        std::copy(r.col_of.begin(), r.col_of.end(), h);
        std::copy(r.colbox.begin(), r.colbox.end(), h + r.ws);
        std::copy(r.row_of.begin(), r.row_of.end(), h + 2 * (int64_t)r.ws);
        std::copy(r.rowbox.begin(), r.rowbox.end(), h + 2 * (int64_t)r.ws + r.hs);
        HIP_TRY2(hipMemcpyAsync(r.tab.p, h, nt * sizeof(int32_t), hipMemcpyHostToDevice, rs));
        r.dco = r.tab.p, r.dcb = r.tab.p + r.ws, r.dro = r.tab.p + 2 * (int64_t)r.ws;
        r.drb = r.dro + r.hs;
        if (tiled) {
            const dim3 tg = tiles(r.ws, r.hs);
            HIP_TRY2(r.bits.alloc((int64_t)tg.x * tg.y * (CT_W * CT_H / 32)));
            r.job.rootbits = r.bits.p;
            hipLaunchKernelGGL(k_ccl_tile<CclMaskSub>, tiles(r.ws, r.hs), dim3(256), 0, rs,
                               CclMaskSub{L.p, nx, st.root[c], r.dco, r.dro}, r.ws, r.hs, r.dcb,
                               r.drb, r.L2.p, r.bits.p);
        } else
            hipLaunchKernelGGL(k_ccl_init_sub, dim3(grid_for(sn, 256, INT32_MAX)), dim3(256), 0,
                               rs, L.p, nx, st.root[c], r.dco, r.dro, r.dcb, r.ws, r.hs,
                               r.L2.p);
        r.job.nx = r.ws, r.job.ny = r.hs, r.job.L = r.L2.p;
        rc = lg_stage1(r.job, r.dcb, r.drb, true, rs, tiled);
        if (rc) return rc;
    }
    HIP_TRY2(sync_all());  // main extents, every region's root counts
    ext_stage2(me);
    for (size_t ri = 0; ri < regs.size(); ++ri) {
        rc = lg_stage2(regs[ri].job, rstream(ri));
        if (rc) return rc;
    }
    // the small regions' rectangles (host) while the GPU labels the large ones
    std::vector<int64_t> small_out;
    std::vector<int64_t> small_at(ncomp + 1, 0);  // component c: small_out[small_at[c], [c+1])
    std::vector<uampoly::Pt> pts;
    for (int32_t c = 0; c < ncomp; ++c) {
        if (small[c]) {
            region_corners(st.y0[c], st.y1[c], &me.xmin[me.off[c]], &me.xmax[me.off[c]], xlo,
                           xhi, ylo, yhi, pts);
            emit_rect(pts, prm->min_approx_area, small_out);
        }
        small_at[c + 1] = (int64_t)small_out.size();
    }
    HIP_TRY2(sync_all());  // every region's component stats
    for (size_t ri = 0; ri < regs.size(); ++ri) {
        Region& r = regs[ri];
        lg_stage3(r.job);
        const std::vector<char> all(r.job.st.cnt.size(), 1);
        rc = ext_stage1(r.ext, r.ws, r.hs, r.L2.p, r.job.cid.p, r.job.st, all, rstream(ri),
                        tiled);
        if (rc) return rc;
    }
    HIP_TRY2(sync_all());  // every region's row extents
    // rectangles in component order (small: the region; large: its pieces, boxes j (x) outer,
    // k (y) inner -- the reference's order)
    // a large region's pieces are independent host work: up to 8 worker threads take regions
    // in turn (the helpers keep their scratch thread_local); joined in component order below
    std::vector<std::vector<int64_t>> rout(regs.size());
    std::atomic<size_t> next{0};
    auto worker = [&] {
        std::vector<uampoly::Pt> rp;
        for (size_t k; (k = next.fetch_add(1)) < regs.size();) {
            Region& r = regs[k];
            ext_stage2(r.ext);
            const CompStats& ps = r.job.st;
            const int32_t np = (int32_t)ps.cnt.size();
            std::vector<int32_t> order(np);
            for (int32_t i = 0; i < np; ++i) order[i] = i;
            std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
                const int ja = r.colbox[ps.x0[a]], jb = r.colbox[ps.x0[b]];
                if (ja != jb) return ja < jb;
                return r.rowbox[ps.y0[a]] < r.rowbox[ps.y0[b]];
            });
            for (int32_t i : order) {
                region_corners(ps.y0[i], ps.y1[i], &r.ext.xmin[r.ext.off[i]],
                               &r.ext.xmax[r.ext.off[i]], r.sxlo, r.sxhi, r.sylo, r.syhi, rp);
                emit_rect(rp, prm->min_approx_area, rout[k]);
            }
        }
    };
    {
        std::vector<std::thread> pool;
        for (size_t k = 1; k < std::min<size_t>(regs.size(), 8); ++k) pool.emplace_back(worker);
        worker();
        for (auto& t : pool) t.join();
    }
    std::vector<int64_t> out;
    out.reserve(small_out.size());
    size_t ri = 0;
    for (int32_t c = 0; c < ncomp; ++c) {
        if (small[c]) {
            out.insert(out.end(), small_out.begin() + small_at[c],
                       small_out.begin() + small_at[c + 1]);
        } else if (large[c]) {
            out.insert(out.end(), rout[ri].begin(), rout[ri].end());
            ++ri;
        }
    }
    const int64_t nr = (int64_t)out.size() / 8;
    *n_rects = (int32_t)nr;
    if (rect_xy)
        for (int64_t i = 0; i < std::min<int64_t>(nr, max_rects) * 8; ++i) rect_xy[i] = out[i];
    if (nr > max_rects)
        return fail(UAM_E_INVALID, "%lld rectangles > max_rects %d", (long long)nr, max_rects);
    return UAM_OK;
}

int uam_argmin(uam_ctx* ctx, const double* values, int64_t groups, int32_t G, int32_t take_sqrt,
               int32_t* best, uam_stream stream) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    if (groups < 0 || G < 1) return fail(UAM_E_INVALID, "groups < 0 or G < 1");
    if (groups == 0) return UAM_OK;
    if (!values || !best) return fail(UAM_E_INVALID, "pointer is NULL");
    DeviceGuard dg(ctx->device);
    hipLaunchKernelGGL(k_argmin, dim3(grid_for(groups, 256, INT32_MAX)), dim3(256), 0,
                       (hipStream_t)stream, values, groups, G, take_sqrt, best);
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}

int uam_path_length(uam_ctx* ctx, const double* pts, int64_t n_paths, int32_t n_points,
                    int32_t n_segments, int32_t smooth, double* out, uam_stream stream) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    if (n_paths < 0 || n_points < 1 || n_segments < 0 || n_segments > n_points - 1)
        return fail(UAM_E_INVALID, "bad sizes n_points=%d n_segments=%d", n_points, n_segments);
    if (n_paths == 0) return UAM_OK;
    if (!pts || !out) return fail(UAM_E_INVALID, "pointer is NULL");
    DeviceGuard dg(ctx->device);
    hipLaunchKernelGGL(k_path_length, dim3(grid_for(n_paths, 256, INT32_MAX)), dim3(256), 0,
                       (hipStream_t)stream, pts, n_paths, n_points, n_segments, smooth, out);
    HIP_TRY(hipGetLastError());
    return UAM_OK;
}


int uam_synchronize(uam_ctx* ctx, uam_stream stream) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    DeviceGuard dg(ctx->device);
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return device_status(ctx);
}

int uam_device_status(uam_ctx* ctx) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    return device_status(ctx);
}

}  // extern "C"

// ---- raster broadcast over RCCL (one broadcast of the record raster, no
// collective in the hot loop).  RCCL is bound at run time (dlopen): the soname librccl.so.1 that
// torch already loaded is reused (one RCCL per process), else the system one; the library loads
// and runs single-GPU work without it.
namespace {
struct Rccl {
    bool tried = false, ok = false;
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclBroadcast) bcast = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
};

Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        r.tried = true;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        r.get_id = (decltype(r.get_id))dlsym(h, "ncclGetUniqueId");
        r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
        r.init_all = (decltype(r.init_all))dlsym(h, "ncclCommInitAll");
        r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
        r.bcast = (decltype(r.bcast))dlsym(h, "ncclBroadcast");
        r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
        r.err = (decltype(r.err))dlsym(h, "ncclGetErrorString");
        r.ok = r.get_id && r.init_rank && r.init_all && r.destroy && r.bcast && r.group_start &&
               r.group_end && r.err;
    });
    return r;
}

#define RCCL_TRY(expr)                                                                     \
    do {                                                                                   \
        ncclResult_t r_ = (expr);                                                          \
        if (r_ != ncclSuccess) return fail(UAM_E_HIP, "%s: %s", #expr, rccl().err(r_));    \
    } while (0)

int need_rccl() {
    return rccl().ok ? UAM_OK : fail(UAM_E_STATE, "RCCL (librccl.so.1) could not be loaded");
}
}  // namespace

static void comm_release(uam_ctx* ctx) {
    if (ctx->comm && rccl().ok) (void)rccl().destroy((ncclComm_t)ctx->comm);
    ctx->comm = nullptr;
}

extern "C" {

int uam_comm_unique_id(uint8_t* id) {
    if (!id) return fail(UAM_E_INVALID, "id is NULL");
    int st = need_rccl();
    if (st) return st;
    ncclUniqueId u;
    RCCL_TRY(rccl().get_id(&u));
    std::memcpy(id, u.internal, UAM_COMM_ID_BYTES);
    return UAM_OK;
}

int uam_comm_init(uam_ctx* ctx, const uint8_t* id, int32_t nranks, int32_t rank) {
    if (!ctx || !id) return fail(UAM_E_INVALID, "ctx/id is NULL");
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return fail(UAM_E_INVALID, "rank %d of %d", rank, nranks);
    int st = need_rccl();
    if (st) return st;
    DeviceGuard dg(ctx->device);
    comm_release(ctx);
    ncclUniqueId u;
    std::memcpy(u.internal, id, UAM_COMM_ID_BYTES);
    ncclComm_t c = nullptr;
    RCCL_TRY(rccl().init_rank(&c, nranks, u, rank));
    ctx->comm = c;
    return UAM_OK;
}

int uam_comm_destroy(uam_ctx* ctx) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    DeviceGuard dg(ctx->device);
    comm_release(ctx);
    return UAM_OK;
}

int uam_bcast_raster(uam_ctx* ctx, void* buf, int64_t bytes, int32_t root, uam_stream stream) {
    if (!ctx) return fail(UAM_E_INVALID, "ctx is NULL");
    if (!ctx->comm) return fail(UAM_E_STATE, "uam_comm_init has not been called");
    if (bytes < 0 || (bytes > 0 && !buf)) return fail(UAM_E_INVALID, "bad broadcast buffer");
    if (bytes == 0) return UAM_OK;
    DeviceGuard dg(ctx->device);
    RCCL_TRY(rccl().bcast(buf, buf, (size_t)bytes, ncclChar, root, (ncclComm_t)ctx->comm,
                          (hipStream_t)stream));
    return UAM_OK;
}

int uam_bcast_raster_group(uam_ctx** ctxs, void** bufs, int32_t n, int64_t bytes, int32_t root,
                           uam_stream* streams) {
    if (!ctxs || !bufs || n < 1) return fail(UAM_E_INVALID, "bad context list");
    if (root < 0 || root >= n) return fail(UAM_E_INVALID, "root %d of %d", root, n);
    if (bytes < 0) return fail(UAM_E_INVALID, "bytes < 0");
    int st = need_rccl();
    if (st) return st;
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i] || (bytes > 0 && !bufs[i])) return fail(UAM_E_INVALID, "context %d", i);
        devs[i] = ctxs[i]->device;
    }
    std::vector<ncclComm_t> comms(n, nullptr);
    {
        DeviceGuard dg(devs[0]);
        RCCL_TRY(rccl().init_all(comms.data(), n, devs.data()));
    }
    for (int i = 0; i < n; ++i) {
        comm_release(ctxs[i]);
        ctxs[i]->comm = comms[i];
    }
    if (bytes == 0) return UAM_OK;
    DeviceGuard dg(devs[0]);
    RCCL_TRY(rccl().group_start());
    for (int i = 0; i < n; ++i) {
        if (hipSetDevice(devs[i]) != hipSuccess) {
            (void)rccl().group_end();
            return fail(UAM_E_HIP, "hipSetDevice(%d)", devs[i]);
        }
        const ncclResult_t r = rccl().bcast(bufs[i], bufs[i], (size_t)bytes, ncclChar, root,
                                            comms[i], streams ? (hipStream_t)streams[i] : nullptr);
        if (r != ncclSuccess) {
            (void)rccl().group_end();
            return fail(UAM_E_HIP, "ncclBroadcast: %s", rccl().err(r));
        }
    }
    RCCL_TRY(rccl().group_end());
    return UAM_OK;
}

}  // extern "C"

