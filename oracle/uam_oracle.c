/*
 * uam_oracle.c -- CPU restatement of the uam_path_planning hot path.
 *
 * TEST INFRASTRUCTURE, NOT PRODUCT.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load this library, and only as the checker / the timed CPU baseline.
 * The product (uam_path_planning_amd, libuampath.so) never links or calls it.
 *
 * Parity pinning: tests/test_oracle_golden.py checks this file against golden vectors that
 * tests/golden/make_golden.py recorded by running the reference's own cost model
 * (geo_simulation_project/path_generation/ *.py) under a numeric casadi stand-in.
 *
 * Every routine restates, in plain float64 C with the reference's operation order, one
 * reference function (file:line relative to /root/reference/geo_simulation_project/):
 *   ineq_h          polygon.py:69-71,98  ball.py:33-37(func)  square.py:29-52(right/left/top/bottom)
 *   psi             path_generation/quadratic_obstacle.py:27-39  (penalty_function)
 *   contains        path_generation/quadratic_obstacle.py:89-94, map.py:41-43 (collides)
 *   region_penalty  path_generation/problem.py:59-82 (get_penalty_function)
 *   total_penalty   path_generation/problem.py:49-56 (get_total_penalty_function)
 *   path loop       path_generation/problem.py:38-44 (get_cost), 84-114 (get_nonlincon),
 *                   130-146 (length_of)
 *   orc_gen_paths   path_generation/solver.py:103-136 (create_x_init, restated through a
 *                   host-computed unit-arc table)
 *   orc_raster_build  map_generation/data_manager.py:14-17 (DEM mask) + the penalty above at
 *                   cell centres (the build's raster mode)
 *   orc_argmin      path_generation/main.py:175-180 (strict <, first index wins)
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_HALFPLANE 0
#define ORC_ELLIPSE 1
#define ORC_AXIS 2

#define ORC_MAX_REGIONS 16

#define ORC_FLAG_NFZ 1u
#define ORC_FLAG_MASK 2u
#define ORC_FLAG_NODATA 4u

typedef struct {
    int32_t n_ineq;
    const int32_t* ineq_kind;    /* [n_ineq] */
    const double* ineq_par;      /* [n_ineq][6] */
    int32_t n_shapes;            /* obstacles first, then regions region-major */
    const int32_t* shape_first;  /* [n_shapes] index into ineq */
    const int32_t* shape_count;  /* [n_shapes] */
    const double* shape_center;  /* [n_shapes][2]; NaN => no normalisation */
    int32_t n_obstacles;         /* shapes [0, n_obstacles) are no-fly obstacles */
    int32_t n_regions;
    const int32_t* region_first; /* [n_regions+1] shape offsets */
} orc_geom;

typedef struct {
    int32_t N;
    int32_t length_smooth, penalty_smooth, obstacle_smooth, maxratio_smooth;
    int32_t quirk_length;        /* 1: get_cost length term as the reference computes it */
    int32_t anchor_mode;         /* 0: anchor = path's own p_0; 1: (anchor_x, anchor_y) */
    int32_t pad_;
    double anchor_x, anchor_y;
    double maxratio, maxalpha, enlargement;
    double altitude;
    double weights[ORC_MAX_REGIONS];
} orc_params;

typedef struct {
    int32_t nx, ny;
    double x0, y_top, dx, dy;
    float nodata, dem_threshold;
} orc_raster;

/* ---- geometry ------------------------------------------------------------------------ */

static double ineq_h(const orc_geom* g, int i, double x0, double x1) {
    const double* p = g->ineq_par + 6 * (int64_t)i;
    switch (g->ineq_kind[i]) {
        case ORC_HALFPLANE: {
            /* polygon.py:69-71: (Pb_y-Pa_y)*(x0-Pa_x) - (Pb_x-Pa_x)*(x1-Pa_y); h = -sgn*line */
            double line = p[3] * (x0 - p[0]) - p[2] * (x1 - p[1]);
            return p[4] * line;
        }
        case ORC_ELLIPSE: {
            /* ball.py: diff=x-c; sumsqr(vertcat(diff0/r1, diff1/r2)) - 1 ; sumsqr from 0 */
            double a = (x0 - p[0]) / p[2];
            double b = (x1 - p[1]) / p[3];
            double s = 0.0;
            s = s + a * a;
            s = s + b * b;
            return s - 1.0;
        }
        default: { /* ORC_AXIS: square.py sides: s*(x_k - c) - r */
            double xk = (p[0] == 0.0) ? x0 : x1;
            return p[3] * (xk - p[1]) - p[2];
        }
    }
}

/* quadratic_obstacle.py:27-39 */
static double psi(const orc_geom* g, int s, double x0, double x1, int smooth, double e) {
    double r = 1.0;
    int f = g->shape_first[s], c = g->shape_count[s];
    for (int i = f; i < f + c; ++i) {
        double h = ineq_h(g, i, x0, x1);
        if (smooth) {
            double m = fmin(h - e, 0.0);
            r = r * (m * m);
        } else {
            r = r * fmin(e - h, 0.0);
        }
    }
    return r;
}

/* quadratic_obstacle.py:89-94 */
static int contains(const orc_geom* g, int s, double x0, double x1) {
    int f = g->shape_first[s], c = g->shape_count[s];
    for (int i = f; i < f + c; ++i)
        if (ineq_h(g, i, x0, x1) > 1e-14) return 0;
    return 1;
}

/* problem.py:72-80: Σ_o ψ(x)/ψ(c) (raw ψ when the centre is NaN), times w */
static double shape_sum(const orc_geom* g, int s0, int s1, double x0, double x1, int smooth,
                        double e) {
    double total = 0.0;
    for (int s = s0; s < s1; ++s) {
        double cx = g->shape_center[2 * s], cy = g->shape_center[2 * s + 1];
        double v = psi(g, s, x0, x1, smooth, e);
        if (isnan(cx) || isnan(cy))
            total = total + v;
        else
            total = total + v / psi(g, s, cx, cy, smooth, e);
    }
    return total;
}

static double region_penalty(const orc_geom* g, const orc_params* p, int r, double x0,
                             double x1) {
    double t = shape_sum(g, g->region_first[r], g->region_first[r + 1], x0, x1,
                         p->penalty_smooth, p->enlargement);
    return p->weights[r] * t;
}

/* problem.py:49-56 */
static double total_penalty(const orc_geom* g, const orc_params* p, double x0, double x1) {
    double pen = 0.0;
    for (int r = 0; r < g->n_regions; ++r) pen = pen + region_penalty(g, p, r, x0, x1);
    return pen;
}

/* Σ_o raw ψ_o(x; obstacle_smooth, e=0): the per-waypoint sum of the no-fly g rows
 * (problem.py:109-112 -- penalty_function(smooth) leaves enlargement at its default 0). */
static double obstacle_psi_sum(const orc_geom* g, const orc_params* p, double x0, double x1) {
    double acc = 0.0;
    for (int s = 0; s < g->n_obstacles; ++s)
        acc = acc + psi(g, s, x0, x1, p->obstacle_smooth, 0.0);
    return acc;
}

static int collides(const orc_geom* g, double x0, double x1) {
    for (int s = 0; s < g->n_obstacles; ++s)
        if (contains(g, s, x0, x1)) return 1;
    return 0;
}

/* ---- point evaluation (Problem.get_*_penalty_function) ------------------------------- */

int orc_eval_points(const orc_geom* g, const orc_params* p, const double* pts, int64_t n,
                    double* phi, double* phi_regions, double* obs_norm, double* psi_raw,
                    int32_t* collide) {
    for (int64_t i = 0; i < n; ++i) {
        double x0 = pts[2 * i], x1 = pts[2 * i + 1];
        if (phi) phi[i] = total_penalty(g, p, x0, x1);
        if (phi_regions)
            for (int r = 0; r < g->n_regions; ++r)
                phi_regions[i * g->n_regions + r] = region_penalty(g, p, r, x0, x1);
        if (obs_norm) /* get_penalty_function(None): obstacles, obstacle_smooth, enlargement */
            obs_norm[i] = 1.0 * shape_sum(g, 0, g->n_obstacles, x0, x1, p->obstacle_smooth,
                                          p->enlargement);
        if (psi_raw) psi_raw[i] = obstacle_psi_sum(g, p, x0, x1);
        if (collide) collide[i] = collides(g, x0, x1);
    }
    return 0;
}

/* ---- candidate generator (solver.py:103-136) ------------------------------------------ */
/* pairs [Q][4] = (x0, y0, xf, yf); utab [D][N][2] unit-arc table; out [Q*D][N+2][2].
 * p_k = C + 0.5*[[vx,-vy],[vy,vx]] u_k with v = x0 - xf, C = (xf + x0)/2. */
static void gen_point(const double* pr, const double* u, double* px, double* py) {
    double vx = pr[0] - pr[2], vy = pr[1] - pr[3];
    double cx = (pr[2] + pr[0]) * 0.5, cy = (pr[3] + pr[1]) * 0.5;
    *px = cx + 0.5 * (vx * u[0] - vy * u[1]);
    *py = cy + 0.5 * (vy * u[0] + vx * u[1]);
}

int orc_gen_paths(const double* pairs, int64_t Q, const double* utab, int32_t D, int32_t N,
                  double* out) {
    int W = N + 2;
    for (int64_t q = 0; q < Q; ++q) {
        const double* pr = pairs + 4 * q;
        for (int d = 0; d < D; ++d) {
            double* o = out + ((q * D + d) * (int64_t)W) * 2;
            o[0] = pr[0];
            o[1] = pr[1];
            for (int k = 0; k < N; ++k)
                gen_point(pr, utab + ((int64_t)d * N + k) * 2, &o[2 * (k + 1)],
                          &o[2 * (k + 1) + 1]);
            o[2 * (N + 1)] = pr[2];
            o[2 * (N + 1) + 1] = pr[3];
        }
    }
    return 0;
}

/* ---- raster build ------------------------------------------------------------------------
 * record (16 B) per cell, row-major, row 0 = north: {phi f32, psi f32, dem f32, flags u32} */
int orc_raster_build(const orc_geom* g, const orc_params* p, const orc_raster* rs,
                     const float* dem, float* rec) {
    for (int64_t iy = 0; iy < rs->ny; ++iy) {
        for (int64_t ix = 0; ix < rs->nx; ++ix) {
            int64_t c = iy * rs->nx + ix;
            double xc = rs->x0 + ((double)ix + 0.5) * rs->dx;
            double yc = rs->y_top - ((double)iy + 0.5) * rs->dy;
            float z = dem ? dem[c] : 0.0f;
            uint32_t fl = 0;
            if (collides(g, xc, yc)) fl |= ORC_FLAG_NFZ;
            /* data_manager.py:14-17 */
            if (rs->dem_threshold == -9999.0f ? (z == -9999.0f) : (z > rs->dem_threshold))
                fl |= ORC_FLAG_MASK;
            if (z == rs->nodata) fl |= ORC_FLAG_NODATA;
            rec[4 * c + 0] = (float)total_penalty(g, p, xc, yc);
            rec[4 * c + 1] = (float)obstacle_psi_sum(g, p, xc, yc);
            rec[4 * c + 2] = z;
            memcpy(&rec[4 * c + 3], &fl, 4);
        }
    }
    return 0;
}

/* ---- path evaluation ------------------------------------------------------------------
 * mode 0 = analytic (reference formulas at the waypoint), 1 = raster (gather the record of
 * the waypoint's cell).  wp [P][W][2], W = N+2 (p_0 = start ... p_{N+1} = goal). */
static double nrm_of(double d2, int smooth) {
    double n = sqrt(d2);
    return smooth ? n * n : n; /* problem.py:94,132: norm_2(.)**2 when smooth */
}

/* Grouped summation (K2g; build-defined, no reference counterpart).  A per-path
 * sum over terms indexed by waypoint: with G > 0 the terms of waypoints [kG, (k+1)G) form a
 * partial sum from +0.0 in index order, and the partials are added to the sum's initial value
 * in group order; with G = 0 every term is added to the running sum in index order, which is
 * the reference's sequential order.  Terms arrive in non-decreasing index order. */
typedef struct {
    double tot, part;
    int grp, G;
} gacc;

static void gacc_init(gacc* a, double init, int G) {
    a->tot = init;
    a->part = 0.0;
    a->grp = 0;
    a->G = G;
}

static void gacc_add(gacc* a, int idx, double v) {
    if (a->G <= 0) {
        a->tot = a->tot + v;
        return;
    }
    const int g = idx / a->G;
    if (g != a->grp) { /* group boundary: flush (empty groups add +0.0, an exact no-op) */
        a->tot = a->tot + a->part;
        a->part = 0.0;
        a->grp = g;
    }
    a->part = a->part + v;
}

static double gacc_done(gacc* a) {
    if (a->G > 0) {
        a->tot = a->tot + a->part;
        a->part = 0.0;
        a->G = 0;
    }
    return a->tot;
}

/* group > 0 (raster mode only): the grouped summation order of the segment-grouped raster
 * evaluation K2g.  The waypoints are cut into groups [kG, min((k+1)G, W)); every per-path sum
 * is formed as per-group partials added in group order (gacc), with each term attached to a
 * waypoint: the Φ/N and ψ terms of waypoint j to j; the length terms of segment p_{j-1} -> p_j
 * (get_cost's L and the true length) to j, get_cost's anchor term to 0; kinematic row k
 * (points k, k+1, k+2) to k + 1.  cost = (N+1)·L + the Φ/N partials.  group = 0 is the
 * reference's sequential order (problem.py:38-44, 84-114, 130-146).  Both sum the same terms
 * and differ by rounding only (≤ 1e-12 relative on the cfg3 batch,
 * tests/test_oracle_golden.py). */
int orc_eval_paths_g(const orc_geom* g, const orc_params* p, int32_t mode, const orc_raster* rs,
                     const float* rec, const double* wp, int64_t P, double* cost, double* lq,
                     double* length, double* kin, double* nfz, int32_t* hits, double* minclr,
                     int32_t* offmap, int32_t* cells, double* g_rows, int32_t group) {
    const int N = p->N, W = N + 2;
    const double mincos = cos(p->maxalpha);
    const double r = p->maxratio_smooth ? p->maxratio * p->maxratio : p->maxratio;
    const int n_rows = 3 * N + g->n_obstacles * W;
    const int G = (mode == 1 && group > 0) ? group : 0;
    double inv_dx = 0, inv_dy = 0;
    if (mode == 1) {
        inv_dx = 1.0 / rs->dx;
        inv_dy = 1.0 / rs->dy;
    }
    for (int64_t pi = 0; pi < P; ++pi) {
        const double* z = wp + pi * (int64_t)W * 2;
        /* length_of (problem.py:130-146): y = [anchor, p_0..p_{N+1}, goal]; N+1 segments */
        double ax = p->anchor_mode ? p->anchor_x : z[0];
        double ay = p->anchor_mode ? p->anchor_y : z[1];
        gacc aL;
        gacc_init(&aL, 0.0, G);
        if (p->quirk_length) {
            double dx = z[0] - ax, dy = z[1] - ay;
            double s = 0.0;
            s = s + dx * dx;
            s = s + dy * dy;
            gacc_add(&aL, 0, nrm_of(s, p->length_smooth));
            for (int k = 1; k <= N; ++k) {
                dx = z[2 * k] - z[2 * k - 2];
                dy = z[2 * k + 1] - z[2 * k - 1];
                s = 0.0;
                s = s + dx * dx;
                s = s + dy * dy;
                gacc_add(&aL, k, nrm_of(s, p->length_smooth));
            }
        } else {
            for (int k = 1; k <= N + 1; ++k) {
                double dx = z[2 * k] - z[2 * k - 2], dy = z[2 * k + 1] - z[2 * k - 1];
                double s = 0.0;
                s = s + dx * dx;
                s = s + dy * dy;
                gacc_add(&aL, k, nrm_of(s, p->length_smooth));
            }
        }
        const double L = gacc_done(&aL);
        /* true polyline length (solver.py:49 length_of(x_sol), non-smooth, all segments) */
        gacc alen;
        gacc_init(&alen, 0.0, G);
        for (int k = 1; k <= N + 1; ++k) {
            double dx = z[2 * k] - z[2 * k - 2], dy = z[2 * k + 1] - z[2 * k - 1];
            double s = 0.0;
            s = s + dx * dx;
            s = s + dy * dy;
            gacc_add(&alen, k, sqrt(s));
        }
        const double len = gacc_done(&alen);
        /* kinematic rows (problem.py:100-107) */
        gacc ak;
        gacc_init(&ak, 0.0, G);
        double* grow = g_rows ? g_rows + pi * (int64_t)n_rows : 0;
        for (int k = 0; k < N; ++k) {
            double ax0 = z[2 * (k + 1)] - z[2 * k], ay0 = z[2 * (k + 1) + 1] - z[2 * k + 1];
            double bx = z[2 * (k + 2)] - z[2 * (k + 1)];
            double by = z[2 * (k + 2) + 1] - z[2 * (k + 1) + 1];
            double sa = 0.0, sb = 0.0, dt = 0.0;
            sa = sa + ax0 * ax0;
            sa = sa + ay0 * ay0;
            sb = sb + bx * bx;
            sb = sb + by * by;
            dt = dt + ax0 * bx;
            dt = dt + ay0 * by;
            double na = nrm_of(sa, p->maxratio_smooth), nb = nrm_of(sb, p->maxratio_smooth);
            double c1 = fmax(0.0, nb - r * na);
            double c2 = fmax(0.0, na / r - nb);
            double c3 = fmax(0.0, mincos - dt / (na * nb));
            gacc_add(&ak, k + 1, c1);
            gacc_add(&ak, k + 1, c2);
            gacc_add(&ak, k + 1, c3);
            if (grow) {
                grow[3 * k] = c1;
                grow[3 * k + 1] = c2;
                grow[3 * k + 2] = c3;
            }
        }
        const double ksum = gacc_done(&ak);
        /* per-waypoint penalty, no-fly rows, clearance */
        gacc ac, an;
        gacc_init(&ac, (double)(N + 1) * L, G);
        gacc_init(&an, 0.0, G);
        double hmax = -INFINITY;
        int32_t nh = 0, off = 0;
        for (int j = 0; j < W; ++j) {
            double x0 = z[2 * j], x1 = z[2 * j + 1];
            if (mode == 0) {
                gacc_add(&ac, j, total_penalty(g, p, x0, x1) / (double)N);
                for (int s = 0; s < g->n_obstacles; ++s) {
                    double v = psi(g, s, x0, x1, p->obstacle_smooth, 0.0);
                    gacc_add(&an, j, v);
                    if (grow) grow[3 * N + s * W + j] = v;
                }
                nh += collides(g, x0, x1);
            } else {
                double fx = floor((x0 - rs->x0) * inv_dx);
                double fy = floor((rs->y_top - x1) * inv_dy);
                int inside = (fx >= 0.0) && (fx < (double)rs->nx) && (fy >= 0.0) &&
                             (fy < (double)rs->ny);
                if (!inside) {
                    ++off;
                    if (cells) cells[pi * W + j] = -1;
                    if (0.0 > hmax) hmax = 0.0; /* off-raster counts as sea level */
                    continue;
                }
                int64_t cell = (int64_t)fy * rs->nx + (int64_t)fx;
                if (cells) cells[pi * W + j] = (int32_t)cell;
                const float* rc = rec + 4 * cell;
                uint32_t fl;
                memcpy(&fl, &rc[3], 4);
                gacc_add(&ac, j, (double)rc[0] / (double)N);
                gacc_add(&an, j, (double)rc[1]);
                nh += (fl & ORC_FLAG_NFZ) ? 1 : 0;
                double terrain = (fl & ORC_FLAG_NODATA) ? 0.0 : (double)rc[2];
                if (terrain > hmax) hmax = terrain;
            }
        }
        const double c = gacc_done(&ac), nsum = gacc_done(&an);
        if (cost) cost[pi] = c;
        if (lq) lq[pi] = L;
        if (length) length[pi] = len;
        if (kin) kin[pi] = ksum;
        if (nfz) nfz[pi] = nsum;
        if (hits) hits[pi] = nh;
        if (offmap) offmap[pi] = off;
        if (minclr) minclr[pi] = (mode == 1) ? p->altitude - hmax : NAN;
    }
    return 0;
}

int orc_eval_paths(const orc_geom* g, const orc_params* p, int32_t mode, const orc_raster* rs,
                   const float* rec, const double* wp, int64_t P, double* cost, double* lq,
                   double* length, double* kin, double* nfz, int32_t* hits, double* minclr,
                   int32_t* offmap, int32_t* cells, double* g_rows) {
    return orc_eval_paths_g(g, p, mode, rs, rec, wp, P, cost, lq, length, kin, nfz, hits, minclr,
                            offmap, cells, g_rows, 0);
}

/* main.py:175-180 over groups of G consecutive paths.  The reference keeps index i when
 * `min_v == 0 or v_i < min_v` with min_v initialised to the sentinel 0, so: the first entry
 * always wins first, later entries replace it on strict '<' (ties keep the first), a NaN never
 * wins, and a best value of exactly 0 is replaced by the next entry (sentinel quirk).  For
 * fval the compared value is sqrt(cost) (solver.py:48), for length the length itself. */
int orc_argmin(const double* v, int64_t groups, int32_t G, int32_t take_sqrt, int32_t* best) {
    for (int64_t q = 0; q < groups; ++q) {
        int32_t bi = 0;
        double bv = 0.0;
        for (int32_t d = 0; d < G; ++d) {
            double x = take_sqrt ? sqrt(v[q * G + d]) : v[q * G + d];
            if (bv == 0.0 || x < bv) {
                bv = x;
                bi = d;
            }
        }
        best[q] = bi;
    }
    return 0;
}

/* ---- volume mode (BASELINE config 5; no reference counterpart) --------------------------
 * Restates the build's own definition (include/uampath.h uam_volume_build /
 * uam_eval_generated3d): voxels [ny][nx][nz] {risk, psi_nfz}, columns [ny][nx]
 * {terrain (0 on nodata), flags}; a waypoint is below the terrain when its layer centre
 * z0 + (iz + 0.5) dz is. */

typedef struct {
    int32_t nx, ny, nz;
    double x0, y_top, dx, dy, z0, dz;
} orc_volume;

int orc_volume_build(const orc_volume* v, const float* rec2, const double* layer_w, float* vox,
                     float* cols) {
    for (int64_t col = 0; col < (int64_t)v->nx * v->ny; ++col) {
        uint32_t f2;
        memcpy(&f2, &rec2[4 * col + 3], 4);
        float terrain = (f2 & ORC_FLAG_NODATA) ? 0.0f : rec2[4 * col + 2];
        uint32_t fl = f2 & (ORC_FLAG_NFZ | ORC_FLAG_MASK | ORC_FLAG_NODATA);
        cols[2 * col] = terrain;
        memcpy(&cols[2 * col + 1], &fl, 4);
        for (int iz = 0; iz < v->nz; ++iz) {
            int64_t o = (col * v->nz + iz) * 2;
            vox[o + 0] = (float)((double)rec2[4 * col] * layer_w[iz]);
            vox[o + 1] = rec2[4 * col + 1];
        }
    }
    return 0;
}

/* pairs6 [Q][6] = (x0, y0, z0, xf, yf, zf) -> wp3 [Q*D][N+2][3]; x/y as orc_gen_paths,
 * z_j = z0 + (zf - z0) * (j / (N+1)) */
int orc_gen_paths3d(const double* pairs6, int64_t Q, const double* utab, int32_t D, int32_t N,
                    double* out) {
    int W = N + 2;
    for (int64_t q = 0; q < Q; ++q) {
        const double* pr6 = pairs6 + 6 * q;
        double pr[4] = {pr6[0], pr6[1], pr6[3], pr6[4]};
        for (int d = 0; d < D; ++d) {
            double* o = out + ((q * D + d) * (int64_t)W) * 3;
            for (int j = 0; j < W; ++j) {
                double px, py;
                if (j == 0) {
                    px = pr[0];
                    py = pr[1];
                } else if (j == W - 1) {
                    px = pr[2];
                    py = pr[3];
                } else {
                    gen_point(pr, utab + ((int64_t)d * N + (j - 1)) * 2, &px, &py);
                }
                o[3 * j] = px;
                o[3 * j + 1] = py;
                o[3 * j + 2] = pr6[2] + (pr6[5] - pr6[2]) * ((double)j / (double)(W - 1));
            }
        }
    }
    return 0;
}

int orc_eval_paths3d(const orc_geom* g, const orc_params* p, const orc_volume* v,
                     const float* vox, const float* cols, const double* wp3, int64_t P,
                     double* cost, double* lq,
                     double* length, double* kin, double* nfz, int32_t* hits, double* minclr,
                     int32_t* offmap, int32_t* below, int32_t* cells) {
    const int N = p->N, W = N + 2;
    double* xy = (double*)malloc(sizeof(double) * 2 * W);
    const double idx = 1.0 / v->dx, idy = 1.0 / v->dy, idz = 1.0 / v->dz;
    for (int64_t pi = 0; pi < P; ++pi) {
        const double* z = wp3 + pi * (int64_t)W * 3;
        for (int j = 0; j < W; ++j) {
            xy[2 * j] = z[3 * j];
            xy[2 * j + 1] = z[3 * j + 1];
        }
        /* geometry-only terms: the 2-D path evaluation in analytic mode with no shapes
         * would recompute penalties; call the shared pieces through orc_eval_paths on a
         * geometry-free copy instead */
        orc_geom g0 = *g;
        g0.n_regions = 0;
        g0.n_obstacles = 0;
        double c2, lq2, len2, k2, n2, mc2;
        int32_t h2, o2;
        orc_eval_paths(&g0, p, 0, NULL, NULL, xy, 1, &c2, &lq2, &len2, &k2, &n2, &h2, &mc2, &o2,
                       NULL, NULL);
        double c = (double)(N + 1) * lq2, ns = 0.0, cm = INFINITY;
        int32_t nh = 0, off = 0, bel = 0;
        for (int j = 0; j < W; ++j) {
            double fx = floor((z[3 * j] - v->x0) * idx);
            double fy = floor((v->y_top - z[3 * j + 1]) * idy);
            double fz = floor((z[3 * j + 2] - v->z0) * idz);
            int in = fx >= 0.0 && fx < (double)v->nx && fy >= 0.0 && fy < (double)v->ny &&
                     fz >= 0.0 && fz < (double)v->nz;
            if (!in) {
                ++off;
                if (cells) cells[pi * W + j] = -1;
                continue;
            }
            int64_t ci = (int64_t)fy * v->nx + (int64_t)fx;
            int64_t vi = ci * v->nz + (int64_t)fz;
            if (cells) cells[pi * W + j] = (int32_t)vi;
            const float* r = vox + 2 * vi;
            const float terrain = cols[2 * ci];
            uint32_t fl;
            memcpy(&fl, &cols[2 * ci + 1], 4);
            c = c + (double)r[0] / (double)N;
            ns = ns + (double)r[1];
            nh += (fl & ORC_FLAG_NFZ) ? 1 : 0;
            bel += (v->z0 + (fz + 0.5) * v->dz < (double)terrain) ? 1 : 0;
            cm = fmin(cm, z[3 * j + 2] - (double)terrain);
        }
        if (cost) cost[pi] = c;
        if (lq) lq[pi] = lq2;
        if (length) length[pi] = len2;
        if (kin) kin[pi] = k2;
        if (nfz) nfz[pi] = ns;
        if (hits) hits[pi] = nh;
        if (minclr) minclr[pi] = cm;
        if (offmap) offmap[pi] = off;
        if (below) below[pi] = bel;
    }
    free(xy);
    return 0;
}

/* ---- generated candidates in the similarity form (K2h / K4h) ----------------
 * The candidates of solver.py:103-136 are circular arcs from x0 to xf; restated through the
 * unit-arc table (orc_gen_paths) they are p_k = C + (1/2) R(v) u_k with v = x0 - xf,
 * R(v) = [[vx, -vy], [vy, vx]], u_1..u_N the table row of displacement d and u_0 = (1, 0),
 * u_{N+1} = (-1, 0) (then p_0 = x0, p_{N+1} = xf).  The path is the unit polyline u under a
 * similarity of scale h = |v| / 2: every chord is h times the unit chord b_k = |u_k - u_{k-1}|
 * and every turn angle is the unit polyline's.  The path terms that depend on the geometry
 * only are therefore per-displacement constants scaled by h (maxratio_smooth = 0):
 *   length_of (problem.py:130-146)   sum_k nrm(p_k - p_{k-1}) = h S1 (nrm = norm_2) or
 *                                    h^2 S2 (smooth: norm_2(.)**2), over k = 1..N (get_cost's
 *                                    L with the quirk, plus its anchor term nrm(p_0 - anchor))
 *                                    or k = 1..N+1 (the true length, solver.py:49)
 *   get_nonlincon rows (problem.py:100-107)  c1 + c2 = h max(0, b_{k+2} - r b_{k+1})
 *                                    + h max(0, b_{k+1}/r - b_{k+2}), c3 = max(0, mincos - cos of
 *                                    the unit turn), summed: h E12 + E3 (0 for h = 0, NaN, inf:
 *                                    the reference's rows are max(0, NaN) = 0 there)
 * Exact in real arithmetic; in float64 these differ from the per-segment sums of the
 * waypoints by rounding only (bench.py's parity.vs_sequential_order measures it on the whole
 * cfg3 batch).  The raster / volume terms are evaluated per waypoint exactly as in
 * orc_eval_paths_g / orc_eval_paths3d at the generated points (gen_point), their sums in the
 * grouped order of `group` (0: sequential).  Build-defined: the definition the GPU's K2h / K4h
 * reproduce bit for bit. */
typedef struct {
    double s1n, s2n, s1a, s2a, e12, e3;
} orc_unit_geo;

/* the unit polyline's sums for one table row u [N][2] (every order below is the definition) */
static void unit_geo(const orc_params* p, const double* u, orc_unit_geo* t) {
    const int N = p->N;
    const double mincos = cos(p->maxalpha), r = p->maxratio;
    double s1n = 0.0, s2n = 0.0, s1a = 0.0, s2a = 0.0, e12 = 0.0, e3 = 0.0;
    double qx = 1.0, qy = 0.0, pdx = 0.0, pdy = 0.0, pb = 0.0;
    for (int k = 1; k <= N + 1; ++k) {
        const double cx = (k <= N) ? u[2 * (k - 1)] : -1.0;
        const double cy = (k <= N) ? u[2 * (k - 1) + 1] : 0.0;
        const double dx = cx - qx, dy = cy - qy;
        const double b = sqrt(dx * dx + dy * dy);
        if (k <= N) {
            s1n = s1n + b;
            s2n = s2n + b * b;
        }
        s1a = s1a + b;
        s2a = s2a + b * b;
        if (k >= 2) { /* row k - 2: chords k - 1 and k */
            e12 = e12 + fmax(0.0, b - r * pb);
            e12 = e12 + fmax(0.0, pb / r - b);
            const double dt = pdx * dx + pdy * dy;
            e3 = e3 + fmax(0.0, mincos - dt / (pb * b));
        }
        qx = cx, qy = cy, pdx = dx, pdy = dy, pb = b;
    }
    t->s1n = s1n, t->s2n = s2n, t->s1a = s1a, t->s2a = s2a, t->e12 = e12, t->e3 = e3;
}

/* the geometry terms of one candidate: pair (x0, y0, xf, yf), the row's unit sums */
static void sim_geo(const orc_params* p, const orc_unit_geo* t, double x0, double y0, double xf,
                    double yf, double* L, double* len, double* ksum) {
    const double vx = x0 - xf, vy = y0 - yf;
    const double s = vx * vx + vy * vy;
    const double h = sqrt(s) * 0.5, h2 = s * 0.25;
    const int ls = p->length_smooth != 0;
    if (p->quirk_length) {
        const double ax = p->anchor_mode ? p->anchor_x : x0;
        const double ay = p->anchor_mode ? p->anchor_y : y0;
        const double dx = x0 - ax, dy = y0 - ay;
        const double a = nrm_of(dx * dx + dy * dy, ls);
        *L = a + (ls ? h2 * t->s2n : h * t->s1n);
    } else {
        *L = ls ? h2 * t->s2a : h * t->s1a;
    }
    *len = h * t->s1a;
    *ksum = (h > 0.0 && h < INFINITY) ? h * t->e12 + t->e3 : 0.0;
}

/* mode 1: raster (rs, rec; pairs [Q][4]); mode 2: volume (v, vox [ny][nx][nz][2],
 * cols [ny][nx][2]; pairs [Q][6] = (x0, y0, z0, xf, yf, zf)).  Path q D + d.  below: volume
 * only.  Returns -1 for maxratio_smooth (its turn rows are not scale-free). */
int orc_eval_generated_h(const orc_geom* g, const orc_params* p, int32_t mode,
                         const orc_raster* rs, const float* rec, const orc_volume* v,
                         const float* vox, const float* cols, const double* pairs, int64_t Q,
                         const double* utab, int32_t D, int32_t group, double* cost, double* lq,
                         double* length, double* kin, double* nfz, int32_t* hits,
                         double* minclr, int32_t* offmap, int32_t* below, int32_t* cells) {
    if (p->maxratio_smooth || (mode != 1 && mode != 2)) return -1;
    const int N = p->N, W = N + 2;
    const int G = group > 0 ? group : 0;
    orc_unit_geo* ug = (orc_unit_geo*)malloc(sizeof(orc_unit_geo) * (size_t)D);
    for (int d = 0; d < D; ++d) unit_geo(p, utab + (int64_t)d * N * 2, &ug[d]);
    const int stride = mode == 1 ? 4 : 6;
    const double idx = mode == 1 ? 1.0 / rs->dx : 1.0 / v->dx;
    const double idy = mode == 1 ? 1.0 / rs->dy : 1.0 / v->dy;
    const double idz = mode == 2 ? 1.0 / v->dz : 0.0;
    for (int64_t q = 0; q < Q; ++q) {
        const double* pr6 = pairs + stride * q;
        const double pr[4] = {pr6[0], pr6[1], pr6[stride == 4 ? 2 : 3], pr6[stride == 4 ? 3 : 4]};
        for (int d = 0; d < D; ++d) {
            const int64_t pi = q * D + d;
            double L, len, ks;
            sim_geo(p, &ug[d], pr[0], pr[1], pr[2], pr[3], &L, &len, &ks);
            gacc ac, an;
            gacc_init(&ac, (double)(N + 1) * L, G);
            gacc_init(&an, 0.0, G);
            double hmax = -INFINITY, cm = INFINITY;
            int32_t nh = 0, off = 0, bel = 0;
            for (int j = 0; j < W; ++j) {
                double x0, x1;
                if (j == 0) {
                    x0 = pr[0], x1 = pr[1];
                } else if (j == W - 1) {
                    x0 = pr[2], x1 = pr[3];
                } else {
                    gen_point(pr, utab + ((int64_t)d * N + (j - 1)) * 2, &x0, &x1);
                }
                if (mode == 1) {
                    const double fx = floor((x0 - rs->x0) * idx);
                    const double fy = floor((rs->y_top - x1) * idy);
                    if (!((fx >= 0.0) && (fx < (double)rs->nx) && (fy >= 0.0) &&
                          (fy < (double)rs->ny))) {
                        ++off;
                        if (cells) cells[pi * W + j] = -1;
                        if (0.0 > hmax) hmax = 0.0; /* off-raster counts as sea level */
                        continue;
                    }
                    const int64_t cell = (int64_t)fy * rs->nx + (int64_t)fx;
                    if (cells) cells[pi * W + j] = (int32_t)cell;
                    const float* rc = rec + 4 * cell;
                    uint32_t fl;
                    memcpy(&fl, &rc[3], 4);
                    gacc_add(&ac, j, (double)rc[0] / (double)N);
                    gacc_add(&an, j, (double)rc[1]);
                    nh += (fl & ORC_FLAG_NFZ) ? 1 : 0;
                    const double terrain = (fl & ORC_FLAG_NODATA) ? 0.0 : (double)rc[2];
                    if (terrain > hmax) hmax = terrain;
                } else {
                    const double z = pr6[2] + (pr6[5] - pr6[2]) * ((double)j / (double)(W - 1));
                    const double fx = floor((x0 - v->x0) * idx);
                    const double fy = floor((v->y_top - x1) * idy);
                    const double fz = floor((z - v->z0) * idz);
                    if (!(fx >= 0.0 && fx < (double)v->nx && fy >= 0.0 && fy < (double)v->ny &&
                          fz >= 0.0 && fz < (double)v->nz)) {
                        ++off;
                        if (cells) cells[pi * W + j] = -1;
                        continue;
                    }
                    const int64_t ci = (int64_t)fy * v->nx + (int64_t)fx;
                    const int64_t vi = ci * v->nz + (int64_t)fz;
                    if (cells) cells[pi * W + j] = (int32_t)vi;
                    const float* r = vox + 2 * vi;
                    const float terrain = cols[2 * ci];
                    uint32_t fl;
                    memcpy(&fl, &cols[2 * ci + 1], 4);
                    gacc_add(&ac, j, (double)r[0] / (double)N);
                    gacc_add(&an, j, (double)r[1]);
                    nh += (fl & ORC_FLAG_NFZ) ? 1 : 0;
                    bel += (v->z0 + (fz + 0.5) * v->dz < (double)terrain) ? 1 : 0;
                    cm = fmin(cm, z - (double)terrain);
                }
            }
            if (cost) cost[pi] = gacc_done(&ac);
            if (lq) lq[pi] = L;
            if (length) length[pi] = len;
            if (kin) kin[pi] = ks;
            if (nfz) nfz[pi] = gacc_done(&an);
            if (hits) hits[pi] = nh;
            if (offmap) offmap[pi] = off;
            if (minclr) minclr[pi] = mode == 1 ? p->altitude - hmax : cm;
            if (below) below[pi] = bel;
        }
    }
    free(ug);
    return 0;
}

/* ---- batched refinement (no pinned reference output) ----------------
 * Restates the build's ALM refinement (include/uampath.h uam_refine): the reference solves
 *   min get_cost(z)  s.t.  get_nonlincon(z) in {0}            (solver.py:82-93)
 * with OpEn's augmented Lagrangian; here per path: outer ALM updates y += c g, c *= rho when
 * sum g^2 did not drop below theta * previous, inner gradient steps on
 *   L = f + sum_i (c/2) (g_i + y_i/c)^2
 * with Armijo backtracking.  Requires penalty_smooth and obstacle_smooth (the reference's
 * main.py options).  Operation order is part of the definition (GPU == oracle bit for bit). */
typedef struct {
    int32_t n_outer, n_inner, max_backtrack, memory;
    double c0, rho, c_max, alpha0, armijo, theta, max_step, inner_tol, delta;
    int32_t n_restart;      /* restarts of a path that ends with sqrt(sum g^2) > delta */
    double restart_margin;  /* km past the obstacle's boundary a restart moves waypoints */
} orc_refine_params;
#define RF_MAXM 8

/* gradient of h_i */
static void ineq_grad(const orc_geom* g, int i, double x0, double x1, double* gx, double* gy) {
    const double* p = g->ineq_par + 6 * (int64_t)i;
    switch (g->ineq_kind[i]) {
        case ORC_HALFPLANE:
            *gx = p[4] * p[3];
            *gy = -(p[4] * p[2]);
            return;
        case ORC_ELLIPSE: {
            double a = (x0 - p[0]) / p[2];
            double b = (x1 - p[1]) / p[3];
            *gx = (2.0 * a) / p[2];
            *gy = (2.0 * b) / p[3];
            return;
        }
        default:
            *gx = (p[0] == 0.0) ? p[3] : 0.0;
            *gy = (p[0] == 0.0) ? 0.0 : p[3];
            return;
    }
}

/* smooth psi = prod_i m_i^2, m_i = min(h_i - e, 0), and (want != 0) its gradient
 * sum_i (2 psi / m_i) grad h_i -- nonzero only where every m_i != 0, i.e. psi != 0.  The value
 * is psi(g, s, x, 1, e) bit for bit. */
static double psi_vg(const orc_geom* g, int s, double x0, double x1, double e, int want,
                     double* dx, double* dy) {
    int f = g->shape_first[s], n = g->shape_count[s];
    double v = 1.0;
    for (int i = f; i < f + n; ++i) {
        double m = fmin(ineq_h(g, i, x0, x1) - e, 0.0);
        v = v * (m * m);
    }
    *dx = 0.0;
    *dy = 0.0;
    if (want && v != 0.0) {
        double ox = 0.0, oy = 0.0;
        for (int i = f; i < f + n; ++i) {
            double m = fmin(ineq_h(g, i, x0, x1) - e, 0.0);
            double coef = (2.0 * v) / m, hx, hy;
            ineq_grad(g, i, x0, x1, &hx, &hy);
            ox = ox + coef * hx;
            oy = oy + coef * hy;
        }
        *dx = ox;
        *dy = oy;
    }
    return v;
}

/* Phi (total_penalty bit for bit, smooth) and, when want, its gradient */
static double phi_vg(const orc_geom* g, const orc_params* p, double x0, double x1, int want,
                     double* dx, double* dy) {
    double pen = 0.0, gx = 0.0, gy = 0.0;
    for (int r = 0; r < g->n_regions; ++r) {
        double t = 0.0, tx = 0.0, ty = 0.0;
        for (int s = g->region_first[r]; s < g->region_first[r + 1]; ++s) {
            double cx = g->shape_center[2 * s], cy = g->shape_center[2 * s + 1];
            double ex, ey;
            double v = psi_vg(g, s, x0, x1, p->enlargement, want, &ex, &ey);
            if (isnan(cx) || isnan(cy)) {
                t = t + v;
                if (want && v != 0.0) {
                    tx = tx + ex;
                    ty = ty + ey;
                }
            } else {
                double nrm = psi(g, s, cx, cy, 1, p->enlargement);
                t = t + v / nrm;
                if (want && v != 0.0) {
                    tx = tx + ex / nrm;
                    ty = ty + ey / nrm;
                }
            }
        }
        pen = pen + p->weights[r] * t;
        gx = gx + p->weights[r] * tx;
        gy = gy + p->weights[r] * ty;
    }
    *dx = gx;
    *dy = gy;
    return pen;
}

typedef struct {
    double c1, c2, c3;          /* row values */
    double d[3][6];             /* d row / d (p_k, p_k+1, p_k+2) as (x, y) triples */
} kin_row;

static void kin_eval(const double* pk, const double* pk1, const double* pk2, double r,
                     double mincos, int ms, int want_grad, kin_row* o) {
    double ax = pk1[0] - pk[0], ay = pk1[1] - pk[1];
    double bx = pk2[0] - pk1[0], by = pk2[1] - pk1[1];
    double sa = 0.0, sb = 0.0, dt = 0.0;
    sa = sa + ax * ax;
    sa = sa + ay * ay;
    sb = sb + bx * bx;
    sb = sb + by * by;
    dt = dt + ax * bx;
    dt = dt + ay * by;
    double ra = sqrt(sa), rb = sqrt(sb);
    double na = ms ? ra * ra : ra, nb = ms ? rb * rb : rb;
    o->c1 = fmax(0.0, nb - r * na);
    o->c2 = fmax(0.0, na / r - nb);
    double den = na * nb;
    o->c3 = fmax(0.0, mincos - dt / den);
    if (!want_grad) return;
    double gax = ms ? 2.0 * ax : ax / ra, gay = ms ? 2.0 * ay : ay / ra;
    double gbx = ms ? 2.0 * bx : bx / rb, gby = ms ? 2.0 * by : by / rb;
    double da[3][2], db[3][2];
    /* c1 = nb - r na */
    da[0][0] = -(r * gax), da[0][1] = -(r * gay), db[0][0] = gbx, db[0][1] = gby;
    /* c2 = na / r - nb */
    da[1][0] = gax / r, da[1][1] = gay / r, db[1][0] = -gbx, db[1][1] = -gby;
    /* c3 = mincos - dt / den */
    double d2 = den * den;
    double qax = bx / den - ((dt * nb) * gax) / d2, qay = by / den - ((dt * nb) * gay) / d2;
    double qbx = ax / den - ((dt * na) * gbx) / d2, qby = ay / den - ((dt * na) * gby) / d2;
    da[2][0] = -qax, da[2][1] = -qay, db[2][0] = -qbx, db[2][1] = -qby;
    for (int t = 0; t < 3; ++t) {
        o->d[t][0] = -da[t][0];
        o->d[t][1] = -da[t][1];
        o->d[t][2] = da[t][0] - db[t][0];
        o->d[t][3] = da[t][1] - db[t][1];
        o->d[t][4] = db[t][0];
        o->d[t][5] = db[t][1];
    }
}

/* The GPU refines one path per 64-lane wavefront, lane l owning waypoints j = l, l+64, ...
 * Path-level sums are therefore defined as: per lane, the sequential sum of its waypoints'
 * terms (ascending j), then the xor butterfly over lanes (offsets 32, 16, ..., 1). */
#define RF_LANES 64
static double wsum(const double* t, int W) {
    double v[RF_LANES], u[RF_LANES];
    for (int l = 0; l < RF_LANES; ++l) {
        v[l] = 0.0;
        for (int j = l; j < W; j += RF_LANES) v[l] = v[l] + t[j];
    }
    for (int off = RF_LANES / 2; off >= 1; off >>= 1) {
        for (int l = 0; l < RF_LANES; ++l) u[l] = v[l] + v[l ^ off];
        for (int l = 0; l < RF_LANES; ++l) v[l] = u[l];
    }
    return v[0];
}

/* waypoint j of z, or of the trial point z + a dr (interior j, a != 0); vectors over the
 * path are indexed by waypoint (v[2j], v[2j+1]; endpoint entries unused) */
static void rpt(const double* z, const double* dr, double a, int N, int j, double* x,
                double* y) {
    *x = z[2 * j];
    *y = z[2 * j + 1];
    if (a != 0.0 && j >= 1 && j <= N) {
        *x = *x + a * dr[2 * j];
        *y = *y + a * dr[2 * j + 1];
    }
}

/* path dot product over the interior waypoints, lane-tree order */
static double wdot(const double* u, const double* v, int N, double* tmp) {
    const int W = N + 2;
    for (int j = 0; j < W; ++j)
        tmp[j] = (j >= 1 && j <= N) ? u[2 * j] * v[2 * j] + u[2 * j + 1] * v[2 * j + 1] : 0.0;
    return wsum(tmp, W);
}

/* norm of the segment (px,py) -> (qx,qy) as get_cost sums it; vx/vy: d/dq of (N+1) * term */
static double seg_term(double px, double py, double qx, double qy, int ls, double sc,
                       double* vx, double* vy) {
    double dx = qx - px, dy = qy - py, s = 0.0;
    s = s + dx * dx;
    s = s + dy * dy;
    double n = sqrt(s);
    if (vx) {
        *vx = ls ? sc * (2.0 * dx) : sc * (dx / n);
        *vy = ls ? sc * (2.0 * dy) : sc * (dy / n);
    }
    return ls ? n * n : n;
}

/* L(z + a dr) = f + sum_i (c/2)(g_i + y_i/c)^2 with f = (N+1) * sum(length terms) +
 * sum(Phi_j / N); per-waypoint terms as the GPU lanes form them; want (a = 0 only): the
 * gradient into gr (waypoint-indexed) and *gn2 = |gr|^2.  Gradient accumulation order per
 * waypoint j: segment ending at j (+), segment starting at j (-), grad Phi / N, kinematic
 * rows k = j-2, j-1, j (c1, c2, c3), obstacle rows s ascending.  yk: kinematic multipliers
 * [3N], yo: obstacle multipliers [S][W]. */
static double refine_L(const orc_geom* g, const orc_params* p, const double* z,
                       const double* dr, double a, double* gr, const double* yk,
                       const double* yo, double c, int want, double* fout, double* gn2) {
    const int N = p->N, W = N + 2, ls = p->length_smooth, ms = p->maxratio_smooth;
    const double r = ms ? p->maxratio * p->maxratio : p->maxratio;
    const double mincos = cos(p->maxalpha), hc = 0.5 * c, dN = (double)N;
    const double sc = (double)(N + 1);
    const int kend = p->quirk_length ? N : N + 1;
    double* tl = (double*)malloc(sizeof(double) * 4 * W);
    double *tphi = tl + W, *taug = tl + 2 * W, *tg = tl + 3 * W;
    for (int j = 0; j < W; ++j) {
        const int inner = want && j >= 1 && j <= N;
        double xj, yj;
        rpt(z, dr, a, N, j, &xj, &yj);
        /* length term of the segment ending at j (anchor segment for j = 0) */
        double lj = 0.0, vx0 = 0.0, vy0 = 0.0;
        if (j == 0) {
            if (p->quirk_length) {
                double ax = p->anchor_mode ? p->anchor_x : xj;
                double ay = p->anchor_mode ? p->anchor_y : yj;
                lj = seg_term(ax, ay, xj, yj, ls, sc, NULL, NULL);
            }
        } else if (j <= kend) {
            double px, py;
            rpt(z, dr, a, N, j - 1, &px, &py);
            lj = seg_term(px, py, xj, yj, ls, sc, inner ? &vx0 : NULL, &vy0);
        }
        tl[j] = lj;
        double ex, ey;
        tphi[j] = phi_vg(g, p, xj, yj, inner, &ex, &ey) / dN;
        double aj = 0.0, gx = 0.0, gy = 0.0;
        if (j < N) {
            double q1[2], q2[2], q0[2] = {xj, yj};
            rpt(z, dr, a, N, j + 1, &q1[0], &q1[1]);
            rpt(z, dr, a, N, j + 2, &q2[0], &q2[1]);
            kin_row kr;
            kin_eval(q0, q1, q2, r, mincos, ms, 0, &kr);
            double gv[3] = {kr.c1, kr.c2, kr.c3};
            for (int t = 0; t < 3; ++t) {
                double tt = gv[t] + yk[3 * j + t] / c;
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
                rpt(z, dr, a, N, j + 1, &qx, &qy);
                seg_term(xj, yj, qx, qy, ls, sc, &vx, &vy);
                gx = gx - vx;
                gy = gy - vy;
            }
            gx = gx + ex / dN;
            gy = gy + ey / dN;
            for (int k = j - 2; k <= j; ++k) {
                if (k < 0 || k >= N) continue;
                double q0[2], q1[2], q2[2];
                rpt(z, dr, a, N, k, &q0[0], &q0[1]);
                rpt(z, dr, a, N, k + 1, &q1[0], &q1[1]);
                rpt(z, dr, a, N, k + 2, &q2[0], &q2[1]);
                kin_row kr;
                kin_eval(q0, q1, q2, r, mincos, ms, 1, &kr);
                double gv[3] = {kr.c1, kr.c2, kr.c3};
                const int q = j - k;
                for (int t = 0; t < 3; ++t) {
                    if (!(gv[t] > 0.0)) continue;
                    double coef = c * (gv[t] + yk[3 * k + t] / c);
                    gx = gx + coef * kr.d[t][2 * q];
                    gy = gy + coef * kr.d[t][2 * q + 1];
                }
            }
        }
        for (int s = 0; s < g->n_obstacles; ++s) {
            double ox, oy;
            double v = psi_vg(g, s, xj, yj, 0.0, inner, &ox, &oy);
            double tt = v + yo[(int64_t)s * W + j] / c;
            aj = aj + hc * (tt * tt);
            if (inner && v != 0.0) {
                double coef = c * tt;
                gx = gx + coef * ox;
                gy = gy + coef * oy;
            }
        }
        taug[j] = aj;
        tg[j] = 0.0;
        if (inner) {
            gr[2 * j] = gx;
            gr[2 * j + 1] = gy;
            tg[j] = gx * gx + gy * gy;
        }
    }
    double f = sc * wsum(tl, W) + wsum(tphi, W);
    double L = f + wsum(taug, W);
    if (want && gn2) *gn2 = wsum(tg, W);
    if (fout) *fout = f;
    free(tl);
    return L;
}

/* outer ALM update: y += c * row for every row; returns sum of row^2 (lane-tree order) */
static double refine_update(const orc_geom* g, const orc_params* p, const double* z,
                            double* yk, double* yo, double c) {
    const int N = p->N, W = N + 2, ms = p->maxratio_smooth;
    const double r = ms ? p->maxratio * p->maxratio : p->maxratio;
    const double mincos = cos(p->maxalpha);
    double* ti = (double*)malloc(sizeof(double) * W);
    for (int j = 0; j < W; ++j) {
        double sj = 0.0;
        if (j < N) {
            kin_row kr;
            kin_eval(&z[2 * j], &z[2 * (j + 1)], &z[2 * (j + 2)], r, mincos, ms, 0, &kr);
            double gv[3] = {kr.c1, kr.c2, kr.c3};
            for (int t = 0; t < 3; ++t) {
                yk[3 * j + t] = yk[3 * j + t] + c * gv[t];
                sj = sj + gv[t] * gv[t];
            }
        }
        for (int s = 0; s < g->n_obstacles; ++s) {
            double v = psi(g, s, z[2 * j], z[2 * j + 1], 1, 0.0);
            yo[(int64_t)s * W + j] = yo[(int64_t)s * W + j] + c * v;
            sj = sj + v * v;
        }
        ti[j] = sj;
    }
    double inf = wsum(ti, W);
    free(ti);
    return inf;
}

/* L-BFGS direction dr = -H g (two-loop recursion over the cnt newest pairs of the ring
 * hs/hy [m][2W], newest at slot head-1) */
static void lbfgs_dir(const double* gr, double* dr, const double* hs, const double* hy,
                      const double* rho, double gamma, int m, int cnt, int head, int N,
                      double* tmp) {
    const int W = N + 2;
    double ai[RF_MAXM];
    for (int j = 1; j <= N; ++j) {
        dr[2 * j] = gr[2 * j];
        dr[2 * j + 1] = gr[2 * j + 1];
    }
    for (int i = 0; i < cnt; ++i) {
        const int sl = (head - 1 - i + m) % m;
        const double* s = hs + (int64_t)sl * 2 * W;
        const double* y = hy + (int64_t)sl * 2 * W;
        ai[i] = rho[sl] * wdot(s, dr, N, tmp);
        for (int j = 1; j <= N; ++j) {
            dr[2 * j] = dr[2 * j] - ai[i] * y[2 * j];
            dr[2 * j + 1] = dr[2 * j + 1] - ai[i] * y[2 * j + 1];
        }
    }
    for (int j = 1; j <= N; ++j) {
        dr[2 * j] = gamma * dr[2 * j];
        dr[2 * j + 1] = gamma * dr[2 * j + 1];
    }
    for (int i = cnt - 1; i >= 0; --i) {
        const int sl = (head - 1 - i + m) % m;
        const double* s = hs + (int64_t)sl * 2 * W;
        const double* y = hy + (int64_t)sl * 2 * W;
        const double b = rho[sl] * wdot(y, dr, N, tmp);
        for (int j = 1; j <= N; ++j) {
            dr[2 * j] = dr[2 * j] + s[2 * j] * (ai[i] - b);
            dr[2 * j + 1] = dr[2 * j + 1] + s[2 * j + 1] * (ai[i] - b);
        }
    }
    for (int j = 1; j <= N; ++j) {
        dr[2 * j] = -dr[2 * j];
        dr[2 * j + 1] = -dr[2 * j + 1];
    }
}

/* distance along the unit direction (ux, uy) from (x0, x1), inside shape s (every h_i < 0),
 * to its boundary: the smallest positive root over the inequalities (each h_i linear in t,
 * or the ellipse's quadratic) */
static double exit_dist(const orc_geom* g, int s, double x0, double x1, double ux, double uy) {
    double t = INFINITY;
    for (int i = g->shape_first[s]; i < g->shape_first[s] + g->shape_count[s]; ++i) {
        const double* q = g->ineq_par + 6 * (int64_t)i;
        const double h = ineq_h(g, i, x0, x1);
        double ti = INFINITY;
        if (g->ineq_kind[i] == ORC_ELLIPSE) {
            const double a0 = (x0 - q[0]) / q[2], b0 = (x1 - q[1]) / q[3];
            const double da = ux / q[2], db = uy / q[3];
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
            ineq_grad(g, i, x0, x1, &gx, &gy);
            double rate = 0.0;
            rate = rate + gx * ux;
            rate = rate + gy * uy;
            if (rate > 0.0) ti = -h / rate;
        }
        if (ti >= 0.0 && ti < t) t = ti;
    }
    return t;
}

/* Restart of a stalled path (build-defined): the obstacle holding the most interior waypoints
 * (ties: the lowest index) has those waypoints moved across the start-goal chord's normal to
 * restart_margin past its boundary, all to the side their mean offset from the obstacle's
 * centre already leans to (+normal on a tie).  Returns 0 when no interior waypoint lies
 * inside an obstacle (nothing to restart from). */
static int refine_restart(const orc_geom* g, const orc_params* p, double* z, double margin,
                          double* tmp) {
    const int N = p->N, W = N + 2;
    int best = -1, bestn = 0;
    for (int s = 0; s < g->n_obstacles; ++s) {
        int n = 0;
        for (int j = 1; j <= N; ++j) n += psi(g, s, z[2 * j], z[2 * j + 1], 1, 0.0) > 0.0;
        if (n > bestn) best = s, bestn = n;
    }
    if (best < 0) return 0;
    const double cx = z[2 * (W - 1)] - z[0], cy = z[2 * (W - 1) + 1] - z[1];
    double l2 = 0.0;
    l2 = l2 + cx * cx;
    l2 = l2 + cy * cy;
    const double len = sqrt(l2);
    if (!(len > 0.0)) return 0;
    const double nx = -cy / len, ny = cx / len;
    double ox = g->shape_center[2 * best], oy = g->shape_center[2 * best + 1];
    if (isnan(ox) || isnan(oy)) ox = 0.5 * (z[0] + z[2 * (W - 1)]), oy = 0.5 * (z[1] + z[2 * (W - 1) + 1]);
    for (int j = 0; j < W; ++j) {
        tmp[j] = 0.0;
        if (j >= 1 && j <= N && psi(g, best, z[2 * j], z[2 * j + 1], 1, 0.0) > 0.0)
            tmp[j] = (z[2 * j] - ox) * nx + (z[2 * j + 1] - oy) * ny;
    }
    const double lean = wsum(tmp, W);
    const double sx = lean < 0.0 ? -nx : nx, sy = lean < 0.0 ? -ny : ny;
    for (int j = 1; j <= N; ++j) {
        if (!(psi(g, best, z[2 * j], z[2 * j + 1], 1, 0.0) > 0.0)) continue;
        const double t = exit_dist(g, best, z[2 * j], z[2 * j + 1], sx, sy);
        if (!(t < INFINITY)) continue;
        const double step = t + margin;
        z[2 * j] = z[2 * j] + step * sx;
        z[2 * j + 1] = z[2 * j + 1] + step * sy;
    }
    return 1;
}

int orc_refine(const orc_geom* g, const orc_params* p, const orc_refine_params* rp, double* wp,
               int64_t P, double* cost, double* infeas, int32_t* iters) {
    const int N = p->N, W = N + 2;
    const int64_t R = 3 * (int64_t)N + (int64_t)g->n_obstacles * W;
    const int m = rp->memory < 0 ? 0 : (rp->memory > RF_MAXM ? RF_MAXM : rp->memory);
    if (!p->penalty_smooth || !p->obstacle_smooth) return -1;
    double* y = (double*)malloc(sizeof(double) * (R > 0 ? R : 1));
    double* gr = (double*)calloc(2 * (size_t)W, sizeof(double));
    double* dr = (double*)calloc(2 * (size_t)W, sizeof(double));
    double* hs = (double*)calloc((size_t)(m > 0 ? m : 1) * 2 * W, sizeof(double));
    double* hy = (double*)calloc((size_t)(m > 0 ? m : 1) * 2 * W, sizeof(double));
    double* tmp = (double*)malloc(sizeof(double) * W);
    double* zbest = (double*)malloc(sizeof(double) * 2 * W);
    for (int64_t pi = 0; pi < P; ++pi) {
        double* z = wp + pi * (int64_t)W * 2;
        double *yk = y, *yo = y + 3 * N;
        double best_inf = INFINITY, f = 0.0, inf = 0.0;
        int32_t used = 0;
        for (int rs = 0; rs <= (rp->n_restart > 0 ? rp->n_restart : 0); ++rs) {
        if (rs > 0 && !refine_restart(g, p, z, rp->restart_margin, tmp)) break;
        for (int64_t i = 0; i < R; ++i) y[i] = 0.0;
        for (int k = 0; k < 2 * W; ++k) gr[k] = dr[k] = 0.0;
        double c = rp->c0, alpha = rp->alpha0, prev = INFINITY;
        inf = 0.0;
        for (int o = 0; o < rp->n_outer; ++o) {
            int cnt = 0, head = 0;
            double rho[RF_MAXM], gamma = 1.0, gn2 = 0.0;
            double Lz = refine_L(g, p, z, dr, 0.0, gr, yk, yo, c, 1, NULL, &gn2);
            for (int it = 0; it < rp->n_inner; ++it) {
                if (!(gn2 > 0.0) || !(gn2 < INFINITY)) break;
                if (sqrt(gn2) <= rp->inner_tol) break;
                double gd = 0.0, dn2 = gn2;
                if (cnt > 0) {
                    lbfgs_dir(gr, dr, hs, hy, rho, gamma, m, cnt, head, N, tmp);
                    gd = wdot(gr, dr, N, tmp);
                    if (!(gd < 0.0)) cnt = 0;
                    else dn2 = wdot(dr, dr, N, tmp);
                }
                if (cnt == 0) {
                    for (int j = 1; j <= N; ++j) {
                        dr[2 * j] = -gr[2 * j];
                        dr[2 * j + 1] = -gr[2 * j + 1];
                    }
                    gd = -gn2;
                    dn2 = gn2;
                }
                double a = fmin(cnt > 0 ? 1.0 : alpha * 2.0, rp->max_step / sqrt(dn2));
                int ok = 0;
                for (int b = 0; b < rp->max_backtrack; ++b) {
                    double Lt = refine_L(g, p, z, dr, a, NULL, yk, yo, c, 0, NULL, NULL);
                    if (Lt <= Lz + (rp->armijo * a) * gd) {
                        ok = 1;
                        break;
                    }
                    a = a * 0.5;
                }
                if (!ok) {
                    if (cnt > 0) {  /* retry along -g */
                        cnt = 0;
                        continue;
                    }
                    break;
                }
                double* hsl = hs + (int64_t)head * 2 * W;
                double* hyl = hy + (int64_t)head * 2 * W;
                for (int j = 1; j <= N; ++j) {
                    for (int e = 0; e < 2; ++e) {
                        const double st = a * dr[2 * j + e];
                        if (m > 0) {
                            hsl[2 * j + e] = st;
                            hyl[2 * j + e] = gr[2 * j + e];
                        }
                        z[2 * j + e] = z[2 * j + e] + st;
                    }
                }
                alpha = a;
                ++used;
                Lz = refine_L(g, p, z, dr, 0.0, gr, yk, yo, c, 1, NULL, &gn2);
                if (m > 0) {
                    for (int j = 1; j <= N; ++j) {
                        hyl[2 * j] = gr[2 * j] - hyl[2 * j];
                        hyl[2 * j + 1] = gr[2 * j + 1] - hyl[2 * j + 1];
                    }
                    const double sy = wdot(hsl, hyl, N, tmp), yy = wdot(hyl, hyl, N, tmp);
                    if (sy > 0.0 && yy > 0.0) {
                        rho[head] = 1.0 / sy;
                        gamma = sy / yy;
                        head = (head + 1) % m;
                        if (cnt < m) ++cnt;
                    }
                }
            }
            inf = refine_update(g, p, z, yk, yo, c);
            if (inf > rp->theta * prev) c = fmin(c * rp->rho, rp->c_max);
            prev = inf;
            if (sqrt(inf) <= rp->delta) break;
        }
        if (rs == 0 || inf < best_inf) {  /* the best attempt by sum g^2 (first on ties) */
            best_inf = inf;
            memcpy(zbest, z, sizeof(double) * 2 * W);
        }
        if (sqrt(inf) <= rp->delta) break;
        }
        memcpy(z, zbest, sizeof(double) * 2 * W);
        inf = best_inf;
        refine_L(g, p, z, dr, 0.0, NULL, yk, yo, rp->c0, 0, &f, NULL);
        if (cost) cost[pi] = f;
        if (infeas) infeas[pi] = inf;
        if (iters) iters[pi] = used;
    }
    free(y);
    free(gr);
    free(dr);
    free(hs);
    free(hy);
    free(tmp);
    free(zbest);
    return 0;
}

/* ======================================================================================
 * Transverse Mercator: geographic JGD2000 / JGD2011 (EPSG:4612 /
 * 6668, lon-lat order as geopandas' to_crs uses) <-> Japan Plane Rectangular CS (EPSG:2443 +
 * zone - 1), the transform pyproj applies at data_manager.py:24-26 / 84-85 and
 * path_generation/main.py:106-115.  Krueger series in n to order 6 (Karney 2011), geodetic
 * from conformal latitude by 2 Newton steps on tau = tan(phi).  Pinned: the reference's own
 * shapefiles (data/processed/{land,populated_area,no_fly_zone}/ .shp) against the plane
 * coordinates they were written from (tests/golden/make_crs_golden.py), <= 3e-14 deg. */
#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif
typedef struct {
    double a, f, k0, lat0_deg, lon0_deg, fe, fn;
} orc_tm;

typedef struct {
    double n, e, e2, A, xi0, lon0, alpha[6], beta[6];
} tm_k;

static void tm_prepare(const orc_tm* t, tm_k* k) {
    const double n = t->f / (2.0 - t->f), n2 = n * n, n3 = n2 * n, n4 = n3 * n, n5 = n4 * n,
                 n6 = n5 * n;
    k->n = n;
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
    /* xi of the origin latitude on the central meridian */
    const double phi0 = t->lat0_deg * (M_PI / 180.0), s0 = sin(phi0);
    const double tt = sinh(atanh(s0) - k->e * atanh(k->e * s0));
    const double xp = atan2(tt, 1.0);
    double xi = xp;
    for (int j = 0; j < 6; ++j) xi = xi + k->alpha[j] * sin(2.0 * (j + 1) * xp);
    k->xi0 = xi;
}

/* Krueger series sum_{j=1..6} c_j sin(2 j zeta), zeta = xi + i eta, by complex Clenshaw
 * summation (as PROJ's tmerc evaluates it): b_k = c_k + 2 cos(2 zeta) b_{k+1} - b_{k+2},
 * S = b_1 sin(2 zeta).  Re S = sum c_j sin(2j xi) cosh(2j eta), Im S = sum c_j cos(2j xi)
 * sinh(2j eta); four transcendentals instead of 24.  The device kr_sum is the same
 * operation sequence. */
static void kr_sum(const double* c, double xi, double eta, double* sr, double* si) {
    const double s2 = sin(2.0 * xi), c2 = cos(2.0 * xi);
    const double sh = sinh(2.0 * eta), ch = cosh(2.0 * eta);
    const double ar = 2.0 * (c2 * ch), ai = -2.0 * (s2 * sh);
    double y0r = 0.0, y0i = 0.0, y1r = 0.0, y1i = 0.0;
    for (int j = 5; j >= 0; --j) {
        const double tr = (ar * y0r - ai * y0i) - y1r + c[j];
        const double ti = (ar * y0i + ai * y0r) - y1i;
        y1r = y0r;
        y1i = y0i;
        y0r = tr;
        y0i = ti;
    }
    const double zr = s2 * ch, zi = c2 * sh;
    *sr = y0r * zr - y0i * zi;
    *si = y0r * zi + y0i * zr;
}

static void tm_fwd1(const orc_tm* t, const tm_k* k, double lon, double lat, double* x,
                    double* y) {
    const double phi = lat * (M_PI / 180.0), dl = lon * (M_PI / 180.0) - k->lon0;
    const double s = sin(phi);
    const double tt = sinh(atanh(s) - k->e * atanh(k->e * s));
    const double xp = atan2(tt, cos(dl));
    const double ep = atanh(sin(dl) / sqrt(1.0 + tt * tt));
    double sr, si;
    kr_sum(k->alpha, xp, ep, &sr, &si);
    const double xi = xp + sr, eta = ep + si;
    *x = t->k0 * k->A * eta + t->fe;
    *y = t->k0 * k->A * (xi - k->xi0) + t->fn;
}

static void tm_inv1(const orc_tm* t, const tm_k* k, double x, double y, double* lon,
                    double* lat) {
    const double kA = t->k0 * k->A;
    const double xi = (y - t->fn) / kA + k->xi0, eta = (x - t->fe) / kA;
    double sr, si;
    kr_sum(k->beta, xi, eta, &sr, &si);
    const double xp = xi - sr, ep = eta - si;
    const double se = sinh(ep), cx = cos(xp);
    const double taup = sin(xp) / sqrt(se * se + cx * cx);
    const double lam = atan2(se, cx);
    const double e = k->e, e2m = 1.0 - k->e2;
    /* Newton from tau'/(1 - e^2) (GeographicLib's start): 2 steps reach the 5-step fixed
     * point to within 1 ulp over |lat| <= 89.9 deg */
    double tau = taup / e2m;
    for (int it = 0; it < 2; ++it) {
        const double r = sqrt(1.0 + tau * tau);
        const double sg = sinh(e * atanh(e * tau / r));
        const double tp = tau * sqrt(1.0 + sg * sg) - sg * r;
        tau = tau + (taup - tp) * (1.0 + e2m * tau * tau) / (e2m * sqrt(1.0 + tp * tp) * r);
    }
    *lat = atan(tau) * (180.0 / M_PI);
    *lon = (lam + k->lon0) * (180.0 / M_PI);
}

void orc_tm_fwd(const orc_tm* t, const double* lonlat, int64_t n, double* xy) {
    tm_k k;
    tm_prepare(t, &k);
    for (int64_t i = 0; i < n; ++i)
        tm_fwd1(t, &k, lonlat[2 * i], lonlat[2 * i + 1], &xy[2 * i], &xy[2 * i + 1]);
}

void orc_tm_inv(const orc_tm* t, const double* xy, int64_t n, double* lonlat) {
    tm_k k;
    tm_prepare(t, &k);
    for (int64_t i = 0; i < n; ++i)
        tm_inv1(t, &k, xy[2 * i], xy[2 * i + 1], &lonlat[2 * i], &lonlat[2 * i + 1]);
}

/* DEM reprojection (build-defined; the reference's merge_test.tif is a
 * plane-CS DEM made outside the repository from the lat/lon mosaic mergeLL.vrt):
 * output cell (ix, iy) centre in plane units -> metres (* unit) -> inverse TM -> source pixel
 * u = (lon - lon0) / dlon, v = (lat_top - lat) / dlat.  resample 0 = nearest (GDAL's default:
 * pixel floor(u), floor(v)); 1 = bilinear on pixel centres when all four neighbours are valid
 * (else nearest).  Outside the source or nodata -> nodata. */
typedef struct {
    int32_t nx, ny;
    double lon0, lat_top, dlon, dlat;
    float nodata;
    int32_t pad;
} orc_geo_grid;

void orc_reproject(const orc_tm* t, const float* src, const orc_geo_grid* g,
                   const orc_raster* dst, double unit, int resample, float* out) {
    tm_k k;
    tm_prepare(t, &k);
    for (int64_t iy = 0; iy < dst->ny; ++iy) {
        for (int64_t ix = 0; ix < dst->nx; ++ix) {
            const double xc = dst->x0 + ((double)ix + 0.5) * dst->dx;
            const double yc = dst->y_top - ((double)iy + 0.5) * dst->dy;
            double lon, lat;
            tm_inv1(t, &k, xc * unit, yc * unit, &lon, &lat);
            const double u = (lon - g->lon0) / g->dlon, v = (g->lat_top - lat) / g->dlat;
            float val = g->nodata;
            const double fu = floor(u), fv = floor(v);
            if (fu >= 0.0 && fu < (double)g->nx && fv >= 0.0 && fv < (double)g->ny) {
                val = src[(int64_t)fv * g->nx + (int64_t)fu];
                if (resample == 1) {
                    const double uu = u - 0.5, vv = v - 0.5;
                    const double bu = floor(uu), bv = floor(vv);
                    if (bu >= 0.0 && bu + 1.0 < (double)g->nx && bv >= 0.0 &&
                        bv + 1.0 < (double)g->ny) {
                        const int64_t i0 = (int64_t)bv * g->nx + (int64_t)bu;
                        const float a00 = src[i0], a01 = src[i0 + 1], a10 = src[i0 + g->nx],
                                    a11 = src[i0 + g->nx + 1];
                        if (a00 != g->nodata && a01 != g->nodata && a10 != g->nodata &&
                            a11 != g->nodata) {
                            const double wu = uu - bu, wv = vv - bv;
                            const double top = (double)a00 + wu * ((double)a01 - (double)a00);
                            const double bot = (double)a10 + wu * ((double)a11 - (double)a10);
                            val = (float)(top + wv * (bot - top));
                        }
                    }
                }
            }
            out[iy * dst->nx + ix] = val;
        }
    }
}

/* ======================================================================================
 * Land polygons from the DEM: load_dem_polygons_from_geotiff
 * (data_manager.py:11-19: mask, rasterio.features.shapes, 4-connectivity) followed by
 * DataProcessor.process_polygons (data_processor.py:15-75).  cv2.minAreaRect + boxPoints are
 * restated in float32 after OpenCV's convexHull / rotatingCalipers / RotatedRect::points;
 * the restatement is pinned on the reference's populated_area output (tests). */
typedef struct {
    double min_area, large_area, min_approx_area;
    int32_t divisions, pad;
} orc_polyproc;

typedef struct {
    float x, y;
} orc_p2f;

static int p2f_cmp(const void* a, const void* b) {
    const orc_p2f *p = (const orc_p2f*)a, *q = (const orc_p2f*)b;
    if (p->x != q->x) return p->x < q->x ? -1 : 1;
    if (p->y != q->y) return p->y < q->y ? -1 : 1;
    return 0;
}

static double p2f_cross(orc_p2f o, orc_p2f a, orc_p2f b) {
    return ((double)a.x - o.x) * ((double)b.y - o.y) - ((double)a.y - o.y) * ((double)b.x - o.x);
}

/* strictly convex hull, counter-clockwise, first vertex = largest (x, y); returns size */
static int orc_hull(orc_p2f* p, int n, orc_p2f* h) {
    qsort(p, n, sizeof(orc_p2f), p2f_cmp);
    int m = 0;
    for (int i = 0; i < n; ++i)
        if (m == 0 || p[i].x != p[m - 1].x || p[i].y != p[m - 1].y) p[m++] = p[i];
    if (m < 3) {
        for (int i = 0; i < m; ++i) h[i] = p[i];
        return m;
    }
    int k = 0;
    for (int i = 0; i < m; ++i) {
        while (k >= 2 && p2f_cross(h[k - 2], h[k - 1], p[i]) <= 0) --k;
        h[k++] = p[i];
    }
    for (int i = m - 2, t = k + 1; i >= 0; --i) {
        while (k >= t && p2f_cross(h[k - 2], h[k - 1], p[i]) <= 0) --k;
        h[k++] = p[i];
    }
    --k;
    int top = 0;
    for (int i = 1; i < k; ++i)
        if (h[i].x > h[top].x || (h[i].x == h[top].x && h[i].y > h[top].y)) top = i;
    orc_p2f* tmp = (orc_p2f*)malloc(sizeof(orc_p2f) * k);
    for (int i = 0; i < k; ++i) tmp[i] = h[(top + i) % k];
    for (int i = 0; i < k; ++i) h[i] = tmp[i];
    free(tmp);
    return k;
}

/* cv2.boxPoints(cv2.minAreaRect(pts)) -> np.intp; pts as doubles (cast to float32) */
void orc_min_area_rect(const double* xy, int64_t n, int64_t* box) {
    orc_p2f* p = (orc_p2f*)malloc(sizeof(orc_p2f) * (n > 0 ? n : 1));
    orc_p2f* h = (orc_p2f*)malloc(sizeof(orc_p2f) * (2 * n + 2));
    for (int64_t i = 0; i < n; ++i) p[i].x = (float)xy[2 * i], p[i].y = (float)xy[2 * i + 1];
    const int m = n > 0 ? orc_hull(p, (int)n, h) : 0;
    float cx, cy, w, hh, ang;
    if (m > 2) {
        float* vx = (float*)malloc(sizeof(float) * m);
        float* vy = (float*)malloc(sizeof(float) * m);
        float* iv = (float*)malloc(sizeof(float) * m);
        int left = 0, bottom = 0, right = 0, top = 0;
        float left_x = h[0].x, right_x = h[0].x, top_y = h[0].y, bottom_y = h[0].y;
        orc_p2f pt0 = h[0];
        for (int i = 0; i < m; ++i) {
            if (pt0.x < left_x) left_x = pt0.x, left = i;
            if (pt0.x > right_x) right_x = pt0.x, right = i;
            if (pt0.y > top_y) top_y = pt0.y, top = i;
            if (pt0.y < bottom_y) bottom_y = pt0.y, bottom = i;
            orc_p2f pt = h[(i + 1) < m ? i + 1 : 0];
            double dx = pt.x - pt0.x, dy = pt.y - pt0.y;
            vx[i] = (float)dx, vy[i] = (float)dy;
            iv[i] = (float)(1. / sqrt(dx * dx + dy * dy));
            pt0 = pt;
        }
        float orientation = 0;
        {
            double ax = vx[m - 1], ay = vy[m - 1];
            for (int i = 0; i < m; ++i) {
                double bx = vx[i], by = vy[i], cv = ax * by - ay * bx;
                if (cv != 0) {
                    orientation = cv > 0 ? 1.f : -1.f;
                    break;
                }
                ax = bx, ay = by;
            }
        }
        float ba = orientation, bb = 0, minarea = FLT_MAX, sa = 0, sw = 0, sb = 0, sh = 0;
        int seq[4] = {bottom, right, top, left}, sl = 0, sbot = 0;
        for (int k = 0; k < m; ++k) {
            float dp[4];
            dp[0] = +ba * vx[seq[0]] + bb * vy[seq[0]];
            dp[1] = -bb * vx[seq[1]] + ba * vy[seq[1]];
            dp[2] = -ba * vx[seq[2]] - bb * vy[seq[2]];
            dp[3] = +bb * vx[seq[3]] - ba * vy[seq[3]];
            float maxcos = dp[0] * iv[seq[0]];
            int me = 0;
            for (int i = 1; i < 4; ++i) {
                float ca = dp[i] * iv[seq[i]];
                if (ca > maxcos) me = i, maxcos = ca;
            }
            const int pi = seq[me];
            const float lx = vx[pi] * iv[pi], ly = vy[pi] * iv[pi];
            if (me == 0) ba = lx, bb = ly;
            else if (me == 1) ba = ly, bb = -lx;
            else if (me == 2) ba = -lx, bb = -ly;
            else ba = -ly, bb = lx;
            seq[me] = (seq[me] + 1 == m) ? 0 : seq[me] + 1;
            float dx = h[seq[1]].x - h[seq[3]].x, dy = h[seq[1]].y - h[seq[3]].y;
            const float width = dx * ba + dy * bb;
            dx = h[seq[2]].x - h[seq[0]].x, dy = h[seq[2]].y - h[seq[0]].y;
            const float height = -dx * bb + dy * ba;
            const float area = width * height;
            if (area <= minarea) {
                minarea = area, sl = seq[3], sa = ba, sw = width, sb = bb, sh = height;
                sbot = seq[0];
            }
        }
        const float A1 = sa, B1 = sb, A2 = -sb, B2 = sa;
        const float C1 = A1 * h[sl].x + h[sl].y * B1, C2 = A2 * h[sbot].x + h[sbot].y * B2;
        const float idet = 1.f / (A1 * B2 - A2 * B1);
        const float px = (C1 * B2 - C2 * B1) * idet, py = (A1 * C2 - A2 * C1) * idet;
        const float o1x = A1 * sw, o1y = B1 * sw, o2x = A2 * sh, o2y = B2 * sh;
        cx = px + (o1x + o2x) * 0.5f;
        cy = py + (o1y + o2y) * 0.5f;
        w = (float)sqrt((double)o1x * o1x + (double)o1y * o1y);
        hh = (float)sqrt((double)o2x * o2x + (double)o2y * o2y);
        ang = (float)atan2((double)o1y, (double)o1x);
        free(vx), free(vy), free(iv);
    } else if (m == 2) {
        cx = (h[0].x + h[1].x) * 0.5f, cy = (h[0].y + h[1].y) * 0.5f;
        double dx = h[1].x - h[0].x, dy = h[1].y - h[0].y;
        w = (float)sqrt(dx * dx + dy * dy), hh = 0;
        ang = (float)atan2(dy, dx);
    } else {
        cx = m ? h[0].x : 0, cy = m ? h[0].y : 0, w = hh = 0, ang = 0;
    }
    ang = (float)(ang * 180 / M_PI);
    const double a_ = ang * M_PI / 180.;
    const float b = (float)cos(a_) * 0.5f, a = (float)sin(a_) * 0.5f;
    float q[8];
    q[0] = cx - a * hh - b * w;
    q[1] = cy + b * hh - a * w;
    q[2] = cx + a * hh - b * w;
    q[3] = cy - b * hh - a * w;
    q[4] = 2 * cx - q[0];
    q[5] = 2 * cy - q[1];
    q[6] = 2 * cx - q[2];
    q[7] = 2 * cy - q[3];
    for (int i = 0; i < 8; ++i) box[i] = (int64_t)q[i];
    free(p), free(h);
}

static double box_area8(const int64_t* b) {
    double s = 0.0;
    for (int i = 0; i < 4; ++i) {
        const int j = (i + 1) & 3;
        s += (double)b[2 * i] * (double)b[2 * j + 1] - (double)b[2 * j] * (double)b[2 * i + 1];
    }
    return fabs(0.5 * s);
}

/* sequential union-find labelling, root = smallest index; cut arrays as uam_dem_polygons */
static int32_t uf_find(int32_t* L, int32_t x) {
    while (L[x] != x) {
        L[x] = L[L[x]];
        x = L[x];
    }
    return x;
}

static void label4(int32_t nx, int32_t ny, const int32_t* colbox, const int32_t* rowbox,
                   int32_t* L) {
    for (int32_t y = 0; y < ny; ++y)
        for (int32_t x = 0; x < nx; ++x) {
            const int64_t i = (int64_t)y * nx + x;
            if (L[i] < 0) continue;
            if (x + 1 < nx && L[i + 1] >= 0 && (!colbox || colbox[x] == colbox[x + 1])) {
                int32_t a = uf_find(L, (int32_t)i), b = uf_find(L, (int32_t)(i + 1));
                if (a != b) L[a > b ? a : b] = a < b ? a : b;
            }
            if (y + 1 < ny && L[i + nx] >= 0 && (!rowbox || rowbox[y] == rowbox[y + 1])) {
                int32_t a = uf_find(L, (int32_t)i), b = uf_find(L, (int32_t)(i + nx));
                if (a != b) L[a > b ? a : b] = a < b ? a : b;
            }
        }
    for (int64_t i = 0; i < (int64_t)nx * ny; ++i)
        if (L[i] >= 0) L[i] = uf_find(L, (int32_t)i);
}

typedef struct {
    int32_t n, cnt, x0, y0, x1, y1, root;
} orc_comp;

/* components of a labelled grid in raster order of their roots, with per-row extents */
static orc_comp* comps_of(int32_t nx, int32_t ny, const int32_t* L, int32_t* ncomp,
                          int32_t** rxmin, int32_t** rxmax, int64_t** roff) {
    const int64_t n = (int64_t)nx * ny;
    int32_t* id = (int32_t*)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
    int32_t nc = 0;
    for (int64_t i = 0; i < n; ++i) id[i] = (L[i] == (int32_t)i) ? nc++ : -1;
    orc_comp* c = (orc_comp*)calloc(nc > 0 ? nc : 1, sizeof(orc_comp));
    for (int32_t k = 0; k < nc; ++k) c[k].x0 = c[k].y0 = INT32_MAX, c[k].x1 = c[k].y1 = -1;
    for (int64_t i = 0; i < n; ++i) {
        if (L[i] < 0) continue;
        orc_comp* q = &c[id[L[i]]];
        const int32_t y = (int32_t)(i / nx), x = (int32_t)(i % nx);
        q->cnt++;
        if (x < q->x0) q->x0 = x;
        if (x > q->x1) q->x1 = x;
        if (y < q->y0) q->y0 = y;
        if (y > q->y1) q->y1 = y;
        q->root = L[i];
    }
    int64_t rows = 0;
    *roff = (int64_t*)malloc(sizeof(int64_t) * (nc > 0 ? nc : 1));
    for (int32_t k = 0; k < nc; ++k) (*roff)[k] = rows, rows += c[k].y1 - c[k].y0 + 1;
    *rxmin = (int32_t*)malloc(sizeof(int32_t) * (rows > 0 ? rows : 1));
    *rxmax = (int32_t*)malloc(sizeof(int32_t) * (rows > 0 ? rows : 1));
    for (int64_t r = 0; r < rows; ++r) (*rxmin)[r] = INT32_MAX, (*rxmax)[r] = -1;
    for (int64_t i = 0; i < n; ++i) {
        if (L[i] < 0) continue;
        const int32_t k = id[L[i]], y = (int32_t)(i / nx), x = (int32_t)(i % nx);
        const int64_t s = (*roff)[k] + (y - c[k].y0);
        if (x < (*rxmin)[s]) (*rxmin)[s] = x;
        if (x > (*rxmax)[s]) (*rxmax)[s] = x;
    }
    free(id);
    *ncomp = nc;
    return c;
}

static int64_t emit_region(const orc_comp* q, const int32_t* mn, const int32_t* mx,
                           const double* xlo, const double* xhi, const double* ylo,
                           const double* yhi, double min_approx, int64_t* out, int64_t nout,
                           int64_t cap) {
    const int32_t rows = q->y1 - q->y0 + 1;
    double* pts = (double*)malloc(sizeof(double) * 8 * rows);
    int64_t np = 0;
    for (int32_t r = 0; r < rows; ++r) {
        if (mn[r] > mx[r]) continue;
        const int32_t row = q->y0 + r;
        const double xs[2] = {xlo[mn[r]], xhi[mx[r]]};
        for (int e = 0; e < 2; ++e) {
            pts[2 * np] = xs[e], pts[2 * np + 1] = yhi[row], ++np;
            pts[2 * np] = xs[e], pts[2 * np + 1] = ylo[row], ++np;
        }
    }
    if (np == 0) {
        free(pts);
        return nout;
    }
    int64_t box[8];
    orc_min_area_rect(pts, np, box);
    free(pts);
    if (!(box_area8(box) > min_approx)) return nout;
    if (nout < cap)
        for (int i = 0; i < 8; ++i) out[8 * nout + i] = box[i];
    return nout + 1;
}

/* -> number of rectangles (rects written up to cap) */
int64_t orc_dem_polygons(const float* dem, const orc_raster* rd, float thr, double unit,
                         const orc_polyproc* pp, int64_t* rects, int64_t cap) {
    const int32_t nx = rd->nx, ny = rd->ny;
    const int64_t n = (int64_t)nx * ny;
    const double X0 = rd->x0 * unit, DX = rd->dx * unit, Y0 = rd->y_top * unit, DY = rd->dy * unit;
    int32_t* L = (int32_t*)malloc(sizeof(int32_t) * n);
    for (int64_t i = 0; i < n; ++i) {
        const float v = dem[i];
        const int m = (thr == -9999.0f) ? (v == -9999.0f) : (v > thr);
        L[i] = m ? (int32_t)i : -1;
    }
    label4(nx, ny, NULL, NULL, L);
    int32_t nc, *mn, *mx;
    int64_t* roff;
    orc_comp* c = comps_of(nx, ny, L, &nc, &mn, &mx, &roff);
    double *xlo = (double*)malloc(sizeof(double) * nx), *xhi = (double*)malloc(sizeof(double) * nx);
    double *ylo = (double*)malloc(sizeof(double) * ny), *yhi = (double*)malloc(sizeof(double) * ny);
    for (int32_t i = 0; i < nx; ++i) xlo[i] = X0 + i * DX, xhi[i] = X0 + (i + 1) * DX;
    for (int32_t j = 0; j < ny; ++j) yhi[j] = Y0 - j * DY, ylo[j] = Y0 - (j + 1) * DY;
    const double cell = fabs(DX * DY);
    const int D = pp->divisions;
    int64_t nout = 0;
    for (int32_t k = 0; k < nc; ++k) {
        const double area = c[k].cnt * cell;
        if (!(area > pp->min_area)) continue;
        if (!(area > pp->large_area)) {
            nout = emit_region(&c[k], mn + roff[k], mx + roff[k], xlo, xhi, ylo, yhi,
                               pp->min_approx_area, rects, nout, cap);
            continue;
        }
        const double minx = X0 + c[k].x0 * DX, maxx = X0 + (c[k].x1 + 1) * DX;
        const double maxy = Y0 - c[k].y0 * DY, miny = Y0 - (c[k].y1 + 1) * DY;
        const double ddx = (maxx - minx) / D, ddy = (maxy - miny) / D;
        const int32_t W0 = c[k].x1 - c[k].x0 + 1, H0 = c[k].y1 - c[k].y0 + 1;
        int32_t *co = (int32_t*)malloc(sizeof(int32_t) * W0 * D),
                *cb = (int32_t*)malloc(sizeof(int32_t) * W0 * D);
        int32_t *ro = (int32_t*)malloc(sizeof(int32_t) * H0 * D),
                *rb = (int32_t*)malloc(sizeof(int32_t) * H0 * D);
        double *sxl = (double*)malloc(sizeof(double) * W0 * D), *sxh = (double*)malloc(sizeof(double) * W0 * D);
        double *syl = (double*)malloc(sizeof(double) * H0 * D), *syh = (double*)malloc(sizeof(double) * H0 * D);
        int32_t ws = 0, hs = 0;
        for (int32_t col = c[k].x0; col <= c[k].x1; ++col)
            for (int j = 0; j < D; ++j) {
                const double lo = fmax(xlo[col], minx + j * ddx), hi = fmin(xhi[col], minx + (j + 1) * ddx);
                if (hi > lo) co[ws] = col, cb[ws] = j, sxl[ws] = lo, sxh[ws] = hi, ++ws;
            }
        for (int32_t row = c[k].y0; row <= c[k].y1; ++row)
            for (int kk = D - 1; kk >= 0; --kk) {
                const double lo = fmax(ylo[row], miny + kk * ddy), hi = fmin(yhi[row], miny + (kk + 1) * ddy);
                if (hi > lo) ro[hs] = row, rb[hs] = kk, syl[hs] = lo, syh[hs] = hi, ++hs;
            }
        int32_t* L2 = (int32_t*)malloc(sizeof(int32_t) * ws * hs);
        for (int32_t t = 0; t < hs; ++t)
            for (int32_t s2 = 0; s2 < ws; ++s2) {
                const int64_t i = (int64_t)t * ws + s2;
                L2[i] = (L[(int64_t)ro[t] * nx + co[s2]] == c[k].root) ? (int32_t)i : -1;
            }
        label4(ws, hs, cb, rb, L2);
        int32_t np2, *pmn, *pmx;
        int64_t* poff;
        orc_comp* pc = comps_of(ws, hs, L2, &np2, &pmn, &pmx, &poff);
        /* boxes j outer, k inner; within a box, raster order of the piece's first cell */
        for (int j = 0; j < D; ++j)
            for (int kk = 0; kk < D; ++kk)
                for (int32_t q = 0; q < np2; ++q)
                    if (cb[pc[q].x0] == j && rb[pc[q].y0] == kk)
                        nout = emit_region(&pc[q], pmn + poff[q], pmx + poff[q], sxl, sxh, syl,
                                           syh, pp->min_approx_area, rects, nout, cap);
        free(pc), free(pmn), free(pmx), free(poff), free(L2);
        free(co), free(cb), free(ro), free(rb), free(sxl), free(sxh), free(syl), free(syh);
    }
    free(c), free(mn), free(mx), free(roff), free(L), free(xlo), free(xhi), free(ylo), free(yhi);
    return nout;
}
