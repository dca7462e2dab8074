/*
 * uampath.h -- C ABI of libuampath.so, the MI355X (gfx950) batched candidate-path cost
 * evaluator for the uam_path_planning hot path.
 *
 * The reference (nomaporon/uam_path_planning) has no FFI: its boundary is the Python class
 * surface of geo_simulation_project/path_generation.  Each entry point below replaces one
 * reference call (file:line relative to /root/reference/geo_simulation_project/); the Python
 * package uam_path_planning_amd keeps those class names and binds these symbols with ctypes
 * (INTEGRATION.md shows the binding a maintainer would add).
 *
 *   uam_set_geometry     RegionMap.add_obstacles / new_region / add_shape(s)_to_region
 *                        (path_generation/region_map.py:14-56) + polygon()/ball()/square()
 *                        inequalities (polygon.py:7-143, ball.py:7-52, square.py:6-65)
 *   uam_set_params       Problem.params / set_weight / options (problem.py:12-34) and the
 *                        OpEn parameter vector p = [xs, xg, maxratio, maxalpha, e, w...]
 *                        (solver.py:60-78)
 *   uam_eval_points      Problem.get_total_penalty_function / get_penalty_function(region|None)
 *                        (problem.py:49-82), QuadraticObstacle.contains / Map.collides
 *                        (quadratic_obstacle.py:89-94, map.py:41-43)
 *   uam_eval_waypoints   Problem.get_cost (problem.py:38-44) + get_nonlincon (84-114) +
 *                        length_of (130-146), batched over paths
 *   uam_eval_generated   Main.run candidate loop (main.py:158-193) with Solver.create_x_init
 *                        (solver.py:103-136) fused on device
 *   uam_gen_paths        Solver.create_x_init (solver.py:103-136), batched
 *   uam_argmin           main.py:175-180 best-candidate selection
 *   uam_path_length      Problem.length_of (problem.py:130-146) for arbitrary point counts
 *   uam_raster_build     map_generation DataManager.load_dem_polygons_from_geotiff mask
 *                        (map_generation/data_manager.py:11-17) + the region / no-fly
 *                        penalty at every cell centre: the per-cell cost record the raster
 *                        mode gathers
 *   uam_dem_mosaic       the VRT tile mosaic (data/raw/nagasaki_geotiff/mergeLL.vrt:1-10)
 *
 * Conventions: all array pointers marked _dev are device pointers (hipMalloc'd or torch
 * CUDA tensors); the caller owns every buffer; the library never frees caller memory.
 * Streams are hipStream_t passed as void* (NULL = default stream).  Calls are asynchronous
 * on that stream except uam_set_geometry.  Every function returns UAM_OK (0) or a negative
 * status; uam_last_error() returns a thread-local message for the last failure.
 */
#ifndef UAMPATH_H
#define UAMPATH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 5): uam_eval_generated gained summary_dev / block / packed_dev and
 * uam_eval_generated3d packed_dev, and the _s / _p entry points were folded into them */
#define UAM_ABI_VERSION 2
#define UAM_MAX_REGIONS 16
#define UAM_RECORD_BYTES 16

enum {
    UAM_OK = 0,
    UAM_E_INVALID = -1, /* bad argument: the reference raises ValueError/AssertionError */
    UAM_E_HIP = -2,     /* HIP runtime failure */
    UAM_E_NOMEM = -3,
    UAM_E_STATE = -4,   /* call order: e.g. eval before set_geometry / set_params */
    UAM_E_VERSION = -5, /* abi_version field does not match UAM_ABI_VERSION */
    UAM_E_DEVICE = -6   /* a device-side consistency check of an earlier call failed: that
                           call's outputs were poisoned (uam_device_status) */
};

/* inequality kinds h(x) <= 0 (parameters p[0..5]) */
enum {
    UAM_INEQ_HALFPLANE = 0, /* polygon edge a->b: h = s*((by-ay)*(x0-ax) - (bx-ax)*(x1-ay));
                               p = {ax, ay, bx-ax, by-ay, s = -sgn, 0} (polygon.py:69-71,98) */
    UAM_INEQ_ELLIPSE = 1,   /* h = ((x0-c0)/r1)^2 + ((x1-c1)/r2)^2 - 1; p = {c0,c1,r1,r2,0,0} */
    UAM_INEQ_AXIS = 2       /* square side h = s*(x_k - c) - r; p = {k, c, r, s, 0, 0} */
};

enum { UAM_MODE_ANALYTIC = 0, UAM_MODE_RASTER = 1, UAM_MODE_VOLUME = 2 };

/* record flag bits (record = {float phi, float psi_nfz, float dem, uint32 flags}; a volume
 * column = {float terrain, uint32 flags}) */
enum { UAM_FLAG_NFZ = 1u, UAM_FLAG_MASK = 2u, UAM_FLAG_NODATA = 4u };

typedef struct uam_ctx uam_ctx;
typedef void* uam_stream; /* hipStream_t */

/* Host-side flat geometry.  Shapes: no-fly obstacles [0, n_obstacles) in add order, then
 * region shapes region-major; region r owns shapes [region_first[r], region_first[r+1]). */
typedef struct {
    uint32_t abi_version;
    int32_t n_ineq;
    const int32_t* ineq_kind;    /* [n_ineq] */
    const double* ineq_par;      /* [n_ineq][6] */
    int32_t n_shapes;
    const int32_t* shape_first;  /* [n_shapes] first inequality */
    const int32_t* shape_count;  /* [n_shapes] number of inequalities (>= 1) */
    const double* shape_center;  /* [n_shapes][2]; NaN => penalty not normalised */
    int32_t n_obstacles;
    int32_t n_regions;           /* <= UAM_MAX_REGIONS */
    const int32_t* region_first; /* [n_regions + 1] */
} uam_geometry;

/* Problem options + OpEn parameter vector. */
typedef struct {
    uint32_t abi_version;
    int32_t N;               /* interior waypoints; a path has W = N + 2 points */
    int32_t length_smooth;   /* problem.py:13-16 */
    int32_t penalty_smooth;
    int32_t obstacle_smooth;
    int32_t maxratio_smooth;
    int32_t quirk_length;    /* 1 = reference get_cost length term: y = [anchor, p_0..p_{N+1}],
                                first N+1 segments (drops p_N->p_{N+1}); 0 = all segments */
    int32_t anchor_mode;     /* 0: anchor = each path's p_0 (segment is 0); 1: anchor_x/y
                                (the map.x_start baked into a reference solver build) */
    double anchor_x, anchor_y;
    double maxratio, maxalpha, enlargement;
    double altitude;         /* cruise altitude for min-clearance (raster mode), metres */
    double weights[UAM_MAX_REGIONS];
} uam_params;

/* Raster geotransform (GeoTIFF convention: row 0 is the northern edge).
 * cell (ix, iy) covers x in [x0 + ix*dx, x0 + (ix+1)*dx), y in (y_top - (iy+1)*dy, y_top - iy*dy];
 * a point maps to ix = floor((x - x0) * (1/dx)), iy = floor((y_top - y) * (1/dy)) in float64. */
typedef struct {
    int32_t nx, ny;
    double x0, y_top, dx, dy;
    float nodata;          /* DEM nodata value (-9999 in the reference DEM) */
    float dem_threshold;   /* data_manager.py:11-17 mask: (dem == -9999) if thr == -9999 else
                              (dem > thr) */
} uam_raster_desc;

/* 3-D risk volume (BASELINE config 5; no reference counterpart; SURVEY §8(d)'s layout): the
 * raster's x/y grid times nz altitude layers [z0 + iz*dz, z0 + (iz+1)*dz) in metres,
 * iz = floor((z - z0) * (1/dz)).  One device buffer (uam_volume_shape): 8-B voxels
 * {float risk, float psi_nfz} [ny][nx][nz] (layer fastest), then at col_offset the 8-B column
 * plane {float terrain (+0 for nodata), uint32 flags} [ny][nx]. */
typedef struct {
    int32_t nx, ny, nz;
    double x0, y_top, dx, dy;
    double z0, dz;
} uam_volume_desc;

/* Per-path outputs (device pointers, any may be NULL).  Index p of a path. */
typedef struct {
    double* cost;          /* get_cost (problem.py:38-44) */
    double* length_q;      /* the length term inside get_cost (quirk per params) */
    double* length;        /* true polyline length, non-smooth (solver.py:49) */
    double* kin_sum;       /* sum of the 3N kinematic g rows (problem.py:100-107) */
    double* nfz_sum;       /* sum of the no-fly g rows (problem.py:109-112) */
    int32_t* nfz_hits;     /* waypoints inside a no-fly zone (Map.collides) */
    double* min_clearance; /* raster: altitude - max terrain over the waypoints; volume: min
                              over waypoints of (waypoint altitude - terrain); analytic NaN */
    int32_t* offmap;       /* raster: waypoints outside the raster */
    int32_t* cells;        /* [P][W] raster cell index iy*nx+ix, -1 off-raster (raster only) */
    double* g_rows;        /* [P][3N + n_obstacles*W] full get_nonlincon vector (analytic) */
    int32_t* best_fval_idx;   /* uam_eval_generated only: [Q] per pair, the displacement index
                                 the reference keeps as "Min fval result" (main.py:175-177) */
    int32_t* best_length_idx; /* [Q] "Min path length result" (main.py:178-180) */
    int32_t* below_terrain;   /* volume mode: waypoints whose altitude layer lies below the
                                 column's terrain */
} uam_path_outputs;

/* Batched refinement: the reference's OpEn ALM problem
 * min get_cost s.t. get_nonlincon in {0} (solver.py:82-93), solved per path by n_outer ALM
 * updates (y += c g; c = min(c rho, c_max) when sum g^2 > theta * previous; stop when
 * sqrt(sum g^2) <= delta) around up to n_inner L-BFGS steps (memory pairs, 0..8; 0 = steepest
 * descent) on L = f + sum (c/2)(g + y/c)^2 with Armijo backtracking, stopping when
 * |grad L| <= inner_tol.  First trial step: 1 (L-BFGS) or 2 * previous step (steepest),
 * capped so the waypoint move is <= max_step (km).  Definition: oracle/uam_oracle.c
 * orc_refine.  Needs penalty_smooth and obstacle_smooth. */
typedef struct {
    int32_t n_outer, n_inner, max_backtrack, memory;
    double c0, rho, c_max, alpha0, armijo, theta, max_step, inner_tol, delta;
    int32_t n_restart;       /* restarts of a path ending with sqrt(sum g^2) > delta (0: none):
                                the obstacle holding most interior waypoints has them moved
                                along the start-goal chord's normal to restart_margin km past
                                its boundary, multipliers and penalty reset; the attempt with
                                the smallest sum g^2 is returned (oracle refine_restart) */
    double restart_margin;
} uam_refine_params;

int uam_abi_version(void);
const char* uam_last_error(void);
int uam_device_count(int* n);

int uam_ctx_create(int device, uam_ctx** out);
void uam_ctx_destroy(uam_ctx* ctx);

/* Copies the geometry to the device (synchronous). */
int uam_set_geometry(uam_ctx* ctx, const uam_geometry* geom);
/* Stores params and computes per-shape normalisers psi(centre) on the device. */
int uam_set_params(uam_ctx* ctx, const uam_params* params, uam_stream stream);

/* Per point (pts_dev [n][2] f64): phi = total penalty, phi_regions [n][n_regions] weighted
 * region penalties, obs_norm = get_penalty_function(None), psi_raw = sum of raw obstacle psi
 * (constraint semantics), collide = Map.collides. */
int uam_eval_points(uam_ctx* ctx, const double* pts_dev, int64_t n, double* phi_dev,
                    double* phi_regions_dev, double* obs_norm_dev, double* psi_raw_dev,
                    int32_t* collide_dev, uam_stream stream);

/* K1: one 16-byte record per cell, row-major.  dem_dev [ny][nx] f32 (NULL = all zero). */
int uam_raster_build(uam_ctx* ctx, const uam_raster_desc* desc, const float* dem_dev,
                     void* rec_dev, uam_stream stream);

/* VRT mosaic: n_tiles tiles of th x tw f32 (tiles_dev [n_tiles][th][tw]) placed at
 * (xoff[t], yoff[t]) (DstRect) into dem_dev [ny][nx]; cells no tile covers keep their value. */
int uam_dem_mosaic(uam_ctx* ctx, const float* tiles_dev, int32_t n_tiles, int32_t th,
                   int32_t tw, const int32_t* xoff_dev, const int32_t* yoff_dev, float* dem_dev,
                   int32_t nx, int32_t ny, uam_stream stream);
/* The mosaic's source tiles (data_manager.py:11-17 over mergeLL.vrt:1-10; build-defined host
 * reader): n_tiles GeoTIFF files (classic little-endian TIFF, one Float32 band in strips, no
 * predictor, uncompressed or deflate), each th x tw, read on up to n_threads host threads
 * (0: the machine's, at most 16) into dst [n_tiles][th][tw] host memory -- page-locked for an
 * asynchronous copy to uam_dem_mosaic's tiles_dev.  A tile that cannot be read fails the call
 * (UAM_E_INVALID, its path in uam_last_error). */
int uam_read_tiles(const char* const* paths, int32_t n_tiles, int32_t th, int32_t tw, float* dst,
                   int32_t n_threads);
/* The same tiles straight into device memory tiles_dev [n_tiles][th][tw] (uam_dem_mosaic's
 * input): read on the thread pool in ~32 MiB chunks into two page-locked buffers the context
 * keeps, each chunk copied on stream while the next one is read.  Returns once the last copy
 * is enqueued (the buffers are reused after their copies complete). */
int uam_load_tiles(uam_ctx* ctx, const char* const* paths, int32_t n_tiles, int32_t th,
                   int32_t tw, float* tiles_dev, int32_t n_threads, uam_stream stream);

/* K4: pairs_dev [Q][4] (x0,y0,xf,yf), utab_dev [D][N][2] unit-arc table -> wp [Q*D][N+2][2]. */
int uam_gen_paths(uam_ctx* ctx, const double* pairs_dev, int64_t n_pairs,
                  const double* utab_dev, int32_t D, double* wp_dev, uam_stream stream);

/* K2 (raster) / K3 (analytic) over explicit waypoints wp_dev [P][N+2][2]. */
int uam_eval_waypoints(uam_ctx* ctx, int32_t mode, const uam_raster_desc* desc,
                       const void* rec_dev, const double* wp_dev, int64_t n_paths,
                       const uam_path_outputs* out, uam_stream stream);

/* K2/K3 with the candidate generator fused: path p = q*D + d.  Raster mode takes two optional
 * derived copies of rec, both built with the same block (uam_raster_summary /
 * uam_raster_pack, below; NULL = none; ignored in analytic mode): summary_dev, the gather-skip
 * bitmap the lane- and wave-per-path forms read, and packed_dev, the packed raster the sorted
 * forms read (K2h by default; without it the sorted batches run K2s on rec).  Every choice
 * gives the same outputs (uam_last_group names the sum order). */
int uam_eval_generated(uam_ctx* ctx, int32_t mode, const uam_raster_desc* desc,
                       const void* rec_dev, const uint32_t* summary_dev, int32_t block,
                       const void* packed_dev, const double* pairs_dev, int64_t n_pairs,
                       const double* utab_dev, int32_t D, const uam_path_outputs* out,
                       uam_stream stream);

/* K2 gather skip (build-defined; no reference counterpart; results unchanged).  A bitmap
 * summary of a record raster: one bit per block x block cells (blocks row-major, nby x nbx;
 * bit b in 32-bit word b / 32), set when every cell of the block has phi == +-0,
 * psi_nfz == +-0, no no-fly flag and a terrain that reads +0.0 (a nodata cell, or a dem value
 * of +0.0f).  K2 / K2s keep the bitmap in LDS and do not gather the records of waypoints in set
 * blocks: they add exactly nothing to cost, no-fly sum and hits, and +0.0 to the terrain
 * maximum, so every output stays bit-identical to uam_eval_generated.  block: a power of two in [1, 1024] with at most 65536 blocks, or 0 =
 * automatic (8, doubled until the blocks fit).  The bitmap holds ceil(nbx * nby / 32) words and
 * must be rebuilt whenever rec changes. */
int uam_raster_summary_shape(const uam_raster_desc* desc, int32_t block, int32_t* block_out,
                             int32_t* nbx, int32_t* nby);
int uam_raster_summary(uam_ctx* ctx, const uam_raster_desc* desc, const void* rec_dev,
                       int32_t block, uint32_t* summary_dev, uam_stream stream);
/* Packed raster (build-defined; no reference counterpart; results unchanged).  A derived copy
 * of rec for the sorted evaluations (K2h / K2g / K2s), 256-B aligned sections:
 *   header  the 2-bit code per summary block (16 per 32-bit word): 0 = every cell has
 *           phi == +-0, psi_nfz == +-0, no no-fly flag and terrain +0.0 as read (nothing to
 *           read); 1 = psi_nfz == +-0 and no flag (phi from the 4-B plane, or phi and terrain
 *           from the 8-B {phi, terrain} plane); 2 = no psi_nfz below zero (phi, |psi_nfz| and
 *           the flag from the 8-B plane); 3 = the 16-B record;
 *           then the terrain bounds: one u16 {ub code, lb code << 8} per bound block (the
 *           smallest power-of-two square of >= 8 cells giving <= 16384 blocks), and one float2
 *           {base, step} per superblock of 4 x 4 bound blocks; a bound decodes as
 *           base + (float)code * step (f32, step a power of two) and holds every cell's terrain
 *           as read (+0 on nodata); {NaN, NaN} where the superblock holds a non-finite terrain;
 *   scratch the bound blocks' {min, max} (float2 each) while packing;
 *   planes  phi (4 B) and the terrain as read (4 B) in 4 x 8-cell blocks (one 128-B line),
 *           {phi, |psi_nfz| | nfz << 31} (8 B) in the same blocks (two 128-B lines) and the
 *           16-B records (four lines), at one index for all four; then {phi, terrain} (8 B) in
 *           4 x 4-cell blocks (one line; K2h's code-1 entry): 40 B per cell in all.
 * K2h reads a waypoint's terrain only where its bound could still be the path's maximum (the
 * maximum is order-free, so min_clearance is unchanged bit for bit); K2g and K2s read it for
 * every waypoint.  K2h addresses the copy by 32-bit offsets: for a copy of 4 GiB or more (about
 * 10^4 x 10^4 cells) it stands aside and the batch runs K2g / K2s on the same copy (slower, same
 * outputs in their documented sum order); packing needs nx, ny < 2^24.  uam_raster_pack_shape
 * gives the bytes of the caller's buffer (4096^2: 640.2 MiB = 56 KiB of header + 128 KiB of
 * scratch + 640 MiB of planes; 8192^2: 2.5 GiB); block as
 * uam_raster_summary
 * (0 = automatic), and the same block must be passed to uam_eval_generated.  Rebuild the copy
 * whenever rec changes. */
int uam_raster_pack_shape(const uam_raster_desc* desc, int32_t block, int32_t* block_out,
                          int64_t* bytes);
int uam_raster_pack(uam_ctx* ctx, const uam_raster_desc* desc, const void* rec_dev,
                    int32_t block, void* packed_dev, uam_stream stream);
/* K5: per group of G consecutive values, the reference's selection rule (main.py:175-180):
 * compare sqrt(v) when take_sqrt (fval = sqrt(cost), solver.py:48), else v. */
int uam_argmin(uam_ctx* ctx, const double* values_dev, int64_t groups, int32_t G,
               int32_t take_sqrt, int32_t* best_dev, uam_stream stream);

/* length_of: pts_dev [n_paths][n_points][2]; sum of the first n_segments segment norms
 * (squared-after-sqrt when smooth). */
int uam_path_length(uam_ctx* ctx, const double* pts_dev, int64_t n_paths, int32_t n_points,
                    int32_t n_segments, int32_t smooth, double* out_dev, uam_stream stream);

/* Waits for stream, then reports uam_device_status (below). */
int uam_synchronize(uam_ctx* ctx, uam_stream stream);
/* Device-side errors.  The sorted forms (K2h / K2g / K4h) check on the device that their
 * counting sort is consistent (every item lands on one position of the order).  A call whose
 * check fails writes NaN to every floating-point output and -1 to every count and selection of
 * the whole batch, and sets a word in page-locked host memory (no copy is issued otherwise).
 * Once the failing call has completed on its stream, uam_device_status returns UAM_E_DEVICE
 * with the text in uam_last_error() and clears the word; UAM_OK otherwise.  uam_synchronize
 * and the next uam_eval_generated* call on ctx report it too (the reference's convention of
 * raising on a failed solve, path_generation/solver.py:22-38, 53-55). */
int uam_device_status(uam_ctx* ctx);

/* Bytes of the volume buffer (256-B aligned sections) and the column plane's byte offset. */
int uam_volume_shape(const uam_volume_desc* desc, int64_t* bytes, int64_t* col_offset);
/* Config 5: build the volume (vol_dev: uam_volume_shape bytes, 256-B aligned) from a 2-D record
 * raster with the same x/y grid (rec2d_dev): risk = phi * layer_w[iz] (f64 product rounded to
 * f32; layer_w_dev [nz] f64), psi_nfz of the column; the column plane holds the column's DEM
 * (+0 for nodata) and its NFZ / MASK / NODATA flags. */
int uam_volume_build(uam_ctx* ctx, const uam_volume_desc* desc, const void* rec2d_dev,
                     const double* layer_w_dev, void* vol_dev, uam_stream stream);
/* Config 5 path evaluation: pairs6_dev [Q][6] = (x0, y0, z0, xf, yf, zf) (km, km, m); x/y
 * candidates as uam_eval_generated, altitude z_j = z0 + (zf - z0) * (j / (N+1)); cost =
 * (N+1) L + sum_j risk(voxel_j) / N; min_clearance = min_j (z_j - terrain of the column);
 * below_terrain counts waypoints whose layer centre z0 + (iz + 0.5) dz lies below it.  D <= 16.
 * packed_dev (uam_volume_pack, below; NULL = none): batches of >= UAM_OPT_SORTED_MIN_PATHS
 * paths (maxratio_smooth off, no cells) run K4h on it -- the (path, group) items sorted on the
 * altitude band and x/y tile of their middle waypoint, grouped partial sums (UAM_OPT_GROUP),
 * the geometry terms in the similarity form (oracle orc_eval_generated_h mode 2;
 * uam_last_kernel "K4h+pack"); every other batch runs on vol_dev. */
int uam_eval_generated3d(uam_ctx* ctx, const uam_volume_desc* desc, const void* vol_dev,
                         const void* packed_dev, const double* pairs6_dev, int64_t n_pairs,
                         const double* utab_dev, int32_t D, const uam_path_outputs* out,
                         uam_stream stream);
/* The packed volume (K4h), 256-B aligned sections:
 *   header  a 2-bit code per 8 x 8 columns (0: risk, psi_nfz +-0 in every layer and no no-fly
 *           flag; 1: psi_nfz +-0 and no flag; 2: no psi_nfz below zero; 3: otherwise), then the
 *           column terrain's bounds in the packed raster's scheme (u16 per bound block of
 *           columns, float2 {base, step} per 4 x 4 bound blocks);
 *   scratch the bound blocks' {min, max} while packing;
 *   4-B risk per voxel in 4 x 8-column blocks of one layer, layer-major (code 1; index i4);
 *   the 4-B column terrain (+0 on nodata) in the same blocks (one layer);
 *   8-B {risk, |psi_nfz| | nfz << 31} per voxel at i4 (code 2);
 *   16-B voxels {float risk, float psi_nfz, float terrain, uint32 flags} in 4 x 2-column
 *   blocks of one layer (one 128-B line; code 3);
 *   8-B {risk, column terrain} voxels in 4 x 4-column blocks of one layer (the
 *   UAM_OPT_K4H_TERRAIN = 1 form's entry): 36 B per voxel + 4 B per column in all.
 * K4h addresses the copy by 32-bit offsets: it stands aside (the batch runs K4 on vol_dev) for a
 * copy of 4 GiB or more or a layer of 2^24 or more entries.
 * K4h reads a waypoint's terrain only where it could still decide min_clearance or
 * below_terrain (the outputs are unchanged bit for bit).  uam_volume_pack derives it from a
 * built volume (vol_dev); packed_dev holds uam_volume_packed_bytes bytes (2.25 GiB at
 * 1024^2 x 64), 256-B aligned.  The copy is not tracked: rebuild it (uam_volume_pack) after
 * any write to vol_dev, including uam_volume_build into the same buffer and uam_bcast_raster. */
int uam_volume_packed_bytes(const uam_volume_desc* desc, int64_t* bytes);
int uam_volume_pack(uam_ctx* ctx, const uam_volume_desc* desc, const void* vol_dev,
                    void* packed_dev, uam_stream stream);

/* ---- Raster broadcast over RCCL / xGMI (the reference has no
 * collective at all -- its only IPC is the solver's TCP socket, path_generation/solver.py:26-38).
 * The record raster (or volume) is built once and broadcast once; the candidate loop of
 * main.py:160-193 then shards by pair with no collective.  RCCL is loaded at run time
 * (librccl.so.1: the one torch already loaded, else the system's); these calls return
 * UAM_E_STATE when it is absent.
 *   multi-process (one process per GPU): rank 0 calls uam_comm_unique_id, the caller ships
 *   the 128 bytes to every rank (e.g. torch.distributed.broadcast_object_list), each rank calls
 *   uam_comm_init (collective: returns once all nranks joined), then uam_bcast_raster.
 *   single process, several GPUs: uam_bcast_raster_group (ncclCommInitAll over the contexts'
 *   devices + one grouped broadcast; the communicators stay with the contexts for later
 *   uam_bcast_raster calls).
 * Asynchronous on the stream(s) given, like every other entry point. */
#define UAM_COMM_ID_BYTES 128
int uam_comm_unique_id(uint8_t* id_out /* [UAM_COMM_ID_BYTES] */);
int uam_comm_init(uam_ctx* ctx, const uint8_t* id /* [UAM_COMM_ID_BYTES] */, int32_t nranks,
                  int32_t rank);
int uam_comm_destroy(uam_ctx* ctx);
int uam_bcast_raster(uam_ctx* ctx, void* buf_dev, int64_t bytes, int32_t root,
                     uam_stream stream);
int uam_bcast_raster_group(uam_ctx** ctxs, void** bufs_dev, int32_t n, int64_t bytes,
                           int32_t root, uam_stream* streams);

/* ---- Coordinate reference systems ------------------------------
 * Transverse Mercator on an ellipsoid (Krueger series to n^6, Karney 2011) between geographic
 * (lon, lat) degrees and plane (x = easting, y = northing) metres -- what pyproj's to_crs does
 * for EPSG:4612/6668 <-> EPSG:2443..2461 in the reference (map_generation/data_manager.py:24-26
 * and 84-85, path_generation/main.py:106-115).  Definition: oracle/uam_oracle.c tm_*. */
typedef struct {
    double a, f, k0, lat0_deg, lon0_deg, false_easting, false_northing;
} uam_tm_params;
/* GRS80 / k0 0.9999 / origin of Japan Plane Rectangular CS zone 1..19 (EPSG:2442 + zone). */
int uam_tm_jprcs(int32_t zone, uam_tm_params* out);
/* Batched transforms of interleaved device arrays [n][2]: lon,lat -> x,y and back. */
int uam_geo_to_plane(uam_ctx* ctx, const uam_tm_params* tm, const double* lonlat_dev,
                     int64_t n, double* xy_dev, uam_stream stream);
int uam_plane_to_geo(uam_ctx* ctx, const uam_tm_params* tm, const double* xy_dev, int64_t n,
                     double* lonlat_dev, uam_stream stream);
/* North-up geographic grid (the mergeLL.vrt mosaic, mergeLL.vrt:1-3): pixel (i, j) covers
 * lon in lon0 + [i, i+1) dlon, lat in lat_top - [j, j+1) dlat. */
typedef struct {
    int32_t nx, ny;
    double lon0, lat_top, dlon, dlat;
    float nodata;
    int32_t pad;
} uam_geo_grid_desc;
/* Reproject a geographic DEM onto the plane raster grid dst (units of dst: unit_m metres):
 * each output cell centre -> inverse TM -> source pixel; resample 0 = nearest, 1 = bilinear
 * when all four neighbours are valid (else nearest); outside / nodata -> src nodata. */
int uam_reproject_dem(uam_ctx* ctx, const uam_tm_params* tm, const float* src_dev,
                      const uam_geo_grid_desc* src, const uam_raster_desc* dst, double unit_m,
                      int32_t resample, float* dst_dev, uam_stream stream);

/* ---- Land / populated-area polygons --------------------------------
 * DataProcessor(min_area, large_area, divisions, min_approx_polygon_area) of
 * map_generation/data_processor.py:9-13 (defaults 750000 m^2, 32000000 m^2, 5, 780000 m^2). */
typedef struct {
    double min_area, large_area, min_approx_area;
    int32_t divisions, pad;
} uam_polyproc_params;
/* DataProcessor.process_polygons (data_processor.py:15-75) on polygons in plane metres (host):
 * unary_union (inputs must have disjoint interiors; shared boundaries merge), area filter,
 * divisions^2 split of large polygons, cv2.minAreaRect + boxPoints + np.intp per polygon /
 * piece, final area filter.  Rings: ring r = xy[ring_start[r] .. ring_start[r+1]) (open or
 * closed), ring_hole[r] != 0 for holes.  Output: *n_rects rectangles, rect_xy[r][4][2]
 * integer metres in cv2.boxPoints order (at most max_rects written; more -> UAM_E_INVALID
 * with *n_rects set).  Definition: oracle/uam_oracle.c orc_process_polygons. */
int uam_process_polygons(const double* xy, const int64_t* ring_start, int32_t n_rings,
                         const int32_t* ring_hole, const uam_polyproc_params* params,
                         int64_t* rect_xy, int32_t max_rects, int32_t* n_rects);

/* The DEM route (DataManager.load_dem_polygons_from_geotiff + process_polygons,
 * map_generation/main.py:27-35): mask (dem == -9999 if threshold == -9999 else
 * dem > threshold, data_manager.py:14-17) -> 4-connected regions (rasterio.features.shapes)
 * labelled on the GPU -> the same approximation as uam_process_polygons, with pixel corners
 * at x0 + i dx, y_top - j dy (times unit_m metres).  Large regions are split into their box
 * pieces by a second labelling on the grid refined at the box edges.  Output as
 * uam_process_polygons (regions in raster order of their first cell).  Definition:
 * oracle/uam_oracle.c orc_dem_polygons.  Work is enqueued on `stream` and, for the large
 * regions, on up to 3 side streams the context owns (UAM_OPT_K8_STREAMS, 1-8, 4 in all);
 * the call synchronises all of them before it returns. */
int uam_dem_polygons(uam_ctx* ctx, const float* dem_dev, const uam_raster_desc* desc,
                     float threshold, double unit_m, const uam_polyproc_params* params,
                     int64_t* rect_xy, int32_t max_rects, int32_t* n_rects, uam_stream stream);

/* Measurement (bench.py's roofline; build-defined).  uam_kernel_timing(ctx, 1) resets and
 * starts timing, 0 stops it: while on, the context records a HIP event pair on the launch
 * stream around every timed path evaluation of uam_eval_generated* -- around the whole launch
 * sequence of K2g and K2s (sorts, evaluation, output launch; K2s's side-stream sorts are
 * joined inside it), around the k_eval_pairs / k_eval_wave launch of the other forms (excluding
 * their pair order and selection launches).  uam_kernel_time waits for those events and returns
 * the summed time and the count since the last call (then resets both).  Every 4096 timed
 * calls the pending pairs are folded into a running total (the timed call waits for the last
 * of them once), so any number of calls may pass between queries. */
int uam_kernel_timing(uam_ctx* ctx, int32_t enable);
int uam_kernel_time(uam_ctx* ctx, double* ms_total, int64_t* launches);
/* The path evaluation the last uam_eval_generated* call on ctx ran: "K2h+pack" (segment-grouped
 * raster with the similarity-form geometry, the default for packed rasters and batches >=
 * UAM_OPT_SORTED_MIN_PATHS paths), "K2g+pack" (the same with per-segment geometry:
 * UAM_OPT_K2G_SIM = 0 or maxratio_smooth), "K4h+pack" (the packed volume, K2h's form),
 * "K2s+pack" / "K2s+skip" / "K2s" (segment-sorted raster, sequential sums), "K2+skip" / "K2"
 * (lane per path), "K2w" (wave per path), "K2d" (D > 16), "K3b", "K3", "K3d", "K4", "K4w";
 * "" before the first call.  The string is static (never freed).  For benchmarks and tests:
 * which kernel a number belongs to. */
const char* uam_last_kernel(const uam_ctx* ctx);

/* Waypoint-group length of the per-path sums of the last uam_eval_generated* call on ctx: G > 0
 * when a segment-grouped evaluation ran -- K2g: cost, length_q, length, kin_sum and nfz_sum
 * formed as per-group partial sums, each term attached to a waypoint of the group
 * [kG, (k+1)G), added in group order (oracle/uam_oracle.c orc_eval_paths_g); K2h / K4h: the
 * raster (volume) terms of cost and nfz_sum so, length_q / length / kin_sum in the similarity
 * form (orc_eval_generated_h) -- 0 for the reference's sequential order (problem.py:38-44,
 * 84-114, 130-146).
 * Tolerance against the sequential order: rounding only.  Measured: <= 8.2e-14 relative on
 * cost and 4.4e-14 on length over the whole cfg3 batch (500k paths), <= 1e-12 on every test
 * map, against the north_star's 1e-5; the selections (best_fval_idx, best_length_idx) agreed
 * on all 100k cfg3 pairs (bench.py parity.vs_sequential_order) -- they can differ only where
 * two candidates of a pair are within that rounding of each other.  A caller that needs the
 * sequential bits sets UAM_OPT_GROUP = 0 (K2s / K4). */
int32_t uam_last_group(const uam_ctx* ctx);

/* Context options: which kernel form runs (results never depend on them, except for the sum
 * order UAM_OPT_GROUP selects, which uam_last_group reports).  Read by the calls that follow.
 *   UAM_OPT_GROUP                K2g waypoints per group, 1..64 (default 21); 0 = no K2g (the
 *                                raster batches it takes run K2s: the reference's sum order)
 *   UAM_OPT_SORTED_MIN_PATHS     smallest raster batch (paths) the sorted forms K2g / K2s take
 *                                (default 65536; smaller batches run K2 / K2w)
 *   UAM_OPT_K2S_SEGMENTS         K2s segments per path, 2..8 (default 2)
 *   UAM_OPT_WAVE_MAX_PATHS       batches of up to this many paths run one wave per path (K2w /
 *                                K4w; default 16384; 0 = never)
 *   UAM_OPT_PAIR_ORDER           1 (default): batches of >= 4096 pairs through the lane-per-path
 *                                kernels in a spatial pair order; 0: in index order
 *   UAM_OPT_K1_ROWS              raster build: cells (rows) per lane, 1, 2 (default), 4, 8
 *   UAM_OPT_K3B_SEGMENT          analytic K3b: waypoints sorted together, 2/4/6/8 (default)/16;
 *                                0 = the lane-per-path K3
 *   UAM_OPT_K3B_POINTS_PER_LANE  analytic K3b evaluation phase: 1 (default) or 2
 *   UAM_OPT_K8_TILED             DEM polygons: 1 (default) tile labelling in LDS, 0 cell-parallel
 *   UAM_OPT_K8_STREAMS           DEM polygons: streams the large regions spread over, 1..8 (4)
 *   UAM_OPT_K2G_TILE_BITS        K2g sort key: 2^b x 2^b tiles over the raster, b = 3..6; 0
 *                                (default) = tiles of ~256 x 256 cells, coarser for batches
 *                                whose sort counts would exceed half their (path, group) items
 *   UAM_OPT_K2G_LDS_FLOOR        K2g / K2h / K4h evaluation: dynamic-LDS floor per workgroup in
 *                                bytes, which caps the workgroups resident per CU; 0 (default):
 *                                none for K2g and K2h (512-item workgroups, 2 per CU by their
 *                                ~62 KiB of tables), 60 000 (2 per CU) for K4h
 *   UAM_OPT_K2G_CHUNK            K2g / K2h / K4h evaluation: gathers in flight per lane,
 *                                6/7/8/11/16/21 (K2g: 7 runs as 6, 16 at two waves per SIMD, 21
 *                                as 16; K2h: 6/7/8/11, 16 and 21 as 11; K4h: 6/7/8/11/16, 21
 *                                as 16);
 *                                0 (default) = 8 for K2g, 7 for K2h, 11 for K4h
 *   UAM_OPT_K2G_CURVE            K2g sort key: tiles in Hilbert (1, default) or Morton (0) order
 *   UAM_OPT_K2G_SIM              1 (default): generated raster batches take K2h, K2g's sort and
 *                                grouped raster sums with the geometry terms (L, length,
 *                                kinematic rows) in the similarity form -- the unit arc's sums
 *                                scaled by |x0 - xf| / 2 (oracle orc_eval_generated_h; needs
 *                                maxratio_smooth = 0); 0: K2g, the geometry per waypoint
 *                                segment in the grouped order (orc_eval_paths_g)
 *   UAM_OPT_K4H_BAND             K4h sort key: altitude layers per band, a power of two
 *                                (default 0: the fewest giving at most 16 bands); tiles from
 *                                UAM_OPT_K2G_TILE_BITS (default 3: 8 x 8 tiles), at most
 *                                4096 (tile, band) bins
 *   UAM_OPT_K2H_LB_STRIDE        K2h / K4h terrain bounds: the histogram launch samples every
 *                                n-th waypoint of each path and seeds the path's items with the
 *                                exact terrain (clearance) of the sample with the best bound
 *                                (1..1024; default 16; 0: no seed); fewer terrain fetches at
 *                                smaller n, more arithmetic in that launch.  Same outputs.
 *   UAM_OPT_K2H_TERRAIN          K2h's terrain: 1 (default) in the entry (8-B {phi, terrain}
 *                                entries, the 16-B records in no-fly / psi blocks), 0 by bounds
 *                                (4-B phi entries, the terrain plane read only where a waypoint
 *                                could still hold the path maximum).  Same outputs.
 *   UAM_OPT_K4H_TERRAIN          K4h's likewise: 0 (default) by bounds (4-B risk / 8-B
 *                                {risk, psi|nfz} voxels, the column terrain only where it could
 *                                still decide an output), 1 in the entry (8-B {risk, terrain}
 *                                voxels, 16-B voxels in no-fly / psi columns).  Same outputs. */
enum {
    UAM_OPT_GROUP = 1,
    UAM_OPT_SORTED_MIN_PATHS = 2,
    UAM_OPT_K2S_SEGMENTS = 3,
    UAM_OPT_WAVE_MAX_PATHS = 4,
    UAM_OPT_PAIR_ORDER = 5,
    UAM_OPT_K1_ROWS = 6,
    UAM_OPT_K3B_SEGMENT = 7,
    UAM_OPT_K3B_POINTS_PER_LANE = 8,
    UAM_OPT_K8_TILED = 9,
    UAM_OPT_K8_STREAMS = 10,
    UAM_OPT_K2G_TILE_BITS = 11,
    UAM_OPT_K2G_LDS_FLOOR = 12,
    UAM_OPT_K2G_CHUNK = 13,
    UAM_OPT_K2G_CURVE = 14,
    UAM_OPT_K2G_SIM = 15,
    UAM_OPT_K4H_BAND = 17,
    UAM_OPT_K2H_LB_STRIDE = 19,
    UAM_OPT_K2H_TERRAIN = 20,
    UAM_OPT_K4H_TERRAIN = 21,
    UAM_OPT_TEST_SORT_FAULT = 22  /* tests only: 1 makes the next sorted calls flag their sort as
                                     inconsistent (the uam_device_status path); 0 (default) off */
};
int uam_set_option(uam_ctx* ctx, int32_t option, int64_t value);
int uam_get_option(const uam_ctx* ctx, int32_t option, int64_t* value);

/* Workspace bytes uam_refine needs for n_paths (after uam_set_geometry/uam_set_params). */
int64_t uam_refine_workspace_bytes(uam_ctx* ctx, int64_t n_paths,
                                   const uam_refine_params* params);
/* Refines wp_dev [P][N+2][2] in place (endpoints fixed); per path: final cost (get_cost),
 * final sum of squared constraint rows, gradient steps taken.  Any output may be NULL. */
int uam_refine(uam_ctx* ctx, double* wp_dev, int64_t n_paths, const uam_refine_params* params,
               void* workspace_dev, int64_t workspace_bytes, double* cost_dev,
               double* infeas_dev, int32_t* iters_dev, uam_stream stream);

#ifdef __cplusplus
}
#endif

#endif /* UAMPATH_H */
