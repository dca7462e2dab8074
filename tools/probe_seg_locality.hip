// Locality probe for a segment-sorted raster evaluation (tools/probe_seg_locality.py): how fast
// can the cfg3 record gathers run when each path is split into segments of L waypoints and the
// (path, segment) items of one segment index are processed in the spatial order of their
// segment, with the state of each path carried in HBM between segment launches?  The probe
// gathers the real records of the real cells (from uam_eval_generated's `cells` output) and
// keeps a per-path f64 sum of the record's first field in waypoint order, so it moves exactly
// the bytes such a kernel would; it is a measurement tool, not a product kernel.
#include <hip/hip_runtime.h>

#include <cstdint>

// workgroup b of nb -> chunk: XCD x = b % 8 walks the contiguous chunk range x * nb / 8 ...
__device__ __forceinline__ int64_t xcd_chunk(int64_t b, int64_t nb) {
    const int64_t x = b & 7, k = b >> 3;
    return x * (nb >> 3) + (x < (nb & 7) ? x : (nb & 7)) + k;
}

struct RGeo {
    double x0, y_top, inv_dx, inv_dy;
    int nx, ny;
};

// the cell of waypoint j of path p (q = p / D, d = p % D), computed like K2's issue_chunk
__device__ __forceinline__ int32_t cell_of(const double* __restrict__ pairs,
                                           const double* __restrict__ utab, int D, int N,
                                           const RGeo& g, int64_t p, int j) {
    const int64_t q = p / D;
    const int d = (int)(p - q * D);
    const double4 pr = reinterpret_cast<const double4*>(pairs)[q];
    double x, y;
    if (j == 0) {
        x = pr.x, y = pr.y;
    } else if (j == N + 1) {
        x = pr.z, y = pr.w;
    } else {
        const double ux = utab[((int64_t)d * N + (j - 1)) * 2], uy = utab[((int64_t)d * N + (j - 1)) * 2 + 1];
        const double vx = pr.x - pr.z, vy = pr.y - pr.w;
        const double cx = (pr.z + pr.x) * 0.5, cy = (pr.w + pr.y) * 0.5;
        x = cx + 0.5 * (vx * ux - vy * uy);
        y = cy + 0.5 * (vy * ux + vx * uy);
    }
    const double fx = floor((x - g.x0) * g.inv_dx), fy = floor((g.y_top - y) * g.inv_dy);
    if (!((fx >= 0.0) && (fx < (double)g.nx) && (fy >= 0.0) && (fy < (double)g.ny))) return -1;
    return (int32_t)fy * g.nx + (int32_t)fx;
}

extern "C" {

// items i -> path order[i]; waypoints [j0, j1) in order; running f64 sum carried in acc
__global__ __launch_bounds__(256) void k_probe_gen(const uint4* __restrict__ rec,
                                                   const double* __restrict__ pairs,
                                                   const double* __restrict__ utab, int D, int N,
                                                   RGeo g, int j0, int j1,
                                                   const int32_t* __restrict__ order, int64_t P,
                                                   double* __restrict__ acc) {
    const int64_t i = xcd_chunk(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const int64_t p = order[i];
    double s = j0 == 0 ? 0.0 : acc[p];
    for (int j = j0; j < j1; j += 8) {
        uint4 r[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int32_t cl = (j + t < j1) ? cell_of(pairs, utab, D, N, g, p, j + t) : -1;
            r[t] = cl >= 0 ? rec[cl] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) s = s + (double)__uint_as_float(r[t].x);
    }
    acc[p] = s;
}

int probe_gen(const void* rec, const double* pairs, const double* utab, int D, int N,
              double x0, double y_top, double inv_dx, double inv_dy, int nx, int ny, int j0, int j1,
              const int32_t* order, int64_t P, double* acc, int lds_pad, void* stream) {
    const RGeo g{x0, y_top, inv_dx, inv_dy, nx, ny};
    hipLaunchKernelGGL(k_probe_gen, dim3((unsigned)((P + 255) / 256)), dim3(256), (size_t)lds_pad,
                       (hipStream_t)stream, (const uint4*)rec, pairs, utab, D, N, g, j0, j1, order,
                       P, acc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}


// baseline: lane = path (items in the given order), all W cells in waypoint order
__global__ __launch_bounds__(256) void k_probe_full(const uint4* __restrict__ rec,
                                                    const int32_t* __restrict__ cells, int W,
                                                    const int32_t* __restrict__ order, int64_t P,
                                                    double* __restrict__ acc) {
    const int64_t i = xcd_chunk(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const int64_t p = order ? order[i] : i;
    const int32_t* c = cells + p * W;
    double s = 0.0;
    for (int j0 = 0; j0 < W; j0 += 8) {
        uint4 r[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int32_t cl = (j0 + t < W) ? c[j0 + t] : -1;
            r[t] = cl >= 0 ? rec[cl] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) s = s + (double)__uint_as_float(r[t].x);
    }
    acc[p] = s;
}

// one segment: lane = item i of the sorted list -> path order[i], cells [j0, j1) of that path;
// the path's running sum is read, advanced in waypoint order and written back
__global__ __launch_bounds__(256) void k_probe_seg(const uint4* __restrict__ rec,
                                                   const int32_t* __restrict__ cells, int W,
                                                   int j0, int j1,
                                                   const int32_t* __restrict__ order, int64_t P,
                                                   double* __restrict__ acc) {
    const int64_t i = xcd_chunk(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const int64_t p = order[i];
    const int32_t* c = cells + p * W;
    double s = j0 == 0 ? 0.0 : acc[p];
    for (int j = j0; j < j1; j += 8) {
        uint4 r[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int32_t cl = (j + t < j1) ? c[j + t] : -1;
            r[t] = cl >= 0 ? rec[cl] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) s = s + (double)__uint_as_float(r[t].x);
    }
    acc[p] = s;
}

int probe_full(const void* rec, const int32_t* cells, int W, const int32_t* order, int64_t P,
               double* acc, void* stream) {
    hipLaunchKernelGGL(k_probe_full, dim3((unsigned)((P + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, (const uint4*)rec, cells, W, order, P, acc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// lds_pad: dynamic LDS per workgroup, to cap the workgroups resident per CU (the window)
int probe_seg(const void* rec, const int32_t* cells, int W, int j0, int j1,
              const int32_t* order, int64_t P, double* acc, int lds_pad, void* stream) {
    hipLaunchKernelGGL(k_probe_seg, dim3((unsigned)((P + 255) / 256)), dim3(256),
                       (size_t)lds_pad, (hipStream_t)stream, (const uint4*)rec, cells, W, j0, j1,
                       order, P, acc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the same segment launch over an 8-B record table (the first two words of each record)
__global__ __launch_bounds__(256) void k_probe_seg8(const uint2* __restrict__ rec,
                                                    const int32_t* __restrict__ cells, int W,
                                                    int j0, int j1,
                                                    const int32_t* __restrict__ order, int64_t P,
                                                    double* __restrict__ acc) {
    const int64_t i = xcd_chunk(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const int64_t p = order[i];
    const int32_t* c = cells + p * W;
    double s = j0 == 0 ? 0.0 : acc[p];
    for (int j = j0; j < j1; j += 8) {
        uint2 r[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int32_t cl = (j + t < j1) ? c[j + t] : -1;
            r[t] = cl >= 0 ? rec[cl] : make_uint2(0, 0);
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) s = s + (double)__uint_as_float(r[t].x);
    }
    acc[p] = s;
}

int probe_seg8(const void* rec, const int32_t* cells, int W, int j0, int j1,
               const int32_t* order, int64_t P, double* acc, int lds_pad, void* stream) {
    hipLaunchKernelGGL(k_probe_seg8, dim3((unsigned)((P + 255) / 256)), dim3(256),
                       (size_t)lds_pad, (hipStream_t)stream, (const uint2*)rec, cells, W, j0, j1,
                       order, P, acc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
