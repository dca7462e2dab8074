// gather_ceiling.hip -- microbenchmark: the rate of independent random gathers (4/8/16-byte
// records) from a table of T bytes on one MI355X, as a function of loads in flight per lane.
// Sets the practical ceiling for the raster path kernel's record gather.
// Indices come from an in-register xorshift hash, so no index traffic is counted.
//   build: hipcc --offload-arch=gfx950 -O3 -o build/gather_ceiling tools/gather_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                         \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

template <int LOADS, int BYTES>
__global__ __launch_bounds__(256) void k_gather(const uint4* __restrict__ tab16,
                                                const uint2* __restrict__ tab8,
                                                const uint32_t* __restrict__ tab4,
                                                uint32_t mask, int iters, uint32_t* out) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    uint32_t s = hash32(tid * 2654435761u + 1u);
    for (int it = 0; it < iters; ++it) {
        uint32_t idx[LOADS];
#pragma unroll
        for (int l = 0; l < LOADS; ++l) {
            s = hash32(s + l);
            idx[l] = s & mask;
        }
        uint32_t v[LOADS];
#pragma unroll
        for (int l = 0; l < LOADS; ++l) {
            if (BYTES == 16) {
                uint4 r = tab16[idx[l]];
                v[l] = r.x ^ r.y ^ r.z ^ r.w;
            } else if (BYTES == 8) {
                uint2 r = tab8[idx[l]];
                v[l] = r.x ^ r.y;
            } else {
                v[l] = tab4[idx[l]];
            }
        }
#pragma unroll
        for (int l = 0; l < LOADS; ++l) acc += v[l];
    }
    if (acc == 0x12345678u) out[tid] = acc;  // keep the loads alive
}

template <int LOADS, int BYTES>
double run(void* tab, size_t table_bytes, int blocks, int iters, uint32_t* out) {
    const size_t n = table_bytes / BYTES;
    const uint32_t mask = (uint32_t)(n - 1);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL((k_gather<LOADS, BYTES>), dim3(blocks), dim3(256), 0, 0,
                           (const uint4*)tab, (const uint2*)tab, (const uint32_t*)tab, mask,
                           iters, out);
    CHECK(hipEventRecord(a));
    const int reps = 5;
    for (int rep = 0; rep < reps; ++rep)
        hipLaunchKernelGGL((k_gather<LOADS, BYTES>), dim3(blocks), dim3(256), 0, 0,
                           (const uint4*)tab, (const uint2*)tab, (const uint32_t*)tab, mask,
                           iters, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double gathers = (double)blocks * 256 * iters * LOADS * reps;
    return gathers / (ms * 1e-3);
}

int main() {
    const size_t max_bytes = (size_t)1 << 30;
    void* tab;
    uint32_t* out;
    CHECK(hipMalloc(&tab, max_bytes));
    CHECK(hipMalloc(&out, 256 * 4096 * sizeof(uint32_t) * 4));
    CHECK(hipMemset(tab, 1, max_bytes));
    const size_t sizes[] = {(size_t)4 << 20, (size_t)64 << 20, (size_t)256 << 20,
                            (size_t)1 << 30};
    const int blocks = 256 * 8;  // 2048 blocks x 256 threads = 8 waves per SIMD if resident
    const int iters = 64;
    printf("{\"probe\":\"gather_ceiling\",\"blocks\":%d,\"threads_per_block\":256}\n", blocks);
    for (size_t tb : sizes) {
        double r;
#define ROW(L, B)                                                                           \
    r = run<L, B>(tab, tb, blocks, iters / L * 4, out);                                     \
    printf("{\"table_MiB\":%zu,\"bytes\":%d,\"loads_in_flight\":%d,\"Ggathers_s\":%.2f,"     \
           "\"GBs_useful\":%.1f}\n",                                                        \
           tb >> 20, B, L, r / 1e9, r * B / 1e9);
        ROW(1, 16) ROW(4, 16) ROW(8, 16) ROW(16, 16)
        ROW(8, 8) ROW(16, 8) ROW(8, 4) ROW(16, 4)
    }
    CHECK(hipFree(tab));
    CHECK(hipFree(out));
    return 0;
}
