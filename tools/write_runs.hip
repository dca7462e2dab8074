// Design probe (round 5, not product code): the cost of K2h's waypoint-cell stores by pattern.
// Every item (path, group) writes a run of RUN 4-B cells at out + path * stride + seg * seg_stride
// in a random item order (as the sorted evaluation meets them); lanes are items.  Patterns:
//   chunks:  the run as CH-cell pieces written at different times (a gap of ~GAP loads between
//            pieces, as K2h's chunks are), or all pieces back to back;
//   layout:  row stride W = 82 cells (the reference's [P][W], runs unaligned), or each group's
//            run at a 32-cell (128-B) aligned slot (row stride 4 x 32);
//   stores:  plain or nontemporal.
// Each lane stages its pieces through LDS so a store instruction writes 64 / CH items' runs
// (K2h's cell staging).  Prints ms per launch; WRITE_SIZE comes from rocprofv3 --pmc.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/write_runs tools/write_runs.hip && /tmp/write_runs
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

constexpr int CH = 7, NSEG = 4, G = 21, W = 82;

template <bool NT, bool SPREAD, bool STORE = true>
__global__ __launch_bounds__(512) void k_runs(const int* __restrict__ order, int n_items,
                                              int* __restrict__ out, int row_stride,
                                              int seg_stride, const float* __restrict__ junk,
                                              float* __restrict__ sink) {
    __shared__ int s_cells[8 * CH * 64];
    const int pos = blockIdx.x * 512 + threadIdx.x;
    const bool live = pos < n_items;
    const int item = live ? order[pos] : 0;
    const int path = item / NSEG, seg = item - path * NSEG;
    const int j0 = seg * G, j1 = live ? min(j0 + G, W) : j0;
    int* sw = s_cells + (threadIdx.x >> 6) * (CH * 64);
    const int lane = threadIdx.x & 63;
    float acc = 0.0f;
    const int nch = 3;
    for (int c = 0; c < nch; ++c) {
        if (SPREAD) {  // ~ a chunk's gathers between the pieces: dependent loads
            unsigned h = (unsigned)item * 2654435761u + c;
            for (int k = 0; k < 6; ++k) {
                acc += junk[h & ((1u << 24) - 1)];
                h = h * 1664525u + 1013904223u + (unsigned)(acc > 1e30f);
            }
        }
        const int jc = j0 + c * CH;
        const int nv = max(0, min(CH, j1 - jc));
        for (int t = 0; t < CH; ++t) sw[t * 64 + lane] = jc + t;
        __builtin_amdgcn_wave_barrier();
        const long base = (long)path * row_stride + (long)seg * seg_stride + c * CH;
        constexpr int IPS = 64 / CH;
        for (int k = 0; k < (64 + IPS - 1) / IPS; ++k) {
            const int it = k * IPS + lane / CH, t = lane % CH;
            const int src = it < 64 ? it : 63;
            const long b_it = __shfl(base, src);
            const int nv_it = __shfl(nv, src);
            if (STORE && lane < IPS * CH && it < 64 && t < nv_it) {
                if (NT)
                    __builtin_nontemporal_store(sw[t * 64 + it], out + b_it + t);
                else
                    out[b_it + t] = sw[t * 64 + it];
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (acc == 12345.0f) sink[0] = acc;
}

int main() {
    const int P = 500000, n = P * NSEG;
    std::vector<int> h(n);
    for (int i = 0; i < n; ++i) h[i] = i;
    srand(7);
    // shuffle in blocks of 64 so items of one path land in different waves (sorted-order-like)
    for (int i = n - 1; i > 0; --i) {
        const int j = (int)(((long)rand() * RAND_MAX + rand()) % (i + 1));
        std::swap(h[i], h[j]);
    }
    int *d_order, *d_out;
    float *d_junk, *d_sink;
    CHECK(hipMalloc(&d_order, (size_t)n * 4));
    CHECK(hipMalloc(&d_out, (size_t)P * 128 * 4));
    CHECK(hipMalloc(&d_junk, (size_t)(1 << 24) * 4));
    CHECK(hipMalloc(&d_sink, 64));
    CHECK(hipMemset(d_junk, 0, (size_t)(1 << 24) * 4));
    CHECK(hipMemcpy(d_order, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int grid = (n + 511) / 512;
    struct V {
        const char* name;
        void (*f)(const int*, int, int*, int, int, const float*, float*);
        int row, seg;
    };
    V vs[] = {
        {"W82 unaligned, NT, spread", k_runs<true, true>, W, G},
        {"W82 unaligned, plain, spread", k_runs<false, true>, W, G},
        {"W82 unaligned, NT, back-to-back", k_runs<true, false>, W, G},
        {"W82 unaligned, plain, back-to-back", k_runs<false, false>, W, G},
        {"128-B slots, NT, spread", k_runs<true, true>, 4 * 32, 32},
        {"128-B slots, plain, spread", k_runs<false, true>, 4 * 32, 32},
        {"128-B slots, NT, back-to-back", k_runs<true, false>, 4 * 32, 32},
        {"128-B slots, plain, back-to-back", k_runs<false, false>, 4 * 32, 32},
        {"gathers only (no stores)", k_runs<true, true, false>, W, G},
    };
    for (const V& v : vs) {
        for (int rep = 0; rep < 3; ++rep)
            hipLaunchKernelGGL(v.f, dim3(grid), dim3(512), 0, 0, d_order, n, d_out, v.row, v.seg,
                               d_junk, d_sink);
        CHECK(hipDeviceSynchronize());
        const int K = 10;
        CHECK(hipEventRecord(e0));
        for (int rep = 0; rep < K; ++rep)
            hipLaunchKernelGGL(v.f, dim3(grid), dim3(512), 0, 0, d_order, n, d_out, v.row, v.seg,
                               d_junk, d_sink);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-40s %.4f ms per launch (%.1f MB of cells)\n", v.name, ms / K,
               (double)P * W * 4 / 1e6);
    }
    return 0;
}
