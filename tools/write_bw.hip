// Design probe (round 5, not product code): the store floor of the waypoint-cells output --
// 164 MB (cfg3: 500k paths x 82 cells x 4 B) written as 16-B stores per lane, a wave writing
// 1 KiB contiguous, plain or nontemporal, one pass per lane or grid-stride loops.  Prints ms
// and TB/s per variant (median of 20).
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/write_bw tools/write_bw.hip && /tmp/write_bw
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void k_fill(v4i* __restrict__ out, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * 256) {
        const v4i w = {(int)i, (int)i + 1, (int)i + 2, (int)i + 3};
        if (NT)
            __builtin_nontemporal_store(w, out + i);
        else
            out[i] = w;
    }
}

int main(int argc, char** argv) {
    // default: the waypoint-cells output; argv[1]: another size in bytes (a multiple of 16)
    const int64_t bytes = argc > 1 ? atoll(argv[1]) : 500000LL * 82 * 4, n4 = bytes / 16;
    v4i* out;
    CHECK(hipMalloc(&out, bytes));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int grids[] = {0, 512, 1024, 2048, 8192};
    for (int nt = 0; nt < 2; ++nt)
        for (int g : grids) {
            const int blocks = g ? g : (int)((n4 + 255) / 256);
            std::vector<float> ts;
            for (int r = 0; r < 23; ++r) {
                CHECK(hipEventRecord(a, 0));
                if (nt)
                    hipLaunchKernelGGL(k_fill<true>, dim3(blocks), dim3(256), 0, 0, out, n4);
                else
                    hipLaunchKernelGGL(k_fill<false>, dim3(blocks), dim3(256), 0, 0, out, n4);
                CHECK(hipEventRecord(b, 0));
                CHECK(hipEventSynchronize(b));
                float ms;
                CHECK(hipEventElapsedTime(&ms, a, b));
                if (r >= 3) ts.push_back(ms);
            }
            std::sort(ts.begin(), ts.end());
            const float ms = ts[ts.size() / 2];
            printf("{\"probe\": \"write_bw\", \"nt\": %d, \"grid\": %d, \"ms\": %.4f, \"TBps\": %.2f}\n",
                   nt, blocks, ms, bytes / (ms * 1e-3) / 1e12);
        }
    CHECK(hipFree(out));
    return 0;
}
