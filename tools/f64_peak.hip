// f64_peak.hip -- microbenchmark: the f64 vector rate of one MI355X (v_fma_f64, v_add_f64,
// v_mul_f64 throughput with CH independent chains per lane), the peak against which the
// refinement kernel K6 (f64 VALU + latency bound) is priced in DESIGN.md §5.  The guide's
// constants table has no f64 vector row, so the number is measured here.
//   build: hipcc --offload-arch=gfx950 -O3 -o build/f64_peak tools/f64_peak.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                         \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// OP 0 = fma (2 flop), 1 = add, 2 = mul
template <int OP, int CH>
__global__ __launch_bounds__(256) void k_f64(double seed, int iters, double* out) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    double v[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = seed + tid * 1e-9 + c;
    const double a = 1.0000000001, b = 1e-12;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            if (OP == 0)
                v[c] = __builtin_fma(v[c], a, b);
            else if (OP == 1)
                v[c] = v[c] + b;
            else
                v[c] = v[c] * a;
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += v[c];
    if (s == 12345.678) out[tid] = s;  // keeps the chains live, never true
}

template <int OP, int CH>
void run(const char* name, int blocks, int iters, double* out) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_f64<OP, CH>), dim3(blocks), dim3(256), 0, 0, 1.0, iters, out);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_f64<OP, CH>), dim3(blocks), dim3(256), 0, 0, 1.0, iters, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double lanes_ops = (double)blocks * 256 * iters * CH * reps;
    const double flop = lanes_ops * (OP == 0 ? 2 : 1);
    printf("{\"op\": \"%s\", \"chains\": %d, \"blocks\": %d, \"ms\": %.3f, \"lane_ops_per_s\": %.4g, "
           "\"tflops\": %.2f}\n",
           name, CH, blocks, ms / reps, lanes_ops / (ms / 1e3), flop / (ms / 1e3) / 1e12);
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 256 * 8 * 4;
    const int iters = argc > 2 ? atoi(argv[2]) : 4096;
    double* out;
    CHECK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(double)));
    run<0, 4>("fma_f64", blocks, iters, out);
    run<0, 8>("fma_f64", blocks, iters, out);
    run<0, 16>("fma_f64", blocks, iters, out);
    run<1, 8>("add_f64", blocks, iters, out);
    run<2, 8>("mul_f64", blocks, iters, out);
    CHECK(hipFree(out));
    return 0;
}
