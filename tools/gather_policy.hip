// gather_policy.hip -- does the memory policy of a random 16-B gather change the L2 miss
// request size (128/64/32 B) and with it the random-gather ceiling?  Variants:
//   0 plain global_load_dwordx4          (default: 128-B line fill per miss)
//   1 __builtin_nontemporal_load         (nt)
//   2 buffer_load aux 0, 3 aux 16 (sc1), 4 aux 17 (sc0 sc1), 5 aux 19 (sc0 sc1 nt), 6 aux 2 (nt)
//   7 plain loads, table from hipExtMallocWithFlags(hipDeviceMallocUncached)
//   8 plain loads, table from hipExtMallocWithFlags(hipDeviceMallocFinegrained)
//   build: hipcc --offload-arch=gfx950 -O3 -o build/gather_policy tools/gather_policy.hip
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

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// POL 0 plain flat load, 1 nt builtin, 2..6 buffer loads with cache-policy aux bits
// (gfx950: sc0 = 1, nt = 2, sc1 = 16), all tracked by the compiler's waitcnt insertion.
template <int POL>
__device__ __forceinline__ uint4 ld(const uint4* base, __amdgpu_buffer_rsrc_t rsrc, uint32_t i) {
    if (POL == 1) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + i));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    if (POL >= 2 && POL <= 6) {
        constexpr int aux = POL == 2 ? 0 : POL == 3 ? 16 : POL == 4 ? 17 : POL == 5 ? 19 : 2;
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, i * 16u, 0, aux));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return base[i];
}

template <int POL>
__global__ __launch_bounds__(256) void k_gather(const uint4* __restrict__ tab, uint32_t mask,
                                                int iters, uint32_t* out) {
    constexpr int L = 8;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint4*>(tab), 0, (int)((mask + 1u) * 16u), 0x00020000);
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    uint32_t s = hash32(tid * 2654435761u + 1u);
    for (int it = 0; it < iters; ++it) {
        uint4 v[L];
#pragma unroll
        for (int l = 0; l < L; ++l) {
            s = hash32(s + l);
            v[l] = ld<POL>(tab, rsrc, s & mask);
        }
#pragma unroll
        for (int l = 0; l < L; ++l) acc += v[l].x ^ v[l].w;
    }
    if (acc == 0x12345678u) out[tid] = acc;
}

template <int POL>
double run(const uint4* tab, size_t bytes, uint32_t* out) {
    const uint32_t mask = (uint32_t)(bytes / 16 - 1);
    const int blocks = 2048, iters = 32;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_gather<POL>, dim3(blocks), dim3(256), 0, 0, tab, mask, iters, out);
    CHECK(hipEventRecord(a));
    const int reps = 5;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(k_gather<POL>, dim3(blocks), dim3(256), 0, 0, tab, mask, iters, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return (double)blocks * 256 * iters * 8 * reps / (ms * 1e-3);
}

int main(int argc, char** argv) {
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    uint32_t* out;
    CHECK(hipMalloc(&out, 2048 * 256 * 4));
    const size_t sizes[] = {(size_t)64 << 20, (size_t)256 << 20, (size_t)1 << 30};
    for (size_t sz : sizes) {
        uint4* plain;
        CHECK(hipMalloc(&plain, sz));
        CHECK(hipMemset(plain, 1, sz));
        uint4* unc = nullptr;
        uint4* fine = nullptr;
        if (hipExtMallocWithFlags((void**)&unc, sz, hipDeviceMallocUncached) != hipSuccess)
            unc = nullptr;
        else
            CHECK(hipMemset(unc, 1, sz));
        if (hipExtMallocWithFlags((void**)&fine, sz, hipDeviceMallocFinegrained) != hipSuccess)
            fine = nullptr;
        else
            CHECK(hipMemset(fine, 1, sz));
        double r[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        if (only < 0 || only == 0) r[0] = run<0>(plain, sz, out);
        if (only < 0 || only == 1) r[1] = run<1>(plain, sz, out);
        if (only < 0 || only == 2) r[2] = run<2>(plain, sz, out);
        if (only < 0 || only == 3) r[3] = run<3>(plain, sz, out);
        if (only < 0 || only == 4) r[4] = run<4>(plain, sz, out);
        if (only < 0 || only == 5) r[5] = run<5>(plain, sz, out);
        if (only < 0 || only == 6) r[6] = run<6>(plain, sz, out);
        if (unc && (only < 0 || only == 7)) r[7] = run<0>(unc, sz, out);
        if (fine && (only < 0 || only == 8)) r[8] = run<0>(fine, sz, out);
        for (int p = 0; p < 9; ++p)
            printf("{\"table_MiB\":%zu,\"policy\":%d,\"Ggathers_s\":%.2f}\n", sz >> 20, p,
                   r[p] / 1e9);
        fflush(stdout);
        CHECK(hipFree(plain));
        if (unc) CHECK(hipFree(unc));
        if (fine) CHECK(hipFree(fine));
    }
    return 0;
}
