// stream_ablate4.hip -- diagnostic build (not shipped): memory-only skeletons of the cfg4
// streaming kernels (block_size 4096, 2^20 blocks: 4 GiB in, 4 GiB out) to find the copy
// ceiling of the one-wave-per-block layout that bit_fast.hip uses.
//   flat<NT>            grid-stride 16-B copy, 2048 threads per CU worth of workgroups
//   wave<DEPTH,NT,WPC>  persistent: one wave per 4 KiB block, 4 x 16 B per lane, DEPTH blocks
//                       of loads in flight per wave (1 = load, then store; 2 = prefetch the next
//                       block while storing this one), WPC 256-thread workgroups per CU
// usage: stream_ablate4 [blocks]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT> __device__ __forceinline__ u32x4 ld(const u32x4* p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}
template <bool NT> __device__ __forceinline__ void st(u32x4* p, u32x4 v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

template <bool NT>
__global__ __launch_bounds__(256) void flat(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        st<NT>(out + i, ld<NT>(in + i));
}

template <bool NT>
__global__ __launch_bounds__(256) void flat4(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n)
{
    // each thread: 4 independent 16-B loads per iteration, wave-coalesced (1 KiB per instruction)
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t b = wave; b * 256 < n; b += nw) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v[k] = ld<NT>(in + b * 256 + 64 * k + lane);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            st<NT>(out + b * 256 + 64 * k + lane, v[k]);
    }
}

template <int DEPTH, bool NT>
__global__ __launch_bounds__(256) void wave_pers(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t nblk)
{
    const size_t lane = threadIdx.x & 63;
    const size_t nw = (size_t)gridDim.x * 4;
    size_t b = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    u32x4 v[DEPTH][4];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
        if (b + d * nw < nblk)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                v[d][k] = ld<NT>(in + (b + d * nw) * 256 + 64 * k + lane);
    for (; b < nblk; b += nw) {
        u32x4 c[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            c[k] = v[0][k];
#pragma unroll
        for (int d = 0; d + 1 < DEPTH; ++d)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                v[d][k] = v[d + 1][k];
        const size_t nx = b + DEPTH * nw;
        if (nx < nblk)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                v[DEPTH - 1][k] = ld<NT>(in + nx * 256 + 64 * k + lane);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            st<NT>(out + b * 256 + 64 * k + lane, c[k]);
    }
}

#define CK(x)                                                                                                          \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) {                                                                                        \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                                           \
            return 1;                                                                                                  \
        }                                                                                                              \
    } while (0)

template <typename F> static float timeit(F f, int reps)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 20; ++i)
        f(); // clock ramp
    (void)hipDeviceSynchronize();
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        (void)hipEventRecord(a, 0);
        f();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main(int argc, char** argv)
{
    const size_t nblk = argc > 1 ? (size_t)atoll(argv[1]) : (1u << 20);
    const size_t bytes = nblk * 4096, n16 = bytes / 16;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    u32x4 *in, *out;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&out, bytes));
    CK(hipMemset(in, 1, bytes));
    CK(hipMemset(out, 0, bytes));
    auto report = [&](const char* name, float ms) {
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n", name, ms, 2.0 * bytes / ms / 1e6,
            2.0 * bytes / ms / 1e6 / 8000.0);
        fflush(stdout);
    };
    const int reps = 20;
    report("flat plain g=8/CU", timeit([&] { flat<false><<<8 * cus, 256>>>(in, out, n16); }, reps));
    report("flat nt g=8/CU", timeit([&] { flat<true><<<8 * cus, 256>>>(in, out, n16); }, reps));
    report("flat plain g=full", timeit([&] { flat<false><<<(n16 + 255) / 256, 256>>>(in, out, n16); }, reps));
    report("flat4 plain g=8/CU", timeit([&] { flat4<false><<<8 * cus, 256>>>(in, out, n16); }, reps));
    report("flat4 nt g=8/CU", timeit([&] { flat4<true><<<8 * cus, 256>>>(in, out, n16); }, reps));
    report("flat4 plain g=full", timeit([&] { flat4<false><<<nblk / 4, 256>>>(in, out, n16); }, reps));
    report("flat4 nt g=full", timeit([&] { flat4<true><<<nblk / 4, 256>>>(in, out, n16); }, reps));
    for (int wpc : { 2, 4, 6, 8 }) {
        char nm[96];
        snprintf(nm, sizeof nm, "wave d1 plain wpc=%d", wpc);
        report(nm, timeit([&] { wave_pers<1, false><<<wpc * cus, 256>>>(in, out, nblk); }, reps));
        snprintf(nm, sizeof nm, "wave d2 plain wpc=%d", wpc);
        report(nm, timeit([&] { wave_pers<2, false><<<wpc * cus, 256>>>(in, out, nblk); }, reps));
        snprintf(nm, sizeof nm, "wave d3 plain wpc=%d", wpc);
        report(nm, timeit([&] { wave_pers<3, false><<<wpc * cus, 256>>>(in, out, nblk); }, reps));
        snprintf(nm, sizeof nm, "wave d2 nt wpc=%d", wpc);
        report(nm, timeit([&] { wave_pers<2, true><<<wpc * cus, 256>>>(in, out, nblk); }, reps));
    }
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
