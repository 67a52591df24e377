// stream_ablate2.hip -- diagnostic build (not shipped): which property of the wave-tile walk costs
// bandwidth vs a flat grid-stride copy.  All variants copy 264 MB -> 264 MB with 16-B nt accesses.
//   flat<G>          grid-stride copy, G workgroups of 256
//   chunk<CH, PERS>  each wave moves 16 KiB per iteration as 16 KiB/CH contiguous chunks of CH bytes;
//                    chunk c of wave w in iteration i is global chunk (i*CPI + c)*Wtot + w, so at
//                    CH = 16 KiB every wave streams its own contiguous 16 KiB (the RS tile walk) and
//                    at CH = 1 KiB concurrent waves cover one contiguous region (flat-copy-like).
//                    PERS = persistent grid (2 WG/CU) vs one iteration per wave.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/stream_ablate2.hip -o tools/stream_ablate2.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void flat(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
}

// 16 KiB per wave-iteration = 1024 pieces of 16 B = 16 per lane
template <int CH>
__global__ __launch_bounds__(256) void chunk(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint64_t niter_total)
{
    constexpr int CPI = 16384 / CH;       // chunks per wave-iteration
    constexpr int PPC = CH / 16;          // pieces per chunk
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wtot = (uint64_t)gridDim.x * 4;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + wave;
    // iteration i of wave w exists while (i * wtot + w) < niter_total (16 KiB units)
    auto addr = [&](uint64_t i, int k) -> uint64_t {
        const uint32_t p = lane + 64 * k;          // piece within the 16 KiB unit
        const uint32_t c = p / PPC, q = p % PPC;   // chunk, piece within chunk
        return ((i * CPI + c) * wtot + w) * (uint64_t)CH + q * 16ull;
    };
    u32x4 L[16];
    uint64_t i = 0;
    if (w < niter_total)
#pragma unroll
        for (int k = 0; k < 16; ++k)
            L[k] = __builtin_nontemporal_load((const u32x4*)(in + addr(0, k)));
    for (; i * wtot + w < niter_total; ++i) {
        u32x4 o[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            o[k] = L[k];
        const bool nx = (i + 1) * wtot + w < niter_total;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            L[k] = __builtin_nontemporal_load((const u32x4*)(in + (nx ? addr(i + 1, k) : (uint64_t)(lane * 16 + k * 1024) % 4096)));
#pragma unroll
        for (int k = 0; k < 16; ++k)
            __builtin_nontemporal_store(o[k], (u32x4*)(out + addr(i, k)));
    }
}

template <class F> float timeit(F f)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    std::vector<float> v;
    for (int r = 0; r < 7; ++r) {
        hipEventRecord(a);
        for (int i = 0; i < 5; ++i)
            f();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        v.push_back(ms / 5 * 1e3f);
    }
    std::sort(v.begin(), v.end());
    return v[3];
}

int main()
{
    const size_t bytes = 16384ull * 16384; // 256 MiB each way
    uint8_t *in, *out;
    hipMalloc(&in, bytes);
    hipMalloc(&out, bytes);
    hipMemset(in, 1, bytes);
    hipMemset(out, 0, bytes);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    auto rep = [&](const char* name, float us) {
        printf("%-30s %7.1f us  %6.0f GB/s\n", name, us, 2.0 * bytes / (us * 1e-6) / 1e9);
    };
    char nm[64];
    for (int g : { 512, 1024, 2048, 4096, 16384, 65536 }) {
        snprintf(nm, sizeof nm, "flat grid=%d", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL(flat, dim3(g), dim3(256), 0, 0, (const u32x4*)in, (u32x4*)out, bytes / 16); }));
    }
    const uint64_t units = bytes / 16384; // 16 KiB units
#define CH(C, G)                                                                                          \
    snprintf(nm, sizeof nm, "chunk CH=%d grid=%d", C, (int)(G));                                        \
    rep(nm, timeit([&] { hipLaunchKernelGGL((chunk<C>), dim3(G), dim3(256), 0, 0, in, out, units); }))
    CH(16384, 2 * cus);
    CH(4096, 2 * cus);
    CH(1024, 2 * cus);
    CH(16384, 4 * cus);
    CH(1024, 4 * cus);
    CH(16384, units / 4);
    CH(1024, units / 4);
    return 0;
}
