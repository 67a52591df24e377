// stream_ablate.hip -- diagnostic build (not shipped): what streaming structure reaches the HBM
// ceiling for the RS(255,249) encode traffic shape (read 2^20 x 249 B packed, write 2^20 x 255 B).
// Variants move the same bytes (payload tile 15936 B in, codeword tile 16320 B out per 64-block
// wave-tile) without any coding work:
//   copy_flat      grid-stride 16 B/lane copy of the same total bytes (reference ceiling)
//   tile_regs<D,L> persistent wave-tiles through VGPRs, prefetch depth D (1 or 2), L = LDS round trip
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/stream_ablate.hip -o tools/stream_ablate.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int IN_P = 996;   // 64 * 249 / 16
constexpr int OUT_P = 1020; // 64 * 255 / 16
constexpr int IN_R = (IN_P + 63) / 64;
constexpr int OUT_R = (OUT_P + 63) / 64;

template <int NT> __device__ __forceinline__ u32x4 ld(const u32x4* p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}
template <int NT> __device__ __forceinline__ void st(u32x4* p, u32x4 v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

template <int NT>
__global__ __launch_bounds__(256) void copy_flat(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t nin,
    size_t nout)
{
    // reads nin pieces, writes nout pieces (nout > nin: the extra pieces re-read modulo nin)
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nout; i += stride) {
        const u32x4 v = i < nin ? ld<NT>(in + i) : u32x4 { 1, 2, 3, 4 };
        st<NT>(out + i, v);
    }
}

template <int D, int LDSRT, int NT, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void tile_regs(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
    uint64_t ntiles)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDSRT ? WAVES * 16384 : 16];
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* tile = lds + (LDSRT ? wave * 16384 : 0);
    const uint64_t stride = (uint64_t)gridDim.x * WAVES;
    uint64_t wt = (uint64_t)blockIdx.x * WAVES + wave;
    u32x4 L[D][IN_R];
    auto load = [&](u32x4(&R)[IN_R], uint64_t t) {
#pragma unroll
        for (int k = 0; k < IN_R; ++k) {
            const uint32_t p = lane + 64 * k;
            if (t < ntiles && (k < IN_P / 64 || p < IN_P))
                R[k] = ld<NT>((const u32x4*)(in + t * 15936) + p);
            else
                R[k] = u32x4 { 0, 0, 0, 0 };
        }
    };
#pragma unroll
    for (int d = 0; d < D; ++d)
        load(L[d], wt + d * stride);
    for (; wt < ntiles; wt += stride) {
        u32x4 o[OUT_R];
        if constexpr (LDSRT) {
#pragma unroll
            for (int k = 0; k < IN_R; ++k) {
                const uint32_t p = lane + 64 * k;
                if (k < IN_P / 64 || p < IN_P)
                    *(u32x4*)(tile + p * 16) = L[0][k];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < OUT_R; ++k) {
                const uint32_t p = lane + 64 * k;
                o[k] = (k < OUT_P / 64 || p < OUT_P) ? *(const u32x4*)(tile + (p % IN_P) * 16) : u32x4 { 0, 0, 0, 0 };
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        } else {
#pragma unroll
            for (int k = 0; k < OUT_R; ++k)
                o[k] = L[0][k < IN_R ? k : IN_R - 1] + u32x4 { (uint32_t)k, 0, 0, 0 };
        }
#pragma unroll
        for (int d = 0; d + 1 < D; ++d)
#pragma unroll
            for (int k = 0; k < IN_R; ++k)
                L[d][k] = L[d + 1][k];
        load(L[D - 1], wt + D * stride);
#pragma unroll
        for (int k = 0; k < OUT_R; ++k) {
            const uint32_t p = lane + 64 * k;
            if (k < OUT_P / 64 || p < OUT_P)
                st<NT>((u32x4*)(out + wt * 16320) + p, o[k]);
        }
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
    const uint64_t nb = 1ull << 20, ntiles = nb / 64;
    uint8_t *in, *out;
    hipMalloc(&in, nb * 249);
    hipMalloc(&out, nb * 255);
    hipMemset(in, 1, nb * 249);
    hipMemset(out, 0, nb * 255);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const double bytes = nb * 504.0;
    auto rep = [&](const char* name, float us) {
        printf("%-34s %7.1f us  %6.0f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
    };
    const size_t nin = nb * 249 / 16, nout = nb * 255 / 16;
    for (int g : { 1024, 4096, 16384 }) {
        char nm[64];
        snprintf(nm, sizeof nm, "copy_flat nt grid=%d", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL(copy_flat<1>, dim3(g), dim3(256), 0, 0, (const u32x4*)in, (u32x4*)out, nin, nout); }));
        snprintf(nm, sizeof nm, "copy_flat plain grid=%d", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL(copy_flat<0>, dim3(g), dim3(256), 0, 0, (const u32x4*)in, (u32x4*)out, nin, nout); }));
    }
#define TR(D, LR, NT, W, WGPERCU)                                                                               \
    rep("tile D" #D " lds" #LR " nt" #NT " waves" #W " x" #WGPERCU, timeit([&] {                                  \
        hipLaunchKernelGGL((tile_regs<D, LR, NT, W>), dim3(WGPERCU * cus), dim3(64 * W), 0, 0, in, out, ntiles); \
    }))
    TR(1, 1, 1, 4, 2);
    TR(1, 0, 1, 4, 2);
    TR(2, 0, 1, 4, 2);
    TR(2, 1, 1, 4, 2);
    TR(1, 0, 1, 4, 4);
    TR(1, 1, 1, 8, 1);
    TR(1, 0, 1, 8, 1);
    TR(1, 0, 1, 4, 3);
    TR(2, 0, 1, 4, 3);
    TR(1, 1, 0, 4, 2);
    return 0;
}
