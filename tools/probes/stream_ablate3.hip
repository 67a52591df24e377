// stream_ablate3.hip -- diagnostic build (not shipped): memory-only skeletons of a
// WORKGROUP-cooperative RS tile (64 blocks: 64*249 B in, 64*255 B out per tile), vs flat copy,
// over a size sweep (tail/ramp vs steady state).
//   wg_oneshot<LDSDMA>    grid = one workgroup per tile; the 256 threads load the tile (4 x 16 B
//                         per lane) into LDS (LDS-DMA or regs + ds_write), barrier, then emit the
//                         out-tile from LDS with a per-block shift (as the codeword layout needs)
//                         straight to global with 16-B stores.
//   wg_pers<NBUF>         persistent: G workgroups walk tiles; NBUF = 2 double-buffers the LDS tile
//                         (next tile's LDS-DMA issued before this tile's emission).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int KB = 249, NB = 255, TB = 64;
constexpr int IN_P = TB * KB / 16, OUT_P = TB * NB / 16; // 996, 1020

__global__ __launch_bounds__(256) void flat(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t nin, size_t nout)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nout; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(in + (i < nin ? i : 0)), out + i);
}

__device__ __forceinline__ void dma16(const uint8_t* g, uint8_t* l)
{
    __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// emit out piece p (16 B) of a tile from the LDS input tile: codeword byte j of block b = j / 255,
// off = j % 255 -> parity (off < 6, fake: 0) or payload byte b*249 + off - 6
__device__ __forceinline__ u32x4 emit_piece(const uint8_t* tile, uint32_t p)
{
    const uint32_t j0 = p * 16;
    const uint32_t b = j0 / NB, off = j0 - b * NB;
    // source of byte j0 (clamped for the parity region) and the 5 aligned dwords around it
    int src = (int)(b * KB + off) - 6;
    src = src < 0 ? 0 : src;
    const uint32_t a = (uint32_t)src & ~3u, sh = ((uint32_t)src & 3u) * 8u;
    const uint32_t* w = (const uint32_t*)(tile + a);
    const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4];
    u32x4 v;
    v.x = __builtin_amdgcn_alignbit(d1, d0, sh);
    v.y = __builtin_amdgcn_alignbit(d2, d1, sh);
    v.z = __builtin_amdgcn_alignbit(d3, d2, sh);
    v.w = __builtin_amdgcn_alignbit(d4, d3, sh);
    return v;
}

template <int LDSDMA>
__global__ __launch_bounds__(256) void wg_oneshot(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint64_t ntiles)
{
    __shared__ __attribute__((aligned(16))) uint8_t tile[IN_P * 16 + 64];
    const uint32_t tid = threadIdx.x;
    const uint64_t t = blockIdx.x;
    const uint8_t* src = in + t * (TB * KB);
    if (LDSDMA) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = tid + 256 * k;
            if (k < 3 || p < IN_P)
                dma16(src + p * 16, tile + 4096 * k + (tid & ~63u) * 16);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        u32x4 L[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = tid + 256 * k;
            if (k < 3 || p < IN_P)
                L[k] = __builtin_nontemporal_load((const u32x4*)(src + p * 16));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = tid + 256 * k;
            if (k < 3 || p < IN_P)
                *(u32x4*)(tile + p * 16) = L[k];
        }
    }
    __syncthreads();
    uint8_t* dst = out + t * (TB * NB);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t p = tid + 256 * k;
        if (k < 3 || p < OUT_P)
            __builtin_nontemporal_store(emit_piece(tile, p), (u32x4*)(dst + p * 16));
    }
}

template <int NBUF>
__global__ __launch_bounds__(256) void wg_pers(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint64_t ntiles)
{
    __shared__ __attribute__((aligned(16))) uint8_t tiles[NBUF][IN_P * 16 + 64];
    const uint32_t tid = threadIdx.x;
    uint64_t t = blockIdx.x;
    auto issue = [&](uint64_t tt, uint8_t* tile) {
        const uint8_t* src = in + tt * (TB * KB);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = tid + 256 * k;
            if (k < 3 || p < IN_P)
                dma16(src + p * 16, tile + 4096 * k + (tid & ~63u) * 16);
        }
    };
    int cur = 0;
    if (t < ntiles)
        issue(t, tiles[0]);
    for (; t < ntiles; t += gridDim.x) {
        const uint64_t nx = t + gridDim.x;
        if (NBUF == 2) {
            if (nx < ntiles) {
                issue(nx, tiles[cur ^ 1]);
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        uint8_t* dst = out + t * (TB * NB);
        u32x4 o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o[k] = emit_piece(tiles[cur], tid + 256 * k);
        __syncthreads();
        if (NBUF == 1 && nx < ntiles)
            issue(nx, tiles[0]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = tid + 256 * k;
            if (k < 3 || p < OUT_P)
                __builtin_nontemporal_store(o[k], (u32x4*)(dst + p * 16));
        }
        if (NBUF == 2)
            cur ^= 1;
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
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (uint64_t nb : { 1ull << 19, 1ull << 20, 1ull << 21, 1ull << 22 }) {
        const uint64_t ntiles = nb / 64;
        uint8_t *in, *out;
        hipMalloc(&in, nb * KB + 4096);
        hipMalloc(&out, nb * NB + 4096);
        hipMemset(in, 1, nb * KB);
        hipMemset(out, 0, nb * NB);
        const double bytes = nb * 504.0;
        auto rep = [&](const char* name, float us) {
            printf("nb=2^%-2d %-28s %7.1f us  %6.0f GB/s\n", __builtin_ctzll(nb), name, us, bytes / (us * 1e-6) / 1e9);
        };
        const size_t nin = nb * KB / 16, nout = nb * NB / 16;
        rep("flat grid=16384", timeit([&] { hipLaunchKernelGGL(flat, dim3(16384), dim3(256), 0, 0, (const u32x4*)in, (u32x4*)out, nin, nout); }));
        rep("flat grid=nout/256", timeit([&] { hipLaunchKernelGGL(flat, dim3((nout + 255) / 256), dim3(256), 0, 0, (const u32x4*)in, (u32x4*)out, nin, nout); }));
        rep("wg_oneshot dma", timeit([&] { hipLaunchKernelGGL(wg_oneshot<1>, dim3(ntiles), dim3(256), 0, 0, in, out, ntiles); }));
        rep("wg_oneshot regs", timeit([&] { hipLaunchKernelGGL(wg_oneshot<0>, dim3(ntiles), dim3(256), 0, 0, in, out, ntiles); }));
        for (int wpc : { 2, 4, 6, 8 }) {
            char nm[64];
            snprintf(nm, sizeof nm, "wg_pers nbuf1 x%d", wpc);
            rep(nm, timeit([&] { hipLaunchKernelGGL(wg_pers<1>, dim3(wpc * cus), dim3(256), 0, 0, in, out, ntiles); }));
            snprintf(nm, sizeof nm, "wg_pers nbuf2 x%d", wpc);
            rep(nm, timeit([&] { hipLaunchKernelGGL(wg_pers<2>, dim3(wpc * cus), dim3(256), 0, 0, in, out, ntiles); }));
        }
        hipFree(in);
        hipFree(out);
    }
    return 0;
}
