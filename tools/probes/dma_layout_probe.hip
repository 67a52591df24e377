// dma_layout_probe.hip -- LDS-DMA throughput of a wave tile (32 rows x 255 B, cfg5 decode input)
// in two layouts: (a) contiguous (lane l of instruction k loads tile bytes 16 (64 k + l)), the
// shipped rs_bs layout; (b) piece-major (lane l of instruction k loads row l % 32, piece 2 k + l / 32:
// source tile + 255 r + 16 i, byte-misaligned), which puts every row at an aligned LDS offset so
// the chain's row reads are conflict-free.  Each wave: DMA, wait, copy the 8 KiB image out with
// coalesced 16-B stores.  Prints median kernel ms over 20 launches per layout, 2^20 rows.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

constexpr int NW = 8, TB = 32, IMG = 8192;

__device__ __forceinline__ void dma16(const uint8_t* g, uint32_t lds_base)
{
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds_base) : "memory", "m0");
}

template <int MODE>
__global__ __launch_bounds__(64 * NW, 1) void probe(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t ntiles)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[NW * IMG];
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* img = lds + wave * IMG;
    const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)img);
    for (uint64_t t = (uint64_t)blockIdx.x * NW + wave; t < ntiles; t += (uint64_t)gridDim.x * NW) {
        const uint8_t* s = src + t * (TB * 255);
        if (MODE != 2)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            uint32_t off;
            if (MODE == 0) {
                off = 16u * (64u * k + lane);
                if (off + 16 > TB * 255)
                    off = TB * 255 - 16;
            } else {
                const uint32_t r = lane & 31u, i = 2u * k + (lane >> 5);
                off = 255u * r + 16u * i;
                if (off + 16 > TB * 255)
                    off = TB * 255 - 16;
            }
            dma16(s + off, base + 1024u * k);
        }
        if (MODE == 2) {
            // register loads of the piece-major pattern (unaligned 16-B global loads), stored out
            uint8_t* d = dst + t * IMG;
            uint4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t r = lane & 31u, i = 2u * k + (lane >> 5);
                uint32_t off = 255u * r + 16u * i;
                if (off + 16 > TB * 255)
                    off = TB * 255 - 16;
                v[k] = *(const uint4*)(s + off);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                __builtin_nontemporal_store(v[k].x, (uint32_t*)(d + 16u * (64u * k + lane)));
                __builtin_nontemporal_store(v[k].y, (uint32_t*)(d + 16u * (64u * k + lane)) + 1);
                __builtin_nontemporal_store(v[k].z, (uint32_t*)(d + 16u * (64u * k + lane)) + 2);
                __builtin_nontemporal_store(v[k].w, (uint32_t*)(d + 16u * (64u * k + lane)) + 3);
            }
            continue;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint8_t* d = dst + t * IMG;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint4 v = *(const uint4*)(img + 16u * (64u * k + lane));
            __builtin_nontemporal_store(v.x, (uint32_t*)(d + 16u * (64u * k + lane)));
            __builtin_nontemporal_store(v.y, (uint32_t*)(d + 16u * (64u * k + lane)) + 1);
            __builtin_nontemporal_store(v.z, (uint32_t*)(d + 16u * (64u * k + lane)) + 2);
            __builtin_nontemporal_store(v.w, (uint32_t*)(d + 16u * (64u * k + lane)) + 3);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
}

int main()
{
    const uint64_t nrows = 1ull << 20, ntiles = nrows / TB;
    uint8_t *src, *dst;
    if (hipMalloc(&src, nrows * 255 + 64) != hipSuccess || hipMalloc(&dst, ntiles * IMG) != hipSuccess)
        return 2;
    hipMemset(src, 0x5A, nrows * 255 + 64);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 3; ++mode) {
            std::vector<float> ms;
            for (int i = 0; i < 25; ++i) {
                hipEventRecord(a, 0);
                if (mode == 0)
                    hipLaunchKernelGGL(probe<0>, dim3(cus), dim3(64 * NW), 0, 0, src, dst, ntiles);
                else if (mode == 1)
                    hipLaunchKernelGGL(probe<1>, dim3(cus), dim3(64 * NW), 0, 0, src, dst, ntiles);
                else
                    hipLaunchKernelGGL(probe<2>, dim3(cus), dim3(64 * NW), 0, 0, src, dst, ntiles);
                hipEventRecord(b, 0);
                hipEventSynchronize(b);
                float m = 0;
                hipEventElapsedTime(&m, a, b);
                if (i >= 5)
                    ms.push_back(m);
            }
            std::sort(ms.begin(), ms.end());
            const double med = ms[ms.size() / 2];
            printf("{\"layout\": \"%s\", \"rep\": %d, \"ms\": %.4f, \"GBps_in\": %.1f, \"GBps_in_out\": %.1f}\n",
                mode == 2 ? "piece-major-regs" : mode ? "piece-major" : "contiguous", rep, med, nrows * 255 / med / 1e6, (nrows * 255 + ntiles * IMG) / med / 1e6);
        }
    return 0;
}
