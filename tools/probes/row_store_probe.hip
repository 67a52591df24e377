// row_store_probe.hip -- can a 2t = 32 decode emit its payload rows straight from registers?
// Each lane pair owns one RS(255,223) block of a 32-block wave tile and holds the block's 223 payload
// bytes in registers, lane c bytes [112 c, 112 c + 112) (111 for c = 1).  The probe writes 2^20 such
// rows (234 MB, packed at the 223-byte stride) in three ways and reports GB/s:
//   coalesced  16-byte aligned pieces, lane l piece 64 k + l (what the LDS-staged emission stores);
//   rows       each lane its own 112 bytes as 7 16-byte stores at 223 b + 112 c + 16 i (unaligned,
//              dword-unaligned for 3 of 4 blocks; the last store of lane 1 is 15 bytes: a 8 + 4 +
//              2 + 1 split);
//   rows_nt    the same with non-temporal stores.
// Diagnostic, not shipped:  make -C tools row_store_probe.bin
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(512) void st_coalesced(uint8_t* __restrict__ out, uint64_t nbytes, uint32_t seed)
{
    const uint64_t npieces = nbytes / 16;
    for (uint64_t p = (uint64_t)blockIdx.x * 512 + threadIdx.x; p < npieces; p += (uint64_t)gridDim.x * 512) {
        const u32x4 v = { (uint32_t)p ^ seed, (uint32_t)p, seed, 7u };
        __builtin_nontemporal_store(v, (u32x4*)(out + 16 * p));
    }
}

template <bool NT>
__global__ __launch_bounds__(512) void st_rows(uint8_t* __restrict__ out, uint64_t nblocks, uint32_t seed)
{
    const uint32_t lane = threadIdx.x & 63u, c = lane & 1u;
    const uint64_t wave = ((uint64_t)blockIdx.x * 512 + threadIdx.x) >> 6, nwaves = ((uint64_t)gridDim.x * 512) >> 6;
    for (uint64_t t = wave; t * 32 < nblocks; t += nwaves) {
        const uint64_t b = t * 32 + (lane >> 1);
        if (b >= nblocks)
            continue;
        uint8_t* dst = out + 223 * b + 112 * c;
        const uint32_t n = c ? 111u : 112u;
#pragma unroll
        for (uint32_t i = 0; i < 7; ++i) {
            const u32x4 v = { (uint32_t)b ^ seed, i, seed, lane };
            if (16 * i + 16 <= n) {
                if constexpr (NT)
                    __builtin_nontemporal_store(v, (u32x4*)(dst + 16 * i));
                else
                    *(u32x4*)(dst + 16 * i) = v;
            } else { // lane 1's last 15 bytes
                *(u32x2*)(dst + 16 * i) = u32x2 { v.x, v.y };
                *(uint32_t*)(dst + 16 * i + 8) = v.z;
                *(uint16_t*)(dst + 16 * i + 12) = (uint16_t)v.w;
                dst[16 * i + 14] = (uint8_t)(v.w >> 16);
            }
        }
    }
}

template <typename F> static float time_it(F launch)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i)
        launch();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < 20; ++i)
        launch();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}

int main()
{
    const uint64_t nb = 1ull << 20, bytes = 223 * nb;
    uint8_t* out;
    (void)hipMalloc(&out, bytes + 64);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const float c = time_it([&] { hipLaunchKernelGGL(st_coalesced, dim3(cus * 8), dim3(512), 0, 0, out, bytes, 1u); });
    const float r = time_it([&] { hipLaunchKernelGGL(st_rows<false>, dim3(cus * 4), dim3(512), 0, 0, out, nb, 2u); });
    const float rn = time_it([&] { hipLaunchKernelGGL(st_rows<true>, dim3(cus * 4), dim3(512), 0, 0, out, nb, 3u); });
    std::printf("{\"bytes\": %llu, \"coalesced_GBps\": %.1f, \"rows_GBps\": %.1f, \"rows_nt_GBps\": %.1f, \"us\": [%.1f, %.1f, %.1f]}\n",
        (unsigned long long)bytes, bytes / (c * 1e6), bytes / (r * 1e6), bytes / (rn * 1e6), c * 1e3, r * 1e3, rn * 1e3);
    const hipError_t e = hipDeviceSynchronize();
    std::printf("{\"status\": \"%s\"}\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
