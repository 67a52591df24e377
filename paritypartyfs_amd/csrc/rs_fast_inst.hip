// rs_fast_inst.hip -- one fast-path instantiation (2t = PPFS_T2), compiled once per 2t.
#include "rs_fast.hpp"

#ifndef PPFS_T2
#error "compile with -DPPFS_T2=<2t>"
#endif

#define PPFS_CAT2(a, b) a##b
#define PPFS_CAT(a, b) PPFS_CAT2(a, b)

using namespace ppfs;

// persistent grid: two 256-thread workgroups per CU (LDS-limited), capped by the work
static uint32_t rs_grid(uint64_t nb)
{
    static int cus[64] = { 0 };
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64)
        dev = 0;
    if (!cus[dev]) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            c = 256;
        cus[dev] = c;
    }
    const uint64_t wave_tiles = (nb + RS_WT - 1) / RS_WT;
    const uint64_t want = (wave_tiles + RS_WAVES - 1) / RS_WAVES;
    const uint64_t cap = 2ull * (uint64_t)cus[dev];
    return (uint32_t)(want < cap ? (want ? want : 1) : cap);
}

extern "C" hipError_t PPFS_CAT(ppfs_rs_fast_encode_t, PPFS_T2)(const uint8_t* d, uint8_t* r, uint64_t nb,
    const uint8_t* tab, hipStream_t s)
{
    const uint32_t grid = rs_grid(nb);
    hipLaunchKernelGGL(rs255_encode_kernel<PPFS_T2>, dim3(grid), dim3(256), 0, s, d, r, nb, tab);
    return hipGetLastError();
}

extern "C" hipError_t PPFS_CAT(ppfs_rs_fast_decode_t, PPFS_T2)(uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb,
    const uint8_t* tab, int wb, hipStream_t s)
{
    const uint32_t grid = rs_grid(nb);
    hipLaunchKernelGGL(rs255_decode_kernel<PPFS_T2>, dim3(grid), dim3(256), 0, s, r, d, st, nb, tab, wb);
    return hipGetLastError();
}
