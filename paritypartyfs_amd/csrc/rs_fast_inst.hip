// rs_fast_inst.hip -- one fast-path instantiation (2t = PPFS_T2), compiled once per 2t.
#include "rs_fast.hpp"
#include "rs_wg.hpp"

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

#if PPFS_T2 <= 8
// workgroup path (2t <= 8): one 256-thread workgroup per 64-block tile, WPC resident per CU
constexpr int ENC_NBUF = 2, ENC_WPC = (4 * wg::lds_bytes<PPFS_T2, false, 2>() <= 163840) ? 4 : 3;
constexpr int DEC_NBUF = 2, DEC_WPC = 3;

static uint32_t rs_wg_grid(uint64_t nb, int wpc)
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
        c = 256;
    const uint64_t tiles = (nb + wg::TB - 1) / wg::TB;
    const uint64_t cap = (uint64_t)wpc * (uint64_t)c;
    return (uint32_t)(tiles < cap ? (tiles ? tiles : 1) : cap);
}
#endif

extern "C" hipError_t PPFS_CAT(ppfs_rs_fast_encode_t, PPFS_T2)(const uint8_t* d, uint8_t* r, uint64_t nb,
    const uint8_t* tab, hipStream_t s)
{
#if PPFS_T2 <= 8
    hipLaunchKernelGGL((wg::rs_wg_encode_kernel<PPFS_T2, ENC_NBUF, ENC_WPC>), dim3(rs_wg_grid(nb, ENC_WPC)), dim3(256), 0, s,
        d, r, nb, tab);
#else
    const uint32_t grid = rs_grid(nb);
    hipLaunchKernelGGL(rs255_encode_kernel<PPFS_T2>, dim3(grid), dim3(256), 0, s, d, r, nb, tab);
#endif
    return hipGetLastError();
}

extern "C" hipError_t PPFS_CAT(ppfs_rs_fast_decode_t, PPFS_T2)(uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb,
    const uint8_t* tab, int wb, hipStream_t s)
{
#if PPFS_T2 <= 8
    hipLaunchKernelGGL((wg::rs_wg_decode_kernel<PPFS_T2, DEC_NBUF, DEC_WPC>), dim3(rs_wg_grid(nb, DEC_WPC)), dim3(256), 0,
        s, r, d, st, nb, tab, wb);
#else
    const uint32_t grid = rs_grid(nb);
    hipLaunchKernelGGL(rs255_decode_kernel<PPFS_T2>, dim3(grid), dim3(256), 0, s, r, d, st, nb, tab, wb);
#endif
    return hipGetLastError();
}
