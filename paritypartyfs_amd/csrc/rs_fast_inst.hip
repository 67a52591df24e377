// rs_fast_inst.hip -- one fast-path instantiation (2t = PPFS_T2), compiled once per 2t.
#include "rs_fast.hpp"

#ifndef PPFS_T2
#error "compile with -DPPFS_T2=<2t>"
#endif

#define PPFS_CAT2(a, b) a##b
#define PPFS_CAT(a, b) PPFS_CAT2(a, b)

using namespace ppfs;

extern "C" hipError_t PPFS_CAT(ppfs_rs_fast_encode_t, PPFS_T2)(const uint8_t* d, uint8_t* r, uint64_t nb,
    const uint8_t* tab, hipStream_t s)
{
    const uint32_t grid = (uint32_t)((nb + RS_TILE - 1) / RS_TILE);
    hipLaunchKernelGGL(rs255_encode_kernel<PPFS_T2>, dim3(grid), dim3(256), 0, s, d, r, nb, tab);
    return hipGetLastError();
}

extern "C" hipError_t PPFS_CAT(ppfs_rs_fast_decode_t, PPFS_T2)(uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb,
    const uint8_t* tab, int wb, hipStream_t s)
{
    const uint32_t grid = (uint32_t)((nb + RS_TILE - 1) / RS_TILE);
    hipLaunchKernelGGL(rs255_decode_kernel<PPFS_T2>, dim3(grid), dim3(256), 0, s, r, d, st, nb, tab, wb);
    return hipGetLastError();
}
