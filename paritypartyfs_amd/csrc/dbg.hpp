#pragma once
// dbg.hpp -- PPFS_ECC_DEBUG builds: device-side bounds checks of the kernels' global accesses.
//
// Build: tools/build_alt.sh debug -DPPFS_ECC_DEBUG=1  (-> _lib/alt/libppfs_ecc_debug.so; run the
// suite on it with PPFS_ECC_LIB=... and PPFS_ECC_SYNC_CHECK=1, tools/gpu_debug_suite.sh).
//
// PPFS_DBG_OK(p, n, base, extent): is [p, p + n) inside [base, base + extent)?  The extents are the
// ones the launch implies (nblocks x bytes per block of that buffer), i.e. what the host entry point
// validated against the caller's buffers.  An access outside is reported (printf, first few per
// translation unit), counted, and SKIPPED, so a bad index shows up as a count and a failing parity
// test instead of a memory fault.  ppfs_ecc_debug_faults() (api.cpp) sums the counters; it
// returns -1 in normal builds, where PPFS_DBG_OK is the constant true and costs nothing.
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef PPFS_ECC_DEBUG

namespace ppfs {
namespace dbg {

static __device__ unsigned long long g_faults; // one counter per translation unit

__device__ __noinline__ inline bool ok(const void* p, uint64_t n, const void* base, uint64_t extent, int line)
{
    const uint64_t a = (uint64_t)(uintptr_t)p, b = (uint64_t)(uintptr_t)base;
    if (n == 0) // an empty range touches nothing (e.g. the payload of 1-byte parity blocks, a null buffer)
        return true;
    if (base != nullptr && a >= b && n <= extent && a - b <= extent - n)
        return true;
    const unsigned long long k = atomicAdd(&g_faults, 1ull);
    if (k < 8)
        printf("PPFS_ECC_DEBUG line %d: access [%p, +%llu) outside [%p, +%llu) (workgroup %u, thread %u)\n", line, p,
            (unsigned long long)n, base, (unsigned long long)extent, blockIdx.x, threadIdx.x);
    return false;
}

} // namespace dbg
} // namespace ppfs

#define PPFS_DBG_OK(p, n, base, extent)                                                                                \
    ppfs::dbg::ok((const void*)(p), (uint64_t)(n), (const void*)(base), (uint64_t)(extent), __LINE__)

// host accessor of this translation unit's counter: extern "C" long long NAME(void)
#define PPFS_DBG_ACCESSOR(NAME)                                                                                        \
    extern "C" long long NAME(void)                                                                                    \
    {                                                                                                                  \
        unsigned long long v = 0;                                                                                      \
        if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(ppfs::dbg::g_faults), sizeof(v)) != hipSuccess)                         \
            return -2;                                                                                                 \
        return (long long)v;                                                                                           \
    }

#else

#define PPFS_DBG_OK(p, n, base, extent) true
#define PPFS_DBG_ACCESSOR(NAME)

#endif
