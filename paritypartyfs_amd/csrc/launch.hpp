#pragma once
// launch.hpp -- kernel launches with an optional timing hook (host code only).
//
// ppfs_ecc_time_next_launch(start, stop) arms the hook for the calling thread: the next engine
// kernel launched through PPFS_LAUNCH records the two events from its own dispatch packet
// (hipExtLaunchKernel), i.e. the kernel's execution time as rocprofv3 measures it, without the
// launch gap that events recorded on the stream around the call also contain.  bench.py uses it
// for roofline.achieved; the hook disarms itself after one launch.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

namespace ppfs {
struct TimeHook {
    hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local TimeHook g_time_hook;
} // namespace ppfs

#define PPFS_LAUNCH(kernel, grid, block, shmem, stream, ...)                                                           \
    do {                                                                                                               \
        if (ppfs::g_time_hook.start) {                                                                                 \
            const hipEvent_t a_ = ppfs::g_time_hook.start, b_ = ppfs::g_time_hook.stop;                                \
            ppfs::g_time_hook = ppfs::TimeHook {};                                                                     \
            hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, a_, b_, 0u, __VA_ARGS__);                        \
        } else {                                                                                                       \
            hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                                       \
        }                                                                                                              \
    } while (0)
