#pragma once
// srv_device.hpp -- device side of the resident small-batch servers (server_box.hpp protocol):
// mailbox polling, system-scope loads / stores, one-round-trip staging from host memory.
// Used by rs_wg.hpp (rs_wg_server_kernel, 2t <= 8) and rs_pair.hpp (rs_pair_server_kernel, 2t > 16).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "server_box.hpp"

namespace ppfs {
namespace srv {

// relaxed system-scope loads bypass the caches without invalidating them (an acquire load would
// invalidate the L2 on every poll, under whatever else runs on the XCD); one acquire fence follows
// a new request
__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys64(const void* p)
{
    return __hip_atomic_load((const uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The next request word, workgroup-uniform, or 0 when the launch should leave (stop, idle_us
// without a request, or SRV_LIFETIME_US since t0).  A request word is never 0 (block count >= 1).
// Lane 0 polls cmd and stop with one 8-byte load (one PCIe round trip), s_sleep between polls,
// and decides alone (its clock); s_cmd is 2 words of LDS.
__device__ __forceinline__ uint32_t next_request(const SrvBox* box, uint32_t seen, uint64_t& last, uint64_t t0,
    uint32_t idle_us, uint32_t* s_cmd)
{
    for (;;) {
        if (threadIdx.x == 0) {
            uint64_t w = 0;
            bool take = false, stop = false;
            for (int spin = 0; spin < 512; ++spin) { // ~50 us between timer checks
                w = ld_sys64(box);
                take = (uint32_t)w != seen;
                stop = (w >> 32) != 0;
                if (take || stop)
                    break;
                __builtin_amdgcn_s_sleep(2);
            }
            const uint64_t now = __builtin_amdgcn_s_memrealtime(); // 100 MHz
            if (take)
                last = now;
            s_cmd[0] = take ? (uint32_t)w : seen;
            // the lifetime holds under a continuous stream of requests too (round 4: a client that
            // posts its next request within the 512-poll window kept one launch resident for good, and
            // a stream sharing its hardware queue -- another context's creation -- waited forever).
            // Leaving with a request pending is safe: the host sees EXITED and relaunches, and the
            // new launch serves every cmd != done.
            s_cmd[1] = stop || now - t0 > 100ull * SRV_LIFETIME_US || (!take && now - last > 100ull * idle_us);
        }
        __syncthreads();
        const uint32_t r = s_cmd[0], leave = s_cmd[1];
        __syncthreads(); // s_cmd is rewritten only after every wave has read it
        if (leave)
            return 0;
        if (r != seen) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); // the request's input bytes, written before cmd
            return r;
        }
    }
}

// The request's outputs are visible to the host, then done = r.
__device__ __forceinline__ void finish_request(SrvBox* box, uint32_t r, uint32_t served)
{
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(&box->served, (uint64_t)served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        st_sys(&box->done, r);
    }
}

// nbytes (<= MAXB) from host-coherent memory (16-byte aligned src, readable up to the next 16
// bytes) into LDS: every thread's loads are issued before any is waited for (one PCIe round trip);
// the loads are unconditional (a branch per load made the compiler wait for each one): past the
// end a thread re-reads the last piece.
template <int NT, int MAXB>
__device__ __forceinline__ void stage_host(uint8_t* dst, const uint8_t* __restrict__ src, uint32_t nbytes, uint32_t tid)
{
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4))); // (a uint4 array went to scratch)
    constexpr int KP = (MAXB / 16 + NT - 1) / NT;
    u32x4 v[KP];
    const uint32_t plast = (nbytes - 1u) / 16u;
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        const uint32_t p = tid + (uint32_t)NT * k;
        v[k] = *(const u32x4*)(src + 16u * min(p, plast));
    }
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        const uint32_t p = tid + (uint32_t)NT * k;
        if (16u * p < nbytes)
            *(u32x4*)(dst + 16u * p) = v[k];
    }
}

} // namespace srv
} // namespace ppfs
