// vote.hip -- 2-of-3 bitwise majority of replicated records.
//
// Reference: SuperBlockManager::_performBitVoting, lib/super_block_manager/src/
// super_block_manager.cpp:133-165: for every bit of the record, majority = (b1 + b2 + b3 >= 2);
// copy k is "damaged" when any of its bits differs from the majority.  PPFS votes over the three
// SuperBlock copies at mount; the batched form here votes nrec records at once (any record size),
// one thread per byte: out = (a & b) | (a & c) | (b & c) as one v_bitop3, and a record's damage
// bits are set with one atomic OR only where a byte disagrees.
#include <hip/hip_runtime.h>

#include "dbg.hpp"
#include <stdint.h>

namespace ppfs {

__global__ __launch_bounds__(256) void vote3_kernel(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
    const uint8_t* __restrict__ c, uint8_t* __restrict__ out, uint64_t rec_bytes, uint64_t nbytes,
    uint32_t* __restrict__ damaged)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes; i += stride) {
        const uint32_t x = a[i], y = b[i], z = c[i];
        const uint32_t m = __builtin_amdgcn_bitop3_b32(x, y, z, 0xE8); // majority
        out[i] = (uint8_t)m;
        const uint32_t bad = (x != m ? 1u : 0u) | (y != m ? 2u : 0u) | (z != m ? 4u : 0u);
        if (bad && damaged)
            atomicOr(&damaged[i / rec_bytes], bad);
    }
}

} // namespace ppfs

extern "C" hipError_t ppfs_vote3_launch(const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* out,
    uint64_t rec_bytes, uint64_t nrec, uint32_t* damaged, hipStream_t s)
{
    const uint64_t nbytes = rec_bytes * nrec;
    if (damaged) {
        const hipError_t e = hipMemsetAsync(damaged, 0, nrec * sizeof(uint32_t), s);
        if (e != hipSuccess)
            return e;
    }
    if (nbytes == 0)
        return hipSuccess;
    const uint64_t want = (nbytes + 255) / 256;
    const uint32_t grid = (uint32_t)(want < 4096 ? want : 4096);
    hipLaunchKernelGGL(ppfs::vote3_kernel, dim3(grid), dim3(256), 0, s, a, b, c, out, rec_bytes, nbytes, damaged);
    return hipGetLastError();
}

// ---- gather of the rows a host decode has to return (api.cpp host_run) ----
// dst row i = src row idx[i] (row_bytes each): the codewords a decode with write-back changed
// (status 1), packed for one D2H copy when they are few.  One workgroup per row, 16-byte pieces
// where source and destination are 16-byte aligned, else bytes.
namespace ppfs {
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint8_t* __restrict__ src, [[maybe_unused]] uint64_t src_rows,
    uint8_t* __restrict__ dst, const uint32_t* __restrict__ idx, uint32_t nrows, uint32_t row_bytes)
{
    for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
        const uint8_t* s = src + (uint64_t)idx[r] * row_bytes;
        uint8_t* d = dst + (uint64_t)r * row_bytes;
        if (!PPFS_DBG_OK(s, row_bytes, src, src_rows * row_bytes) || !PPFS_DBG_OK(d, row_bytes, dst, (uint64_t)nrows * row_bytes))
            continue;
        if ((((uintptr_t)s | (uintptr_t)d | row_bytes) & 15u) == 0) {
            for (uint32_t p = threadIdx.x; 16u * p < row_bytes; p += blockDim.x)
                *(uint4*)(d + 16u * p) = *(const uint4*)(s + 16u * p);
        } else {
            for (uint32_t b = threadIdx.x; b < row_bytes; b += blockDim.x)
                d[b] = s[b];
        }
    }
}
} // namespace ppfs

// ---- patch list of a decode's write-back (api.cpp host_run_chunks) ----
// The bytes a decode with write-back changed, for the host to patch into its image instead of
// copying every changed codeword back: block b with status[b] == 1 gets (pos << 8 | byte) for each
// byte where cur differs from orig (the codeword before the decode) in patch[b S .. b S + S - 1],
// in position order, its unused slots ~0; a block with more than S changed bytes gets 0xFFFFFFFE in
// slot 0 (the host fetches that codeword whole).  Other blocks' slots are not written.  With
// `image` (a device pointer to the caller's page-locked image, row b at image + b n) the changed
// bytes are stored there instead, over the link, and no list is made.  One wave per block, byte
// loads coalesced across the lanes, a ballot prefix for the slot of each change.
namespace ppfs {
__global__ __launch_bounds__(256) void patch_list_kernel(const uint8_t* __restrict__ cur, const uint8_t* __restrict__ orig,
    const uint8_t* __restrict__ status, uint32_t n, uint64_t nb, uint32_t S, uint32_t* __restrict__ patch,
    uint8_t* __restrict__ image)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t b = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); b < nb; b += nw) {
        if (!PPFS_DBG_OK(status + b, 1, status, nb) || status[b] != 1)
            continue;
        const uint8_t* c = cur + b * n;
        const uint8_t* o = orig + b * n;
        uint32_t* slot = patch + b * S;
        uint32_t cnt = 0;
        for (uint32_t j0 = 0; j0 < n; j0 += 64u) {
            const uint32_t j = j0 + lane;
            const uint32_t cv = j < n && PPFS_DBG_OK(c + j, 1, cur, nb * n) ? c[j] : 0u;
            const uint32_t ov = j < n && PPFS_DBG_OK(o + j, 1, orig, nb * n) ? o[j] : 0u;
            const bool d = j < n && cv != ov;
            if (image) {
                if (d)
                    image[b * n + j] = (uint8_t)cv;
                continue;
            }
            const uint64_t m = __builtin_amdgcn_ballot_w64(d);
            const uint32_t idx = cnt + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
            if (d && idx < S && PPFS_DBG_OK(slot + idx, 4, patch, nb * S * 4))
                slot[idx] = j << 8 | cv;
            cnt += (uint32_t)__builtin_popcountll(m);
        }
        if (image)
            continue;
        if (cnt > S) {
            if (lane == 0 && PPFS_DBG_OK(slot, 4, patch, nb * S * 4))
                slot[0] = 0xFFFFFFFEu;
        } else {
            for (uint32_t j = cnt + lane; j < S; j += 64u)
                if (PPFS_DBG_OK(slot + j, 4, patch, nb * S * 4))
                    slot[j] = 0xFFFFFFFFu;
        }
    }
}
} // namespace ppfs

extern "C" hipError_t ppfs_patch_list_launch(const uint8_t* cur, const uint8_t* orig, const uint8_t* status, uint32_t n,
    uint64_t nb, uint32_t S, uint32_t* patch, uint8_t* image, hipStream_t s)
{
    if (nb == 0)
        return hipSuccess;
    const uint64_t want = (nb + 3) / 4;
    const uint32_t grid = (uint32_t)(want < 8192 ? want : 8192);
    hipLaunchKernelGGL(ppfs::patch_list_kernel, dim3(grid), dim3(256), 0, s, cur, orig, status, n, nb, S, patch, image);
    return hipGetLastError();
}

// ---- device copy at the HBM ceiling (measurement reference for bench.py's roofline) ----
// One thread per 16 bytes over a full grid (workgroups dispatched in address order: one
// contiguous window of HBM in flight), plain 16-byte loads and stores; ragged ends by bytes.
// The same shape reached 6.26 TB/s on 8.6 GB (tools/probes/stream_ablate4.hip).
namespace ppfs {
__global__ __launch_bounds__(256) void copy16_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
    uint64_t n16, uint64_t head, uint64_t bytes)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n16)
        *(uint4*)(dst + head + 16 * i) = *(const uint4*)(src + head + 16 * i);
    if (i < head)
        dst[i] = src[i];
    const uint64_t tail0 = head + 16 * n16;
    if (i < bytes - tail0)
        dst[tail0 + i] = src[tail0 + i];
}
} // namespace ppfs

extern "C" hipError_t ppfs_copy_launch(uint8_t* dst, const uint8_t* src, uint64_t bytes, hipStream_t s)
{
    if (bytes == 0)
        return hipSuccess;
    // 16-byte body where src and dst share their alignment, bytes elsewhere
    uint64_t head = ((uintptr_t)src ^ (uintptr_t)dst) & 15u ? bytes : ((16u - ((uintptr_t)src & 15u)) & 15u);
    if (head > bytes)
        head = bytes;
    const uint64_t n16 = (bytes - head) / 16;
    const uint64_t tail = bytes - head - 16 * n16;
    const uint64_t work = n16 > head ? (n16 > tail ? n16 : tail) : (head > tail ? head : tail);
    const uint64_t grid = (work + 255) / 256;
    if (grid > 0x7FFFFFFFull)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(ppfs::copy16_kernel, dim3((uint32_t)grid), dim3(256), 0, s, dst, src, n16, head, bytes);
    return hipGetLastError();
}

// ---- fault injection: one byte per block (bench step, tests) ----
// Block b of a raw image at `stride` bytes per block gets byte pos[b] replaced by val[b] (mode 0)
// or XORed with it (mode 1); pos[b] >= stride skips the block.  The counterpart of the
// reference's bit flipper (usage_simulator/simulation/src/bit_flipper.cpp), used by bench.py to
// corrupt every codeword of a step: torch's index_put_ of the same bytes reads 8-byte indices and
// costs ~2x this kernel.  Each thread takes 4 consecutive blocks: one
// 4-byte load of their positions and one of their values, then four byte stores.  (Round 4: store
// instructions over 64 consecutive blocks instead, 16 KiB spans: 33 vs 30 us, r4zj; 8 or 16 blocks
// per thread with byte loads: 31.3 vs 30.0 us, r4zk; round 5: non-temporal byte stores and the
// blocks in reverse order, no gain, r5k.)
namespace ppfs {
template <int MODE>
__global__ __launch_bounds__(256) void inject_kernel(uint8_t* __restrict__ raw, uint64_t stride, uint64_t nblocks,
    const uint8_t* __restrict__ pos, const uint8_t* __restrict__ val)
{
    const uint64_t nq = (nblocks + 3) / 4, qi = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= nq)
        return;
    const uint64_t b0 = 4 * qi;
    uint32_t p4, v4;
    if (b0 + 4 <= nblocks && ((uintptr_t)(pos + b0) & 3u) == 0 && ((uintptr_t)(val + b0) & 3u) == 0) {
        p4 = *(const uint32_t*)(pos + b0);
        v4 = *(const uint32_t*)(val + b0);
    } else {
        p4 = v4 = 0xFFFFFFFFu;
        for (uint64_t j = 0; j < 4 && b0 + j < nblocks; ++j) {
            p4 = (p4 & ~(0xFFu << (8 * j))) | ((uint32_t)pos[b0 + j] << (8 * j));
            v4 = (v4 & ~(0xFFu << (8 * j))) | ((uint32_t)val[b0 + j] << (8 * j));
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t p = (p4 >> (8 * j)) & 0xFFu;
        if (b0 + j >= nblocks || p >= stride)
            continue;
        uint8_t* d = raw + (b0 + j) * stride + p;
        const uint8_t v = (uint8_t)(v4 >> (8 * j));
        const uint8_t w = MODE == 0 ? v : (uint8_t)(*d ^ v);
        *d = w;
    }
}
} // namespace ppfs

extern "C" hipError_t ppfs_inject_launch(uint8_t* raw, uint64_t stride, uint64_t nblocks, const uint8_t* pos,
    const uint8_t* val, int mode, hipStream_t s)
{
    if (nblocks == 0)
        return hipSuccess;
    const uint64_t grid = ((nblocks + 3) / 4 + 255) / 256;
    if (grid > 0x7FFFFFFFull)
        return hipErrorInvalidValue;
    if (mode == 0)
        hipLaunchKernelGGL(ppfs::inject_kernel<0>, dim3((uint32_t)grid), dim3(256), 0, s, raw, stride, nblocks, pos, val);
    else
        hipLaunchKernelGGL(ppfs::inject_kernel<1>, dim3((uint32_t)grid), dim3(256), 0, s, raw, stride, nblocks, pos, val);
    return hipGetLastError();
}

// Completion flag of the small-batch launch path (api.cpp wait_flag): queued after a call's
// kernels on the same stream, it makes their outputs visible system-wide and stores `v` (release)
// into host-coherent memory, where the host spins on it.  Cheaper than hipStreamSynchronize's
// completion signal (measured 6.4 vs 10.3 us for one empty kernel, tools/probes/latency_probe.cpp).
namespace ppfs {
__global__ __launch_bounds__(64) void flag_kernel(uint32_t* flag, uint32_t v)
{
    __threadfence_system();
    if (threadIdx.x == 0)
        __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
} // namespace ppfs

extern "C" hipError_t ppfs_flag_launch(uint32_t* flag, uint32_t v, hipStream_t s)
{
    hipLaunchKernelGGL(ppfs::flag_kernel, dim3(1), dim3(64), 0, s, flag, v);
    return hipGetLastError();
}

// src holds src_rows rows; idx[i] < src_rows
extern "C" hipError_t ppfs_gather_rows_launch(const uint8_t* src, uint64_t src_rows, uint8_t* dst, const uint32_t* idx,
    uint32_t nrows, uint32_t row_bytes, hipStream_t s)
{
    if (nrows == 0)
        return hipSuccess;
    const uint32_t grid = nrows < 4096u ? nrows : 4096u;
    hipLaunchKernelGGL(ppfs::gather_rows_kernel, dim3(grid), dim3(256), 0, s, src, src_rows, dst, idx, nrows, row_bytes);
    return hipGetLastError();
}

PPFS_DBG_ACCESSOR(ppfs_dbg_faults_vote)

// Positive control of the PPFS_ECC_DEBUG checks (tests/test_gpu_hygiene.py): a gather of row 5
// from a 4-row source must be reported and skipped.  Returns the number of reports (the counter is
// restored afterwards, so the suite's per-test accounting is unaffected); -1 in normal builds.
#ifdef PPFS_ECC_DEBUG
extern "C" long long ppfs_ecc_debug_selftest(void)
{
    uint8_t *src = nullptr, *dst = nullptr;
    uint32_t* idx = nullptr;
    const uint32_t bad = 5;
    unsigned long long before = 0, after = 0;
    long long r = -2;
    if (hipMalloc(&src, 4 * 16) == hipSuccess && hipMalloc(&dst, 16) == hipSuccess && hipMalloc(&idx, 4) == hipSuccess
        && hipMemcpy(idx, &bad, 4, hipMemcpyHostToDevice) == hipSuccess
        && hipMemcpyFromSymbol(&before, HIP_SYMBOL(ppfs::dbg::g_faults), sizeof(before)) == hipSuccess
        && ppfs_gather_rows_launch(src, 4, dst, idx, 1, 16, nullptr) == hipSuccess && hipDeviceSynchronize() == hipSuccess
        && hipMemcpyFromSymbol(&after, HIP_SYMBOL(ppfs::dbg::g_faults), sizeof(after)) == hipSuccess
        && hipMemcpyToSymbol(HIP_SYMBOL(ppfs::dbg::g_faults), &before, sizeof(before)) == hipSuccess)
        r = (long long)(after - before);
    (void)hipFree(src);
    (void)hipFree(dst);
    (void)hipFree(idx);
    return r;
}
#else
extern "C" long long ppfs_ecc_debug_selftest(void) { return -1; }
#endif
