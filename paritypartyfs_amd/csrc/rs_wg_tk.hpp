#pragma once
// rs_wg_tk.hpp -- the t <= 4 RS encode (rs_wg.hpp's ring of 3 LDS tile buffers, 2 workgroups per
// CU) with its tiles handed out dynamically: per-XCD ticket counters keep the tiles in flight one
// window of HBM and let fast workgroups take more tiles (the persistent static walk's copy skeleton
// measured 96 vs 91.6 us against dynamic tiles).  The counters live in a per-context
// buffer, one set per stream that runs them through the context (api.cpp ctr_for): launches on one
// stream are ordered, and the kernel's last workgroup zeroes its set for the next one.
#include "rs_wg.hpp"

namespace ppfs {
namespace wg {

// ------------------------------------------------------------------------------------
// Dynamic tiles with the ticket in a worker wave: the 4-wave ring encode of rs_wg_encode_kernel
// (NBUF = 3) with its tile sequence from per-XCD ticket counters, as in the ablation
// rs_wg_encode_dyn_kernel (rs_wg_ablate.hpp) but without its fifth wave.  Waves 1-3 issue all of a tile's LDS-DMA
// (at most 6 instructions each: for 2t <= 8 wave 1 issues 6 and waves 2-3 issue 5, which the
// loop's wait counts tolerate, vm_wait_newer rounding down to a multiple of 4) and wave 0 none, so wave 0's vector-memory queue holds only its stores
// and the ticket atomics: the compiler's wait for a returned ticket (issued at the top of
// iteration j, published in LDS at its end) never waits for a tile DMA.  Ticket j is the tile of
// iteration j + 3 (read at the top of iteration j + 1 for the DMA two tiles ahead); the prologue
// takes three.  The last workgroup resets the counters for the next launch on the stream.  The
// loop's ticket is an atomicInc (uinc_wrap), which the compiler's atomic optimizer leaves alone: an
// optimised atomicAdd would be combined across lanes and waited for at once.
// ------------------------------------------------------------------------------------
template <int NPIECE>
__device__ __forceinline__ void dma_tile192(uint8_t* dst, const uint8_t* __restrict__ src, uint32_t tid,
    [[maybe_unused]] const uint8_t* gbase, [[maybe_unused]] uint64_t extent)
{
    constexpr int KI = (NPIECE + 191) / 192;
    const uint32_t w = tid - 64u; // waves 1-3
    const uint32_t lbase = __builtin_amdgcn_readfirstlane(lds_addr(dst) + (w & ~63u) * 16u);
#pragma unroll
    for (int k = 0; k < KI; ++k) {
        const uint32_t p = w + 192u * (uint32_t)k;
        if (((k + 1) * 192 <= NPIECE || p < (uint32_t)NPIECE) && PPFS_DBG_OK(src + (size_t)p * 16, 16, gbase, extent))
            dma16(src + (size_t)p * 16, __builtin_amdgcn_readfirstlane(lbase + 3072u * (uint32_t)k));
    }
}

template <int T2, int WPC = 2, int NTST = 1>
__global__ __launch_bounds__(256, WPC) void rs_wg_encode_tk_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables, uint32_t* __restrict__ ctr)
{
    constexpr int NBUF = 3;
    using L = RsWgLayout<T2>;
    using D = Lds<T2, false, NBUF, false>;
    constexpr int BUF = D::BUFB;
    constexpr int LDS_ALLOC = lds_alloc<D::BYTES + 64, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * K / 16;
    constexpr int OUT_PIECES = TB * 255 / 16;
    constexpr uint32_t KD = (IN_PIECES + 191) / 192; // DMA instructions per tile of a DMA wave
    constexpr uint32_t OFF_TK = D::BYTES;              // 4 ticket slots: slot i & 3 = tile of iteration i
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    uint32_t* const s_tk = (uint32_t*)(lds + OFF_TK);
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const bool dmaw = wave != 0, tk_lane = wave == 0 && lane == 0;
    const uint32_t row = lane_row(lane);
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    const uint32_t nx = gridDim.x < 8u ? gridDim.x : 8u, xc = blockIdx.x % nx;
    uint32_t* const my_ctr = ctr + 32u * xc; // 128-byte lines
    for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += NTHR)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    if (tid < 128)
        *(uint64_t*)(lds + D::OFF_PAR + 8 * tid) = 0;
    if (tk_lane) {
        const uint32_t base = atomicAdd(my_ctr, 3u);
#pragma unroll
        for (uint32_t j = 0; j < 3; ++j)
            s_tk[j] = (base + j) * nx + xc;
    }
    __syncthreads();
    uint64_t q0 = __builtin_amdgcn_readfirstlane(s_tk[0]), q1 = __builtin_amdgcn_readfirstlane(s_tk[1]);
    uint32_t cur = 0, pc = 0, hist = 0, iter = 0;
    if (dmaw) {
        if (q0 < nfull)
            dma_tile192<IN_PIECES>(lds + D::OFF_BUF + PAD, data + q0 * (TB * K), tid, data, nblocks * K);
        const bool go = q1 < nfull;
        if (go)
            dma_tile192<IN_PIECES>(lds + D::OFF_BUF + BUF + PAD, data + q1 * (TB * K), tid, data, nblocks * K);
        hist = go ? 1u : 0u;
        vm_wait_newer(KD * hist); // tile q0 landed, q1 may fly
    }
    while (q0 < nfull) {
        barrier_lds(); // A: tile q0 in LDS, the last emission reads done, the next ticket published
        const uint64_t ahead = __builtin_amdgcn_readfirstlane(s_tk[(iter + 2u) & 3u]);
        // no initial value: writing the register outside wave 0's branch would make every wave wait
        // for the previous ticket (the compiler tracks its pending write per register)
        uint32_t tk;
        if (tk_lane)
            tk = atomicInc(my_ctr, 0xFFFFFFFFu); // the tile of iteration iter + 3
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        const bool go = ahead < nfull;
        if (dmaw && go)
            dma_tile192<IN_PIECES>(lds + D::OFF_BUF + ring_add(cur, NBUF - 1, NBUF) * BUF + PAD, data + ahead * (TB * K),
                tid, data, nblocks * K);
        hist = (hist << 1) | (go ? 1u : 0u);
        if (wave == 0)
            *(uint64_t*)(lds + D::OFF_PAR + (pc ^ 1u) * 512u + 8u * lane) = 0;
        phase_remainder<T2, K, D::NMAP>(lds, buf, par, wave, row);
        barrier_lds(); // B: parity slots complete
        uint8_t* dst = raw + q0 * (TB * 255);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = tid + 256u * k;
            const uint4 o = enc_piece<T2>(lds, buf, par, p);
            if ((k < 3 || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, raw, nblocks * 255u))
                st_nt<NTST>(dst + 16u * p, o);
        }
        ++iter;
        if (dmaw) {
            // the next tile's DMA (issued an iteration ago) landed; the stores since, and this
            // iteration's DMA, may fly
            const uint32_t st = 4u * (iter < 2u ? iter : 2u);
            vm_wait_newer(st + KD * (hist & 1u));
        }
        if (tk_lane)
            s_tk[(iter + 2u) & 3u] = tk * nx + xc; // the tile of (iteration iter - 1) + 3
        cur = ring_add(cur, 1, NBUF);
        pc ^= 1u;
        q0 = q1;
        q1 = ahead;
    }
    if (q0 == nfull && nfull < ntiles) { // the partial tile
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        const uint64_t t = nfull;
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        if (PPFS_DBG_OK(data + t * (TB * K), nb * K, data, nblocks * K))
            stage_bytes(lds + buf + PAD, data + t * (TB * K), nb * K, tid);
        barrier_lds();
        phase_remainder<T2, K, D::NMAP>(lds, buf, par, wave, row);
        barrier_lds();
        uint8_t* dst = raw + t * (TB * 255);
        const uint32_t nout = nb * 255u;
        for (uint32_t p = tid; 16u * p < nout; p += NTHR) {
            const uint4 v = enc_piece<T2>(lds, buf, par, p);
            if (!PPFS_DBG_OK(dst + 16u * p, min(16u, nout - 16u * p), raw, nblocks * 255u))
                continue;
            if (16u * p + 16u <= nout)
                *(uint4*)(dst + 16u * p) = v;
            else
                st_bytes(dst + 16u * p, v, nout - 16u * p);
        }
    }
    if (tk_lane) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // this workgroup's last ticket has returned
        if (atomicAdd(ctr + 32u * 8u, 1u) == gridDim.x - 1) { // every workgroup has taken its last ticket
            for (uint32_t x = 0; x < nx; ++x)
                __hip_atomic_store(ctr + 32u * x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ctr + 32u * 8u, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ------------------------------------------------------------------------------------
// The t <= 4 decode (rs_wg_decode_kernel, double-buffered, 3 workgroups per CU) on the same
// ticket scheme: waves 1-3 issue the DMA, wave 0 (the corrector) takes the tickets.  With two
// buffers ticket j is the tile of iteration j + 2 (read at the top of iteration j + 1 for the DMA
// one tile ahead); the prologue takes two.  Counter set: the second half of the stream's set
// (api.cpp ctr_for), so an encode and a decode on one stream never share counters.
// ------------------------------------------------------------------------------------
template <int T2, int WPC = 3, int NTST = 1>
__global__ __launch_bounds__(256, WPC) void rs_wg_decode_tk_kernel(uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks, const uint8_t* __restrict__ tables, int write_back,
    uint32_t* __restrict__ ctr)
{
    constexpr int NBUF = 2;
    using L = RsWgLayout<T2>;
    using D = Lds<T2, true, NBUF>;
    constexpr int LDS_ALLOC = lds_alloc<D::BYTES + 64, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * 255 / 16;
    constexpr int OUT_PIECES = TB * K / 16;
    constexpr uint32_t OFF_TK = D::BYTES; // 4 ticket slots: slot i & 3 = tile of iteration i
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    uint32_t* const s_tk = (uint32_t*)(lds + OFF_TK);
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const bool dmaw = wave != 0, tk_lane = wave == 0 && lane == 0;
    const uint32_t row = lane_row(lane);
    const bool wb = write_back != 0, want = data != nullptr;
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    const uint32_t nx = gridDim.x < 8u ? gridDim.x : 8u, xc = blockIdx.x % nx;
    uint32_t* const my_ctr = ctr + 32u * xc;
    for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += NTHR)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    if (tid < 128)
        *(uint64_t*)(lds + D::OFF_PAR + 8 * tid) = 0;
    if (tk_lane) {
        const uint32_t base = atomicAdd(my_ctr, 2u);
        s_tk[0] = base * nx + xc;
        s_tk[1] = (base + 1u) * nx + xc;
    }
    __syncthreads();
    uint64_t q0 = __builtin_amdgcn_readfirstlane(s_tk[0]);
    uint32_t cur = 0, pc = 0, iter = 0;
    if (dmaw) {
        if (q0 < nfull)
            dma_tile192<IN_PIECES>(lds + D::OFF_BUF + PAD, raw + q0 * (TB * 255), tid, raw, nblocks * 255u);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    while (q0 < nfull) {
        barrier_lds(); // A: tile q0 in LDS, the last emission reads done, the next ticket published
        const uint64_t q1 = __builtin_amdgcn_readfirstlane(s_tk[(iter + 1u) & 3u]);
        uint32_t tk; // no initial value (see the encode)
        if (tk_lane)
            tk = atomicInc(my_ctr, 0xFFFFFFFFu); // the tile of iteration iter + 2
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        if (dmaw && q1 < nfull)
            dma_tile192<IN_PIECES>(lds + D::OFF_BUF + (cur ^ 1u) * BUF + PAD, raw + q1 * (TB * 255), tid, raw,
                nblocks * 255u);
        if (wave == 0)
            *(uint64_t*)(lds + D::OFF_PAR + (pc ^ 1u) * 512u + 8u * lane) = 0;
        phase_remainder<T2, 255>(lds, buf, par, wave, row);
        barrier_lds(); // B: remainders complete
        if (wave == 0) {
            const uint32_t st = phase_correct<T2>(lds, buf, par, row, true, raw, q0 * TB + row, wb, nblocks * 255u);
            if (status && PPFS_DBG_OK(status + q0 * TB + row, 1, status, nblocks))
                status[q0 * TB + row] = (uint8_t)st;
        }
        barrier_lds(); // C: corrections patched into the LDS rows
        if (want) {
            uint8_t* dst = data + q0 * (TB * K);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t p = tid + 256u * k;
                const uint4 o = dec_piece<T2>(lds, buf, p);
                if ((k < 3 || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, data, nblocks * K))
                    st_nt<NTST>(dst + 16u * p, o);
            }
        }
        ++iter;
        if (dmaw) { // the next tile's DMA landed; this tile's stores may fly
            if (want)
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (tk_lane)
            s_tk[(iter + 1u) & 3u] = tk * nx + xc; // the tile of (iteration iter - 1) + 2
        cur ^= 1u;
        pc ^= 1u;
        q0 = q1;
    }
    if (q0 == nfull && nfull < ntiles) { // the partial tile
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        const uint64_t t = nfull;
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        if (PPFS_DBG_OK(raw + t * (TB * 255), nb * 255u, raw, nblocks * 255u))
            stage_bytes(lds + buf + PAD, raw + t * (TB * 255), nb * 255u, tid);
        barrier_lds();
        phase_remainder<T2, 255>(lds, buf, par, wave, row);
        barrier_lds();
        if (wave == 0) {
            const bool valid = row < nb;
            const uint32_t st = phase_correct<T2>(lds, buf, par, row, valid, raw, t * TB + row, wb, nblocks * 255u);
            if (status && valid && PPFS_DBG_OK(status + t * TB + row, 1, status, nblocks))
                status[t * TB + row] = (uint8_t)st;
        }
        barrier_lds();
        if (want) {
            uint8_t* dst = data + t * (TB * K);
            const uint32_t nout = nb * (uint32_t)K;
            for (uint32_t p = tid; 16u * p < nout; p += NTHR) {
                const uint4 v = dec_piece<T2>(lds, buf, p);
                if (!PPFS_DBG_OK(dst + 16u * p, min(16u, nout - 16u * p), data, nblocks * K))
                    continue;
                if (16u * p + 16u <= nout)
                    *(uint4*)(dst + 16u * p) = v;
                else
                    st_bytes(dst + 16u * p, v, nout - 16u * p);
            }
        }
    }
    if (tk_lane) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (atomicAdd(ctr + 32u * 8u, 1u) == gridDim.x - 1) {
            for (uint32_t x = 0; x < nx; ++x)
                __hip_atomic_store(ctr + 32u * x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ctr + 32u * 8u, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

} // namespace wg
} // namespace ppfs
