#pragma once
// rs_wg_tk_ablate.hpp -- ablation (built with -DPPFS_WG_TKN=NBUF): the ticket encode of rs_wg_tk.hpp
// over a ring of NBUF tile buffers (3..6) instead of 3.  q0 of the next iteration is read from its
// ticket slot after the iteration's end (the slot was published NBUF - 1 iterations earlier).
#include "rs_wg_tk.hpp"

namespace ppfs {
namespace wg {

template <int T2, int NBUF, int WPC = 2, int NTST = 1>
__global__ __launch_bounds__(256, WPC) void rs_wg_encode_tkn_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables, uint32_t* __restrict__ ctr)
{
    static_assert(NBUF >= 3 && NBUF <= 6, "ring depth");
    using L = RsWgLayout<T2>;
    using D = Lds<T2, false, NBUF, false>;
    constexpr int BUF = D::BUFB;
    constexpr int LDS_ALLOC = lds_alloc<D::BYTES + 64, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * K / 16;
    constexpr int OUT_PIECES = TB * 255 / 16;
    constexpr uint32_t KD = (IN_PIECES + 191) / 192; // DMA instructions per tile of a DMA wave
    constexpr uint32_t OFF_TK = D::BYTES;              // 8 ticket slots: slot i & 7 = tile of iteration i
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
        const uint32_t base = atomicAdd(my_ctr, (uint32_t)NBUF);
#pragma unroll
        for (uint32_t j = 0; j < (uint32_t)NBUF; ++j)
            s_tk[j] = (base + j) * nx + xc;
    }
    __syncthreads();
    uint64_t q0 = __builtin_amdgcn_readfirstlane(s_tk[0]);
    uint32_t cur = 0, pc = 0, hist = 0, iter = 0;
    if (dmaw) {
        if (q0 < nfull)
            dma_tile192<IN_PIECES>(lds + D::OFF_BUF + PAD, data + q0 * (TB * K), tid, data, nblocks * K);
#pragma unroll
        for (int j = 1; j <= NBUF - 2; ++j) {
            const uint64_t qj = __builtin_amdgcn_readfirstlane(s_tk[j]);
            const bool go = qj < nfull;
            if (go)
                dma_tile192<IN_PIECES>(lds + D::OFF_BUF + j * BUF + PAD, data + qj * (TB * K), tid, data, nblocks * K);
            hist = (hist << 1) | (go ? 1u : 0u);
        }
        vm_wait_newer(KD * __builtin_popcount(hist)); // tile q0 landed, the later ones may fly
    }
    while (q0 < nfull) {
        barrier_lds(); // A: tile q0 in LDS, the last emission reads done, the next ticket published
        const uint64_t ahead = __builtin_amdgcn_readfirstlane(s_tk[(iter + NBUF - 1u) & 7u]);
        // no initial value: writing the register outside wave 0's branch would make every wave wait
        // for the previous ticket (the compiler tracks its pending write per register)
        uint32_t tk;
        if (tk_lane)
            tk = atomicInc(my_ctr, 0xFFFFFFFFu); // the tile of iteration iter + NBUF
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
            const uint32_t st = 4u * (iter < (uint32_t)(NBUF - 1) ? iter : (uint32_t)(NBUF - 1));
            vm_wait_newer(st + KD * __builtin_popcount(hist & ((1u << (NBUF - 2)) - 1u)));
        }
        if (tk_lane)
            s_tk[(iter + NBUF - 1u) & 7u] = tk * nx + xc; // the tile of (iteration iter - 1) + NBUF
        cur = ring_add(cur, 1, NBUF);
        pc ^= 1u;
        q0 = __builtin_amdgcn_readfirstlane(s_tk[iter & 7u]);
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

} // namespace wg
} // namespace ppfs
