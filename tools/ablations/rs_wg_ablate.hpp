// rs_wg_ablate.hpp -- ABLATION ONLY (built with -DPPFS_WG_DYN=N or -DPPFS_WG_ENC_W8=NBUF,
// tools/build_alt.sh): two encode variants of rs_wg.hpp's 2t <= 8 RS kernels, both correct (295 GPU
// tests) and not faster in the bench step (profiles/r2_ablations/dyn_tiles_kablate.jsonl,
// w8_encode_ab.jsonl).  Their tables (RsWgLayout MAP32, CTR) stay in every context's blob.
#pragma once
#include "rs_wg.hpp"

namespace ppfs {
namespace wg {

// ------------------------------------------------------------------------------------
// Dynamic tiles (PPFS_WG_DYN): the same ring, but a workgroup's next tile comes from a ticket
// counter instead of t + G, so the tiles in flight stay one window of HBM however far the
// workgroups drift apart (a full grid gets that from the dispatcher's address order).  NX = min(8,
// G) counters, one per XCD (workgroup w uses counter w % NX; ticket k of counter x is tile
// k NX + x): one counter for the whole chip serialises ~12 ns per ticket, twice the kernel.  A
// fifth wave takes the tickets: its only vector-memory operations are the counter atomics, so
// waiting for one never waits for a tile DMA (the other waves' counted vmcnt is untouched).  The
// ticket for the DMA of iteration j + 2 is taken in iteration j and published in LDS in iteration
// j + 1.  Tiles >= the full-tile count end a workgroup's walk (tile == nfull is the partial tile,
// if any); the last workgroup to finish zeroes the counters for the next launch on the stream.
// FAKE (ablation): the static walk's tiles through the same machinery, no atomics.
// ------------------------------------------------------------------------------------
template <int T2, int NBUF = 3, int WPC = 2, int MODE = 3, int NTST = 1, bool FAKE = false>
__global__ __launch_bounds__(320, WPC) void rs_wg_encode_dyn_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables, uint32_t* __restrict__ ctr)
{
    static_assert(NBUF >= 3 && NBUF <= 4, "ring of tile buffers");
    using L = RsWgLayout<T2>;
    using D = Lds<T2, false, NBUF, false>;
    constexpr int BUF = D::BUFB;
    constexpr int LDS_ALLOC = lds_alloc<D::BYTES + 64, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * K / 16;
    constexpr int OUT_PIECES = TB * 255 / 16;
    constexpr int NPRO = NBUF + 1; // ring tickets + the DMA tickets of iterations 0 and 1
    constexpr uint32_t OFF_TK = D::BYTES; // NPRO prologue tiles, then 2 per-iteration slots
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    uint32_t* const s_tk = (uint32_t*)(lds + OFF_TK);
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const bool worker = wave < 4;
    const uint32_t row = lane_row(lane);
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    const uint32_t nx = gridDim.x < 8u ? gridDim.x : 8u, xc = blockIdx.x % nx;
    uint32_t* const my_ctr = ctr + 32u * xc; // 128-byte lines
    if (worker) {
        for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += NTHR)
            *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
        if (tid < 128)
            *(uint64_t*)(lds + D::OFF_PAR + 8 * tid) = 0;
    }
    const uint32_t gx = gridDim.x / nx;
    uint32_t fk = blockIdx.x / nx;
    if (!worker && lane == 0) {
        if constexpr (FAKE) {
#pragma unroll
            for (int j = 0; j < NPRO; ++j)
                s_tk[j] = (fk + j * gx) * nx + xc;
            fk += NPRO * gx;
        } else {
            const uint32_t base = atomicAdd(my_ctr, (uint32_t)NPRO);
#pragma unroll
            for (int j = 0; j < NPRO; ++j)
                s_tk[j] = (base + j) * nx + xc;
        }
    }
    __syncthreads();
    // q[j]: the tiles in the ring (current first); uniform
    uint32_t q[NBUF - 1];
#pragma unroll
    for (int j = 0; j < NBUF - 1; ++j)
        q[j] = __builtin_amdgcn_readfirstlane(s_tk[j]);
    uint32_t cur = 0, pc = 0;
    uint32_t hist = 0, iter = 0;
    if (worker) {
        if (q[0] < nfull)
            dma_tile<IN_PIECES>(lds + D::OFF_BUF + PAD, data + (uint64_t)q[0] * (TB * K), tid, data, nblocks * K);
#pragma unroll
        for (int j = 1; j <= NBUF - 2; ++j) {
            const bool go = q[j] < nfull;
            if (go)
                dma_tile<IN_PIECES>(lds + D::OFF_BUF + j * BUF + PAD, data + (uint64_t)q[j] * (TB * K), tid, data, nblocks * K);
            hist = (hist << 1) | (go ? 1u : 0u);
        }
        vm_wait_newer(4u * __builtin_popcount(hist));
    }
    uint32_t pend = 0; // ticket wave, lane 0: the atomic of the previous iteration
    while (q[0] < nfull) {
        barrier_lds(); // A
        const uint32_t ahead = __builtin_amdgcn_readfirstlane(iter < 2 ? s_tk[NBUF - 1 + iter] : s_tk[NPRO + (iter & 1u)]);
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        const uint64_t t = q[0];
        const bool go = ahead < nfull;
        if (worker) {
            if (go)
                dma_tile<IN_PIECES>(lds + D::OFF_BUF + ring_add(cur, NBUF - 1, NBUF) * BUF + PAD, data + (uint64_t)ahead * (TB * K),
                    tid, data, nblocks * K);
            if (wave == 0)
                *(uint64_t*)(lds + D::OFF_PAR + (pc ^ 1u) * 512u + 8u * lane) = 0;
            if constexpr (MODE & 1)
                phase_remainder<T2, K, D::NMAP>(lds, buf, par, wave, row);
        } else if (lane == 0) {
            // publish last iteration's ticket (for iteration iter + 1), take the one for iter + 2
            if (iter >= 1)
                s_tk[NPRO + ((iter + 1u) & 1u)] = pend * nx + xc;
            if constexpr (FAKE) {
                pend = fk;
                fk += gx;
            } else {
                pend = atomicAdd(my_ctr, 1u);
            }
        }
        hist = (hist << 1) | (go ? 1u : 0u);
        barrier_lds(); // B
        if (worker) {
            uint8_t* dst = raw + t * (TB * 255);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t p = tid + 256u * k;
                uint4 o;
                if constexpr (MODE & 2)
                    o = enc_piece<T2>(lds, buf, par, p);
                else
                    o = *(const uint4*)(lds + buf + PAD + 16u * (p < 996u ? p : p - 64u));
                if ((k < 3 || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, raw, nblocks * 255u))
                    st_nt<NTST>(dst + 16u * p, o);
            }
            ++iter;
            const uint32_t st = 4u * (iter < (uint32_t)(NBUF - 1) ? iter : (uint32_t)(NBUF - 1));
            vm_wait_newer(st + 4u * __builtin_popcount(hist & ((1u << (NBUF - 2)) - 1u)));
        } else {
            ++iter;
        }
#pragma unroll
        for (int j = 0; j < NBUF - 2; ++j)
            q[j] = q[j + 1];
        q[NBUF - 2] = ahead;
        cur = ring_add(cur, 1, NBUF);
        pc ^= 1u;
    }
    if (q[0] == nfull && nfull < ntiles) { // the partial tile
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        const uint64_t t = nfull;
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        if (worker && PPFS_DBG_OK(data + t * (TB * K), nb * K, data, nblocks * K))
            stage_bytes(lds + buf + PAD, data + t * (TB * K), nb * K, tid);
        barrier_lds();
        if (worker)
            phase_remainder<T2, K, D::NMAP>(lds, buf, par, wave, row);
        barrier_lds();
        if (worker) {
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
    }
    if (!worker && lane == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // this workgroup's last ticket has returned
        if (atomicAdd(ctr + 32u * 8u, 1u) == gridDim.x - 1) { // every workgroup has taken its last ticket
            for (uint32_t x = 0; x < nx; ++x)
                __hip_atomic_store(ctr + 32u * x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ctr + 32u * 8u, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ------------------------------------------------------------------------------------
// 8-wave encode (PPFS_WG_ENC_W8): a 512-thread workgroup per tile, wave s computing the remainder of
// 32-byte segment s of every row (4 slicing steps instead of 8) and moving it with the MAP32 table
// of x^(32 s); 2 DMA and 2 emission pieces per thread.  Same ring of LDS tile buffers and counted
// waits as rs_wg_encode_kernel; twice the waves per CU for the same bytes in flight.
// ------------------------------------------------------------------------------------
template <int T2, int LEN, int S>
__device__ __forceinline__ void seg8_one(uint32_t (&s)[2], const uint8_t* lds, uint32_t row, uint32_t wave)
{
    if constexpr (S < 8) {
        if (wave == (uint32_t)S) {
            seg_remainder<T2, LEN, S, 32>(s, lds, row);
            if constexpr (S > 0)
                seg_map<T2, S>(s, lds); // LDS holds MAP32 at OFF_MAP: map S-1 = x^(q + 32 S)
        } else {
            seg8_one<T2, LEN, S + 1>(s, lds, row, wave);
        }
    }
}

template <int T2, int LEN>
__device__ __forceinline__ void phase_remainder8(uint8_t* lds, uint32_t buf, uint32_t par, uint32_t wave, uint32_t blk)
{
    uint32_t s[2];
    seg8_one<T2, LEN, 0>(s, lds, buf + PAD + (uint32_t)LEN * blk, wave);
    const uint64_t v = ((uint64_t)s[1] << 32) | s[0];
    __hip_atomic_fetch_xor((unsigned long long*)(lds + par + 8u * blk), (unsigned long long)v, __ATOMIC_RELAXED,
        __HIP_MEMORY_SCOPE_WORKGROUP);
}

// LDS-DMA of NPIECE 16-byte pieces by 512 threads: piece p = tid + 512 k, exactly 2 per wave
template <int NPIECE>
__device__ __forceinline__ void dma_tile512(uint8_t* dst, const uint8_t* __restrict__ src, uint32_t tid,
    [[maybe_unused]] const uint8_t* base, [[maybe_unused]] uint64_t extent)
{
    static_assert(NPIECE > 512 + 448 && NPIECE <= 1024, "2 pieces per thread, every wave active in each");
    const uint32_t lbase = __builtin_amdgcn_readfirstlane(lds_addr(dst) + (tid & ~63u) * 16u);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t p = tid + 512u * k;
        if ((k < 1 || p < (uint32_t)NPIECE) && PPFS_DBG_OK(src + (size_t)p * 16, 16, base, extent))
            dma16(src + (size_t)p * 16, lbase + 8192u * k);
    }
}

template <int T2> struct Lds8 {
    using L = RsWgLayout<T2>;
    static constexpr int TBL = L::OFF_MAP + 7 * L::MAP_STRIDE; // SL + MAP32 (copied to OFF_MAP)
    static constexpr int OFF_PAR = TBL;
    static constexpr int OFF_BUF = OFF_PAR + 1024 + 64;
    static_assert(OFF_BUF % 16 == 0 && TBL % 16 == 0, "aligned buffers");
};

template <int T2, int NBUF = 3, int WPC = 2, int NTST = 1>
__global__ __launch_bounds__(512, WPC) void rs_wg_encode8_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables)
{
    static_assert(NBUF >= 3 && NBUF <= 4, "ring of tile buffers");
    using L = RsWgLayout<T2>;
    using D = Lds8<T2>;
    constexpr int NT = 512;
    constexpr int BYTES = D::OFF_BUF + NBUF * BUF;
    constexpr int LDS_ALLOC = lds_alloc<BYTES, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * K / 16;   // 996 for 2t = 6
    constexpr int OUT_PIECES = TB * 255 / 16; // 1020
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t row = lane_row(lane);
    for (uint32_t p = tid; p < (uint32_t)L::OFF_MAP / 16; p += NT) // SL
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    for (uint32_t p = tid; p < 7u * L::MAP_STRIDE / 16; p += NT) // MAP32
        *(uint4*)(lds + L::OFF_MAP + 16 * p) = *(const uint4*)(tables + L::OFF_MAP32 + 16 * p);
    if (tid < 128)
        *(uint64_t*)(lds + D::OFF_PAR + 8 * tid) = 0;
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    uint64_t t = blockIdx.x;
    uint32_t cur = 0, pc = 0;
    if (t < nfull)
        dma_tile512<IN_PIECES>(lds + D::OFF_BUF + PAD, data + t * (TB * K), tid, data, nblocks * K);
    uint32_t hist = 0, iter = 0;
#pragma unroll
    for (int j = 1; j <= NBUF - 2; ++j) {
        const bool go = t + j * gridDim.x < nfull;
        if (go)
            dma_tile512<IN_PIECES>(lds + D::OFF_BUF + j * BUF + PAD, data + (t + j * gridDim.x) * (TB * K), tid, data,
                nblocks * K);
        hist = (hist << 1) | (go ? 1u : 0u);
    }
    vm_wait_newer(2u * __builtin_popcount(hist)); // tile t landed, the later ones may fly
    for (; t < nfull; t += gridDim.x) {
        barrier_lds(); // A: tile t in LDS, last tile's emission reads done
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        {
            const uint64_t ahead = t + (uint64_t)(NBUF - 1) * gridDim.x;
            const bool go = ahead < nfull;
            if (go)
                dma_tile512<IN_PIECES>(lds + D::OFF_BUF + ring_add(cur, NBUF - 1, NBUF) * BUF + PAD, data + ahead * (TB * K),
                    tid, data, nblocks * K);
            hist = (hist << 1) | (go ? 1u : 0u);
        }
        if (wave == 0)
            *(uint64_t*)(lds + D::OFF_PAR + (pc ^ 1u) * 512u + 8u * lane) = 0;
        phase_remainder8<T2, K>(lds, buf, par, wave, row);
        barrier_lds(); // B: parity slots complete
        uint8_t* dst = raw + t * (TB * 255);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t p = tid + 512u * k;
            const uint4 o = enc_piece<T2>(lds, buf, par, p);
            if ((k < 1 || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, raw, nblocks * 255u))
                st_nt<NTST>(dst + 16u * p, o);
        }
        // tile t + G landed: count every operation issued after its DMA (2 stores and 2 DMA
        // instructions per wave and tile; fewer newer operations only lower the count)
        ++iter;
        const uint32_t st = 2u * (iter < (uint32_t)(NBUF - 1) ? iter : (uint32_t)(NBUF - 1));
        vm_wait_newer(st + 2u * __builtin_popcount(hist & ((1u << (NBUF - 2)) - 1u)));
        cur = ring_add(cur, 1, NBUF);
        pc ^= 1u;
    }
    if (t == nfull && nfull < ntiles) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        if (PPFS_DBG_OK(data + t * (TB * K), nb * K, data, nblocks * K))
            for (uint32_t i = tid; i < nb * K; i += NT)
                lds[buf + PAD + i] = data[t * (TB * K) + i];
        barrier_lds();
        phase_remainder8<T2, K>(lds, buf, par, wave, row);
        barrier_lds();
        uint8_t* dst = raw + t * (TB * 255);
        const uint32_t nout = nb * 255u;
        for (uint32_t p = tid; 16u * p < nout; p += NT) {
            const uint4 v = enc_piece<T2>(lds, buf, par, p);
            if (!PPFS_DBG_OK(dst + 16u * p, min(16u, nout - 16u * p), raw, nblocks * 255u))
                continue;
            if (16u * p + 16u <= nout)
                *(uint4*)(dst + 16u * p) = v;
            else
                st_bytes(dst + 16u * p, v, nout - 16u * p);
        }
    }
}

} // namespace wg
} // namespace ppfs
