#pragma once
// ABLATION ONLY (not built into libppfs_ecc.so; tools/build_alt.sh with
// RS_INST=tools/ablations/rs_fast_inst_ablate.hip).  The nibble-table pair launch kernels for
// 16 < 2t <= 32, superseded for 2t = 32 by the byte-slice kernels of
// csrc/rs_bs.hpp; their shared pieces (pair_remainder, pair_correct, the server) stay in
// csrc/rs_pair.hpp.
#include "rs_pair.hpp"

namespace ppfs {
namespace pair {
template <int T2, int WPC = 3, int NBUF = 2, int NTST = 1>
__global__ __launch_bounds__(NTHR, 2) void rs_pair_encode_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables)
{
    using L = RsPairLayout<T2>;
    using D = Lds<T2, false, NBUF>;
    constexpr int LDS_ALLOC = wg::lds_alloc<D::BYTES, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * K / 16;
    constexpr int OUT_PIECES = TB * 255 / 16; // 1020
    constexpr int KOUT = (OUT_PIECES + NTHR - 1) / NTHR;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t c = lane_col(lane), blk = 32u * wave + lane_blk(lane);
    const uint32_t tb = L::OFF_SL + 256u * c; // offset in lds[]
    for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += NTHR)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    uint64_t t = blockIdx.x;
    uint32_t cur = 0;
    if (t < nfull)
        dma_tile128<IN_PIECES>(lds + D::OFF_BUF + PAD, data + t * (TB * K), tid, data, nblocks * K);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (; t < nfull; t += gridDim.x) {
        barrier_lds(); // A: tile t in LDS, the last tile's emission reads done
        const uint32_t buf = D::OFF_BUF + cur * BUF;
        const uint64_t nx = t + gridDim.x;
        if (NBUF == 2 && nx < nfull)
            dma_tile128<IN_PIECES>(lds + D::OFF_BUF + (cur ^ 1u) * BUF + PAD, data + nx * (TB * K), tid, data, nblocks * K);
        uint32_t s[4];
        pair_remainder<K>(s, lds, buf + PAD + (uint32_t)K * blk, tb, c);
        *(uint4*)(lds + D::OFF_PAR + 32u * blk + 16u * c) = make_uint4(s[0], s[1], s[2], s[3]);
        barrier_lds(); // B: parity slots complete
        uint8_t* dst = raw + t * (TB * 255);
        // opaque per iteration: keeps the pieces' loop-invariant index maths (b, off, masks) from
        // being hoisted out of the tile loop, where it held ~150 VGPRs and starved the lookups
        uint32_t tid_o = tid;
        asm volatile("" : "+v"(tid_o));
#pragma unroll
        for (int k = 0; k < KOUT; ++k) {
            const uint32_t p = tid_o + (uint32_t)NTHR * k;
            const uint4 o = col_enc_piece<T2>(lds, buf, D::OFF_PAR, p);
            if ((k + 1) * NTHR <= OUT_PIECES || p < (uint32_t)OUT_PIECES)
                st_nt<NTST>(dst + 16u * p, o);
        }
        if constexpr (NBUF == 1) {
            barrier_lds(); // every wave's emission reads done: the buffer is free
            if (nx < nfull)
                dma_tile128<IN_PIECES>(lds + D::OFF_BUF + PAD, data + nx * (TB * K), tid, data, nblocks * K);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // other workgroups overlap this wait
        } else {
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); // next tile's DMA landed; stores may fly
        }
        cur ^= (NBUF == 2) ? 1u : 0u;
    }
    if (t == nfull && nfull < ntiles) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint32_t buf = D::OFF_BUF + cur * BUF;
        stage_bytes128(lds + buf + PAD, data + t * (TB * K), nb * K, tid);
        barrier_lds();
        uint32_t s[4];
        pair_remainder<K>(s, lds, buf + PAD + (uint32_t)K * blk, tb, c);
        *(uint4*)(lds + D::OFF_PAR + 32u * blk + 16u * c) = make_uint4(s[0], s[1], s[2], s[3]);
        barrier_lds();
        uint8_t* dst = raw + t * (TB * 255);
        const uint32_t nout = nb * 255u;
        for (uint32_t p = tid; 16u * p < nout; p += NTHR) {
            const uint4 v = col_enc_piece<T2>(lds, buf, D::OFF_PAR, p);
            if (16u * p + 16u <= nout)
                *(uint4*)(dst + 16u * p) = v;
            else
                st_bytes(dst + 16u * p, v, nout - 16u * p);
        }
    }
}

// NW waves per workgroup (32 blocks each), tiles of TBK = 32 NW blocks; the tables are shared by
// the NW waves, so larger workgroups fit more waves per CU (NW = 4: 4 x 40.9 KB, 16 waves).
template <int T2, int WPC = 6, int NW = 2, int NTST = 1>
__global__ __launch_bounds__(64 * NW, 2) void rs_pair_encode_img_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables)
{
    static_assert(T2 % 16 == 0, "aligned image pieces need 16 | 2t");
    using L = RsPairLayout<T2>;
    constexpr int TBL = L::ENC_BYTES;
    constexpr int IMG = TBL;
    constexpr int TBK = 32 * NW, NT = 64 * NW;
    constexpr int BYTES = IMG + img_bytes<TBK>();
    constexpr int LDS_ALLOC = wg::lds_alloc<BYTES, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    static_assert(IMG % 16 == 0, "aligned image");
    constexpr int K = L::K;
    constexpr int PIECES = TBK * 255 / 16; // in and out (1020 at 64 blocks)
    constexpr int KP = (PIECES + NT - 1) / NT;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t c = lane_col(lane), blk = spread_blk<2 * NW>(wave, lane);
    const uint32_t tb = L::OFF_SL + 256u * c;
    for (uint32_t p = tid; p < (uint32_t)TBL / 16; p += NT)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    const uint32_t img_base = __builtin_amdgcn_readfirstlane(lds_addr(lds + IMG) + (tid & ~63u) * 16u);
    auto dma_img = [&](const uint8_t* __restrict__ src) {
#pragma unroll
        for (int k = 0; k < KP; ++k) {
            const uint32_t i = tid + (uint32_t)NT * k;
            const int so = img_src<T2>(i);
            if (((k + 1) * NT <= PIECES || i < (uint32_t)PIECES) && so >= 0 && PPFS_DBG_OK(src + so, 16, data, nblocks * K))
                dma16(src + so, img_base + 16u * NT * k);
        }
    };
    const uint64_t nfull = nblocks / TBK, ntiles = (nblocks + TBK - 1) / TBK;
    uint64_t t = blockIdx.x;
    if (t < nfull)
        dma_img(data + t * (TBK * K));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t row = IMG + 255u * blk + (uint32_t)T2;
    uint8_t* const gap = lds + IMG + 255u * blk + 16u * c; // this lane's 16 parity bytes
    for (; t < nfull; t += gridDim.x) {
        barrier_lds(); // A: tile t in the image, the last tile's emission reads done
        uint32_t s[4];
        pair_remainder<K>(s, lds, row, tb, c);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            gap[k] = (uint8_t)(s[k >> 2] >> (8 * (k & 3)));
        barrier_lds(); // B: parity in the image
        uint8_t* dst = raw + t * (TBK * 255);
#pragma unroll
        for (int k = 0; k < KP; ++k) {
            const uint32_t i = tid + (uint32_t)NT * k;
            if (((k + 1) * NT <= PIECES || i < (uint32_t)PIECES) && PPFS_DBG_OK(dst + 16u * i, 16, raw, nblocks * 255u))
                st_nt<NTST>(dst + 16u * i, ld16(lds, IMG + 16u * i));
        }
        barrier_lds(); // C: the image is free
        const uint64_t nx = t + gridDim.x;
        if (nx < nfull)
            dma_img(data + nx * (TBK * K));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // other workgroups overlap this wait
    }
    if (t == nfull && nfull < ntiles) {
        // the one partial tile (nblocks % TBK blocks), staged byte by byte into the image
        barrier_lds();
        const uint32_t nb = (uint32_t)(nblocks - t * TBK);
        const uint8_t* src = data + t * (TBK * K);
        if (!PPFS_DBG_OK(src, nb * (uint32_t)K, data, nblocks * K))
            return;
        for (uint32_t j = tid; j < nb * (uint32_t)K; j += NT) {
            const uint32_t b = j / (uint32_t)K;
            lds[row - 255u * blk + 255u * b + (j - (uint32_t)K * b)] = src[j];
        }
        barrier_lds();
        uint32_t s[4];
        pair_remainder<K>(s, lds, row, tb, c);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            gap[k] = (uint8_t)(s[k >> 2] >> (8 * (k & 3)));
        barrier_lds();
        uint8_t* dst = raw + t * (TBK * 255);
        const uint32_t nout = nb * 255u;
        for (uint32_t i = tid; 16u * i < nout; i += NT) {
            const uint4 v = ld16(lds, IMG + 16u * i);
            if (!PPFS_DBG_OK(dst + 16u * i, min(16u, nout - 16u * i), raw, nblocks * 255u))
                continue;
            if (16u * i + 16u <= nout)
                *(uint4*)(dst + 16u * i) = v;
            else
                st_bytes(dst + 16u * i, v, nout - 16u * i);
        }
    }
}

template <int T2, int WPC = 3, int NBUF = 2, int NTST = 1, bool RM = (T2 == 32)>
__global__ __launch_bounds__(NTHR, (WPC >= 5 ? 3 : 2)) void rs_pair_decode_kernel(uint8_t* __restrict__ raw,
    uint8_t* __restrict__ data, uint8_t* __restrict__ status, uint64_t nblocks, const uint8_t* __restrict__ tables,
    int write_back)
{
    using L = RsPairLayout<T2>;
    using D = Lds<T2, true, NBUF>;
    constexpr int LDS_ALLOC = wg::lds_alloc<D::BYTES, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * 255 / 16; // 1020
    constexpr int OUT_PIECES = TB * K / 16;
    constexpr int KOUT = (OUT_PIECES + NTHR - 1) / NTHR;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t c = lane_col(lane), blk = spread_blk<NTHR / 32>(wave, lane);
    const uint32_t tb = L::OFF_SL + 256u * c; // offset in lds[]
    const bool wb = write_back != 0, want = data != nullptr;
    const uint32_t slot = D::OFF_PAR + 32u * blk;
    for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += NTHR)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    uint64_t t = blockIdx.x;
    uint32_t cur = 0;
    if (t < nfull)
        dma_tile128<IN_PIECES>(lds + D::OFF_BUF + PAD, raw + t * (TB * 255), tid, raw, nblocks * 255u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (; t < nfull; t += gridDim.x) {
        barrier_lds(); // A
        const uint32_t buf = D::OFF_BUF + cur * BUF;
        const uint64_t nx = t + gridDim.x;
        if (NBUF == 2 && nx < nfull)
            dma_tile128<IN_PIECES>(lds + D::OFF_BUF + (cur ^ 1u) * BUF + PAD, raw + nx * (TB * 255), tid, raw, nblocks * 255u);
        const uint32_t row = buf + PAD + 255u * blk;
        uint32_t s[4];
        if constexpr (RM)
            pair_cmodg<T2>(s, lds, row, tb, c);
        else
            pair_remainder<255>(s, lds, row, tb, c);
        *(uint4*)(lds + slot + 16u * c) = make_uint4(s[0], s[1], s[2], s[3]); // read by the general path
        wave_fence();
        const uint32_t st = pair_correct<T2, RM>(
            lds, L::OFF_GF, tables + (RM ? L::OFF_XPM : L::OFF_XP), row, slot, c, s, true, raw, t * TB + blk, wb, nblocks * 255u);
        if (status && c == 0 && PPFS_DBG_OK(status + t * TB + blk, 1, status, nblocks))
            status[t * TB + blk] = (uint8_t)st;
        barrier_lds(); // C: corrections patched into the LDS rows
        uint8_t* dst = want ? data + t * (TB * K) : nullptr;
        uint32_t tid_o = tid; // see the encode kernel
        asm volatile("" : "+v"(tid_o));
        if (want) {
#pragma unroll
            for (int k = 0; k < KOUT; ++k) {
                const uint32_t p = tid_o + (uint32_t)NTHR * k;
                const uint4 o = dec_piece<T2>(lds, buf, p);
                if (((k + 1) * NTHR <= OUT_PIECES || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, data, nblocks * K))
                    st_nt<NTST>(dst + 16u * p, o);
            }
        }
        if constexpr (NBUF == 1) {
            barrier_lds(); // emission reads done: the buffer is free
            if (nx < nfull)
                dma_tile128<IN_PIECES>(lds + D::OFF_BUF + PAD, raw + nx * (TB * 255), tid, raw, nblocks * 255u);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // other workgroups overlap this wait
        } else if (want) {
            asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        cur ^= (NBUF == 2) ? 1u : 0u;
    }
    if (t == nfull && nfull < ntiles) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint32_t buf = D::OFF_BUF + cur * BUF;
        if (PPFS_DBG_OK(raw + t * (TB * 255), nb * 255u, raw, nblocks * 255u))
            stage_bytes128(lds + buf + PAD, raw + t * (TB * 255), nb * 255u, tid);
        barrier_lds();
        const uint32_t row = buf + PAD + 255u * blk;
        uint32_t s[4];
        if constexpr (RM)
            pair_cmodg<T2>(s, lds, row, tb, c);
        else
            pair_remainder<255>(s, lds, row, tb, c);
        *(uint4*)(lds + slot + 16u * c) = make_uint4(s[0], s[1], s[2], s[3]);
        wave_fence();
        const bool valid = blk < nb;
        const uint32_t st = pair_correct<T2, RM>(
            lds, L::OFF_GF, tables + (RM ? L::OFF_XPM : L::OFF_XP), row, slot, c, s, valid, raw, t * TB + blk, wb, nblocks * 255u);
        if (status && valid && c == 0 && PPFS_DBG_OK(status + t * TB + blk, 1, status, nblocks))
            status[t * TB + blk] = (uint8_t)st;
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
}

} // namespace pair
} // namespace ppfs
