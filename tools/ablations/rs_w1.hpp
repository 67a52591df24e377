#pragma once
// rs_w1.hpp -- wave-independent RS(255, 255-2t) encode / decode for gfx950, 2t <= 8 (the headline
// RS(255,249), t = 3).
//
// Reference semantics: lib/blockdevice/src/rs_block_device.cpp (encode :95-117, decode :119-183),
// the maths of rs_wg.hpp: slicing-by-8 over the nibble tables of RsWgLayout (top-aligned 8-byte
// state), r' = x^2t c(x) mod g for decode, the syndromes / single-error closed form / BM / roots /
// Forney of phase_correct, and the emission helpers enc_piece / dec_piece.
//
// Work decomposition.  rs_wg.hpp splits a 64-block tile over the four waves of a workgroup (one
// 64-byte segment of every row per wave, x^(64 s) maps, three workgroup barriers per tile); its
// memory pipeline is then coupled across the workgroup (the persistent skeleton
// alone costs 96 us against an 88 us copy).  Here one workgroup of NW waves per CU shares only
// the tables (encode: the 2 KiB slicing tables), and every wave works ALONE on its own 64-block
// tiles: lane = block, the whole row in one slicing chain (32 steps), no segment maps, no barrier
// in the tile loop.  Tiles come in by LDS-DMA (NBUF = 1: the next tile's DMA is issued once the
// emission has read the buffer; other waves cover the wait) or by register prefetch (NBUF = 0:
// plain loads of the next tile during this tile's compute, written to LDS after the emission).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rs_wg.hpp"

namespace ppfs {
namespace w1 {

using wg::dma16;
using wg::lds_addr;
using wg::st_bytes;
using wg::st_nt;

constexpr int TB = 64; // blocks per wave tile (lane = block)

// per-wave LDS: tile buffer (PAD + 64 rows + 32 B over-read slack) | 64 x 8 B parity / remainder
// slots (+ 64 B: enc_piece reads the slot of block b + 1)
template <int T2, bool DEC> struct W1Wave {
    static constexpr int K = 255 - T2;
    static constexpr int ROWB = DEC ? 255 : K;
    static constexpr int BUFB = (wg::PAD + TB * ROWB + 32 + 15) / 16 * 16;
    static constexpr int OFF_PAR = BUFB;
    static constexpr int BYTES = BUFB + TB * 8 + 64;
    static constexpr int IN_PIECES = TB * ROWB / 16; // 996 (encode, 2t = 6) / 1020 (decode)
    static constexpr int KIN = (IN_PIECES + 63) / 64;
};

template <int T2, int NW, bool DEC> struct W1Lds {
    using L = RsWgLayout<T2>;
    using W = W1Wave<T2, DEC>;
    static constexpr int TBL = DEC ? L::TABLE_BYTES : L::OFF_MAP; // encode: the slicing tables only
    static constexpr int OFF_W = (TBL + 15) / 16 * 16;
    static constexpr int BYTES = OFF_W + NW * W::BYTES;
    static_assert(BYTES <= 163840, "one workgroup per CU: 160 KiB of LDS");
    static_assert(W::BYTES % 16 == 0, "aligned wave areas");
};

// LDS-DMA of one wave tile: piece i = lane + 64 k (16 B) lands at buf + PAD + 16 i
template <int NPIECE>
__device__ __forceinline__ void dma_rows(uint32_t base, const uint8_t* __restrict__ src, uint32_t lane,
    [[maybe_unused]] const uint8_t* gbase, [[maybe_unused]] uint64_t extent)
{
    constexpr int KI = (NPIECE + 63) / 64;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
        const uint32_t i = lane + 64u * (uint32_t)k;
        if (((k + 1) * 64 <= NPIECE || i < (uint32_t)NPIECE) && PPFS_DBG_OK(src + 16u * i, 16, gbase, extent))
            dma16(src + 16u * i, __builtin_amdgcn_readfirstlane(base + 1024u * (uint32_t)k));
    }
}

// register prefetch of one wave tile (NBUF = 0): every lane loads (the last instruction's idle
// lanes re-read the tile's last piece) so that pf stays in registers
template <int NPIECE>
__device__ __forceinline__ void load_rows(u32x4 (&pf)[(NPIECE + 63) / 64], const uint8_t* __restrict__ src, uint32_t lane,
    [[maybe_unused]] const uint8_t* gbase, [[maybe_unused]] uint64_t extent)
{
    constexpr int KI = (NPIECE + 63) / 64;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
        uint32_t i = lane + 64u * (uint32_t)k;
        i = i < (uint32_t)NPIECE ? i : (uint32_t)NPIECE - 1u;
        if (PPFS_DBG_OK(src + 16u * i, 16, gbase, extent))
            pf[k] = *(const u32x4*)(src + 16u * i);
    }
}

template <int NPIECE>
__device__ __forceinline__ void put_rows(uint8_t* lds, uint32_t buf, const u32x4 (&pf)[(NPIECE + 63) / 64], uint32_t lane)
{
    constexpr int KI = (NPIECE + 63) / 64;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
        const uint32_t i = lane + 64u * (uint32_t)k;
        if ((k + 1) * 64 <= NPIECE || i < (uint32_t)NPIECE)
            *(u32x4*)(lds + buf + wg::PAD + 16u * i) = pf[k];
    }
}

// the whole-row slicing chain of the lane's block: s = sum_j row[j] x^(2t + j) mod g
template <int T2, int LEN>
__device__ __forceinline__ void row_remainder(uint32_t (&s)[2], const uint8_t* lds, uint32_t row)
{
    wg::seg_remainder<T2, LEN, 0, 256>(s, lds, row);
}

// MODE (ablation builds only; the engine uses 3): bit 0 = remainder chain, bit 1 = codeword
// emission (else a plain copy out of the tile buffer, same bytes moved)
template <int T2, int NW, int NBUF = 1, int MODE = 3, int NTST = 1>
__global__ __launch_bounds__(64 * NW, 1) void rs_w1_encode_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables)
{
    static_assert(NBUF == 0 || NBUF == 1, "NBUF");
    using D = W1Lds<T2, NW, false>;
    using W = W1Wave<T2, false>;
    constexpr int K = W::K;
    constexpr int OUT_PIECES = TB * 255 / 16; // 1020
    constexpr int KO = (OUT_PIECES + 63) / 64;
    __shared__ __attribute__((aligned(16))) uint8_t lds[D::BYTES];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += 64u * NW)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    __syncthreads();
    const uint32_t r = wg::lane_row(lane);
    const uint32_t buf = D::OFF_W + wave * (uint32_t)W::BYTES, par = buf + W::OFF_PAR;
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(lds + buf + wg::PAD));
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    const uint64_t S = (uint64_t)gridDim.x * NW;
    uint64_t t = (uint64_t)blockIdx.x * NW + wave;
    [[maybe_unused]] u32x4 pf[W::KIN];
    if (t < nfull) {
        if constexpr (NBUF == 0) {
            load_rows<W::IN_PIECES>(pf, data + t * (TB * K), lane, data, nblocks * K);
            put_rows<W::IN_PIECES>(lds, buf, pf, lane);
        } else {
            dma_rows<W::IN_PIECES>(base, data + t * (TB * K), lane, data, nblocks * K);
        }
    }
    for (; t < nfull; t += S) {
        const uint64_t nx = t + S;
        if constexpr (NBUF == 0) {
            if (nx < nfull)
                load_rows<W::IN_PIECES>(pf, data + nx * (TB * K), lane, data, nblocks * K);
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if constexpr (MODE & 1) {
            uint32_t s[2];
            row_remainder<T2, K>(s, lds, buf + wg::PAD + (uint32_t)K * r);
            *(uint2*)(lds + par + 8u * r) = make_uint2(s[0], s[1]);
        }
        wave_fence(); // every lane's parity slot written
        uint8_t* dst = raw + t * (TB * 255);
#pragma unroll
        for (int k = 0; k < KO; ++k) {
            uint32_t p = lane + 64u * (uint32_t)k;
            asm volatile("" : "+v"(p)); // this piece's index maths starts after the last store
            uint4 o;
            if constexpr (MODE & 2)
                o = wg::enc_piece<T2>(lds, buf, par, p);
            else
                o = *(const uint4*)(lds + buf + wg::PAD + 16u * (p < (uint32_t)W::IN_PIECES ? p : p - 64u));
            if (((k + 1) * 64 <= OUT_PIECES || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, raw, nblocks * 255u))
                st_nt<NTST>(dst + 16u * p, o);
            asm volatile("" ::: "memory"); // one piece live at a time
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the tile buffer is read
        if (nx < nfull) {
            if constexpr (NBUF == 0)
                put_rows<W::IN_PIECES>(lds, buf, pf, lane);
            else
                dma_rows<W::IN_PIECES>(base, data + nx * (TB * K), lane, data, nblocks * K);
        }
    }
    if (t == nfull && nfull < ntiles) {
        // the one partial tile (nblocks % 64 blocks), staged byte by byte
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint8_t* src = data + t * (TB * K);
        if (!PPFS_DBG_OK(src, nb * (uint32_t)K, data, nblocks * K))
            return;
        for (uint32_t j = lane; j < nb * (uint32_t)K; j += 64u)
            lds[buf + wg::PAD + j] = src[j];
        wave_fence();
        uint32_t s[2];
        row_remainder<T2, K>(s, lds, buf + wg::PAD + (uint32_t)K * r);
        *(uint2*)(lds + par + 8u * r) = make_uint2(s[0], s[1]);
        wave_fence();
        uint8_t* dst = raw + t * (TB * 255);
        const uint32_t nout = nb * 255u;
        for (uint32_t p = lane; 16u * p < nout; p += 64u) {
            const uint4 v = wg::enc_piece<T2>(lds, buf, par, p);
            if (!PPFS_DBG_OK(dst + 16u * p, min(16u, nout - 16u * p), raw, nblocks * 255u))
                continue;
            if (16u * p + 16u <= nout)
                *(uint4*)(dst + 16u * p) = v;
            else
                st_bytes(dst + 16u * p, v, nout - 16u * p);
        }
    }
}

// Decode with status and write-back: r' per lane over the whole codeword, phase_correct (its
// syndrome / correction tables and GF block in LDS), payload emission from the corrected rows.
template <int T2, int NW, int NBUF = 1, int NTST = 1>
__global__ __launch_bounds__(64 * NW, 1) void rs_w1_decode_kernel(uint8_t* __restrict__ raw,
    uint8_t* __restrict__ data, uint8_t* __restrict__ status, uint64_t nblocks, const uint8_t* __restrict__ tables,
    int write_back)
{
    static_assert(NBUF == 0 || NBUF == 1, "NBUF");
    using D = W1Lds<T2, NW, true>;
    using W = W1Wave<T2, true>;
    constexpr int K = W::K;
    constexpr int OUT_PIECES = TB * K / 16; // 996 for 2t = 6
    constexpr int KO = (OUT_PIECES + 63) / 64;
    __shared__ __attribute__((aligned(16))) uint8_t lds[D::BYTES];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += 64u * NW)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    __syncthreads();
    const uint32_t r = wg::lane_row(lane);
    const uint32_t buf = D::OFF_W + wave * (uint32_t)W::BYTES, par = buf + W::OFF_PAR;
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(lds + buf + wg::PAD));
    const bool wb = write_back != 0, want = data != nullptr;
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    const uint64_t S = (uint64_t)gridDim.x * NW;
    uint64_t t = (uint64_t)blockIdx.x * NW + wave;
    [[maybe_unused]] u32x4 pf[W::KIN];
    if (t < nfull) {
        if constexpr (NBUF == 0) {
            load_rows<W::IN_PIECES>(pf, raw + t * (TB * 255), lane, raw, nblocks * 255u);
            put_rows<W::IN_PIECES>(lds, buf, pf, lane);
        } else {
            dma_rows<W::IN_PIECES>(base, raw + t * (TB * 255), lane, raw, nblocks * 255u);
        }
    }
    for (; t < nfull; t += S) {
        const uint64_t nx = t + S;
        if constexpr (NBUF == 0) {
            if (nx < nfull)
                load_rows<W::IN_PIECES>(pf, raw + nx * (TB * 255), lane, raw, nblocks * 255u);
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        uint32_t s[2];
        row_remainder<T2, 255>(s, lds, buf + wg::PAD + 255u * r);
        *(uint2*)(lds + par + 8u * r) = make_uint2(s[0], s[1]);
        wave_fence();
        const uint32_t st = wg::phase_correct<T2>(lds, buf, par, r, true, raw, t * TB + r, wb, nblocks * 255u);
        if (status && PPFS_DBG_OK(status + t * TB + r, 1, status, nblocks))
            status[t * TB + r] = (uint8_t)st;
        wave_fence(); // corrections patched into the rows
        if (want) {
            uint8_t* dst = data + t * (TB * K);
#pragma unroll
            for (int k = 0; k < KO; ++k) {
                uint32_t p = lane + 64u * (uint32_t)k;
                asm volatile("" : "+v"(p));
                if (((k + 1) * 64 <= OUT_PIECES || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, data, nblocks * K))
                    st_nt<NTST>(dst + 16u * p, wg::dec_piece<T2>(lds, buf, p));
                asm volatile("" ::: "memory");
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (nx < nfull) {
            if constexpr (NBUF == 0)
                put_rows<W::IN_PIECES>(lds, buf, pf, lane);
            else
                dma_rows<W::IN_PIECES>(base, raw + nx * (TB * 255), lane, raw, nblocks * 255u);
        }
    }
    if (t == nfull && nfull < ntiles) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint8_t* src = raw + t * (TB * 255);
        if (!PPFS_DBG_OK(src, nb * 255u, raw, nblocks * 255u))
            return;
        for (uint32_t j = lane; j < nb * 255u; j += 64u)
            lds[buf + wg::PAD + j] = src[j];
        wave_fence();
        uint32_t s[2];
        row_remainder<T2, 255>(s, lds, buf + wg::PAD + 255u * r);
        *(uint2*)(lds + par + 8u * r) = make_uint2(s[0], s[1]);
        wave_fence();
        const bool valid = r < nb;
        const uint32_t st = wg::phase_correct<T2>(lds, buf, par, r, valid, raw, t * TB + r, wb, nblocks * 255u);
        if (status && valid && PPFS_DBG_OK(status + t * TB + r, 1, status, nblocks))
            status[t * TB + r] = (uint8_t)st;
        wave_fence();
        if (want) {
            uint8_t* dst = data + t * (TB * K);
            const uint32_t nout = nb * (uint32_t)K;
            for (uint32_t p = lane; 16u * p < nout; p += 64u) {
                const uint4 v = wg::dec_piece<T2>(lds, buf, p);
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

} // namespace w1
} // namespace ppfs
