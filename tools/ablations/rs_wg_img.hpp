#pragma once
// ABLATION ONLY (not built into libppfs_ecc.so; tools/build_alt.sh, -DPPFS_WG_ENC_IMG=1): the
// full-grid image encode of DESIGN.md 4.1 (a third fewer VALU instructions, slower from HBM).
#include "rs_wg.hpp"

namespace ppfs {
namespace wg {

// ------------------------------------------------------------------------------------
// Encode into a codeword image (full grid: one 64-block tile per workgroup).
// The tile is DMA'd straight into the OUTPUT layout: codeword j of the tile at LDS IMG + 255 j,
// payload at IMG + 255 j + 2t.  Output piece i (16 bytes at image offset 16 i) takes its payload
// bytes from tile payload offset 16 i - 2t (b + 1), b = the block of the piece's last byte; the
// LDS-DMA reads that source at any byte alignment (checked on gfx950: tools/probes/dma_align_test.hip).
// Two kinds of pieces cannot be one contiguous source and are assembled in registers instead:
// piece 0 (block 0's parity, then its payload from offset 0) and the pieces in which block b's
// 2t parity bytes sit between the tail of block b-1's payload and the head of block b's.  After the
// remainder the parity bytes go into the image gaps, and the emission is a plain aligned 16-byte
// copy of the image: no windows, masks or parity merges per piece (those were a third of the
// VALU instructions of rs_wg_encode_kernel's tile loop).
// ------------------------------------------------------------------------------------
// 16 bytes v shifted up by N bytes within the piece (bytes [0, N) zero)
template <int N> __device__ __forceinline__ uint4 shift_up(uint4 v)
{
    static_assert(N % 2 == 0 && N > 0 && N < 16, "even byte shift");
    const uint32_t w[4] = { v.x, v.y, v.z, v.w };
    uint32_t o[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int q = m - N / 4; // source dword of o[m]'s top bytes
        const uint32_t hi = q >= 0 ? w[q >= 0 ? q : 0] : 0u;
        const uint32_t lo = q - 1 >= 0 ? w[q - 1 >= 0 ? q - 1 : 0] : 0u;
        o[m] = (N % 4) ? __builtin_amdgcn_alignbit(hi, lo, 32 - 8 * (N % 4)) : hi;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

template <int T2, int WPC = 6, int NTST = 1>
__global__ __launch_bounds__(256, WPC) void rs_wg_encode_img_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables)
{
    using L = RsWgLayout<T2>;
    constexpr int K = L::K;
    constexpr int TBL = L::OFF_SYN;             // SL + MAP
    constexpr int OFF_PAR = TBL;                // 64 x 8 B remainder slots
    constexpr int IMG = OFF_PAR + 512 + 64;     // + slack: row reads run up to 8 bytes past a row
    constexpr int BYTES = IMG + TB * 255 + 80;  // the last row's word reads run past the image
    constexpr int LDS_ALLOC = lds_alloc<BYTES, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840 && IMG % 16 == 0, "LDS for WPC workgroups per CU");
    constexpr int PIECES = TB * 255 / 16; // 1020, in and out
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t row = lane_row(lane);
    for (uint32_t p = tid; p < (uint32_t)TBL / 16; p += NTHR)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    if (tid < 64)
        *(uint64_t*)(lds + OFF_PAR + 8 * tid) = 0;
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    const uint64_t t = blockIdx.x;
    if (t >= ntiles)
        return;
    const uint8_t* __restrict__ src = data + t * (TB * K);
    uint8_t* dst = raw + t * (TB * 255);
    if (t < nfull) {
        const uint32_t img_base = __builtin_amdgcn_readfirstlane(lds_addr(lds + IMG) + (tid & ~63u) * 16u);
        uint4 fix[4];
        uint32_t fix_mask = 0; // bit k: piece tid + 256 k is assembled in registers
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = tid + 256u * k;
            const uint32_t e = 16u * i + 15u, b = e / 255u, off = e - 255u * b;
            const uint32_t s0 = 255u * b; // block b's first codeword byte
            // block b's parity sits between block b-1's payload tail and block b's payload head
            const bool straddle = off >= (uint32_t)T2 && 16u * i < s0;
            if (i >= (uint32_t)PIECES)
                continue;
            if (i == 0 || straddle) {
                fix_mask |= 1u << k;
                if (i == 0) {
                    fix[k] = shift_up<T2>(*(const uint4*)src); // [2t parity gap][payload 0 .. 16-2t)
                } else {
                    // bytes [0, s0 - 16 i) from block b-1, the rest from block b (gap overwritten later)
                    const uint4 A = *(const uint4*)(src + 16u * i - (uint32_t)T2 * b);
                    const uint4 B = *(const uint4*)(src + 16u * i - (uint32_t)T2 * (b + 1u));
                    const M128 m = range_mask(0, s0 - 16u * i);
                    fix[k] = make_uint4(bfi((uint32_t)m.lo, A.x, B.x), bfi((uint32_t)(m.lo >> 32), A.y, B.y),
                        bfi((uint32_t)m.hi, A.z, B.z), bfi((uint32_t)(m.hi >> 32), A.w, B.w));
                }
            } else {
                // the piece's bytes are payload of block b (and block b's parity gap, if it ends there)
                const uint32_t so = off >= (uint32_t)T2 ? 16u * i - (uint32_t)T2 * (b + 1u) : 16u * i - (uint32_t)T2 * b;
                dma16(src + so, img_base + 4096u * (uint32_t)k);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (fix_mask & (1u << k))
                *(uint4*)(lds + IMG + 16u * (tid + 256u * (uint32_t)k)) = fix[k];
        barrier_lds(); // A: the image holds every payload
        phase_remainder_row<T2, K>(lds, IMG + 255u * row + (uint32_t)T2, OFF_PAR, wave, row);
        barrier_lds(); // B: parity slots complete
        if (wave == 0) {
            const uint64_t pv = *(const uint64_t*)(lds + OFF_PAR + 8u * lane);
#pragma unroll
            for (int q = 0; q < T2; ++q)
                lds[IMG + 255u * lane + (uint32_t)q] = (uint8_t)(pv >> (8 * (8 - T2 + q)));
        }
        barrier_lds(); // C: the image is the codeword tile
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = tid + 256u * k;
            if (k < 3 || i < (uint32_t)PIECES)
                st_nt<NTST>(dst + 16u * i, *(const uint4*)(lds + IMG + 16u * i));
        }
        return;
    }
    // the one partial tile (nblocks % 64 blocks), staged byte by byte into the image
    const uint32_t nb = (uint32_t)(nblocks - t * TB);
    for (uint32_t j = tid; j < nb * (uint32_t)K; j += NTHR) {
        const uint32_t b = j / (uint32_t)K;
        lds[IMG + 255u * b + (uint32_t)T2 + (j - (uint32_t)K * b)] = src[j];
    }
    barrier_lds();
    phase_remainder_row<T2, K>(lds, IMG + 255u * row + (uint32_t)T2, OFF_PAR, wave, row);
    barrier_lds();
    if (wave == 0 && lane < nb) {
        const uint64_t pv = *(const uint64_t*)(lds + OFF_PAR + 8u * lane);
#pragma unroll
        for (int q = 0; q < T2; ++q)
            lds[IMG + 255u * lane + (uint32_t)q] = (uint8_t)(pv >> (8 * (8 - T2 + q)));
    }
    barrier_lds();
    const uint32_t nout = nb * 255u;
    for (uint32_t i = tid; 16u * i < nout; i += NTHR) {
        const uint4 v = *(const uint4*)(lds + IMG + 16u * i);
        if (16u * i + 16u <= nout)
            *(uint4*)(dst + 16u * i) = v;
        else
            st_bytes(dst + 16u * i, v, nout - 16u * i);
    }
}
} // namespace wg
} // namespace ppfs
