#pragma once
// rs_emit.hpp -- emission helpers of the RS(255, 255-2t) workgroup kernels with 8 < 2t <= 32
// (rs_pair.hpp): 16-byte output pieces of a 64-block tile assembled from the LDS codeword / payload
// rows and the parity slots, and the in-LDS + HBM byte fix of a correction.
//
// Reference semantics: lib/blockdevice/src/rs_block_device.cpp
//   codeword byte i = coefficient of x^i: parity in bytes [0,2t), payload in [2t,n) (_encodeBlock
//   :95-117); the corrected codeword is written back whole (:175-180), here byte by byte.
//
// (The column-split kernels these helpers were first written for -- four lanes per block,
// byte-indexed tables -- lost to the pair kernels and live on as an ablation in
// tools/ablations/rs_col.hpp)
#include <hip/hip_runtime.h>

#include "dbg.hpp"
#include <stdint.h>

#include "gf_common.hpp"
#include "rs_wg.hpp"

namespace ppfs {
namespace col {

using wg::bfi;
using wg::M128;
using wg::range_mask;

constexpr int TB = 64;                   // blocks per tile
constexpr int PAD = 48;                  // front pad of a tile buffer
constexpr int BUF = PAD + TB * 255 + 96; // 16464: windows read up to 2t + 20 bytes past a piece

// 16 bytes at any LDS byte address, from the two aligned 16-byte pieces that cover them.
// Emission lanes read consecutive 16-byte pieces: as ds_read_b128 a 16-lane group then covers
// the 64 banks exactly, where five ds_read_b32 per lane (lane stride 4 dwords) hit each bank
// 4 times per 32-lane group.  The per-lane dword offset is selected with two v_bfi levels.
__device__ __forceinline__ void win16(uint32_t (&X)[4], const uint8_t* lds, uint32_t addr)
{
    const uint32_t a16 = addr & ~15u;
    const uint4 A = *(const uint4*)(lds + a16), B = *(const uint4*)(lds + a16 + 16);
    const uint32_t D[8] = { A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w };
    const uint32_t sh = (addr & 3u) * 8u;
    // masks, not selects: LLVM folds a select between array elements into a dynamic index (scratch)
    const uint32_t m2 = 0u - ((addr >> 3) & 1u), m1 = 0u - ((addr >> 2) & 1u);
    uint32_t F[6], E[5];
#pragma unroll
    for (int i = 0; i < 6; ++i)
        F[i] = bfi(m2, D[i + 2], D[i]);
#pragma unroll
    for (int i = 0; i < 5; ++i)
        E[i] = bfi(m1, F[i + 1], F[i]);
#pragma unroll
    for (int m = 0; m < 4; ++m)
        X[m] = __builtin_amdgcn_alignbit(E[m + 1], E[m], sh);
}

__device__ __forceinline__ uint32_t mword(const M128& mk, int m)
{
    return (uint32_t)((m < 2 ? mk.lo : mk.hi) >> ((m & 1) * 32));
}

// Encode emission: 16 bytes of the codeword tile at piece p.  Codeword byte j of block b = j / 255
// (off = j % 255) is parity byte off (slot byte POFF + off) if off < 2t, else payload byte
// K b + off - 2t; a piece may run into block b+1 (off > 239), whose parity and payload follow.
template <int T2>
__device__ __forceinline__ uint4 col_enc_piece(const uint8_t* lds, uint32_t buf, uint32_t par, uint32_t p)
{
    constexpr uint32_t K = 255 - T2, POFF = 32 - T2;
    const uint32_t j0 = p * 16u, b = j0 / 255u, off = j0 - 255u * b;
    const uint32_t S = buf + PAD + K * b + off - T2;   // payload source of output byte 0
    const uint32_t kb = off > 239u ? 255u - off : 16u; // first byte of block b+1 in the piece
    const uint32_t c0 = off < (uint32_t)T2 ? min((uint32_t)T2 - off, 16u) : 0u; // leading parity bytes
    const uint32_t e1 = min(kb + (uint32_t)T2, 16u);   // end of block b+1's parity bytes
    uint32_t X[4], Y[4], P0[4], P1[4];
    win16(X, lds, S);
    win16(Y, lds, S - T2); // block b+1 payload: 2t bytes behind
    win16(P0, lds, par + 32u * b + POFF + (c0 ? off : 0u));
    win16(P1, lds, par + 32u * (b + 1u) + POFF - kb);
    const M128 mY = range_mask(e1, 16), mP1 = range_mask(kb, e1), mP0 = range_mask(0, c0);
    uint32_t o[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        uint32_t v = bfi(mword(mY, m), Y[m], X[m]);
        v = bfi(mword(mP1, m), P1[m], v);
        o[m] = bfi(mword(mP0, m), P0[m], v);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// Decode emission: 16 bytes of the payload tile at piece p: payload byte j of block b = j / K
// (off = j % K) is codeword byte 255 b + 2t + off; past the block end the source skips block
// b+1's 2t parity bytes.
template <int T2> __device__ __forceinline__ uint4 col_dec_piece(const uint8_t* lds, uint32_t buf, uint32_t p)
{
    constexpr uint32_t K = 255 - T2;
    const uint32_t j0 = p * 16u, b = j0 / K, off = j0 - K * b;
    const uint32_t S = buf + PAD + 255u * b + T2 + off;
    const uint32_t kb = off > K - 16u ? K - off : 16u;
    uint32_t X[4], Z[4];
    win16(X, lds, S);
    win16(Z, lds, S + T2);
    const M128 mZ = range_mask(kb, 16);
    uint32_t o[4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
        o[m] = bfi(mword(mZ, m), Z[m], X[m]);
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// codeword byte `pos` of the LDS row ^= ev, and the same byte in HBM with write-back
// (raw_bytes: extent of raw_g, PPFS_ECC_DEBUG bounds checks)
__device__ __forceinline__ void col_fix(uint8_t* lds, uint32_t row, uint8_t* __restrict__ raw_g, uint64_t gblk, bool wb,
    uint32_t pos, uint32_t ev, [[maybe_unused]] uint64_t raw_bytes)
{
    if (ev == 0)
        return;
    const uint8_t fixed = (uint8_t)(lds[row + pos] ^ ev);
    lds[row + pos] = fixed;
    if (wb && PPFS_DBG_OK(raw_g + gblk * 255u + pos, 1, raw_g, raw_bytes))
        wb_byte(raw_g + gblk * 255u + pos, fixed);
}

} // namespace col
} // namespace ppfs
