#pragma once
// rs_pair.hpp -- workgroup RS(255, 255-2t) encode / decode for gfx950 with 16 < 2t <= 32
// (cfg5: t = 16, RS(255, 223)), conflict-free LDS lookups.
//
// Reference semantics: lib/blockdevice/src/rs_block_device.cpp (encode :95-117, decode :119-183;
// see rs_wg.hpp for the line map).
//
// The column kernels of tools/ablations/rs_col.hpp (four lanes per block, byte-indexed tables) are bound by LDS
// bank conflicts: a 32-lane ds_read_b64 group holds 8 blocks whose random table entries collide
// (PMC: 56 % of LDS cycles are conflict cycles).  This design makes every lookup conflict-free:
//   - Two lanes per block; lane c holds the 16-byte column [16c, 16c+16) of the block's 32-byte
//     top-aligned remainder (coefficient q at byte 32 - 2t + q).
//   - Slicing-by-8 over NIBBLE tables whose column halves are 256-byte planes: 16 entries x 16 B
//     = exactly the 64 LDS banks.  A ds_read_b128 is serviced in four 16-lane groups,
//     {0-3,12-15,20-27}, {4-11,16-19,28-31} and the same +32 (MI355X_MICROARCH.md, LDS); lanes
//     are assigned so that each group holds one column only, so all 16 lanes of a group read one
//     plane -- distinct entries sit in distinct banks, equal entries broadcast.  Column of lane l
//     = parity of bits 2-4 of l; the partner of lane l is lane l ^ 4 (DPP row_shl:4 / row_shr:4
//     with bank masks).
//   - Per 8 payload bytes: exchange the top dwords with the partner, fold the state's top 8 bytes
//     into the chunk, shift the state 8 bytes up (column 1 takes column 0's top half), and XOR in
//     16 table entries (one ds_read_b128 each, address = one SDWA add).
//   - 64-block tiles, 128-thread workgroups (2 waves, 32 blocks each), 3 per CU; LDS-DMA double
//     buffering and the emission of rs_emit.hpp / rs_wg.hpp.
//   - Decode correction per pair: S_1, S_2 and the XP-row check for a single error, else all 2t
//     syndromes (16 per lane) and the reference's BM / roots / Forney in lane 0, out of line.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf_common.hpp"
#include "rs_emit.hpp"
#include "srv_device.hpp"
#include "rs_fast.hpp"
#include "rs_layout.hpp"
#include "rs_wg.hpp"

namespace ppfs {
namespace pair {

using col::col_dec_piece;
using col::col_enc_piece;
using col::col_fix;
using wg::barrier_lds;
using wg::dma16;
using wg::lds_addr;
using wg::st_bytes;
using wg::st_nt;

constexpr int TB = 64;    // blocks per tile
constexpr int NTHR = 128; // threads per workgroup: 2 waves x 32 blocks x 2 lanes
static_assert(col::PAD == 48 && col::BUF == 16464, "emission helpers assume rs_emit.hpp's tile buffer");
constexpr int PAD = col::PAD, BUF = col::BUF;
constexpr int wpc_of(int wpc, int nbuf, int = 1, int = 0) { return (void)nbuf, wpc; }

// value of the partner lane: lane ^ 4 (XM = 4, this file's kernels) or lane ^ 1 (XM = 1, the
// byte-slice kernels of rs_bs.hpp)
template <int XM = 4> __device__ __forceinline__ uint32_t pair_xchg(uint32_t v)
{
    static_assert(XM == 4 || XM == 1, "partner lane");
    if constexpr (XM == 1)
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false); // quad_perm [1,0,3,2]
    // row_shl:4 writes banks 0 and 2 (lanes with bit 2 clear take lane + 4), row_shr:4 banks 1, 3
    const int x = __builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xF, 0x5, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(x, (int)v, 0x114, 0xF, 0xA, false);
}

// column of a lane: one column per ds_read_b128 lane group
__device__ __forceinline__ uint32_t lane_col(uint32_t lane) { return __builtin_popcount((lane >> 2) & 7u) & 1u; }
// block (0..31) of a lane within its wave: lanes l and l ^ 4 share it
__device__ __forceinline__ uint32_t lane_blk(uint32_t lane) { return ((lane >> 3) << 2) | (lane & 3u); }

// Block of a lane for tiles whose rows sit at a 255-byte stride (codewords, the encode image):
// half-wave h (32 lanes, 16 blocks) takes blocks h, h + NH, h + 2 NH, ... (NH = halves per
// workgroup), so the 16 rows a ds_read_b32 group reads start 255 NH / 4 dwords apart -- distinct
// banks -- where 16 consecutive blocks (63.75 dwords apart) pile onto ~4 banks.
template <int NH> __device__ __forceinline__ uint32_t spread_blk(uint32_t wave, uint32_t lane)
{
    return (uint32_t)NH * lane_blk(lane & 31u) + 2u * wave + (lane >> 5);
}

// base + byte K of x (one v_add_u32_sdwa)
template <int K> __device__ __forceinline__ uint32_t add_byte(uint32_t x, uint32_t base)
{
    uint32_t r;
    if constexpr (K == 0)
        asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD"
            : "=v"(r) : "v"(x), "v"(base));
    else if constexpr (K == 1)
        asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
            : "=v"(r) : "v"(x), "v"(base));
    else if constexpr (K == 2)
        asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
            : "=v"(r) : "v"(x), "v"(base));
    else
        asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
            : "=v"(r) : "v"(x), "v"(base));
    return r;
}

__device__ __forceinline__ uint4 ld16(const uint8_t* lds, uint32_t addr) { return *(const uint4*)(lds + addr); }

__device__ __forceinline__ void xor4(uint32_t (&a)[4], const uint4& e)
{
    a[0] ^= e.x;
    a[1] ^= e.y;
    a[2] ^= e.z;
    a[3] ^= e.w;
}

// the 16 nibble lookups of one chunk (lo, hi): entries XORed into acc.  tb = lane's plane base
// (SL + 256 c, offset into lds[]); table t = 2i + h sits at tb + 512 t.
// TS: byte stride between the 16 tables (512: the pair layout's two column planes per table;
// 256: one plane per table, the lane-per-block slicing tables of 8 < 2t <= 16 used by the solo
// kernels)
template <int TS = 512>
__device__ __forceinline__ void pair_lookups(uint32_t (&acc)[4], const uint8_t* lds, uint32_t tb, uint32_t lo, uint32_t hi)
{
    const uint32_t Ll = (lo << 4) & 0xF0F0F0F0u, Hl = lo & 0xF0F0F0F0u;
    const uint32_t Lh = (hi << 4) & 0xF0F0F0F0u, Hh = hi & 0xF0F0F0F0u;
    uint4 e[16];
    e[0] = ld16(lds, add_byte<0>(Ll, tb) + 0 * TS);
    e[1] = ld16(lds, add_byte<0>(Hl, tb) + 1 * TS);
    e[2] = ld16(lds, add_byte<1>(Ll, tb) + 2 * TS);
    e[3] = ld16(lds, add_byte<1>(Hl, tb) + 3 * TS);
    e[4] = ld16(lds, add_byte<2>(Ll, tb) + 4 * TS);
    e[5] = ld16(lds, add_byte<2>(Hl, tb) + 5 * TS);
    e[6] = ld16(lds, add_byte<3>(Ll, tb) + 6 * TS);
    e[7] = ld16(lds, add_byte<3>(Hl, tb) + 7 * TS);
    e[8] = ld16(lds, add_byte<0>(Lh, tb) + 8 * TS);
    e[9] = ld16(lds, add_byte<0>(Hh, tb) + 9 * TS);
    e[10] = ld16(lds, add_byte<1>(Lh, tb) + 10 * TS);
    e[11] = ld16(lds, add_byte<1>(Hh, tb) + 11 * TS);
    e[12] = ld16(lds, add_byte<2>(Lh, tb) + 12 * TS);
    e[13] = ld16(lds, add_byte<2>(Hh, tb) + 13 * TS);
    e[14] = ld16(lds, add_byte<3>(Lh, tb) + 14 * TS);
    e[15] = ld16(lds, add_byte<3>(Hh, tb) + 15 * TS);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        auto w = [&](int i) -> uint32_t { return q == 0 ? e[i].x : q == 1 ? e[i].y : q == 2 ? e[i].z : e[i].w; };
        uint32_t a = xor3(acc[q], w(0), w(1));
        a = xor3(a, w(2), w(3));
        a = xor3(a, w(4), w(5));
        a = xor3(a, w(6), w(7));
        a = xor3(a, w(8), w(9));
        a = xor3(a, w(10), w(11));
        a = xor3(a, w(12), w(13));
        acc[q] = xor3(a, w(14), w(15));
    }
}

// Remainder column c of a LEN-byte row at LDS byte `row` (s = state bytes [16c, 16c+16)).
// SOLO (2t <= 16): one lane per block holds the whole state as column 1 (column 0 is all zero):
// no partner exchange, c = 1, tables at a 256-byte stride.
template <int LEN, bool SOLO = false>
__device__ __forceinline__ void pair_remainder(uint32_t (&s)[4], const uint8_t* lds, uint32_t row, uint32_t tb, uint32_t c)
{
    constexpr int TS = SOLO ? 256 : 512;
    if constexpr (SOLO)
        c = 1;
    constexpr int NC = (LEN + 7) / 8;
    constexpr int TOPN = LEN - 8 * (NC - 1);
    const uint32_t sh = (row & 3u) * 8u;
    const uint32_t* w = (const uint32_t*)(lds + (row & ~3u));
    const uint32_t cm = c ? ~0u : 0u;
    uint32_t up = w[2 * NC];
#pragma unroll
    for (int j = NC - 1; j >= 0; --j) {
        const uint32_t d1 = w[2 * j + 1], d0 = w[2 * j];
        uint32_t hi = __builtin_amdgcn_alignbit(up, d1, sh); // payload bytes 8j+4 .. 8j+7
        uint32_t lo = __builtin_amdgcn_alignbit(d1, d0, sh); // payload bytes 8j .. 8j+3
        up = d0;
        if (j == NC - 1) {
            if constexpr (TOPN < 4) {
                lo &= (1u << (8 * TOPN)) - 1u;
                hi = 0;
            } else if constexpr (TOPN == 4) {
                hi = 0;
            } else if constexpr (TOPN < 8) {
                hi &= (1u << (8 * (TOPN - 4))) - 1u;
            }
            s[0] = s[1] = s[2] = s[3] = 0;
            pair_lookups<TS>(s, lds, tb, lo, hi);
        } else {
            const uint32_t p2 = SOLO ? 0u : pair_xchg(s[2]), p3 = SOLO ? 0u : pair_xchg(s[3]);
            lo ^= c ? s[2] : p2; // fold the top 8 coefficients (column 1's upper half)
            hi ^= c ? s[3] : p3;
            uint32_t n[4] = { p2 & cm, p3 & cm, s[0], s[1] }; // state * x^8
            pair_lookups<TS>(n, lds, tb, lo, hi);
            s[0] = n[0];
            s[1] = n[1];
            s[2] = n[2];
            s[3] = n[3];
        }
    }
}

template <int XM = 4> __device__ __forceinline__ uint32_t pair_or(uint32_t v) { return v | pair_xchg<XM>(v); }

// General correction (2+ errors), out of line; both lanes of the pair: lane c computes S_i for
// i = 16c+1 .. 16c+16 into the block's slot (over r', which both lanes have read), then lane 0
// runs BM / roots / Forney (rs_fast.hpp).
// RM: the state is c mod g (coefficient q has exponent i q in S_i) instead of x^2t c mod g
// TAG: a separate instance per calling kernel (the server's looser register budget must not
// become the decode kernel's: an out-of-line function is compiled once for all its callers)
template <int T2, bool RM = false, int TAG = 0>
__device__ __noinline__ void pair_correct_general(uint8_t* lds, uint32_t goff, uint32_t row, uint32_t slot, uint32_t c,
    uint8_t* __restrict__ raw_g, uint64_t gblk, bool wb, uint64_t raw_bytes)
{
    const Gf gf { lds + goff };
    const uint4 r0 = *(const uint4*)(lds + slot), r1 = *(const uint4*)(lds + slot + 16);
    const uint32_t rw[8] = { r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w };
    wave_fence(); // both lanes hold r' before the slot is overwritten
    uint32_t sw[4] = { 0u, 0u, 0u, 0u };
#pragma unroll
    for (int ii = 0; ii < 16; ++ii) {
        const uint32_t i = 16u * c + 1u + (uint32_t)ii;
        uint32_t e = RM ? 0u : (255u * 32u - i * (uint32_t)T2) % 255u; // i (q - 2t) (RM: i q) mod 255 at q = 0
        uint32_t sacc = 0;
#pragma unroll
        for (int q = 0; q < T2; ++q) {
            constexpr int P0 = 32 - T2;
            const uint32_t rv = (rw[(P0 + q) >> 2] >> (8 * ((P0 + q) & 3))) & 0xFFu;
            const uint32_t v = gf.exp(gf.log(rv) + e);
            sacc ^= rv ? v : 0u;
            e += i;
            e = e >= 255u ? e - 255u : e;
        }
        sw[ii >> 2] |= (i <= (uint32_t)T2 ? sacc : 0u) << (8 * (ii & 3));
    }
    *(uint4*)(lds + slot + 16u * c) = make_uint4(sw[0], sw[1], sw[2], sw[3]);
    wave_fence();
    if (c == 0) {
        uint32_t S[T2];
        const uint4 s0 = *(const uint4*)(lds + slot), s1 = *(const uint4*)(lds + slot + 16);
        const uint32_t sw8[8] = { s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w };
#pragma unroll
        for (int i = 0; i < T2; ++i)
            S[i] = (sw8[i >> 2] >> (8 * (i & 3))) & 0xFFu;
        rs_correct_general<T2>(S, gf, [&](uint32_t pos, uint32_t ev) { col_fix(lds, row, raw_g, gblk, wb, pos, ev, raw_bytes); });
    }
}

// Decode correction for the pair's block; s = the lane's column of r' = x^2t c(x) mod g.  Single
// error: S_1, S_2 -> X = S_2/S_1, e = S_1/X, confirmed iff r' == e * XP row LOG X.
template <int T2, bool RM = false, int TAG = 0, int XM = 4>
__device__ __forceinline__ uint32_t pair_correct(uint8_t* lds, uint32_t goff, const uint8_t* __restrict__ xp, uint32_t row,
    uint32_t slot,
    uint32_t c, const uint32_t (&s)[4], bool valid, uint8_t* __restrict__ raw_g, uint64_t gblk, bool wb, uint64_t raw_bytes)
{
    const bool err = valid && pair_or<XM>(s[0] | s[1] | s[2] | s[3]) != 0u;
    if (!__builtin_amdgcn_ballot_w64(err))
        return 0u;
    const Gf gf { lds + goff };
    // state byte 16c+k is coefficient q = 16c+k-POFF; exponent i (q - 2t) = i (16c + k - 32)
    uint32_t s1 = 0, s2 = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t rb = (s[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const uint32_t lb = gf.log(rb), u = 16u * c + (uint32_t)k;
        // exponent i (q - 2t) for i = 1, 2 (q = u, 2t = 32); RM: i q
        const uint32_t v1 = gf.exp(lb + u + (RM ? 0u : 223u)), v2 = gf.exp(lb + 2u * u + (RM ? 0u : 191u));
        s1 ^= rb ? v1 : 0u;
        s2 ^= rb ? v2 : 0u;
    }
    s1 ^= pair_xchg<XM>(s1);
    s2 ^= pair_xchg<XM>(s2);
    const uint32_t l1 = gf.log(s1), l2 = gf.log(s2);
    uint32_t lx = l2 + 255u - l1;
    lx = lx >= 255u ? lx - 255u : lx;
    uint32_t le = l1 + 255u - lx;
    le = le >= 255u ? le - 255u : le;
    const uint4 xr = *(const uint4*)(xp + 32u * lx + 16u * c); // XP rows stay in global memory (L2)
    const uint32_t xw[4] = { xr.x, xr.y, xr.z, xr.w };
    uint32_t bad = (s1 == 0u || s2 == 0u) ? 1u : 0u;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t x = (xw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const uint32_t rb = (s[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const uint32_t ev = x == 0xFFu ? 0u : gf.exp(le + x);
        bad |= ev != rb ? 1u : 0u;
    }
    const bool geo = err && pair_or<XM>(bad) == 0u;
    if (geo && c == 0)
        col_fix(lds, row, raw_g, gblk, wb, lx, gf.exp(le), raw_bytes);
    if (err && !geo)
        pair_correct_general<T2, RM, TAG>(lds, goff, row, slot, c, raw_g, gblk, wb, raw_bytes);
    return err ? 1u : 0u;
}

// Decode emission for 2t a multiple of 16: payload piece p starts at codeword byte
// 16 p + 2t (b + 1) of the tile, a 16-byte aligned LDS address, and the bytes past block b's end
// (from kb on) come from 2t further on.  Two aligned ds_read_b128 and one byte mask, where
// col_dec_piece's windows (any alignment) cost four reads and the funnel shifts.
template <int T2> __device__ __forceinline__ uint4 pair_dec_piece(const uint8_t* lds, uint32_t buf, uint32_t p)
{
    static_assert(T2 % 16 == 0, "aligned payload pieces need 16 | 2t");
    constexpr uint32_t K = 255 - T2;
    const uint32_t j0 = p * 16u, b = j0 / K, off = j0 - K * b;
    const uint32_t S = buf + PAD + j0 + (uint32_t)T2 * (b + 1u);
    const uint32_t kb = off > K - 16u ? K - off : 16u;
    const uint4 X = ld16(lds, S), Z = ld16(lds, S + (uint32_t)T2);
    const wg::M128 mZ = wg::range_mask(kb, 16);
    const uint32_t x[4] = { X.x, X.y, X.z, X.w }, z[4] = { Z.x, Z.y, Z.z, Z.w };
    uint32_t o[4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
        o[m] = wg::bfi(col::mword(mZ, m), z[m], x[m]);
    return make_uint4(o[0], o[1], o[2], o[3]);
}

template <int T2> __device__ __forceinline__ uint4 dec_piece(const uint8_t* lds, uint32_t buf, uint32_t p)
{
    if constexpr (T2 % 16 == 0)
        return pair_dec_piece<T2>(lds, buf, p);
    else
        return col_dec_piece<T2>(lds, buf, p);
}

// LDS-DMA of a tile by 128 threads: piece p = tid + 128 k lands at dst + 16 p.
template <int NPIECE>
__device__ __forceinline__ void dma_tile128(uint8_t* dst, const uint8_t* __restrict__ src, uint32_t tid,
    [[maybe_unused]] const uint8_t* gbase, [[maybe_unused]] uint64_t extent)
{
    constexpr int K = (NPIECE + NTHR - 1) / NTHR;
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(dst) + (tid & ~63u) * 16u);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t p = tid + (uint32_t)NTHR * k;
        if (((k + 1) * NTHR <= NPIECE || p < (uint32_t)NPIECE) && PPFS_DBG_OK(src + (size_t)p * 16, 16, gbase, extent))
            dma16(src + (size_t)p * 16, base + 16u * NTHR * k);
    }
}

__device__ __forceinline__ void stage_bytes128(uint8_t* dst, const uint8_t* __restrict__ src, uint32_t nbytes, uint32_t tid)
{
    for (uint32_t i = tid; i < nbytes; i += NTHR)
        dst[i] = src[i];
}

// LDS plan (single __shared__ array at LDS address 0): tables | remainder / syndrome slots
// (65 x 32 B + slack) | NBUF tile buffers.  NBUF = 2: the next tile's DMA is issued at the top of
// an iteration; NBUF = 1: after this tile's emission reads (more workgroups per CU overlap it).
template <int T2, bool DEC, int NBUF> struct Lds {
    using L = RsPairLayout<T2>;
    // decode copies SL + GF; the XP rows (8 KiB, read once per single-error block) stay in
    // global memory so that one more workgroup fits a CU
    static constexpr int TBL = DEC ? L::OFF_XP : L::ENC_BYTES;
    static constexpr int OFF_PAR = TBL;
    static constexpr int OFF_BUF = OFF_PAR + 2080;
    static constexpr int BYTES = OFF_BUF + NBUF * BUF;
    static_assert(OFF_BUF % 16 == 0 && TBL % 16 == 0, "aligned buffers");
};


// ---- Encode into a codeword image (2t a multiple of 16) ----
// The tile is DMA'd straight into the OUTPUT layout: codeword j of the tile at LDS IMG + 255 j,
// payload at IMG + 255 j + 2t.  Output piece i (bytes [16 i, 16 i + 16) of the tile's codewords)
// takes its payload bytes from tile payload offset 16 i - 2t (b + 1), b = the block of those bytes:
// a 16-byte aligned source, so every piece is one LDS-DMA lane.  The parity bytes (registers after
// the remainder) are then written into the gaps [255 j, 255 j + 2t) and the emission is a plain
// aligned copy of the image: no per-piece windows, masks or parity merges (those were 42 % of the
// VALU instructions of rs_pair_encode_kernel's tile loop).
// image bytes of a TBK-block tile, + slack: the rows' last word reads run past the image
template <int TBK> constexpr int img_bytes() { return TBK * 255 + 64; }

// tile payload offset of output piece i, or -1 when the piece holds parity bytes only
template <int T2> __device__ __forceinline__ int img_src(uint32_t i)
{
    const uint32_t e = 16u * i + 15u, b = e / 255u, off = e - 255u * b;
    if (off >= (uint32_t)T2)
        return (int)(16u * i) - T2 * (int)(b + 1u); // payload of block b (from 255 b + 2t on)
    if (16u * i >= 255u * b)
        return -1; // inside block b's parity
    return (int)(16u * i) - T2 * (int)b; // ends block b-1's payload, then block b's parity
}


// c mod g of the LDS codeword row: the remainder of the payload (as encode) XOR the stored parity
// -- K bytes through the lookups instead of all 255 for x^2t c mod g (28 chunks, not 32)
template <int T2>
__device__ __forceinline__ void pair_cmodg(uint32_t (&s)[4], const uint8_t* lds, uint32_t row, uint32_t tb, uint32_t c)
{
    static_assert(T2 == 32, "state byte q = coefficient q");
    pair_remainder<255 - T2>(s, lds, row + (uint32_t)T2, tb, c);
    const uint32_t a = row + 16u * c, sh = (a & 3u) * 8u;
    const uint32_t* w = (const uint32_t*)(lds + (a & ~3u));
    uint32_t d[5];
#pragma unroll
    for (int m = 0; m < 5; ++m)
        d[m] = w[m];
#pragma unroll
    for (int m = 0; m < 4; ++m)
        s[m] ^= __builtin_amdgcn_alignbit(d[m + 1], d[m], sh);
}

// RM: decode from c mod g (pair_cmodg) and the x^p mod g rows; else from x^2t c mod g
// ---- Solo encode into a codeword image (2t = 16): one lane per block ----
// The state fits one 16-byte column, so a lane owns a block: half the lookups per block of the
// pair kernels.  Tables: the lane-per-block slicing tables (16 tables x 16 nibbles x 16 B, top-
// aligned entries = column 1 of the pair layout).  Tiles of 64 NW blocks into the output image as
// rs_pair_encode_img_kernel; half-wave h takes rows h + 2 NW i so a ds_read_b32 group's 32 rows
// start on distinct banks (4 rows apart at NW = 2).
template <int T2, int WPC = 4, int NW = 2, int NTST = 1>
__global__ __launch_bounds__(64 * NW, 2) void rs_solo_encode_img_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables)
{
    static_assert(T2 == 16, "parity bytes = the lane's 16 state bytes; aligned image pieces need 16 | 2t");
    constexpr int TBL = 16 * 256;
    constexpr int IMG = TBL;
    constexpr int TBK = 64 * NW, NT = 64 * NW;
    constexpr int BYTES = IMG + img_bytes<TBK>();
    constexpr int LDS_ALLOC = wg::lds_alloc<BYTES, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = 255 - T2;
    constexpr int PIECES = TBK * 255 / 16;
    constexpr int KP = (PIECES + NT - 1) / NT;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t blk = (uint32_t)(2 * NW) * (lane & 31u) + 2u * wave + (lane >> 5);
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
    uint8_t* const gap = lds + IMG + 255u * blk; // the block's 16 parity bytes
    for (; t < nfull; t += gridDim.x) {
        barrier_lds(); // A: tile t in the image, the last tile's emission reads done
        uint32_t s[4];
        pair_remainder<K, true>(s, lds, row, 0u, 1u);
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
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (t == nfull && nfull < ntiles) {
        barrier_lds();
        const uint32_t nb = (uint32_t)(nblocks - t * TBK);
        const uint8_t* src = data + t * (TBK * K);
        if (!PPFS_DBG_OK(src, nb * (uint32_t)K, data, nblocks * K))
            return;
        for (uint32_t j = tid; j < nb * (uint32_t)K; j += NT) {
            const uint32_t b = j / (uint32_t)K;
            lds[IMG + T2 + 255u * b + (j - (uint32_t)K * b)] = src[j];
        }
        barrier_lds();
        uint32_t s[4];
        pair_remainder<K, true>(s, lds, row, 0u, 1u);
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


// Resident small-batch server for 16 < 2t <= 32 (server_box.hpp; the 2t <= 8 twin is
// rs_wg_server_kernel): one 128-thread workgroup, the decode tables in LDS (the XP rows stay in
// global memory as in the decode kernel), requests of <= 64 blocks from the context's zero-copy
// buffer.  Decode is the partial-tile path of rs_pair_decode_kernel; encode stages the payloads
// contiguously (one round trip) and copies them into the codeword image of
// rs_pair_encode_img_kernel inside LDS.
template <int T2, bool RM>
__global__ __launch_bounds__(NTHR, 1) void rs_pair_server_kernel(SrvBox* box, uint8_t* zc, uint64_t zc_bytes,
    const uint8_t* __restrict__ tables, uint32_t gen, uint32_t idle_us)
{
    static_assert(T2 % 16 == 0, "codeword image pieces need 16 | 2t");
    using L = RsPairLayout<T2>;
    using D = Lds<T2, true, 1>;
    constexpr int K = L::K;
    constexpr int IMG = D::OFF_BUF;           // encode: the codeword image (64 x 255 + 64 <= BUF)
    constexpr int STG = D::BYTES;             // encode: the payloads as read (64 K bytes)
    static_assert(img_bytes<TB>() <= BUF && IMG % 16 == 0, "image in the tile buffer");
    __shared__ __attribute__((aligned(16))) uint8_t lds[STG + TB * K + 16];
    __shared__ uint32_t s_cmd[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t c = lane_col(lane), blk = spread_blk<NTHR / 32>(wave, lane);
    const uint32_t tb = L::OFF_SL + 256u * c;
    const uint32_t slot = D::OFF_PAR + 32u * blk;
    for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += NTHR)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t last = t0;
    uint32_t seen = srv::ld_sys(&box->done), served = 0;
    if (tid == 0)
        srv::st_sys(&box->alive, gen);
    for (;;) {
        const uint32_t r = srv::next_request(box, seen, last, t0, idle_us, s_cmd);
        if (r == 0)
            break;
        const SrvCmd cmd = srv_cmd_unpack(r);
        const uint32_t op = cmd.op, nb = cmd.nb;
        const SrvLayout lay = srv_layout(nb, (uint32_t)K, 255u);
        uint8_t* data = zc + lay.data;
        uint8_t* raw = zc + lay.raw;
        uint8_t* status = zc + lay.status;
        const bool ok = nb >= 1 && nb <= (uint32_t)TB && PPFS_DBG_OK(data, nb * K, zc, zc_bytes)
            && PPFS_DBG_OK(raw, nb * 255u, zc, zc_bytes) && PPFS_DBG_OK(status, nb, zc, zc_bytes);
        if (ok && (op == SRV_DECODE || op == SRV_WRITE)) {
            const uint32_t buf = D::OFF_BUF;
            srv::stage_host<NTHR, TB * 255>(lds + buf + PAD, raw, nb * 255u, tid);
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
            const uint32_t st = pair_correct<T2, RM, 1>(lds, L::OFF_GF, tables + (RM ? L::OFF_XPM : L::OFF_XP), row,
                slot, c, s, valid, raw, blk, op == SRV_DECODE && cmd.write_back, nb * 255u);
            if (valid && c == 0)
                status[blk] = (uint8_t)st;
            barrier_lds();
            if (op == SRV_DECODE && cmd.want_data) {
                const uint32_t nout = nb * (uint32_t)K;
                for (uint32_t p = tid; 16u * p < nout; p += NTHR) {
                    const uint4 v = dec_piece<T2>(lds, buf, p);
                    if (16u * p + 16u <= nout)
                        *(uint4*)(data + 16u * p) = v;
                    else
                        st_bytes(data + 16u * p, v, nout - 16u * p);
                }
            }
            barrier_lds();
        }
        if (ok && (op == SRV_ENCODE || op == SRV_WRITE)) {
            srv::stage_host<NTHR, TB * K + 16>(lds + STG, data, nb * (uint32_t)K, tid);
            barrier_lds();
            for (uint32_t j = tid; j < nb * (uint32_t)K; j += NTHR) { // payload b -> image row b
                const uint32_t b = j / (uint32_t)K;
                lds[IMG + 255u * b + (uint32_t)T2 + (j - (uint32_t)K * b)] = lds[STG + j];
            }
            barrier_lds();
            uint32_t s[4];
            pair_remainder<K>(s, lds, IMG + 255u * blk + (uint32_t)T2, tb, c);
            uint8_t* const gap = lds + IMG + 255u * blk + 16u * c; // this lane's 16 parity bytes
#pragma unroll
            for (int k = 0; k < 16; ++k)
                gap[k] = (uint8_t)(s[k >> 2] >> (8 * (k & 3)));
            barrier_lds();
            const uint32_t nout = nb * 255u;
            for (uint32_t i = tid; 16u * i < nout; i += NTHR) {
                const uint4 v = ld16(lds, IMG + 16u * i);
                if (16u * i + 16u <= nout)
                    *(uint4*)(raw + 16u * i) = v;
                else
                    st_bytes(raw + 16u * i, v, nout - 16u * i);
            }
            barrier_lds();
        }
        seen = r;
        srv::finish_request(box, r, ++served);
    }
    if (tid == 0)
        srv::st_sys(&box->alive, gen | SRV_EXITED);
}

} // namespace pair
} // namespace ppfs
