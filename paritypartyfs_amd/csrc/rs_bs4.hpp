#pragma once
// rs_bs4.hpp -- RS(255,223) decode (2t = 32, cfg5) with FOUR lanes per block (round 4).
//
// Reference semantics: lib/blockdevice/src/rs_block_device.cpp (decode :119-183), as rs_bs.hpp's
// decode: c mod g = the payload's remainder XOR the stored parity, a single error confirmed against
// the x^p mod g row, anything else all 32 syndromes and BM / roots / Forney out of line.
//
// Why four lanes: rs_bs.hpp's decode gives a block two lanes (16 state bytes each) and a wave 32
// blocks, so its 8,160-byte wave image, the 64 KiB byte table and the correction tables fill the
// LDS at 8 waves (2 per SIMD), and each lane's 28-step slicing chain is dependent LDS latency that 2
// waves per SIMD cannot hide (a timing ablation with half the steps took the clean decode from
// 137-143 to 89 us).  Here lane c of a block holds state bytes [8c, 8c+8),
// a wave decodes 16 blocks (4,080-byte image), and 16 waves fit the same LDS: 4 per SIMD.
//   - Same byte table (RsPairLayout::OFF_BS): row v (256 B) holds chunk positions q = 0..7 x the
//     32-byte entry, so quarter c of position q is the 8-byte slot 32 q + 8 c -- one ds_read_b64
//     per chunk byte and lane.  A ds_read_b64 is serviced per 32 lanes (8 blocks x 4 quarters); the
//     8 blocks of a group have distinct rotations k (block k looks up chunk byte (m + k) mod 8 at
//     lookup m), so the 32 lanes read 32 distinct slots = all 64 banks: conflict-free for any bytes.
//   - The fold (top 8 state bytes, quarter 3) and the x^8 shift (quarter c takes quarter c - 1) are
//     quad_perm DPP moves folded into the XOR / AND.
//   - Correction per quad: the S12 table gives each lane its 8 state bytes' share of S_1, S_2 (a quad
//     XOR), the XP row its 8 bytes to confirm; quarter 0 patches and writes back.
#include "rs_bs.hpp"

namespace ppfs {
namespace bs4 {

using bs::addr_sel;
using bs::OFF_TAB;
using bs::TAB_BYTES;
using wg::lds_addr;
using wg::st_bytes;
using wg::st_nt;

constexpr int TBQ = 16;                       // blocks per wave tile
constexpr int IMGQ = TBQ * 255;               // 4,080 B: one wave tile's codeword image
constexpr int IMGQ_PIECES = IMGQ / 16;        // 255 16-byte pieces
constexpr int KPQ = (IMGQ_PIECES + 63) / 64;  // 4 load / put instructions per tile

// quad_perm DPP controls
constexpr int QP_TOP = 0xFF;   // [3,3,3,3]: quarter 3 to every lane of the quad
constexpr int QP_SHIFT = 0x90; // [0,0,1,2]: quarter c takes quarter c - 1 (quarter 0: masked)
constexpr int QP_X1 = 0xB1;    // [1,0,3,2]
constexpr int QP_X2 = 0x4E;    // [2,3,0,1]
template <int J> constexpr int qp_bcast() { return J * 0x55; } // [J,J,J,J]

template <int CTRL> __device__ __forceinline__ uint32_t qdpp(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t quad_or(uint32_t v)
{
    v |= qdpp<QP_X1>(v);
    return v | qdpp<QP_X2>(v);
}
__device__ __forceinline__ uint32_t quad_xor(uint32_t v)
{
    v ^= qdpp<QP_X1>(v);
    return v ^ qdpp<QP_X2>(v);
}

// lane constants: quarter, block in the wave tile, rotation and the v_perm selectors
struct QLane {
    uint32_t c, blk;
    uint32_t sel_lo, sel_hi; // rotated chunk: byte m = chunk byte (m + k) mod 8 (v_perm of hi:lo)
    uint32_t off_a, off_b;   // slot offsets 32 ((m + k) mod 8) + 8 c, m = 0..3 / 4..7, one per byte
};

__device__ __forceinline__ QLane q_lane(uint32_t lane)
{
    QLane L;
    L.c = lane & 3u;
    L.blk = lane >> 2;
    const uint32_t k = L.blk & 7u; // lanes 0-31: blocks 0-7, lanes 32-63: blocks 8-15
    uint32_t sl = 0, sh = 0, oa = 0, ob = 0;
#pragma unroll
    for (uint32_t m = 0; m < 4; ++m) {
        sl |= ((m + k) & 7u) << (8 * m);
        sh |= ((m + 4u + k) & 7u) << (8 * m);
        oa |= (32u * ((m + k) & 7u) + 8u * L.c) << (8 * m);
        ob |= (32u * ((m + 4u + k) & 7u) + 8u * L.c) << (8 * m);
    }
    L.sel_lo = sl;
    L.sel_hi = sh;
    L.off_a = oa;
    L.off_b = ob;
    return L;
}

// the 8 byte lookups of one chunk (lo, hi = chunk bytes 0-3 / 4-7), XORed into acc
__device__ __forceinline__ void q_lookups(uint32_t (&acc)[2], const uint8_t* lds, const QLane& L, uint32_t lo, uint32_t hi)
{
    const uint32_t rl = __builtin_amdgcn_perm(hi, lo, L.sel_lo), rh = __builtin_amdgcn_perm(hi, lo, L.sel_hi);
    uint2 e[8];
    e[0] = *(const uint2*)(lds + OFF_TAB + __builtin_amdgcn_perm(L.off_a, rl, addr_sel<0>()));
    e[1] = *(const uint2*)(lds + OFF_TAB + __builtin_amdgcn_perm(L.off_a, rl, addr_sel<1>()));
    e[2] = *(const uint2*)(lds + OFF_TAB + __builtin_amdgcn_perm(L.off_a, rl, addr_sel<2>()));
    e[3] = *(const uint2*)(lds + OFF_TAB + __builtin_amdgcn_perm(L.off_a, rl, addr_sel<3>()));
    e[4] = *(const uint2*)(lds + OFF_TAB + __builtin_amdgcn_perm(L.off_b, rh, addr_sel<0>()));
    e[5] = *(const uint2*)(lds + OFF_TAB + __builtin_amdgcn_perm(L.off_b, rh, addr_sel<1>()));
    e[6] = *(const uint2*)(lds + OFF_TAB + __builtin_amdgcn_perm(L.off_b, rh, addr_sel<2>()));
    e[7] = *(const uint2*)(lds + OFF_TAB + __builtin_amdgcn_perm(L.off_b, rh, addr_sel<3>()));
    uint32_t a = xor3(acc[0], e[0].x, e[1].x), b = xor3(acc[1], e[0].y, e[1].y);
    a = xor3(a, e[2].x, e[3].x);
    b = xor3(b, e[2].y, e[3].y);
    a = xor3(a, e[4].x, e[5].x);
    b = xor3(b, e[4].y, e[5].y);
    acc[0] = xor3(a, e[6].x, e[7].x);
    acc[1] = xor3(b, e[6].y, e[7].y);
}

// Remainder quarter c of the 223-byte payload row at LDS byte `row`: slicing-by-8 Horner steps from
// the top chunk down (the top chunk holds 223 - 8 * 27 = 7 bytes)
__device__ __forceinline__ void q_remainder(uint32_t (&s)[2], const uint8_t* lds, uint32_t row, const QLane& L)
{
    constexpr int LEN = 223, NC = (LEN + 7) / 8, TOPN = LEN - 8 * (NC - 1);
    static_assert(TOPN == 7, "top chunk");
    const uint32_t sh = (row & 3u) * 8u;
    const uint32_t* w = (const uint32_t*)(lds + (row & ~3u));
    uint32_t cm = L.c ? ~0u : 0u;
    asm("" : "+v"(cm)); // a mask, not a select: keeps (dpp & cm) one v_and_b32_dpp
    // the top chunk (7 bytes) starts the state
    uint32_t up = w[2 * NC], d1 = w[2 * NC - 1], d0 = w[2 * NC - 2];
    {
        const uint32_t hi = __builtin_amdgcn_alignbit(up, d1, sh) & ((1u << (8 * (TOPN - 4))) - 1u);
        const uint32_t lo = __builtin_amdgcn_alignbit(d1, d0, sh);
        up = d0;
        s[0] = s[1] = 0;
        q_lookups(s, lds, L, lo, hi);
    }
    // the other 27 chunks in a rolled loop (the unrolled chain hoisted all 57 payload dwords into
    // registers and spilled at 4 waves per SIMD); the next chunk's dwords are read a step ahead
    d1 = w[2 * NC - 3];
    d0 = w[2 * NC - 4];
#pragma unroll 3
    for (int j = NC - 2; j >= 0; --j) {
        const uint32_t hi0 = __builtin_amdgcn_alignbit(up, d1, sh); // payload bytes 8j+4 .. 8j+7
        const uint32_t lo0 = __builtin_amdgcn_alignbit(d1, d0, sh); // payload bytes 8j .. 8j+3
        up = d0;
        if (j > 0) {
            d1 = w[2 * j - 1];
            d0 = w[2 * j - 2];
        }
        // fold the top 8 coefficients (quarter 3) into the chunk; state * x^8: quarter c takes
        // quarter c - 1, quarter 0 zeros
        const uint32_t lo = lo0 ^ qdpp<QP_TOP>(s[0]), hi = hi0 ^ qdpp<QP_TOP>(s[1]);
        uint32_t n[2] = { qdpp<QP_SHIFT>(s[0]) & cm, qdpp<QP_SHIFT>(s[1]) & cm };
        q_lookups(n, lds, L, lo, hi);
        s[0] = n[0];
        s[1] = n[1];
    }
}

// c mod g of the LDS codeword row (255 B at `row`): the payload's remainder XOR the stored parity
__device__ __forceinline__ void q_cmodg(uint32_t (&s)[2], const uint8_t* lds, uint32_t row, const QLane& L)
{
    q_remainder(s, lds, row + 32u, L);
    const uint32_t a = row + 8u * L.c, sh = (a & 3u) * 8u;
    const uint32_t* w = (const uint32_t*)(lds + (a & ~3u));
    const uint32_t d0 = w[0], d1 = w[1], d2 = w[2];
    s[0] ^= __builtin_amdgcn_alignbit(d1, d0, sh);
    s[1] ^= __builtin_amdgcn_alignbit(d2, d1, sh);
}

// General correction (2+ errors), out of line; the four lanes of a block take it together.  Every
// lane gathers the 32-byte c mod g state; lane c computes S_i, i = 8c+1 .. 8c+8 (coefficient q has
// exponent i q); quarter 0 gathers S_1..S_32 and runs BM / roots / Forney (rs_fast.hpp).
__device__ __noinline__ void q_correct_general(uint8_t* lds, const uint8_t* gfp, uint32_t row, uint32_t c, uint32_t s0,
    uint32_t s1, uint8_t* __restrict__ raw_g, uint64_t gblk, bool wb, uint64_t raw_bytes)
{
    constexpr int T2 = 32;
    const Gf gf { gfp };
    const uint32_t rw[8] = { qdpp<qp_bcast<0>()>(s0), qdpp<qp_bcast<0>()>(s1), qdpp<qp_bcast<1>()>(s0),
        qdpp<qp_bcast<1>()>(s1), qdpp<qp_bcast<2>()>(s0), qdpp<qp_bcast<2>()>(s1), qdpp<qp_bcast<3>()>(s0),
        qdpp<qp_bcast<3>()>(s1) };
    uint32_t sw[2] = { 0u, 0u };
#pragma unroll
    for (int ii = 0; ii < 8; ++ii) {
        const uint32_t i = 8u * c + 1u + (uint32_t)ii;
        uint32_t e = 0, sacc = 0;
#pragma unroll
        for (int q = 0; q < T2; ++q) {
            const uint32_t rv = (rw[q >> 2] >> (8 * (q & 3))) & 0xFFu;
            const uint32_t v = gf.exp(gf.log(rv) + e);
            sacc ^= rv ? v : 0u;
            e += i;
            e = e >= 255u ? e - 255u : e;
        }
        sw[ii >> 2] |= sacc << (8 * (ii & 3));
    }
    const uint32_t all[8] = { qdpp<qp_bcast<0>()>(sw[0]), qdpp<qp_bcast<0>()>(sw[1]), qdpp<qp_bcast<1>()>(sw[0]),
        qdpp<qp_bcast<1>()>(sw[1]), qdpp<qp_bcast<2>()>(sw[0]), qdpp<qp_bcast<2>()>(sw[1]), qdpp<qp_bcast<3>()>(sw[0]),
        qdpp<qp_bcast<3>()>(sw[1]) };
    if (c == 0) {
        uint32_t S[T2];
#pragma unroll
        for (int i = 0; i < T2; ++i)
            S[i] = (all[i >> 2] >> (8 * (i & 3))) & 0xFFu;
        rs_correct_general<T2>(S, gf, [&](uint32_t pos, uint32_t ev) { col::col_fix(lds, row, raw_g, gblk, wb, pos, ev, raw_bytes); });
    }
}

// Decode correction for the quad's block (rs_bs.hpp bs_correct with quarters): single error X =
// S_2 / S_1, e = S_1 / X, confirmed iff c mod g == e (x^p mod g); else the general path
__device__ __forceinline__ uint32_t q_correct(uint8_t* lds, const uint8_t* gfp, const uint8_t* s12p, const uint8_t* __restrict__ xp,
    uint32_t row, uint32_t c, const uint32_t (&s)[2], bool valid, uint8_t* __restrict__ raw_g, uint64_t gblk, bool wb,
    uint64_t raw_bytes)
{
    const bool err = valid && quad_or(s[0] | s[1]) != 0u;
    if (!__builtin_amdgcn_ballot_w64(err))
        return 0u;
    const Gf gf { gfp };
    const uint16_t* t = (const uint16_t*)s12p + 256u * 8u * c; // state byte u = 8c + k
    uint32_t s12 = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        s12 ^= t[256 * k + ((s[k >> 2] >> (8 * (k & 3))) & 0xFFu)];
    s12 = quad_xor(s12);
    const uint32_t s1 = s12 & 0xFFu, s2 = s12 >> 8;
    const uint32_t l1 = gf.log(s1), l2 = gf.log(s2);
    uint32_t lx = l2 + 255u - l1;
    lx = lx >= 255u ? lx - 255u : lx;
    uint32_t le = l1 + 255u - lx;
    le = le >= 255u ? le - 255u : le;
    const uint2 xr = *(const uint2*)(xp + 32u * lx + 8u * c);
    const uint32_t xw[2] = { xr.x, xr.y };
    uint32_t bad = (s1 == 0u || s2 == 0u) ? 1u : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t x = (xw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const uint32_t rb = (s[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const uint32_t ev = x == 0xFFu ? 0u : gf.exp(le + x);
        bad |= ev != rb ? 1u : 0u;
    }
    const bool geo = err && quad_or(bad) == 0u;
    if (geo && c == 0)
        col::col_fix(lds, row, raw_g, gblk, wb, lx, gf.exp(le), raw_bytes);
    if (err && !geo)
        q_correct_general(lds, gfp, row, c, s[0], s[1], raw_g, gblk, wb, raw_bytes);
    return err ? 1u : 0u;
}

// register prefetch of a wave tile: image piece i = lane + 64 k from src + 16 i (every lane loads;
// pieces past the image re-read the last one, so pf stays in registers)
__device__ __forceinline__ void q_load(u32x4 (&pf)[KPQ], const uint8_t* __restrict__ src, uint32_t lane,
    [[maybe_unused]] const uint8_t* gbase, [[maybe_unused]] uint64_t extent)
{
#pragma unroll
    for (int k = 0; k < KPQ; ++k) {
        const uint32_t i = lane + 64u * (uint32_t)k;
        const uint32_t so = 16u * (i < (uint32_t)IMGQ_PIECES ? i : (uint32_t)IMGQ_PIECES - 1u);
        if (PPFS_DBG_OK(src + so, 16, gbase, extent))
            pf[k] = *(const u32x4*)(src + so);
    }
}
__device__ __forceinline__ void q_put(uint8_t* lds, uint32_t img, const u32x4 (&pf)[KPQ], uint32_t lane)
{
#pragma unroll
    for (int k = 0; k < KPQ; ++k) {
        const uint32_t i = lane + 64u * (uint32_t)k;
        if ((k + 1) * 64 <= IMGQ_PIECES || i < (uint32_t)IMGQ_PIECES)
            *(u32x4*)(lds + img + 16u * i) = pf[k];
    }
}

// LDS-DMA of an encode wave tile: image piece i = lane + 64 k at img + 16 i from the payloads
// (pair::img_src: the piece's codeword bytes, parity gaps filled after the remainder)
template <int T2>
__device__ __forceinline__ void q_dma_payload(uint32_t img_base, const uint8_t* __restrict__ src, uint32_t lane,
    [[maybe_unused]] const uint8_t* gbase, [[maybe_unused]] uint64_t extent)
{
#pragma unroll
    for (int k = 0; k < KPQ; ++k) {
        const uint32_t i = lane + 64u * (uint32_t)k;
        const int so = pair::img_src<T2>(i);
        if (((k + 1) * 64 <= IMGQ_PIECES || i < (uint32_t)IMGQ_PIECES) && so >= 0 && PPFS_DBG_OK(src + so, 16, gbase, extent))
            wg::dma16(src + so, __builtin_amdgcn_readfirstlane(img_base + 1024u * (uint32_t)k));
    }
}

// Encode (2t = 32) with four lanes per block: workgroup b's wave w takes 16-block wave tiles
// b NW + w + j S; a tile's payloads are LDS-DMA'd into the codeword layout of the wave's image, the
// remainder quarters written into the parity gaps, and the image stored as whole 16-byte pieces.
template <int T2, int NW, int NTST = 1>
__global__ __launch_bounds__(64 * NW, 1) void rs_bs4_encode_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables)
{
    static_assert(T2 == 32, "quad byte-slice path: 2t = 32");
    using L = RsPairLayout<T2>;
    constexpr int K = L::K;
    constexpr int BYTES = TAB_BYTES + NW * IMGQ + 64;
    static_assert(BYTES <= 163840, "one workgroup per CU: 160 KiB of LDS");
    __shared__ __attribute__((aligned(16))) uint8_t lds[BYTES];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    for (uint32_t p = tid; p < (uint32_t)TAB_BYTES / 16; p += 64u * NW)
        *(uint4*)(lds + OFF_TAB + 16 * p) = *(const uint4*)(tables + L::OFF_BS + 16 * p);
    __syncthreads();
    const QLane Ln = q_lane(lane);
    const uint32_t img = TAB_BYTES + wave * (uint32_t)IMGQ;
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(lds + img));
    const uint32_t row = img + 255u * Ln.blk;
    const uint64_t nfull = nblocks / TBQ, ntiles = (nblocks + TBQ - 1) / TBQ;
    const uint64_t S = (uint64_t)gridDim.x * NW;
    uint64_t t = (uint64_t)blockIdx.x * NW + wave;
    if (t < nfull)
        q_dma_payload<T2>(base, data + t * (TBQ * K), lane, data, nblocks * K);
    for (; t < nfull; t += S) {
        const uint64_t nx = t + S;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // this tile's DMA (and the last tile's stores)
        uint32_t s[2];
        q_remainder(s, lds, row + (uint32_t)T2, Ln);
        uint8_t* const gap = lds + row + 8u * Ln.c; // parity bytes [8c, 8c + 8) of the block
#pragma unroll
        for (int k = 0; k < 8; ++k)
            gap[k] = (uint8_t)(s[k >> 2] >> (8 * (k & 3)));
        wave_fence();
        uint8_t* dst = raw + t * (TBQ * 255);
#pragma unroll
        for (int k = 0; k < KPQ; ++k) {
            const uint32_t i = lane + 64u * (uint32_t)k;
            if (((k + 1) * 64 <= IMGQ_PIECES || i < (uint32_t)IMGQ_PIECES) && PPFS_DBG_OK(dst + 16u * i, 16, raw, nblocks * 255u))
                st_nt<NTST>(dst + 16u * i, *(const uint4*)(lds + img + 16u * i));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the image is read: free for the next DMA
        if (nx < nfull)
            q_dma_payload<T2>(base, data + nx * (TBQ * K), lane, data, nblocks * K);
    }
    if (t == nfull && nfull < ntiles) { // the one partial tile (nblocks % 16 blocks), staged byte by byte
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t nb = (uint32_t)(nblocks - t * TBQ);
        const uint8_t* src = data + t * (TBQ * K);
        if (!PPFS_DBG_OK(src, nb * (uint32_t)K, data, nblocks * K))
            return;
        for (uint32_t j = lane; j < nb * (uint32_t)K; j += 64u) {
            const uint32_t b = j / (uint32_t)K;
            lds[img + 255u * b + (uint32_t)T2 + (j - (uint32_t)K * b)] = src[j];
        }
        wave_fence();
        uint32_t s[2];
        q_remainder(s, lds, row + (uint32_t)T2, Ln);
        if (Ln.blk < nb) {
            uint8_t* const gap = lds + row + 8u * Ln.c;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                gap[k] = (uint8_t)(s[k >> 2] >> (8 * (k & 3)));
        }
        wave_fence();
        uint8_t* dst = raw + t * (TBQ * 255);
        const uint32_t nout = nb * 255u;
        for (uint32_t i = lane; 16u * i < nout; i += 64u) {
            const uint4 v = *(const uint4*)(lds + img + 16u * i);
            if (!PPFS_DBG_OK(dst + 16u * i, min(16u, nout - 16u * i), raw, nblocks * 255u))
                continue;
            if (16u * i + 16u <= nout)
                *(uint4*)(dst + 16u * i) = v;
            else
                st_bytes(dst + 16u * i, v, nout - 16u * i);
        }
    }
}

// LDS: the 64 KiB byte table | GF block | S12 table | x^p mod g rows | NW wave images | 64 B slack
// (the emission's second window runs past the last image)
template <int NW> struct QLds {
    static constexpr int OFF_GF = TAB_BYTES;
    static constexpr int OFF_S12 = OFF_GF + GF_BYTES;
    static constexpr int OFF_XP = OFF_S12 + 32 * 256 * 2;
    static constexpr int OFF_IMG = OFF_XP + 256 * 32;
    static constexpr int BYTES = OFF_IMG + NW * IMGQ + 64;
    static_assert(BYTES <= 163840, "one workgroup per CU: 160 KiB of LDS");
    static_assert(OFF_IMG % 16 == 0 && IMGQ % 16 == 0, "aligned images");
};

// Decode with status and write-back: workgroup b's wave w takes 16-block wave tiles b NW + w + j S
// (S = grid NW), the next tile prefetched into registers while this one is decoded.
template <int T2, int NW, int NTST = 1>
__global__ __launch_bounds__(64 * NW, 1) void rs_bs4_decode_kernel(uint8_t* __restrict__ raw,
    uint8_t* __restrict__ data, uint8_t* __restrict__ status, uint64_t nblocks, const uint8_t* __restrict__ tables,
    int write_back)
{
    static_assert(T2 == 32, "quad byte-slice path: 2t = 32");
    using L = RsPairLayout<T2>;
    using D = QLds<NW>;
    constexpr int K = L::K;
    constexpr int OUT_PIECES = TBQ * K / 16; // 223
    constexpr int KO = (OUT_PIECES + 63) / 64;
    static_assert(TBQ * K % 16 == 0, "whole output pieces per tile");
    __shared__ __attribute__((aligned(16))) uint8_t lds[D::BYTES];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    for (uint32_t p = tid; p < (uint32_t)TAB_BYTES / 16; p += 64u * NW)
        *(uint4*)(lds + OFF_TAB + 16 * p) = *(const uint4*)(tables + L::OFF_BS + 16 * p);
    for (uint32_t p = tid; p < (uint32_t)GF_BYTES / 16; p += 64u * NW)
        *(uint4*)(lds + D::OFF_GF + 16 * p) = *(const uint4*)(tables + L::OFF_GF + 16 * p);
    for (uint32_t p = tid; p < (uint32_t)L::S12_BYTES / 16; p += 64u * NW)
        *(uint4*)(lds + D::OFF_S12 + 16 * p) = *(const uint4*)(tables + L::OFF_S12 + 16 * p);
    for (uint32_t p = tid; p < 255u * 2u; p += 64u * NW)
        *(uint4*)(lds + D::OFF_XP + 16 * p) = *(const uint4*)(tables + L::OFF_XPM + 16 * p);
    __syncthreads();
    const uint8_t* const gfp = lds + D::OFF_GF;
    const uint8_t* const s12p = lds + D::OFF_S12;
    const uint8_t* const xpm = lds + D::OFF_XP;
    const QLane Ln = q_lane(lane);
    const bool wb = write_back != 0, want = data != nullptr;
    const uint32_t img = D::OFF_IMG + wave * (uint32_t)IMGQ;
    const uint32_t row = img + 255u * Ln.blk;
    const uint64_t nfull = nblocks / TBQ, ntiles = (nblocks + TBQ - 1) / TBQ;
    const uint64_t S = (uint64_t)gridDim.x * NW;
    uint64_t t = (uint64_t)blockIdx.x * NW + wave;
    u32x4 pf[KPQ];
    if (t < nfull) {
        q_load(pf, raw + t * (TBQ * 255), lane, raw, nblocks * 255u);
        q_put(lds, img, pf, lane);
    }
    for (; t < nfull; t += S) {
        const uint64_t nx = t + S;
        if (nx < nfull)
            q_load(pf, raw + nx * (TBQ * 255), lane, raw, nblocks * 255u);
        uint32_t s[2];
        q_cmodg(s, lds, row, Ln);
        const uint64_t gblk = t * TBQ + Ln.blk;
        const uint32_t st = q_correct(lds, gfp, s12p, xpm, row, Ln.c, s, true, raw, gblk, wb, nblocks * 255u);
        if (status && Ln.c == 0 && PPFS_DBG_OK(status + gblk, 1, status, nblocks))
            status[gblk] = (uint8_t)st;
        wave_fence(); // corrections patched into the image rows
        if (want) {
            uint8_t* dst = data + t * (TBQ * K);
            uint4 v[KO];
#pragma unroll
            for (int k = 0; k < KO; ++k) {
                uint32_t p = lane + 64u * (uint32_t)k;
                asm volatile("" : "+v"(p));
                v[k] = pair::pair_dec_piece<T2>(lds, img - pair::PAD, p < (uint32_t)OUT_PIECES ? p : 0u);
            }
#pragma unroll
            for (int k = 0; k < KO; ++k) {
                const uint32_t p = lane + 64u * (uint32_t)k;
                if (((k + 1) * 64 <= OUT_PIECES || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, data, nblocks * K))
                    st_nt<NTST>(dst + 16u * p, v[k]);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the image is read: free for the next tile
        if (nx < nfull)
            q_put(lds, img, pf, lane);
        wave_fence();
    }
    if (t == nfull && nfull < ntiles) { // the one partial tile (nblocks % 16 blocks), staged byte by byte
        const uint32_t nb = (uint32_t)(nblocks - t * TBQ);
        const uint8_t* src = raw + t * (TBQ * 255);
        if (!PPFS_DBG_OK(src, nb * 255u, raw, nblocks * 255u))
            return;
        for (uint32_t j = lane; j < nb * 255u; j += 64u)
            lds[img + j] = src[j];
        wave_fence();
        uint32_t s[2];
        q_cmodg(s, lds, row, Ln);
        const bool valid = Ln.blk < nb;
        const uint64_t gblk = t * TBQ + Ln.blk;
        const uint32_t st = q_correct(lds, gfp, s12p, xpm, row, Ln.c, s, valid, raw, gblk, wb, nblocks * 255u);
        if (status && valid && Ln.c == 0 && PPFS_DBG_OK(status + gblk, 1, status, nblocks))
            status[gblk] = (uint8_t)st;
        wave_fence();
        if (want) {
            uint8_t* dst = data + t * (TBQ * K);
            const uint32_t nout = nb * (uint32_t)K;
            for (uint32_t p = lane; 16u * p < nout; p += 64u) {
                const uint4 v = pair::pair_dec_piece<T2>(lds, img - pair::PAD, p);
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

} // namespace bs4
} // namespace ppfs
