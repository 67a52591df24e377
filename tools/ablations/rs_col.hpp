// ABLATION ONLY (not built into libppfs_ecc.so): include with -I paritypartyfs_amd/csrc.
#pragma once
// rs_col.hpp -- workgroup RS(255, 255-2t) encode / decode for gfx950 with 8 < 2t <= 32
// (cfg5: t = 16, RS(255, 223)).
//
// Reference semantics: lib/blockdevice/src/rs_block_device.cpp
//   encode  _encodeBlock :95-117   c(x) = m(x) x^2t + (m(x) x^2t mod g(x)); byte i = coeff of x^i,
//                                  parity in bytes [0,2t), payload in [2t,n)
//   decode  _fixBlockAndExtract :119-183 (syndromes :131-141, all-zero fast return :143-146,
//           Berlekamp-Massey :234-269, roots over all 255 field values :271-280, Omega :224-232,
//           Forney :210-222, whole-codeword write-back :175-180)
//
// Why a second workgroup design: rs_wg.hpp splits a row into four segments, one per wave, and
// moves the segment remainders into place with x^(64 s) map tables.  With a 2t-byte remainder
// those maps are 2t x 2 nibble tables of 2t-byte entries each -- 32 KiB per map at 2t = 32 -- and a
// lane's 32-byte state plus its 16 in-flight entries do not fit the register budget (the old
// lane-per-block kernel spilled).  Here the STATE is split instead:
//   - Tile = 64 blocks, one 256-thread workgroup; wave w owns blocks 16w..16w+15, four lanes per
//     block (a quad).  Lane c of a quad holds bytes [8c, 8c+8) of the block's 32-byte top-aligned
//     remainder state (coefficient q at byte 32 - 2t + q).
//   - Slicing-by-4 over byte-indexed tables: per 4 payload bytes, fold the state's top dword
//     (column 3, broadcast across the quad by a DPP quad_perm) into the chunk, shift the state up
//     one dword (column c <- column c-1, DPP quad_perm), and XOR in four table entries; each lane
//     reads only its 8-byte column of an entry (ds_read_b64).  Byte tables halve the LDS bytes of
//     nibble tables (32 B of table per payload byte), which is what bounds this kernel.
//   - No maps and no cross-wave combine: each quad runs its block's whole chain (56 / 64 steps).
//   - Tiles arrive by LDS-DMA double buffering and leave by 16-byte non-temporal stores assembled
//     from the LDS rows and parity slots, as in rs_wg.hpp (whose helpers this file reuses).
//   - Decode correction runs per quad, right after the quad's remainder (no workgroup barrier):
//     a single error is recognised from S_1, S_2 and one row of the XP table (col_correct); other
//     blocks compute all 2t syndromes (8 per lane, log / exp) and run the reference's BM / roots /
//     Forney (rs_fast.hpp) in lane 0, out of line (col_correct_general).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf_common.hpp"
#include "rs_fast.hpp"
#include "rs_layout.hpp"
#include "rs_wg.hpp"
#include "rs_emit.hpp"

namespace ppfs {
// Column-split RS path (rs_col.hpp), 8 < 2t <= 32: the remainder is a 32-byte top-aligned state
// (coefficient q at byte 32 - 2t + q), four lanes per block each holding one 8-byte column.
//   SL   slicing-by-4, byte-indexed: table k, value v -> v * x^(2t+k) mod g as a 32-byte entry
//        (4 tables x 256 x 32 B); lane c reads bytes [8c, 8c+8) of an entry
//   GF   the 1 KiB EXP2 / LOG / QS block of gf_common.hpp
//   XP   decode only: row p (32 B, state layout) = LOG of each coefficient of x^(p+2t) mod g, 0xFF
//        for a zero coefficient -- the remainder of a single error e at byte p is e * row p,
//        which is how the decoder confirms the single-error case (see rs_col.hpp)
template <int T2> struct RsColLayout {
    static_assert(T2 > 8 && T2 <= 32 && (T2 % 2) == 0, "column RS path: 2t in (8, 32]");
    static constexpr int N = 255, K = N - T2;
    static constexpr int ES = 32;
    static constexpr int TBL = 256 * ES;
    static constexpr int OFF_SL = 0;
    static constexpr int OFF_GF = OFF_SL + 4 * TBL;
    static constexpr int OFF_XP = OFF_GF + GF_BYTES;
    static constexpr int ENC_BYTES = OFF_GF;              // what encode loads
    static constexpr int TABLE_BYTES = OFF_XP + 255 * 32; // what decode loads
    static constexpr int POFF = 32 - T2; // state byte of parity / remainder coefficient 0
};

constexpr int rs_col_table_bytes() { return 4 * 256 * 32 + GF_BYTES + 255 * 32; }


namespace col {

using wg::barrier_lds;
using wg::bfi;
using wg::dma_tile;
using wg::M128;
using wg::range_mask;
using wg::st_bytes;
using wg::st_nt;
using wg::stage_bytes;

constexpr int NTHR = 256;                // threads per workgroup

// quad_perm DPP controls
constexpr int QP_BCAST3 = 0xFF; // [3,3,3,3]: column 3 to every lane of the quad
constexpr int QP_SHIFT = 0x90;  // [0,0,1,2]: column c-1 to lane c (lane 0 masked off by the caller)

__device__ __forceinline__ uint32_t quad_bcast3(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, QP_BCAST3, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t quad_shift(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, QP_SHIFT, 0xF, 0xF, false);
}

// table entry column of byte K of f: 8 bytes at tb + K * 8 KiB + 32 * byte
template <int K> __device__ __forceinline__ uint2 col_entry(const uint8_t* tb, uint32_t f)
{
    const uint32_t v = (f >> (8 * K)) & 0xFFu;
    return *(const uint2*)(tb + K * 8192 + v * 32u);
}

// Remainder column c of a LEN-byte row at LDS byte `row`: (lo, hi) = state bytes [8c, 8c+8) of
// sum_j B[j] x^(2t + j) mod g.  tb = SL tables + 8c; cmask = all ones for c > 0, else 0.
template <int LEN>
__device__ __forceinline__ void col_remainder(uint32_t& lo_out, uint32_t& hi_out, const uint8_t* lds, uint32_t row,
    const uint8_t* tb, uint32_t cmask)
{
    constexpr int NC = (LEN + 3) / 4;
    constexpr int TOPN = LEN - 4 * (NC - 1);
    const uint32_t sh = (row & 3u) * 8u;
    const uint32_t* w = (const uint32_t*)(lds + (row & ~3u));
    uint32_t lo = 0, hi = 0;
    uint32_t up = w[NC];
#pragma unroll
    for (int j = NC - 1; j >= 0; --j) {
        const uint32_t dn = w[j];
        uint32_t f = __builtin_amdgcn_alignbit(up, dn, sh); // payload bytes 4j .. 4j+3
        up = dn;
        if (j == NC - 1) {
            if constexpr (TOPN < 4)
                f &= (1u << (8 * TOPN)) - 1u;
            const uint2 e0 = col_entry<0>(tb, f), e1 = col_entry<1>(tb, f);
            const uint2 e2 = col_entry<2>(tb, f), e3 = col_entry<3>(tb, f);
            lo = xor3(e0.x, e1.x, e2.x) ^ e3.x;
            hi = xor3(e0.y, e1.y, e2.y) ^ e3.y;
        } else {
            f ^= quad_bcast3(hi);                        // fold the top 4 coefficients
            const uint32_t shl = quad_shift(hi) & cmask; // state * x^4: dword d <- dword d-1
            const uint2 e0 = col_entry<0>(tb, f), e1 = col_entry<1>(tb, f);
            const uint2 e2 = col_entry<2>(tb, f), e3 = col_entry<3>(tb, f);
            const uint32_t nhi = xor3(lo, e0.y, e1.y) ^ xor3(e2.y, e3.y, 0u);
            lo = xor3(shl, e0.x, e1.x) ^ xor3(e2.x, e3.x, 0u);
            hi = nhi;
        }
    }
    lo_out = lo;
    hi_out = hi;
}


__device__ __forceinline__ uint32_t quad_xor(uint32_t v)
{
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false); // quad_perm [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false); // quad_perm [2,3,0,1]
    return v;
}
__device__ __forceinline__ uint32_t quad_or(uint32_t v)
{
    v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    return v;
}


// General correction (2+ errors; out of line so its registers do not weigh on the streaming path).
// Called by all four lanes of a quad whose block is not a single error: lane c computes S_i for
// i = 8c+1 .. 8c+8 (S_i = r'(a^i) a^(-2t i), rs_block_device.cpp:131-141) into the block's
// syndrome slot; lane 0 then runs the reference's BM / roots / Forney (rs_fast.hpp).
template <int T2>
__device__ __noinline__ void col_correct_general(uint8_t* lds, uint32_t row, uint32_t slot, uint32_t syn, uint32_t c,
    uint8_t* __restrict__ raw_g, uint64_t gblk, bool wb)
{
    using L = RsColLayout<T2>;
    const Gf gf { lds + L::OFF_GF };
    const uint4 r0 = *(const uint4*)(lds + slot), r1 = *(const uint4*)(lds + slot + 16);
    const uint32_t rw[8] = { r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w };
    uint32_t sw[2] = { 0u, 0u };
#pragma unroll
    for (int ii = 0; ii < 8; ++ii) {
        const uint32_t i = 8u * c + 1u + (uint32_t)ii;
        uint32_t e = (255u * 32u - i * (uint32_t)T2) % 255u; // i (q - 2t) mod 255 at q = 0
        uint32_t s = 0;
#pragma unroll
        for (int q = 0; q < T2; ++q) {
            constexpr int P0 = 32 - T2;
            const uint32_t rv = (rw[(P0 + q) >> 2] >> (8 * ((P0 + q) & 3))) & 0xFFu;
            const uint32_t v = gf.exp(gf.log(rv) + e);
            s ^= rv ? v : 0u;
            e += i;
            e = e >= 255u ? e - 255u : e;
        }
        sw[ii >> 2] |= (i <= (uint32_t)T2 ? s : 0u) << (8 * (ii & 3));
    }
    *(uint2*)(lds + syn + 8u * c) = make_uint2(sw[0], sw[1]);
    wave_fence();
    if (c == 0) {
        uint32_t S[T2];
        const uint4 s0 = *(const uint4*)(lds + syn), s1 = *(const uint4*)(lds + syn + 16);
        const uint32_t sw8[8] = { s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w };
#pragma unroll
        for (int i = 0; i < T2; ++i)
            S[i] = (sw8[i >> 2] >> (8 * (i & 3))) & 0xFFu;
        rs_correct_general<T2>(S, gf, [&](uint32_t pos, uint32_t ev) { col_fix(lds, row, raw_g, gblk, wb, pos, ev); });
    }
}

// Decode correction for the quad's block; (lo, hi) = the lane's column of r' = x^2t c(x) mod g.
// Single-error fast path: S_1 and S_2 from the quad (each lane its 8 coefficients, DPP XOR), the
// candidate X = S_2 / S_1 (position p = LOG X) and e = S_1 / X, confirmed iff r' == e * (x^(p+2t)
// mod g) (the XP row).  That equality holds exactly when every S_i = e X^i, i.e. when the
// syndromes are geometric -- the case in which the reference's BM returns 1 + X x and corrects
// byte p by e (rs_fast.hpp rs_geometric).  Anything else takes col_correct_general.
template <int T2>
__device__ __forceinline__ uint32_t col_correct(uint8_t* lds, uint32_t row, uint32_t slot, uint32_t syn, uint32_t c,
    uint32_t lo, uint32_t hi, bool valid, uint8_t* __restrict__ raw_g, uint64_t gblk, bool wb)
{
    using L = RsColLayout<T2>;
    const bool err = valid && quad_or(lo | hi) != 0u;
    if (!__builtin_amdgcn_ballot_w64(err))
        return 0u;
    const Gf gf { lds + L::OFF_GF };
    // state byte 8c+k is coefficient q = 8c+k-POFF; exponent i (q - 2t) = i (8c + k - 32)
    uint32_t rb[8], s1 = 0, s2 = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        rb[k] = ((k < 4 ? lo : hi) >> (8 * (k & 3))) & 0xFFu;
        const uint32_t lb = gf.log(rb[k]), u = 8u * c + (uint32_t)k;
        const uint32_t v1 = gf.exp(lb + u + 223u), v2 = gf.exp(lb + 2u * u + 191u);
        s1 ^= rb[k] ? v1 : 0u;
        s2 ^= rb[k] ? v2 : 0u;
    }
    s1 = quad_xor(s1);
    s2 = quad_xor(s2);
    const uint32_t l1 = gf.log(s1), l2 = gf.log(s2);
    uint32_t lx = l2 + 255u - l1;
    lx = lx >= 255u ? lx - 255u : lx;
    uint32_t le = l1 + 255u - lx;
    le = le >= 255u ? le - 255u : le;
    const uint2 xr = *(const uint2*)(lds + L::OFF_XP + 32u * lx + 8u * c);
    uint32_t bad = (s1 == 0u || s2 == 0u) ? 1u : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t x = ((k < 4 ? xr.x : xr.y) >> (8 * (k & 3))) & 0xFFu;
        const uint32_t ev = x == 0xFFu ? 0u : gf.exp(le + x);
        bad |= ev != rb[k] ? 1u : 0u;
    }
    const bool geo = err && quad_or(bad) == 0u;
    if (geo && c == 0)
        col_fix(lds, row, raw_g, gblk, wb, lx, gf.exp(le));
    if (err && !geo)
        col_correct_general<T2>(lds, row, slot, syn, c, raw_g, gblk, wb);
    return err ? 1u : 0u;
}

// LDS plan: tables | parity/remainder slots (65 x 32 B + slack) | syndrome slots | 2 tile buffers
template <int T2, bool DEC> struct Lds {
    using L = RsColLayout<T2>;
    static constexpr int TBL = DEC ? L::TABLE_BYTES : L::ENC_BYTES;
    static constexpr int OFF_PAR = TBL;
    static constexpr int OFF_SYN = OFF_PAR + 66 * 32;
    static constexpr int OFF_BUF = OFF_SYN + (DEC ? TB * 32 : 0);
    static constexpr int BYTES = OFF_BUF + 2 * BUF;
    static_assert(OFF_BUF % 16 == 0 && L::TABLE_BYTES % 16 == 0 && BUF % 16 == 0, "aligned buffers");
};

template <int T2, bool DEC> constexpr int lds_bytes() { return Lds<T2, DEC>::BYTES; }

// Quad of a thread: block 16 w + lane / 4 of the tile, column lane % 4
struct Quad {
    uint32_t blk, c, cmask;
};
__device__ __forceinline__ Quad quad_of(uint32_t wave, uint32_t lane)
{
    const uint32_t c = lane & 3u;
    return Quad { 16u * wave + (lane >> 2), c, c ? ~0u : 0u };
}

template <int T2, int WPC = 2, int NTST = 1>
__global__ __launch_bounds__(256, WPC) void rs_col_encode_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables)
{
    using L = RsColLayout<T2>;
    using D = Lds<T2, false>;
    constexpr int LDS_ALLOC = wg::lds_alloc<D::BYTES, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * K / 16;
    constexpr int OUT_PIECES = TB * 255 / 16; // 1020
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const Quad qd = quad_of(wave, lane);
    const uint8_t* tb = lds + L::OFF_SL + 8u * qd.c;
    for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += NTHR)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    uint64_t t = blockIdx.x;
    uint32_t cur = 0;
    if (t < nfull)
        dma_tile<IN_PIECES>(lds + D::OFF_BUF + PAD, data + t * (TB * K), tid);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (; t < nfull; t += gridDim.x) {
        barrier_lds(); // A: tile t in LDS, the last tile's emission reads done
        const uint32_t buf = D::OFF_BUF + cur * BUF;
        const uint64_t nx = t + gridDim.x;
        if (nx < nfull)
            dma_tile<IN_PIECES>(lds + D::OFF_BUF + (cur ^ 1u) * BUF + PAD, data + nx * (TB * K), tid);
        uint32_t lo, hi;
        col_remainder<K>(lo, hi, lds, buf + PAD + (uint32_t)K * qd.blk, tb, qd.cmask);
        *(uint2*)(lds + D::OFF_PAR + 32u * qd.blk + 8u * qd.c) = make_uint2(lo, hi);
        barrier_lds(); // B: parity slots complete
        uint8_t* dst = raw + t * (TB * 255);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = tid + 256u * k;
            const uint4 o = col_enc_piece<T2>(lds, buf, D::OFF_PAR, p);
            if (k < 3 || p < (uint32_t)OUT_PIECES)
                st_nt<NTST>(dst + 16u * p, o);
        }
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); // next tile's DMA landed; stores may fly
        cur ^= 1u;
    }
    if (t == nfull && nfull < ntiles) {
        // the one partial tile (nblocks % 64 blocks)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint32_t buf = D::OFF_BUF + cur * BUF;
        stage_bytes(lds + buf + PAD, data + t * (TB * K), nb * K, tid);
        barrier_lds();
        uint32_t lo, hi;
        col_remainder<K>(lo, hi, lds, buf + PAD + (uint32_t)K * qd.blk, tb, qd.cmask);
        *(uint2*)(lds + D::OFF_PAR + 32u * qd.blk + 8u * qd.c) = make_uint2(lo, hi);
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

template <int T2, int WPC = 2, int NTST = 1>
__global__ __launch_bounds__(256, WPC) void rs_col_decode_kernel(uint8_t* __restrict__ raw,
    uint8_t* __restrict__ data, uint8_t* __restrict__ status, uint64_t nblocks, const uint8_t* __restrict__ tables,
    int write_back)
{
    using L = RsColLayout<T2>;
    using D = Lds<T2, true>;
    constexpr int LDS_ALLOC = wg::lds_alloc<D::BYTES, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * 255 / 16; // 1020
    constexpr int OUT_PIECES = TB * K / 16;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const Quad qd = quad_of(wave, lane);
    const uint8_t* tb = lds + L::OFF_SL + 8u * qd.c;
    const bool wb = write_back != 0, want = data != nullptr;
    const uint32_t slot = D::OFF_PAR + 32u * qd.blk, syn = D::OFF_SYN + 32u * qd.blk;
    for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += NTHR)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    uint64_t t = blockIdx.x;
    uint32_t cur = 0;
    if (t < nfull)
        dma_tile<IN_PIECES>(lds + D::OFF_BUF + PAD, raw + t * (TB * 255), tid);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (; t < nfull; t += gridDim.x) {
        barrier_lds(); // A
        const uint32_t buf = D::OFF_BUF + cur * BUF;
        const uint64_t nx = t + gridDim.x;
        if (nx < nfull)
            dma_tile<IN_PIECES>(lds + D::OFF_BUF + (cur ^ 1u) * BUF + PAD, raw + nx * (TB * 255), tid);
        const uint32_t row = buf + PAD + 255u * qd.blk;
        uint32_t lo, hi;
        col_remainder<255>(lo, hi, lds, row, tb, qd.cmask);
        *(uint2*)(lds + slot + 8u * qd.c) = make_uint2(lo, hi); // read only by the general path
        wave_fence(); // the quad's slot is complete (same wave)
        const uint32_t st = col_correct<T2>(lds, row, slot, syn, qd.c, lo, hi, true, raw, t * TB + qd.blk, wb);
        if (status && qd.c == 0)
            status[t * TB + qd.blk] = (uint8_t)st;
        barrier_lds(); // C: corrections patched into the LDS rows
        if (want) {
            uint8_t* dst = data + t * (TB * K);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t p = tid + 256u * k;
                const uint4 o = col_dec_piece<T2>(lds, buf, p);
                if (k < 3 || p < (uint32_t)OUT_PIECES)
                    st_nt<NTST>(dst + 16u * p, o);
            }
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        cur ^= 1u;
    }
    if (t == nfull && nfull < ntiles) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint32_t buf = D::OFF_BUF + cur * BUF;
        stage_bytes(lds + buf + PAD, raw + t * (TB * 255), nb * 255u, tid);
        barrier_lds();
        const uint32_t row = buf + PAD + 255u * qd.blk;
        uint32_t lo, hi;
        col_remainder<255>(lo, hi, lds, row, tb, qd.cmask);
        *(uint2*)(lds + slot + 8u * qd.c) = make_uint2(lo, hi);
        wave_fence();
        const bool valid = qd.blk < nb;
        const uint32_t st = col_correct<T2>(lds, row, slot, syn, qd.c, lo, hi, valid, raw, t * TB + qd.blk, wb);
        if (status && valid && qd.c == 0)
            status[t * TB + qd.blk] = (uint8_t)st;
        barrier_lds();
        if (want) {
            uint8_t* dst = data + t * (TB * K);
            const uint32_t nout = nb * (uint32_t)K;
            for (uint32_t p = tid; 16u * p < nout; p += NTHR) {
                const uint4 v = col_dec_piece<T2>(lds, buf, p);
                if (16u * p + 16u <= nout)
                    *(uint4*)(dst + 16u * p) = v;
                else
                    st_bytes(dst + 16u * p, v, nout - 16u * p);
            }
        }
    }
}

} // namespace col
} // namespace ppfs
