#pragma once
// rs_wg.hpp -- workgroup-cooperative Reed-Solomon RS(255, 255-2t) encode / decode for gfx950, 2t <= 8.
//
// Reference semantics: lib/blockdevice/src/rs_block_device.cpp
//   encode  _encodeBlock :95-117   c(x) = m(x) x^2t + (m(x) x^2t mod g(x)); byte i = coeff of x^i,
//                                  parity in bytes [0,2t), payload in [2t,n)
//   decode  _fixBlockAndExtract :119-183 (syndromes :131-141, all-zero fast return :143-146,
//           Berlekamp-Massey :234-269, roots over all 255 field values :271-280, Omega :224-232,
//           Forney :210-222, whole-codeword write-back :175-180)
//
// Work decomposition (one 256-thread workgroup = 4 waves per 64-block tile):
//   - The tile's packed rows (64 x 249 B payloads or 64 x 255 B codewords, contiguous in HBM) are
//     brought into LDS by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave-instruction, 4 per
//     lane), double-buffered: tile i+1 is in flight while tile i is computed.  Waits are counted
//     (vmcnt) and the barriers are raw s_barrier, so the prefetch stays in flight across them.
//   - Phase 1, remainder: lane l of wave s owns block l and computes the remainder of bytes
//     [64s, 64s+64) of its row (slicing-by-8 over nibble tables), then moves it to its place with
//     the x^(64 s) map, and XOR-accumulates it into the block's 8-byte slot in LDS (ds_xor_b64).
//     The four segment chains run in parallel in four waves: 8 slicing steps per lane, not 32.
//   - Phase 2 (decode only, wave 0): blocks with a non-zero remainder run the reference's
//     correction (syndromes by nibble tables, single-error closed form, else BM / roots / Forney)
//     and patch their bytes in the LDS tile and, with write-back, in HBM.
//   - Phase 3, emission: every thread assembles 16-byte pieces of the OUTPUT tile straight from
//     the LDS input rows (funnel shifts; parity bytes inserted at block starts) and stores them
//     with 16-byte non-temporal stores.  No output staging in LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dbg.hpp"
#include "gf_common.hpp"
#include "rs_fast.hpp"
#include "rs_layout.hpp"
#include "srv_device.hpp"

namespace ppfs {
namespace wg {

constexpr int TB = 64;      // blocks per tile
constexpr int NTHR = 256;   // threads per workgroup
constexpr int PAD = 16;     // front pad of a tile buffer (emission reads up to 2t bytes before row 0)
constexpr int BUF = 16368;  // PAD + 64*255 + 32: decode emission reads up to 28 B past a piece start


__device__ __forceinline__ void barrier_lds()
{
    // every wave's LDS ops done, then the workgroup barrier; no vmcnt: LDS-DMA may stay in flight
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One LDS-DMA wave-instruction (global_load_lds_dwordx4: 16 B per lane to lds_base + 16 * lane).
// Issued from inline asm on purpose: hipcc tracks a builtin LDS-DMA and then waits vmcnt(0) before
// every later LDS read, which would drain the next tile's prefetch.  The waits for these loads are
// the explicit counted vmcnt in the kernels.  (M0 write -> LDS-DMA needs one wait state.)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm" // m0 is reserved; nothing else in these kernels uses it
__device__ __forceinline__ void dma16(const uint8_t* g, uint32_t lds_base)
{
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g),
                 "s"(lds_base)
                 : "memory", "m0");
}
#pragma clang diagnostic pop

__device__ __forceinline__ uint32_t lds_addr(const uint8_t* p)
{
    return (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)p;
}

// LDS-DMA of NPIECE 16-byte pieces: piece p = tid + 256k lands at dst + 16p (wave-uniform base
// dst + 1024 * (4k + wave), + 16 * lane implicit).  Exactly 4 instructions per wave.
// (base, extent): the global buffer the tile lies in (PPFS_ECC_DEBUG bounds checks, dbg.hpp)
template <int NPIECE>
__device__ __forceinline__ void dma_tile(uint8_t* dst, const uint8_t* __restrict__ src, uint32_t tid,
    [[maybe_unused]] const uint8_t* base, [[maybe_unused]] uint64_t extent)
{
    static_assert(NPIECE > 768 && NPIECE <= 1024, "4 pieces per thread, every wave active in each");
    const uint32_t lbase = __builtin_amdgcn_readfirstlane(lds_addr(dst) + (tid & ~63u) * 16u);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t p = tid + 256u * k;
        if ((k < 3 || p < (uint32_t)NPIECE) && PPFS_DBG_OK(src + (size_t)p * 16, 16, base, extent))
            dma16(src + (size_t)p * 16, lbase + 4096u * k);
    }
}

__device__ __forceinline__ uint2 ld8(const uint8_t* p) { return *(const uint2*)p; }

// (x >> 8k) & 0x78: byte k of x, masked to a nibble * 8 (one v_and_b32_sdwa for k > 0)
__device__ __forceinline__ uint32_t sel78(uint32_t x, int k)
{
    uint32_t r;
    switch (k & 3) {
    case 0:
        return x & 0x78u;
    case 1:
        asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
            : "=v"(r) : "v"(x), "s"(0x78u));
        return r;
    case 2:
        asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
            : "=v"(r) : "v"(x), "s"(0x78u));
        return r;
    default:
        asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
            : "=v"(r) : "v"(x), "s"(0x78u));
        return r;
    }
}

// s ^= XOR of N 8-byte entries
template <int N> __device__ __forceinline__ void xor_entries(uint32_t (&s)[2], const uint2 (&e)[N])
{
    uint32_t a = s[0], b = s[1];
    int i = 0;
#pragma unroll
    for (; i + 1 < N; i += 2) {
        a = xor3(a, e[i].x, e[i + 1].x);
        b = xor3(b, e[i].y, e[i + 1].y);
    }
    if (i < N) {
        a ^= e[i].x;
        b ^= e[i].y;
    }
    s[0] = a;
    s[1] = b;
}

// One slicing step: s <- (s x^8 + sum_i byte_i x^(2t+i)) mod g, top-aligned 8-byte state.
// NB = bytes of the chunk that may be non-zero when FIRST (state still zero).
template <bool FIRST, int NB>
__device__ __forceinline__ void step8(uint32_t (&s)[2], uint32_t lo, uint32_t hi, const uint8_t* sl)
{
    if constexpr (!FIRST) {
        lo ^= s[0];
        hi ^= s[1];
    }
    constexpr int NL = FIRST ? NB : 8;
    const uint32_t ll = lo << 3, lh = lo >> 1, hl = hi << 3, hh = hi >> 1;
    uint2 e[2 * NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        const uint32_t xl = i < 4 ? ll : hl, xh = i < 4 ? lh : hh;
        e[2 * i] = ld8(sl + (2 * i) * 128 + sel78(xl, i));
        e[2 * i + 1] = ld8(sl + (2 * i + 1) * 128 + sel78(xh, i));
    }
    // the whole 8-byte state was folded into the chunk: the new state is the XOR of the entries
    s[0] = 0;
    s[1] = 0;
    xor_entries<2 * NL>(s, e);
}

// The same step through the 5-bit field tables (rs_layout.hpp SL5): field i = bits [5i, 5i+5) of the
// 64-bit chunk lo | hi << 32 (field 6 straddles the two words, field 12 has 4 bits)
template <bool FIRST, int NB>
__device__ __forceinline__ void step13(uint32_t (&s)[2], uint32_t lo, uint32_t hi, const uint8_t* t5)
{
    if constexpr (!FIRST) {
        lo ^= s[0];
        hi ^= s[1];
    }
    constexpr int NF = FIRST ? (8 * NB + 4) / 5 : 13;
    uint2 e[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        uint32_t f;
        if (5 * i + 5 <= 32)
            f = __builtin_amdgcn_ubfe(lo, 5 * i, 5);
        else if (5 * i >= 32)
            f = __builtin_amdgcn_ubfe(hi, 5 * i - 32, 5);
        else
            f = __builtin_amdgcn_alignbit(hi, lo, 30) & 31u;
        e[i] = ld8(t5 + i * 256 + f * 8u);
    }
    s[0] = 0;
    s[1] = 0;
    xor_entries<NF>(s, e);
}

// r = sum_j B[SEG S + j] x^(2t + j) mod g over segment S (SEG bytes) of a LEN-byte row at LDS byte `row`.
// XOFF > 0 (the SLX layout, round 3): the LAST slicing step (bottom chunk) reads the segment's own
// tables at LDS byte XOFF + 2048 (S - 1), SL with x^(64 S) folded in.  That step maps the whole
// folded state, so the result is already r x^(64 S) mod g: no x^(64 S) map round after the chain.
// T5: the 5-bit field tables, SL5 at LDS 0 and the segment's SLX5 at XOFF + SL5_BYTES (S - 1)
template <int T2, int LEN, int S, int SEG = 64, int XOFF = 0, bool T5 = false>
__device__ __forceinline__ void seg_remainder(uint32_t (&s)[2], const uint8_t* lds, uint32_t row)
{
    constexpr int LO = SEG * S;
    constexpr int LS = (LEN - LO) < SEG ? (LEN - LO) : SEG;
    constexpr int NC = (LS + 7) / 8;
    constexpr int TOPN = LS - 8 * (NC - 1);
    constexpr int NR = 2 * NC + 1;
    const uint32_t a0 = row + LO;
    const uint32_t sh = (a0 & 3u) * 8u;
    const uint32_t* w = (const uint32_t*)(lds + (a0 & ~3u));
    uint32_t R[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q)
        R[q] = w[q];
#pragma unroll
    for (int c = NC - 1; c >= 0; --c) {
        constexpr int XSTRIDE = T5 ? RsWgLayout<T2>::SL5_BYTES : 2048;
        const uint8_t* sl = (XOFF > 0 && S > 0 && c == 0) ? lds + XOFF + XSTRIDE * (S > 0 ? S - 1 : 0)
                                                          : lds + (T5 ? 0 : RsWgLayout<T2>::OFF_SL);
        uint32_t lo = __builtin_amdgcn_alignbit(R[2 * c + 1], R[2 * c], sh);
        uint32_t hi = __builtin_amdgcn_alignbit(R[2 * c + 2], R[2 * c + 1], sh);
        if (c == NC - 1) {
            if constexpr (TOPN < 4) {
                lo &= (1u << (8 * TOPN)) - 1u;
                hi = 0;
            } else if constexpr (TOPN == 4) {
                hi = 0;
            } else if constexpr (TOPN < 8) {
                hi &= (1u << (8 * (TOPN - 4))) - 1u;
            }
            if constexpr (T5)
                step13<true, TOPN>(s, lo, hi, sl);
            else
                step8<true, TOPN>(s, lo, hi, sl);
        } else {
            if constexpr (T5)
                step13<false, 8>(s, lo, hi, sl);
            else
                step8<false, 8>(s, lo, hi, sl);
        }
    }
}

// s <- s(x) * x^(SEG S) mod g through the segment's map tables (S >= 1; SEG = 64, or 32 for the
// 8-wave encode, which copies MAP32 to OFF_MAP)
template <int T2, int S> __device__ __forceinline__ void seg_map(uint32_t (&s)[2], const uint8_t* lds)
{
    using L = RsWgLayout<T2>;
    const uint8_t* mp = lds + L::OFF_MAP + (S - 1) * L::MAP_STRIDE;
    uint2 e[2 * T2];
#pragma unroll
    for (int q = 0; q < T2; ++q) {
        const int P = 8 - T2 + q;
        const uint32_t x = s[P >> 2];
        e[2 * q] = ld8(mp + (2 * q) * 128 + sel78(x << 3, P & 3));
        e[2 * q + 1] = ld8(mp + (2 * q + 1) * 128 + sel78(x >> 1, P & 3));
    }
    s[0] = 0;
    s[1] = 0;
    xor_entries<2 * T2>(s, e);
}

// Block (row of the tile) owned by a lane in phases 1 and 2: lanes 0-31 take the even rows, 32-63
// the odd ones.  Rows sit 255 (or 249) bytes apart, so consecutive rows start in nearly the same
// LDS bank; a 32-lane half reading every other row hits each bank at most twice (4-way -> 2-way
// for 255-byte rows).
__device__ __forceinline__ uint32_t lane_row(uint32_t lane) { return ((lane & 31u) << 1) | (lane >> 5); }

// Phase 1 for this wave's segment of block `blk`: XOR its remainder into the block's slot
template <int T2, int LEN, int NMAP = 3, int XOFF = 0, bool T5 = false>
__device__ __forceinline__ void phase_remainder_row(uint8_t* lds, uint32_t row, uint32_t par, uint32_t wave, uint32_t blk);

// NMAP = x^(64 s) maps in LDS: 3 (one per segment), or 2 (x^64, x^128; segment 3 applies both,
// which frees 2t x 256 B of LDS for the compact encode layout); 1 = no maps: the SLX last-step
// tables at LDS byte XOFF (seg_remainder)
template <int T2, int LEN, int NMAP = 3, int XOFF = 0, bool T5 = false>
__device__ __forceinline__ void phase_remainder(uint8_t* lds, uint32_t buf, uint32_t par, uint32_t wave, uint32_t blk)
{
    phase_remainder_row<T2, LEN, NMAP, XOFF, T5>(lds, buf + PAD + (uint32_t)LEN * blk, par, wave, blk);
}

// the same for a LEN-byte row at LDS byte `row` (any row layout)
template <int T2, int LEN, int NMAP, int XOFF, bool T5>
__device__ __forceinline__ void phase_remainder_row(uint8_t* lds, uint32_t row, uint32_t par, uint32_t wave, uint32_t blk)
{
    static_assert(!T5 || NMAP == 1, "5-bit tables: the SLX layout");
    static_assert(NMAP == 1 || NMAP == 2 || NMAP == 3, "x^(64 s) maps, or SLX tables");
    static_assert(NMAP != 1 || XOFF > 0, "SLX tables need their LDS offset");
    uint32_t s[2];
    if constexpr (NMAP == 1) {
        switch (wave) {
        case 0:
            seg_remainder<T2, LEN, 0, 64, XOFF, T5>(s, lds, row);
            break;
        case 1:
            seg_remainder<T2, LEN, 1, 64, XOFF, T5>(s, lds, row);
            break;
        case 2:
            seg_remainder<T2, LEN, 2, 64, XOFF, T5>(s, lds, row);
            break;
        default:
            seg_remainder<T2, LEN, 3, 64, XOFF, T5>(s, lds, row);
            break;
        }
    } else switch (wave) {
    case 0:
        seg_remainder<T2, LEN, 0>(s, lds, row);
        break;
    case 1:
        seg_remainder<T2, LEN, 1>(s, lds, row);
        seg_map<T2, 1>(s, lds);
        break;
    case 2:
        seg_remainder<T2, LEN, 2>(s, lds, row);
        seg_map<T2, 2>(s, lds);
        break;
    default:
        seg_remainder<T2, LEN, 3>(s, lds, row);
        if constexpr (NMAP == 3) {
            seg_map<T2, 3>(s, lds);
        } else {
            seg_map<T2, 1>(s, lds); // x^192 = x^64 x^128
            seg_map<T2, 2>(s, lds);
        }
        break;
    }
    const uint64_t v = ((uint64_t)s[1] << 32) | s[0];
    __hip_atomic_fetch_xor((unsigned long long*)(lds + par + 8u * blk), (unsigned long long)v, __ATOMIC_RELAXED,
        __HIP_MEMORY_SCOPE_WORKGROUP);
}

// bytes [lo, hi) of a 16-byte piece as a 128-bit mask (lo <= hi, both in [0, 16])
struct M128 {
    uint64_t lo, hi;
};
__device__ __forceinline__ uint64_t ones_below(uint32_t nbytes) // bytes [0, n) of a u64, n in [0, 8]
{
    return nbytes >= 8 ? ~0ull : ((1ull << (8 * nbytes)) - 1ull);
}
__device__ __forceinline__ M128 range_mask(uint32_t lo, uint32_t hi)
{
    const uint32_t l0 = lo < 8 ? lo : 8, h0 = hi < 8 ? hi : 8;
    const uint32_t l1 = lo > 8 ? lo - 8 : 0, h1 = hi > 8 ? hi - 8 : 0;
    return M128 { ones_below(h0) & ~ones_below(l0), ones_below(h1 < 8 ? h1 : 8) & ~ones_below(l1 < 8 ? l1 : 8) };
}
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }

// The emission's unaligned LDS window: the n dwords at LDS byte S & ~3 (S any byte).  (Round 3: 8-byte
// aligned reads with a dword select measured slower, emission 1,747 vs 1,573 cycles per tile.)
template <int N> __device__ __forceinline__ void lds_window(uint32_t (&d)[N], const uint8_t* lds, uint32_t S)
{
    const uint32_t* w = (const uint32_t*)(lds + (S & ~3u));
#pragma unroll
    for (int i = 0; i < N; ++i)
        d[i] = w[i];
}

// Encode emission: 16 bytes of the codeword tile at piece p, from the LDS payload rows and the
// combined parity slots.  Codeword byte j of block b = j / 255 (off = j % 255): parity byte off if
// off < 2t, else payload byte K b + off - 2t.  A piece may run into block b+1 (off > 239).
template <int T2>
__device__ __forceinline__ uint4 enc_piece(const uint8_t* lds, uint32_t buf, uint32_t par, uint32_t p)
{
    constexpr uint32_t K = 255 - T2;
    const uint32_t j0 = p * 16u, b = j0 / 255u, off = j0 - 255u * b;
    const uint32_t S = buf + PAD + K * b + off - T2; // LDS byte of output byte 0's payload source
    const uint32_t sh = (S & 3u) * 8u;
    uint32_t d[5];
    lds_window(d, lds, S);
    uint32_t X[4], Y[4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
        X[m] = __builtin_amdgcn_alignbit(d[m + 1], d[m], sh);
    // after the block boundary the source runs 2t bytes behind: Y byte k = X byte k - 2t
    constexpr int q2 = T2 / 4, r2 = T2 % 4;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const uint32_t hi = (m - q2 >= 0) ? X[m - q2 >= 0 ? m - q2 : 0] : 0u;
        const uint32_t lo = (m - q2 - 1 >= 0) ? X[m - q2 - 1 >= 0 ? m - q2 - 1 : 0] : 0u;
        Y[m] = r2 ? __builtin_amdgcn_alignbit(hi, lo, 16) : hi;
    }
    // parity bytes of blocks b and b+1, byte q at byte q
    const uint64_t P0 = *(const uint64_t*)(lds + par + 8u * b) >> (8 * (8 - T2));
    const uint64_t P1 = *(const uint64_t*)(lds + par + 8u * b + 8u) >> (8 * (8 - T2));
    const uint32_t kb = off > 239u ? 255u - off : 16u;    // first byte of block b+1 in the piece
    const uint32_t c0 = off < (uint32_t)T2 ? T2 - off : 0u; // leading parity bytes of block b
    // parity of b: bytes [0, c0) = P0 bytes off.. ; parity of b+1: bytes [kb, kb+2t) = P1 << 8 kb
    const uint64_t pb0 = P0 >> (8 * (c0 ? off : 0u));
    const uint64_t p1lo = kb < 8 ? (P1 << (8 * kb)) : 0ull;
    const uint64_t p1hi = kb < 8 ? (kb ? (P1 >> (64 - 8 * kb)) : 0ull) : (kb < 16 ? (P1 << (8 * (kb - 8))) : 0ull);
    const M128 mY = range_mask(kb + T2 < 16 ? kb + T2 : 16, 16);
    const M128 mP1 = range_mask(kb, kb + T2 < 16 ? kb + T2 : 16);
    const uint64_t mP0 = ones_below(c0);
    uint32_t o[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const uint64_t my = m < 2 ? mY.lo : mY.hi, mp = m < 2 ? mP1.lo : mP1.hi, pp = m < 2 ? p1lo : p1hi;
        const int sh32 = (m & 1) * 32;
        uint32_t v = bfi((uint32_t)(my >> sh32), Y[m], X[m]);
        v = bfi((uint32_t)(mp >> sh32), (uint32_t)(pp >> sh32), v);
        if (m < 2)
            v = bfi((uint32_t)(mP0 >> sh32), (uint32_t)(pb0 >> sh32), v);
        o[m] = v;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// Decode emission: 16 bytes of the payload tile at piece p from the (corrected) LDS codeword rows:
// payload byte j of block b = j / K (off = j % K) is codeword byte 255 b + 2t + off.
template <int T2> __device__ __forceinline__ uint4 dec_piece(const uint8_t* lds, uint32_t buf, uint32_t p)
{
    constexpr uint32_t K = 255 - T2;
    const uint32_t j0 = p * 16u, b = j0 / K, off = j0 - K * b;
    const uint32_t S = buf + PAD + 255u * b + T2 + off;
    const uint32_t sh = (S & 3u) * 8u;
    uint32_t d[7];
    lds_window(d, lds, S);
    uint32_t X[6];
#pragma unroll
    for (int m = 0; m < 6; ++m)
        X[m] = __builtin_amdgcn_alignbit(d[m + 1], d[m], sh);
    // past the block end the source skips block b+1's 2t parity bytes: Z byte k = X byte k + 2t
    constexpr int q2 = T2 / 4, r2 = T2 % 4;
    const uint32_t kb = off > K - 16u ? K - off : 16u;
    const M128 mZ = range_mask(kb, 16);
    uint32_t o[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        uint32_t Z;
        if constexpr (r2 != 0)
            Z = __builtin_amdgcn_alignbit(X[m + q2 + 1], X[m + q2], 8 * r2);
        else
            Z = X[m + q2];
        const uint64_t mz = m < 2 ? mZ.lo : mZ.hi;
        o[m] = bfi((uint32_t)(mz >> ((m & 1) * 32)), Z, X[m]);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// Output stores: NT = 1 non-temporal (the other cache policies measured no faster step, DESIGN.md
// Appendix A, round 5 store policy), NT = 0 plain
template <int NT = 1> __device__ __forceinline__ void st_nt(uint8_t* dst, uint4 v)
{
    if constexpr (NT) {
        const u32x4 u = { v.x, v.y, v.z, v.w };
        __builtin_nontemporal_store(u, (u32x4*)dst);
    } else {
        *(uint4*)dst = v;
    }
}

// byte-bounded store of a piece (partial tiles): bytes [0, n) of v
__device__ __forceinline__ void st_bytes(uint8_t* dst, uint4 v, uint32_t n)
{
    const uint32_t w[4] = { v.x, v.y, v.z, v.w };
    for (uint32_t k = 0; k < n && k < 16; ++k)
        dst[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
}

// partial-tile staging (nbytes < one tile): plain loads into the LDS buffer
__device__ __forceinline__ void stage_bytes(uint8_t* dst, const uint8_t* __restrict__ src, uint32_t nbytes, uint32_t tid)
{
    for (uint32_t i = tid; i < nbytes; i += NTHR)
        dst[i] = src[i];
}

// Decode phase 2 (wave 0, lane = block): the reference correction for blocks with r' != 0.
// fix(pos, e) patches codeword byte pos of the lane's row (LDS) and, with write-back, in HBM.
template <int T2>
__device__ __forceinline__ uint32_t phase_correct(uint8_t* lds, uint32_t buf, uint32_t par, uint32_t r, bool valid,
    uint8_t* __restrict__ raw_g, uint64_t blk, bool wb, [[maybe_unused]] uint64_t raw_bytes)
{
    using L = RsWgLayout<T2>;
    const uint64_t rem = *(const uint64_t*)(lds + par + 8u * r);
    const bool err = valid && rem != 0;
    if (__builtin_amdgcn_ballot_w64(err)) {
        const Gf gf { lds + L::OFF_GF };
        uint32_t S[T2];
        bool geo = false;
        uint32_t gpos = 0, ge = 0;
        const uint32_t row = buf + PAD + 255u * r;
        if (err) {
            // syndromes as a linear map of r' (nibble tables)
            uint32_t s[2] = { 0, 0 };
            uint2 e[2 * T2];
            const uint8_t* sy = lds + L::OFF_SYN;
            const uint32_t r0 = (uint32_t)rem, r1 = (uint32_t)(rem >> 32);
#pragma unroll
            for (int q = 0; q < T2; ++q) {
                const int P = 8 - T2 + q;
                const uint32_t x = P < 4 ? r0 : r1;
                e[2 * q] = ld8(sy + (2 * q) * 128 + sel78(x << 3, P & 3));
                e[2 * q + 1] = ld8(sy + (2 * q + 1) * 128 + sel78(x >> 1, P & 3));
            }
            xor_entries<2 * T2>(s, e);
#pragma unroll
            for (int i = 0; i < T2; ++i)
                S[i] = (s[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            geo = rs_geometric<T2>(S, gf, gpos, ge);
        }
        auto fix = [&](uint32_t pos, uint32_t e) {
            if (e == 0)
                return;
            const uint8_t fixed = (uint8_t)(lds[row + pos] ^ e);
            lds[row + pos] = fixed;
            if (wb && PPFS_DBG_OK(raw_g + blk * 255u + pos, 1, raw_g, raw_bytes))
                wb_byte(raw_g + blk * 255u + pos, fixed);
        };
        if (__builtin_amdgcn_ballot_w64(err && !geo)) {
            if (err) {
                if (geo)
                    fix(gpos, ge);
                else
                    rs_correct_general<T2>(S, gf, fix);
            }
        } else if (err && geo) {
            fix(gpos, ge);
        }
    }
    return err ? 1u : 0u;
}

// ------------------------------------------------------------------------------------
// Kernels: persistent workgroups walk 64-block tiles t = blockIdx.x, += gridDim.x.
// NBUF = LDS tile buffers: 2 = the next tile's DMA is issued at the top of an iteration (a whole
// tile of compute ahead); 3, 4 = a ring, the DMA NBUF - 1 tiles ahead (fewer workgroups per CU fit); 1 = it is issued after this tile's emission reads (cross-workgroup
// overlap hides it); 0 = full grid: one tile per workgroup (the grid covers the batch, workgroups
// dispatched in address order), emission pieces computed and stored one at a time (few live
// registers, so WPC workgroups fit a CU without spills).  WPC = resident workgroups per CU (the
// launch bound; persistent grids are WPC x CUs).
// ------------------------------------------------------------------------------------
// Ring of NBUF >= 3 tile buffers: the DMA of tile t + (NBUF-1) G is issued at the top of the
// iteration of tile t.  Counted waits: the DMA and store instructions are 4 per wave per tile, and
// a wave's vector-memory operations complete in issue order, so "tile t + G has landed" is
// vmcnt(#operations issued after its DMA).  `hist` holds one bit per DMA slot (1 = issued; bit 0
// the latest); a skipped DMA (past the last tile) means fewer newer operations and a lower count.
__device__ __forceinline__ uint32_t ring_add(uint32_t c, uint32_t d, uint32_t n) { return c + d >= n ? c + d - n : c + d; }

// s_waitcnt vmcnt(m) for the largest m in {0, 4, ..., 24} with m <= n (n wave-uniform)
__device__ __forceinline__ void vm_wait_newer(uint32_t n)
{
    if (n >= 24)
        asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (n >= 20)
        asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if (n >= 16)
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (n >= 12)
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (n >= 8)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 4)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// COMPACT (encode only): 2 maps (phase_remainder NMAP = 2) and tile buffers sized for the 64
// payload rows (PAD + 64 K + 32) instead of 64 codewords, so 3 ring buffers fit 3 workgroups / CU
// MAPS = 1: the SLX last-step tables (3 x 2 KiB, seg_remainder) instead of the maps: the encode holds
// SL + SLX (OFF_SLX = L::OFF_MAP), the decode the whole decode table prefix + SLX after it.
// MAPS = 2 (encode): the 5-bit field tables SL5 + SLX5 (OFF_SLX = L::SL5_BYTES)
template <int T2, bool DEC, int NBUF, bool COMPACT = false, int MAPS = 0> struct Lds {
    using L = RsWgLayout<T2>;
    static_assert(!(DEC && COMPACT), "compact layout: encode only");
    static_assert(MAPS >= 0 && MAPS <= 2, "x^(64 s) maps, SLX tables, or (encode) SL5 + SLX5");
    static_assert(MAPS != 2 || !DEC, "5-bit tables: encode only");
    static constexpr int NMAP = MAPS ? 1 : COMPACT ? 2 : 3;
    static constexpr int OFF_SLX = MAPS == 2 ? L::SL5_BYTES : MAPS == 1 ? (DEC ? L::TABLE_BYTES : L::OFF_MAP) : 0;
    static constexpr int TBL = MAPS == 2 ? OFF_SLX + L::SLX5_BYTES : MAPS == 1 ? OFF_SLX + L::SLX_BYTES
        : DEC ? L::TABLE_BYTES : L::OFF_MAP + NMAP * L::MAP_STRIDE; // encode: SL + MAP only
    static constexpr int OFF_PAR = TBL;                              // 2 x 64 x 8 B remainder slots
    static constexpr int OFF_BUF = OFF_PAR + 1024 + 64;             // + slack: par[b+1] over-read
    static constexpr int BUFB = COMPACT ? (PAD + TB * L::K + 32 + 15) / 16 * 16 : BUF; // one tile buffer
    static constexpr int BYTES = OFF_BUF + (NBUF ? NBUF : 1) * BUFB;
    static_assert(OFF_BUF % 16 == 0 && TBL % 16 == 0, "aligned buffers");
};

template <int T2, bool DEC, int NBUF, bool COMPACT = false> constexpr int lds_bytes() { return Lds<T2, DEC, NBUF, COMPACT>::BYTES; }

// LDS declared per workgroup: at least the layout, and more than 1/(WPC+1) of the CU's 160 KiB, so
// exactly WPC workgroups are resident per CU -- a WPC x CUs persistent grid is then balanced
// (a smaller footprint would let some CUs take WPC+1 workgroups and others fewer).
template <int BYTES, int WPC> constexpr int lds_alloc()
{
    constexpr int floor_plus = (163840 / (WPC + 1) + 512) & ~511;
    return BYTES > floor_plus ? BYTES : floor_plus;
}

// MODE (ablation builds only; the engine uses 3): bit 0 = remainder phase, bit 1 = codeword
// emission (else a plain 16-byte copy out of the LDS tile, same bytes moved)
template <int T2, int NBUF = 2, int WPC = 4, int MODE = 3, int NTST = 1, bool COMPACT = false>
__global__ __launch_bounds__(256, WPC) void rs_wg_encode_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables)
{
    using L = RsWgLayout<T2>;
    using D = Lds<T2, false, NBUF, COMPACT>;
    constexpr int BUF = D::BUFB;
    constexpr int LDS_ALLOC = lds_alloc<D::BYTES, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * K / 16;   // 996 for 2t = 6
    constexpr int OUT_PIECES = TB * 255 / 16; // 1020
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t row = lane_row(lane);
    for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += NTHR)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    if (tid < 128)
        *(uint64_t*)(lds + D::OFF_PAR + 8 * tid) = 0;
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    uint64_t t = blockIdx.x;
    uint32_t cur = 0, pc = 0; // tile buffer, parity-slot set
    if (t < nfull)
        dma_tile<IN_PIECES>(lds + D::OFF_BUF + PAD, data + t * (TB * K), tid, data, nblocks * K);
    uint32_t hist = 0, iter = 0;
    if constexpr (NBUF >= 3) {
#pragma unroll
        for (int j = 1; j <= NBUF - 2; ++j) {
            const bool go = t + j * gridDim.x < nfull;
            if (go)
                dma_tile<IN_PIECES>(lds + D::OFF_BUF + j * BUF + PAD, data + (t + j * gridDim.x) * (TB * K), tid, data, nblocks * K);
            hist = (hist << 1) | (go ? 1u : 0u);
        }
        vm_wait_newer(4u * __builtin_popcount(hist)); // tile t landed, the later ones may fly
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    for (; t < nfull; t += gridDim.x) {
        barrier_lds(); // A: tile t in LDS (every wave's pieces), last tile's emission reads done
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        const uint64_t nx = t + gridDim.x;
        if (NBUF == 2 && nx < nfull)
            dma_tile<IN_PIECES>(lds + D::OFF_BUF + (cur ^ 1u) * BUF + PAD, data + nx * (TB * K), tid, data, nblocks * K);
        if constexpr (NBUF >= 3) { // NBUF - 1 tiles ahead, into the buffer tile t - G used
            const uint64_t ahead = t + (uint64_t)(NBUF - 1) * gridDim.x;
            const bool go = ahead < nfull;
            if (go)
                dma_tile<IN_PIECES>(lds + D::OFF_BUF + ring_add(cur, NBUF - 1, NBUF) * BUF + PAD, data + ahead * (TB * K), tid, data, nblocks * K);
            hist = (hist << 1) | (go ? 1u : 0u);
        }
        if (wave == 0)
            *(uint64_t*)(lds + D::OFF_PAR + (pc ^ 1u) * 512u + 8u * lane) = 0;
        if constexpr (MODE & 1)
            phase_remainder<T2, K, D::NMAP>(lds, buf, par, wave, row);
        barrier_lds(); // B: parity slots complete
        uint8_t* dst = raw + t * (TB * 255);
        uint4 o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t p = tid + 256u * k;
            if constexpr (NBUF == 0)
                asm volatile("" : "+v"(p)); // this piece's index maths starts after the last store
            if constexpr (MODE & 2)
                o[k] = enc_piece<T2>(lds, buf, par, p);
            else
                o[k] = *(const uint4*)(lds + buf + PAD + 16u * (p < 996u ? p : p - 64u));
            if (NBUF != 1 && (k < 3 || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, raw, nblocks * 255u))
                st_nt<NTST>(dst + 16u * p, o[k]); // store as soon as the piece is assembled
            if constexpr (NBUF == 0)
                asm volatile("" ::: "memory"); // one piece live at a time
        }
        if (NBUF == 1) {
            barrier_lds(); // every wave's emission reads done: the buffer is free
            if (nx < nfull)
                dma_tile<IN_PIECES>(lds + D::OFF_BUF + PAD, data + nx * (TB * K), tid, data, nblocks * K);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t p = tid + 256u * k;
                if ((k < 3 || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, raw, nblocks * 255u))
                    st_nt<NTST>(dst + 16u * p, o[k]);
            }
        }
        // next tile's DMA landed; this tile's stores (NBUF >= 3: and every store and DMA issued
        // after that DMA) may fly
        if constexpr (NBUF >= 3) {
            ++iter;
            const uint32_t st = 4u * (iter < (uint32_t)(NBUF - 1) ? iter : (uint32_t)(NBUF - 1));
            vm_wait_newer(st + 4u * __builtin_popcount(hist & ((1u << (NBUF - 2)) - 1u)));
            cur = ring_add(cur, 1, NBUF);
        } else {
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            cur ^= (NBUF == 2) ? 1u : 0u;
        }
        pc ^= 1u;
    }
    if (t == nfull && nfull < ntiles) {
        // the one partial tile (nblocks % 64 blocks)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
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
}


// MODE (ablation builds only; the engine uses 7): bit 0 = remainder phase, bit 1 = payload
// emission (else a plain 16-byte copy), bit 2 = correction phase
template <int T2, int NBUF = 2, int WPC = 3, int MODE = 7, int NTST = 1>
__global__ __launch_bounds__(256, WPC) void rs_wg_decode_kernel(uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks, const uint8_t* __restrict__ tables, int write_back,
    uint8_t* __restrict__ raw_wb)
{
    using L = RsWgLayout<T2>;
    using D = Lds<T2, true, NBUF>;
    constexpr int LDS_ALLOC = lds_alloc<D::BYTES, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * 255 / 16; // 1020
    constexpr int OUT_PIECES = TB * K / 16;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t row = lane_row(lane);
    const bool wb = write_back != 0, want = data != nullptr;
    uint8_t* const wbp = raw_wb ? raw_wb : raw; // write-back target (rs_wg_tk.hpp rs_wg_decode_tk_kernel)
    for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += NTHR)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    if (tid < 128)
        *(uint64_t*)(lds + D::OFF_PAR + 8 * tid) = 0;
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    uint64_t t = blockIdx.x;
    uint32_t cur = 0, pc = 0;
    if (t < nfull)
        dma_tile<IN_PIECES>(lds + D::OFF_BUF + PAD, raw + t * (TB * 255), tid, raw, nblocks * 255u);
    uint32_t hist = 0, iter = 0;
    if constexpr (NBUF >= 3) {
#pragma unroll
        for (int j = 1; j <= NBUF - 2; ++j) {
            const bool go = t + j * gridDim.x < nfull;
            if (go)
                dma_tile<IN_PIECES>(lds + D::OFF_BUF + j * BUF + PAD, raw + (t + j * gridDim.x) * (TB * 255), tid, raw, nblocks * 255u);
            hist = (hist << 1) | (go ? 1u : 0u);
        }
        vm_wait_newer(4u * __builtin_popcount(hist));
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    for (; t < nfull; t += gridDim.x) {
        barrier_lds(); // A
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        const uint64_t nx = t + gridDim.x;
        if (NBUF == 2 && nx < nfull)
            dma_tile<IN_PIECES>(lds + D::OFF_BUF + (cur ^ 1u) * BUF + PAD, raw + nx * (TB * 255), tid, raw, nblocks * 255u);
        if constexpr (NBUF >= 3) {
            const uint64_t ahead = t + (uint64_t)(NBUF - 1) * gridDim.x;
            const bool go = ahead < nfull;
            if (go)
                dma_tile<IN_PIECES>(lds + D::OFF_BUF + ring_add(cur, NBUF - 1, NBUF) * BUF + PAD, raw + ahead * (TB * 255), tid, raw, nblocks * 255u);
            hist = (hist << 1) | (go ? 1u : 0u);
        }
        if (wave == 0)
            *(uint64_t*)(lds + D::OFF_PAR + (pc ^ 1u) * 512u + 8u * lane) = 0;
        if constexpr (MODE & 1)
            phase_remainder<T2, 255>(lds, buf, par, wave, row);
        barrier_lds(); // B: remainders complete
        if ((MODE & 4) && wave == 0) {
            const uint32_t st = phase_correct<T2>(lds, buf, par, row, true, wbp, t * TB + row, wb, nblocks * 255u);
            if (status && PPFS_DBG_OK(status + t * TB + row, 1, status, nblocks))
                status[t * TB + row] = (uint8_t)st;
        }
        barrier_lds(); // C: corrections patched into the LDS rows
        uint4 o[4];
        uint8_t* dst = want ? data + t * (TB * K) : nullptr;
        if (want) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t p = tid + 256u * k;
                if constexpr (NBUF == 0)
                    asm volatile("" : "+v"(p));
                if constexpr (MODE & 2)
                    o[k] = dec_piece<T2>(lds, buf, p);
                else
                    o[k] = *(const uint4*)(lds + buf + PAD + 16u * p);
                if (NBUF != 1 && (k < 3 || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, data, nblocks * K))
                    st_nt<NTST>(dst + 16u * p, o[k]);
                if constexpr (NBUF == 0)
                    asm volatile("" ::: "memory");
            }
        }
        if (NBUF == 1) {
            barrier_lds();
            if (nx < nfull)
                dma_tile<IN_PIECES>(lds + D::OFF_BUF + PAD, raw + nx * (TB * 255), tid, raw, nblocks * 255u);
            if (want) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t p = tid + 256u * k;
                    if ((k < 3 || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, data, nblocks * K))
                        st_nt<NTST>(dst + 16u * p, o[k]);
                }
            }
        }
        // as in encode (no output stores without `data`); the wave-0 status / write-back stores
        // only add newer operations, which keeps the count a lower bound
        if constexpr (NBUF >= 3) {
            ++iter;
            const uint32_t st = want ? 4u * (iter < (uint32_t)(NBUF - 1) ? iter : (uint32_t)(NBUF - 1)) : 0u;
            vm_wait_newer(st + 4u * __builtin_popcount(hist & ((1u << (NBUF - 2)) - 1u)));
            cur = ring_add(cur, 1, NBUF);
        } else {
            if (want)
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            cur ^= (NBUF == 2) ? 1u : 0u;
        }
        pc ^= 1u;
    }
    if (t == nfull && nfull < ntiles) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        if (PPFS_DBG_OK(raw + t * (TB * 255), nb * 255u, raw, nblocks * 255u))
            stage_bytes(lds + buf + PAD, raw + t * (TB * 255), nb * 255u, tid);
        barrier_lds();
        phase_remainder<T2, 255>(lds, buf, par, wave, row);
        barrier_lds();
        if (wave == 0) {
            const bool valid = row < nb;
            const uint32_t st = phase_correct<T2>(lds, buf, par, row, valid, wbp, t * TB + row, wb, nblocks * 255u);
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
}

// ------------------------------------------------------------------------------------
// Resident small-batch server (per-block readBlock / writeBlock calls, <= 64 blocks): one
// workgroup stays on the GPU with the tables in LDS and serves requests posted in host-coherent
// memory (server_box.hpp), reading its inputs from and writing its outputs to the context's
// zero-copy buffer.  A request costs two PCIe round trips instead of a kernel launch and a stream
// synchronize.  The tile work is the partial-tile path of the kernels above.
// ------------------------------------------------------------------------------------
template <int T2>
__global__ __launch_bounds__(256, 1) void rs_wg_server_kernel(SrvBox* box, uint8_t* zc, uint64_t zc_bytes,
    const uint8_t* __restrict__ tables, uint32_t gen, uint32_t idle_us)
{
    using L = RsWgLayout<T2>;
    using D = Lds<T2, true, 1>; // all tables (encode uses SL + MAP of the same layout)
    constexpr int K = L::K;
    __shared__ __attribute__((aligned(16))) uint8_t lds[D::BYTES];
    __shared__ uint32_t s_cmd[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t row = lane_row(lane);
    const uint32_t buf = D::OFF_BUF, par = D::OFF_PAR;
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
            if (wave == 0)
                *(uint64_t*)(lds + par + 8u * lane) = 0;
            srv::stage_host<NTHR, TB * 255>(lds + buf + PAD, raw, nb * 255u, tid);
            barrier_lds();
            phase_remainder<T2, 255>(lds, buf, par, wave, row);
            barrier_lds();
            if (wave == 0) {
                const bool valid = row < nb;
                const uint32_t st = phase_correct<T2>(lds, buf, par, row, valid, raw, row, op == SRV_DECODE && cmd.write_back,
                    nb * 255u);
                if (valid)
                    status[row] = (uint8_t)st;
            }
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
            barrier_lds(); // the buffer and slots are free
        }
        if (ok && (op == SRV_ENCODE || op == SRV_WRITE)) {
            if (wave == 0)
                *(uint64_t*)(lds + par + 8u * lane) = 0;
            srv::stage_host<NTHR, TB * 255>(lds + buf + PAD, data, nb * (uint32_t)K, tid);
            barrier_lds();
            phase_remainder<T2, K>(lds, buf, par, wave, row);
            barrier_lds();
            const uint32_t nout = nb * 255u;
            for (uint32_t p = tid; 16u * p < nout; p += NTHR) {
                const uint4 v = enc_piece<T2>(lds, buf, par, p);
                if (16u * p + 16u <= nout)
                    *(uint4*)(raw + 16u * p) = v;
                else
                    st_bytes(raw + 16u * p, v, nout - 16u * p);
            }
            barrier_lds();
        }
        seen = r;
        srv::finish_request(box, r, ++served);
    }
    if (tid == 0)
        srv::st_sys(&box->alive, gen | SRV_EXITED);
}

} // namespace wg
} // namespace ppfs
