// bit_fast.hip -- Hamming SECDED and single-parity kernels for 1, 2 and 4 KiB blocks (gfx950).
//
// The BASELINE cfg4 shape (block_size 4096, 2^20 blocks: 4 GiB in, 4 GiB out per launch) is pure
// streaming; these kernels keep every byte's work to a few VALU ops so they run at the HBM rate.
// One wave per block, NP = block_size / 1024 pieces of 16 B per lane, coalesced: lane l of a wave
// holds raw bytes [16 (64 k + l), +16) for k < NP, i.e. big-endian raw words w = 256 k + 4 l + u.
// The grid covers the batch (one wave per block, workgroups dispatched in address order); see
// BF_PREFETCH below.  Smaller blocks use bit_kernels.hip.
//
// Reference semantics (lib/blockdevice/src/hamming_block_device.cpp, MSB-first bit numbering of
// lib/common/include/ppfs/common/bit_helpers.hpp:8-52):
//   - payload bit i sits at raw position r(i) = the i-th integer >= 3 that is not a power of two;
//     for r in (2^j, 2^(j+1)) that is r = i + j + 2 (HammingDataBitsIterator :180-198), so raw
//     word w >= 1 is one funnel of the payload bit stream at offset 32 w - j - 2, j = log2(32 w);
//   - parity bit 2^j = bit j of the XOR of the positions of the set payload bits; bit 0 makes the
//     total parity even (_encodeData :76-109); raw bits after the last payload bit L keep their
//     old contents (the reference only writes payload and parity positions);
//   - decode (_readAndFixBlock :21-65): over the used bits [0, L] (plus parity positions past L,
//     none for block_size >= 1024): odd parity -> flip bit (XOR of set positions), write back
//     that byte, status 1; even parity and a non-zero XOR -> BlockDevice_CorrectionError (5).
// Parity (parity_block_device.cpp:31-97): even parity over the raw block, the fix bit is the LSB
// of the last byte, whose other bits keep their old contents.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dbg.hpp"
#include "gf_common.hpp"
#include "launch.hpp"

namespace ppfs {
namespace bf {

typedef unsigned int bf_u32x4 __attribute__((ext_vector_type(4)));
// streamed global traffic: every block is read once and written once.  Non-temporal variants on
// cfg4 (bs 4096, 2^20 blocks): NT loads 0-7 % slower except the parity encode's payload (below); NT
// stores 1-3 % faster on encode, 4-5 % slower on decode -- the encode outputs use them (gst16_raw:
// on the full grid, r1l, Hamming encode 1.51 -> 1.46 ms, parity 1.59 -> 1.55 ms), everything else
// is plain.
__device__ __forceinline__ uint4 gld16(const uint8_t* p) { return *(const uint4*)p; }
__device__ __forceinline__ void gst16(uint8_t* p, uint4 v) { *(uint4*)p = v; }
__device__ __forceinline__ void gst16_raw(uint8_t* p, uint4 v)
{
    const bf_u32x4 u = { v.x, v.y, v.z, v.w };
    __builtin_nontemporal_store(u, (bf_u32x4*)p);
}

// PPFS_ECC_DEBUG (dbg.hpp): a load outside its buffer reads zeros (and is reported); normal
// builds compile this to gld16
__device__ __forceinline__ uint4 gld16c(const uint8_t* p, const uint8_t* base, uint64_t extent)
{
    return PPFS_DBG_OK(p, 16, base, extent) ? gld16(p) : make_uint4(0, 0, 0, 0);
}

// Payload loads of the parity encode: non-temporal (round 5, r5nt A/Bs on cfg4, 3 interleaved
// rounds: 1,394-1,401 vs 1,484-1,491 us in the configs leg).  The Hamming encode gains as much
// (1,422-1,425 vs 1,465-1,470 us) but the 1-error decode timed right after it then runs 1,642-1,658
// vs 1,579-1,589 us, so it keeps plain loads; the CRC encode is slower with them (1,636-1,640 vs
// 1,606-1,608 us), and so is every decode / check (Hamming +3 %, parity +4 %, CRC +3 %).
constexpr bool PAR_ENC_NTLD = true, HAM_ENC_NTLD = false;
template <bool NT> __device__ __forceinline__ uint4 gld16p(const uint8_t* p, const uint8_t* base, uint64_t extent)
{
    if constexpr (NT) {
        if (!PPFS_DBG_OK(p, 16, base, extent))
            return make_uint4(0, 0, 0, 0);
        const bf_u32x4 v = __builtin_nontemporal_load((const bf_u32x4*)p);
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return gld16c(p, base, extent);
    }
}

constexpr int WAVES = 4;
// Grid and prefetch.  The kernels launch one wave per block over the whole batch (a full grid,
// not a persistent one): the dispatcher then walks workgroups in address order, so the blocks in
// flight form one contiguous window of HBM.  A persistent grid-stride walk spreads them over
// gridDim x 4 KiB and ran 9-22 % slower on cfg4 (A/B in DESIGN.md section 4.3).  With one block
// per wave a register prefetch of the next block is dead weight (measured: no gain, Appendix A);
// a wave loads its next block at the loop end, which only runs for grids capped below the batch.
// Blocks per wave of the Hamming / parity kernels: one group of WV blocks per workgroup (more, in
// one contiguous range: slower, r4m).
constexpr int BF_BPW = 1;

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// Workgroup -> block range, XCD-local (round 6).  The dispatcher places workgroup b on XCD b % 8
// (MI355X_MICROARCH.md: the placement is for speed only, so this is a bijection on [0, gridDim.x)
// whatever it is); remapped, each XCD's workgroups take one contiguous range of blocks, so
// neighbouring blocks -- which share the 128-B lines at their unaligned payload-row boundaries, where
// each writes a partial 16-B piece -- meet in one L2 instead of two (the workgroups in flight are
// then 8 contiguous HBM windows, one per XCD).  Configs leg, 3 interleaved rounds (r6m): Hamming
// decode clean 1.471-1.473 vs 1.515-1.522 ms, 1-error 1.510-1.525 vs 1.586-1.597, encode
// 1.403-1.413 vs 1.419; parity check 1.387-1.391 vs 1.438-1.445, encode 1.318-1.321 vs 1.327-1.329;
// CRC check 1.584-1.600 vs 1.609-1.614; the CRC encode (24 blocks per workgroup, so its boundaries
// were mostly inside one workgroup) 1.548-1.555 vs 1.543-1.547 keeps the dispatch order.
template <bool XCD> __device__ __forceinline__ uint32_t bf_wg()
{
    const uint32_t b = blockIdx.x, G = gridDim.x;
    if (!XCD || G < 64u)
        return b;
    const uint32_t x = b & 7u, r = b >> 3, per = G >> 3, rem = G & 7u;
    return x * per + (x < rem ? x : rem) + r;
}

// Hamming decode: the LDS image stores issued before the syndrome reduction (round 5), so they
// complete under its DPP chain (after it: configs leg, 3 interleaved rounds, r5hei: clean
// 1.512-1.523 vs 1.531 ms, 1-error 1.582-1.590 vs 1.588-1.602 ms).  Status bytes and corrected-byte
// write-backs of the Hamming decode and the CRC / parity checks are stored after the payload
// emission (round 5; before it: r5late, parity check 1.439-1.441 vs 1.467-1.469 ms, Hamming 1-error
// 1.576-1.579 vs 1.578-1.587 ms, clean 1.500-1.511 vs 1.509-1.513, CRC check within noise).

// XOR over the 64 lanes of a wave, returned wave-uniform: a DPP butterfly inside each row of 16
// lanes, then row broadcasts 15 and 31 (lane 63 ends with the total).
__device__ __forceinline__ uint32_t wave_xor(uint32_t v)
{
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);        // quad_perm [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);        // quad_perm [2,3,0,1]
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);       // row_half_mirror
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);       // row_mirror
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false); // row_bcast:15
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false); // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// 32 bits of a big-endian bit stream in LDS starting at absolute bit position `bit` (the stream's
// bit 0 is the MSB of byte 0 of `base`); reads two aligned dwords.
__device__ __forceinline__ uint32_t be_fetch32(const uint8_t* base, uint32_t bit)
{
    const uint32_t* w = (const uint32_t*)(base + ((bit >> 5) << 2));
    const uint64_t v = ((uint64_t)bswap(w[0]) << 32) | bswap(w[1]);
    return (uint32_t)(v >> (32 - (bit & 31u)));
}

// top n bits (MSB side) of a word, n in [0, 32]
__device__ __forceinline__ uint32_t top_bits(uint32_t n) { return n >= 32 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> n); }

// syndrome contribution of the positions q (MSB-first) set in the XOR of a lane's words
__device__ __forceinline__ uint32_t qbits(uint32_t x)
{
    return (__builtin_popcount(x & 0x55555555u) & 1u) | ((__builtin_popcount(x & 0x33333333u) & 1u) << 1)
        | ((__builtin_popcount(x & 0x0F0F0F0Fu) & 1u) << 2) | ((__builtin_popcount(x & 0x00FF00FFu) & 1u) << 3)
        | ((__builtin_popcount(x & 0x0000FFFFu) & 1u) << 4);
}

struct HamFast {
    uint32_t bs, ds, L;
    uint64_t data_bytes; // nblocks * ds: the payload buffer's end (no vector load may pass it)
};

// ------------------------------------------------------------------------------------
// Hamming encode
// ------------------------------------------------------------------------------------
// The payload row (ds bytes at any alignment) is staged as the 16-byte pieces of the aligned
// superset [a0, a0 + 16 npc) into the wave's LDS buffer; pieces past the buffer end (last block
// only) are loaded byte by byte.  NPL = pieces per lane in the prefetch registers.
template <int NP> struct HamEncStage {
    static constexpr int NPL = NP + 1; // superset <= 64 NP + 1 pieces
    uint4 v[NPL];
};

template <int NP, bool NTL = false>
__device__ __forceinline__ void ham_stage_load(HamEncStage<NP>& s, const uint8_t* __restrict__ data, uint64_t blk,
    const HamFast& a, uint32_t lane)
{
    const uint64_t start = blk * a.ds, a0 = start & ~15ull;
    const uint32_t npc = (uint32_t)((start + a.ds - a0 + 15) >> 4);
#pragma unroll
    for (int k = 0; k < HamEncStage<NP>::NPL; ++k) {
        const uint32_t p = 64u * k + lane;
        const uint64_t g = a0 + 16ull * p;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (p < npc) {
            if (g + 16 <= a.data_bytes) {
                v = gld16p<NTL>(data + g, data, a.data_bytes);
            } else { // the batch's last bytes: one flat predicated load per byte (no nested
                     // divergence, which spilled the exec masks of 16 levels into SGPRs)
                const uint32_t nb = g < a.data_bytes ? (uint32_t)(a.data_bytes - g) : 0u;
                uint32_t w[4] = { 0, 0, 0, 0 };
#pragma unroll
                for (uint32_t b = 0; b < 16; ++b)
                    if (b < nb)
                        w[b >> 2] |= (uint32_t)data[g + b] << (8 * (b & 3));
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
        s.v[k] = v;
    }
}

template <int NP>
__device__ __forceinline__ void ham_stage_write(uint8_t* buf, const HamEncStage<NP>& s, uint32_t lane)
{
#pragma unroll
    for (int k = 0; k < HamEncStage<NP>::NPL; ++k)
        *(uint4*)(buf + 16u * (64u * k + lane)) = s.v[k];
}

// bytes [lo, hi) of a 16-byte piece (the partial first / last piece of an unaligned row: the
// other bytes belong to the neighbouring rows, written by other waves): whole dwords where the
// range covers them, single bytes at the two ends
__device__ __forceinline__ void store_piece_part(uint8_t* dst, const uint32_t (&o)[4], uint32_t lo, uint32_t hi)
{
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t d0 = 4 * u;
        if (lo <= d0 && d0 + 4 <= hi) {
            *(uint32_t*)(dst + d0) = o[u];
        } else {
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (d0 + b >= lo && d0 + b < hi)
                    dst[d0 + b] = (uint8_t)(o[u] >> (8 * b));
        }
    }
}

template <int NP, int WV>
__global__ __launch_bounds__(64 * WV) void ham_fast_encode_kernel(const uint8_t* __restrict__ data, uint8_t* __restrict__ raw,
    const uint8_t* __restrict__ skip, uint64_t nblocks_all, HamFast a)
{
    constexpr int BUF = (NP + 1) * 1024 + 32; // NP + 1 staged pieces per lane + read slack
    __shared__ __attribute__((aligned(16))) uint8_t lds[WV * BUF];
    const uint32_t lane = lane_id(), wave = wave_id();
    uint8_t* buf = lds + wave * BUF;
    const uint32_t nwords = a.bs / 4, lastw = nwords - 1;
    const uint64_t wg0 = (uint64_t)bf_wg<true>() * (WV * BF_BPW);
    const uint64_t nblocks = nblocks_all < wg0 + WV * BF_BPW ? nblocks_all : wg0 + WV * BF_BPW;
    const uint64_t stride = WV;
    uint64_t blk = wg0 + wave;
    HamEncStage<NP> st;
    if (blk < nblocks)
        ham_stage_load<NP, HAM_ENC_NTLD>(st, data, blk, a, lane);
    for (; blk < nblocks; blk += stride) {
        ham_stage_write<NP>(buf, st, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint64_t nx = blk + stride;
        const uint32_t m = (uint32_t)((blk * a.ds) & 15u); // payload byte 0 sits at LDS byte m
        uint8_t* rb = raw + blk * a.bs;
        const bool skipped = skip && PPFS_DBG_OK(skip + blk, 1, skip, nblocks_all) && skip[blk] == 5;
        // old raw tail word (bits past L keep their contents): the last word of the block.  (Round 4
        // measured the alternative for whole-byte tails -- no read, the last piece stored without
        // them: 2 % slower on cfg4, the partial-sector write costs more than the 4-byte read's line,
        // which is the 1.039x of the read bytes.)
        uint32_t old_tail = 0;
        if (lane == 63 && PPFS_DBG_OK(rb + 4 * lastw, 4, raw, nblocks_all * a.bs))
            old_tail = bswap(*(const uint32_t*)(rb + 4 * lastw));
        uint32_t X[NP][4];
        uint32_t ax = 0, aw = 0;
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const uint32_t w0 = 256u * k + 4u * lane;
            if (k == 0 && lane == 0) {
                // words 0-3: positions 0..127 hold parity bits 0,1,2,4,8,16,32,64
                const uint32_t D = be_fetch32(buf, 8 * m);
                X[0][0] = (((D >> 31) & 1u) << 28) | (((D >> 28) & 7u) << 24) | (((D >> 21) & 0x7Fu) << 16)
                    | ((D >> 6) & 0x7FFFu);
                X[0][1] = be_fetch32(buf, 8 * m + 32 - 5 - 2) & 0x7FFFFFFFu;  // j = 5, parity at 32
                X[0][2] = be_fetch32(buf, 8 * m + 64 - 6 - 2) & 0x7FFFFFFFu;  // j = 6, parity at 64
                X[0][3] = be_fetch32(buf, 8 * m + 96 - 6 - 2);
            } else {
                const uint32_t j = 36u - (uint32_t)__builtin_clz(w0); // log2(32 w0)
                const uint32_t o = 8 * m + 32 * w0 - j - 2;           // stream bit of word w0, position 0
                // the 5 dwords from word o / 32: two 16-byte-aligned reads and a dword select, as in
                // ham_mid_piece (5 dword reads of windows 16 B apart: 4-way bank conflicts)
                const uint32_t q = (o >> 7) << 4, d = (o >> 5) & 3u, s = o & 31u;
                const uint4 wa = *(const uint4*)(buf + q), wb = *(const uint4*)(buf + q + 16u);
                const uint32_t W[8] = { wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w };
                const uint32_t m1 = (d & 1u) ? ~0u : 0u, m2 = (d & 2u) ? ~0u : 0u;
                uint32_t F[7], E[5];
#pragma unroll
                for (int i = 0; i < 7; ++i)
                    F[i] = (m1 & W[i + 1]) | (~m1 & W[i]);
#pragma unroll
                for (int i = 0; i < 5; ++i)
                    E[i] = bswap((m2 & F[i + 2]) | (~m2 & F[i]));
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    X[k][u] = (uint32_t)((((uint64_t)E[u] << 32) | E[u + 1]) >> (32 - s));
                if ((w0 & (w0 - 1)) == 0)
                    X[k][0] &= 0x7FFFFFFFu; // position 32 w0 = 2^j is a parity bit
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t w = w0 + u;
                if (32 * w + 31 > a.L) // bits past the last payload bit are not payload
                    X[k][u] &= top_bits(a.L >= 32 * w ? a.L - 32 * w + 1 : 0);
                ax ^= X[k][u];
                aw ^= (__builtin_popcount(X[k][u]) & 1u) ? w : 0u;
            }
        }
        // syndrome S = XOR of the positions of the set payload bits, and the payload parity
        const uint32_t red = wave_xor(((aw << 5 | qbits(ax)) << 1) | (__builtin_popcount(ax) & 1u));
        const uint32_t S = red >> 1;
        const uint32_t bit0 = (red ^ (uint32_t)__builtin_popcount(S)) & 1u; // total parity even
        if (!skipped) {
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                const uint32_t w0 = 256u * k + 4u * lane;
                if (k == 0 && lane == 0) {
                    X[0][0] |= (bit0 << 31) | ((S & 1u) << 30) | (((S >> 1) & 1u) << 29) | (((S >> 2) & 1u) << 27)
                        | (((S >> 3) & 1u) << 23) | (((S >> 4) & 1u) << 15);
                    X[0][1] |= ((S >> 5) & 1u) << 31;
                    X[0][2] |= ((S >> 6) & 1u) << 31;
                } else if ((w0 & (w0 - 1)) == 0 && 32 * w0 < 8 * a.bs) {
                    const uint32_t j = 36u - (uint32_t)__builtin_clz(w0);
                    X[k][0] |= ((S >> j) & 1u) << 31;
                }
                if (k == NP - 1 && lane == 63) {
                    const uint32_t keep = ~top_bits(a.L - 32 * lastw + 1);
                    X[k][3] = (X[k][3] & ~keep) | (old_tail & keep);
                }
                if (PPFS_DBG_OK(rb + 16u * (64u * k + lane), 16, raw, nblocks_all * a.bs))
                    gst16_raw(rb + 16u * (64u * k + lane),
                        make_uint4(bswap(X[k][0]), bswap(X[k][1]), bswap(X[k][2]), bswap(X[k][3])));
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); // LDS reads done before the rewrite
        __builtin_amdgcn_wave_barrier();
        if (nx < nblocks)
            ham_stage_load<NP, HAM_ENC_NTLD>(st, data, nx, a, lane);
    }
}

// ------------------------------------------------------------------------------------
// Hamming decode
// ------------------------------------------------------------------------------------
// payload bits [i, i + 32) for 0 <= i < 64, from the corrected raw image in LDS (big-endian
// stream).  Below raw bit 72 the parity positions 1,2,4,8,16,32,64 interleave with the payload,
// so payload bits 0..63 are gathered with fixed masks from raw words 0-2; payload bits 64..
// continue at raw bit 72 with no parity position before raw bit 128.
__device__ __forceinline__ uint32_t ham_head32(const uint8_t* img, uint32_t i)
{
    const uint32_t* w = (const uint32_t*)img;
    const uint32_t W0 = bswap(w[0]), W1 = bswap(w[1]), W2 = bswap(w[2]);
    // payload 0 <- raw 3; 1-3 <- 5-7; 4-10 <- 9-15; 11-25 <- 17-31; 26-56 <- 33-63; 57-63 <- 65-71
    const uint32_t hi = (((W0 >> 28) & 1u) << 31) | (((W0 >> 24) & 7u) << 28) | (((W0 >> 16) & 0x7Fu) << 21)
        | ((W0 & 0x7FFFu) << 6) | ((W1 >> 25) & 0x3Fu);
    const uint32_t lo = ((W1 & 0x1FFFFFFu) << 7) | ((W2 >> 24) & 0x7Fu);
    const uint64_t P = ((uint64_t)hi << 32) | lo;                    // payload bits 0..63
    const uint32_t head = (uint32_t)((P << i) >> 32);                    // payload bits [i, min(i + 32, 64))
    const uint32_t tail = i > 32 ? be_fetch32(img, 72) >> (64 - i) : 0u; // payload bits 64.. from raw 72
    return head | tail;
}

// payload bits [i, i + 32) for i >= 64: at most one parity position (the next power of two)
// among their raw positions; bits before it from the raw stream at r(i), after it at r(i) + 1
__device__ __forceinline__ uint32_t ham_mid32(const uint8_t* img, uint32_t i)
{
    uint32_t j = 31u - (uint32_t)__builtin_clz(i + 2);
    if (i + j + 2 >= (2u << j))
        j++;
    const uint32_t r = i + j + 2, n = (2u << j) - r;
    const uint32_t A = be_fetch32(img, r), B = be_fetch32(img, r + 1);
    const uint32_t mk = top_bits(n);
    return (A & mk) | (B & ~mk);
}

// payload bytes [b0, b0 + 16) (b0 >= 8) of the corrected raw image: payload bits [i0, i0 + 128)
// sit at raw bits [r0, ...) with at most one parity position inside (the next power of two): bits
// before it come from the raw stream at r0 (A), bits after it from r0 + 1 (B).  Most pieces hold
// no parity position (n >= 128): A only.
__device__ __forceinline__ void ham_mid_piece(const uint8_t* img, uint32_t b0, uint32_t (&o)[4])
{
    const uint32_t i0 = 8u * b0;
    uint32_t j = 31u - (uint32_t)__builtin_clz(i0 + 2);
    if (i0 + j + 2 >= (2u << j))
        j++;
    const uint32_t r0 = i0 + j + 2;
    const uint32_t n = (2u << j) - r0; // payload bits before the parity position
    // the 5 dwords from raw word r0 / 32: two 16-byte-aligned reads and a dword select (round 4:
    // 5 dword reads of windows 16 B apart put 32 lanes on 8 banks, 4-way conflicts; a ds_read_b128
    // lane group reading consecutive 16-byte pieces is conflict-free)
    const uint32_t q = (r0 >> 7) << 4, d = (r0 >> 5) & 3u, sft = r0 & 31u;
    const uint4 wa = *(const uint4*)(img + q), wb = *(const uint4*)(img + q + 16u);
    const uint32_t W[8] = { wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w };
    // bitwise selects (v_bfi_b32): a ?: on the lane's d compiles to a dynamic index into scratch
    const uint32_t m1 = (d & 1u) ? ~0u : 0u, m2 = (d & 2u) ? ~0u : 0u;
    uint32_t F[7], E[5];
#pragma unroll
    for (int i = 0; i < 7; ++i)
        F[i] = (m1 & W[i + 1]) | (~m1 & W[i]);
#pragma unroll
    for (int i = 0; i < 5; ++i)
        E[i] = bswap((m2 & F[i + 2]) | (~m2 & F[i]));
    if (n >= 128) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
            o[u] = bswap((uint32_t)((((uint64_t)E[u] << 32) | E[u + 1]) >> (32 - sft)));
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t pair = ((uint64_t)E[u] << 32) | E[u + 1];
            const uint32_t A = (uint32_t)(pair >> (32 - sft));
            const uint32_t B = (uint32_t)(pair >> (31 - sft));
            const int32_t c = (int32_t)n - 32 * u;
            const uint32_t mk = top_bits(c <= 0 ? 0u : (uint32_t)c);
            o[u] = bswap((A & mk) | (B & ~mk));
        }
    }
}

template <int NP, int WV>
__global__ __launch_bounds__(64 * WV) void ham_fast_decode_kernel(uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks_all, int write_back, HamFast a)
{
    constexpr int BUF = NP * 1024 + 16; // raw image + zero slack
    __shared__ __attribute__((aligned(16))) uint8_t lds[WV * BUF];
    const uint32_t lane = lane_id(), wave = wave_id();
    uint8_t* img = lds + wave * BUF;
    const uint32_t lastw = a.bs / 4 - 1;
    const uint64_t wg0 = (uint64_t)bf_wg<true>() * (WV * BF_BPW);
    const uint64_t nblocks = nblocks_all < wg0 + WV * BF_BPW ? nblocks_all : wg0 + WV * BF_BPW;
    const uint64_t stride = WV;
    uint64_t blk = wg0 + wave;
    uint4 R[NP];
    if (blk < nblocks) {
#pragma unroll
        for (int k = 0; k < NP; ++k)
            R[k] = gld16c(raw + blk * a.bs + 16u * (64u * k + lane), raw, nblocks_all * a.bs);
    }
    for (; blk < nblocks; blk += stride) {
        uint32_t X[NP][4];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            X[k][0] = R[k].x;
            X[k][1] = R[k].y;
            X[k][2] = R[k].z;
            X[k][3] = R[k].w;
        }
        const uint64_t nx = blk + stride;
        // Syndrome (round 4: fewer VALU).  S = XOR of the positions of the set bits = (XOR over odd-
        // parity words w of w) << 5 | qbits(XOR of all words).  Parity is byte-order free, so the
        // words stay in memory order and only the XOR of all words is byte-swapped.  The odd-parity
        // word XOR is built from the parities of word groups (parity(a) ^ parity(b) = parity(a ^ b)):
        // the lane's word w = 256 k + 4 lane + u contributes 4 lane if odd, plus 256 k + u, whose bits
        // are the parities of the words with that bit of k or u set.  Only the block's last word (lane
        // 63, piece NP - 1, u = 3) holds bits past L, which are not part of the code.
        if (data) {
#pragma unroll
            for (int k = 0; k < NP; ++k)
                *(uint4*)(img + 16u * (64u * k + lane)) = make_uint4(X[k][0], X[k][1], X[k][2], X[k][3]);
            if (lane < 4)
                *(uint32_t*)(img + NP * 1024 + 4 * lane) = 0;
        }
        uint32_t xk[NP][4];
#pragma unroll
        for (int k = 0; k < NP; ++k)
#pragma unroll
            for (int u = 0; u < 4; ++u)
                xk[k][u] = X[k][u];
        if (lane == 63)
            xk[NP - 1][3] &= bswap(top_bits(a.L - 32u * lastw + 1u));
        uint32_t ax = 0, xu0 = 0, xu1 = 0, xk0 = 0, xk1 = 0;
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const uint32_t g = xk[k][0] ^ xk[k][1] ^ xk[k][2] ^ xk[k][3];
            ax ^= g;
            xu0 ^= xk[k][1] ^ xk[k][3];
            xu1 ^= xk[k][2] ^ xk[k][3];
            if (k & 1)
                xk0 ^= g;
            if (k & 2)
                xk1 ^= g;
        }
        const uint32_t pall = __builtin_popcount(ax) & 1u;
        const uint32_t aw = (pall ? 4u * lane : 0u) | (__builtin_popcount(xu0) & 1u) | ((__builtin_popcount(xu1) & 1u) << 1)
            | ((__builtin_popcount(xk0) & 1u) << 8) | ((__builtin_popcount(xk1) & 1u) << 9);
        const uint32_t red = wave_xor(((aw << 5 | qbits(bswap(ax))) << 1) | pall);
        const uint32_t S = red >> 1, par = red & 1u;
        const uint32_t st = par ? 1u : (S ? 5u : 0u);
        uint8_t* rb = raw + blk * a.bs;
        // the owner lane of bit S (raw word S >> 5 = 256 k + 4 lane + u) flips it in the LDS image
        // below and writes the corrected byte back from there (round 4: it read the byte back from
        // global memory, a dependent load in every corrected block); without a payload output there
        // is no image, and the byte is patched in place
        const bool owner = par && ((S >> 7) & 63u) == lane;
        if (!data && owner && write_back && PPFS_DBG_OK(rb + (S >> 3), 1, raw, nblocks_all * a.bs))
            rb[S >> 3] = (uint8_t)(rb[S >> 3] ^ (0x80u >> (S & 7u)));
        if (data && st != 5) {
            // the correction, after the image stores of the same wave (LDS ops of a wave run in order)
            if (owner) {
                __hip_atomic_fetch_xor((uint32_t*)(img + ((S >> 5) << 2)), 0x80u << (8 * ((S >> 3) & 3u)) >> (S & 7u),
                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            // payload row [blk ds, +ds) as 16-byte pieces of the global 16-byte grid
            const uint64_t start = blk * a.ds, a0 = start & ~15ull;
            const uint32_t m = (uint32_t)(start - a0);
            const uint32_t npc = (m + a.ds + 15) >> 4;
            auto store = [&](uint32_t p, int32_t b0, const uint32_t (&o)[4]) {
                uint8_t* dst = data + a0 + 16ull * p;
                [[maybe_unused]] const int32_t lo = b0 < 0 ? -b0 : 0, hi = b0 + 16 > (int32_t)a.ds ? (int32_t)a.ds - b0 : 16;
                if (!PPFS_DBG_OK(dst + lo, hi - lo, data, a.data_bytes))
                    return;
                if (b0 >= 0 && b0 + 16 <= (int32_t)a.ds)
                    gst16(dst, make_uint4(o[0], o[1], o[2], o[3]));
                else
                    store_piece_part(dst, o, b0 < 0 ? (uint32_t)(-b0) : 0u,
                        b0 + 16 > (int32_t)a.ds ? (uint32_t)((int32_t)a.ds - b0) : 16u);
            };
            // piece k = 0: the row's first bytes (payload bits below 64, several parity
            // positions) sit in the pieces of lanes 0 and 1 only
            {
                const int32_t b0 = (int32_t)(16 * lane) - (int32_t)m;
                uint32_t o[4];
                if (b0 >= 8) {
                    ham_mid_piece(img, (uint32_t)b0, o);
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int32_t i = 8 * (b0 + 4 * u);
                        uint32_t v;
                        if (i < 0)
                            v = i <= -32 ? 0u : ham_head32(img, 0) >> (uint32_t)(-i);
                        else if (i < 64)
                            v = ham_head32(img, (uint32_t)i);
                        else
                            v = ham_mid32(img, (uint32_t)i);
                        o[u] = bswap(v);
                    }
                }
                store(lane, b0, o);
            }
            // pieces k >= 1: no head path; one rolled loop keeps the live state to one piece
#pragma unroll 1
            for (int k = 1; k <= NP; ++k) {
                const uint32_t p = 64u * k + lane;
                if (p >= npc)
                    break;
                const int32_t b0 = (int32_t)(16 * p) - (int32_t)m;
                uint32_t o[4];
                ham_mid_piece(img, (uint32_t)b0, o);
                store(p, b0, o);
            }
            // the corrected byte (the owner lane: after its flip)
            if (owner && write_back && PPFS_DBG_OK(rb + (S >> 3), 1, raw, nblocks_all * a.bs))
                rb[S >> 3] = img[S >> 3];
        }
        if (status && lane == 0 && PPFS_DBG_OK(status + blk, 1, status, nblocks_all))
            status[blk] = (uint8_t)st;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        (void)lastw;
        if (nx < nblocks) {
#pragma unroll
            for (int k = 0; k < NP; ++k)
                R[k] = gld16c(raw + nx * a.bs + 16u * (64u * k + lane), raw, nblocks_all * a.bs);
        }
    }
}

// ------------------------------------------------------------------------------------
// Parity
// ------------------------------------------------------------------------------------
// raw piece p (16 B) of the row from the payload superset pieces own = p and nxt = p + 1, with
// the payload starting m bytes into piece 0 (m wave-uniform: a uniform branch per dword offset)
__device__ __forceinline__ uint4 shift_pieces(uint4 own, uint4 nxt, uint32_t m)
{
    const uint32_t W[8] = { own.x, own.y, own.z, own.w, nxt.x, nxt.y, nxt.z, nxt.w };
    const uint32_t sh = 8 * (m & 3u);
    uint32_t o[4];
    switch (m >> 2) {
#define PPFS_SHIFT_CASE(D)                                                                                             \
    case D:                                                                                                            \
        for (int u = 0; u < 4; ++u)                                                                                    \
            o[u] = __builtin_amdgcn_alignbit(W[u + D + 1], W[u + D], sh);                                              \
        break;
        PPFS_SHIFT_CASE(0)
        PPFS_SHIFT_CASE(1)
        PPFS_SHIFT_CASE(2)
    default:
        PPFS_SHIFT_CASE(3)
#undef PPFS_SHIFT_CASE
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// The neighbour pieces of a wave's 16-byte pieces by whole-wave DPP moves (VALU; round 4 replaced
// ds_bpermute + v_readlane: CRC check -0.5 %, the rest unchanged, r4w): next_piece gives lane l
// own[l + 1] and lane 63 nxt[0] (wave_rol:1 of nxt, then wave_shl:1 of own over it -- lane 63 has
// no wave_shl source and keeps the rotated value); prev_piece the mirror (wave_ror:1, wave_shr:1:
// lane 0 gets prv[63], or zero for the first piece)
__device__ __forceinline__ uint32_t next_lane(uint32_t own, uint32_t nxt)
{
    const int r = __builtin_amdgcn_mov_dpp((int)nxt, 0x134, 0xF, 0xF, false);        // wave_rol:1
    return (uint32_t)__builtin_amdgcn_update_dpp(r, (int)own, 0x130, 0xF, 0xF, false); // wave_shl:1
}
__device__ __forceinline__ uint32_t prev_lane(uint32_t own, uint32_t prv)
{
    const int r = __builtin_amdgcn_mov_dpp((int)prv, 0x13C, 0xF, 0xF, false);        // wave_ror:1
    return (uint32_t)__builtin_amdgcn_update_dpp(r, (int)own, 0x138, 0xF, 0xF, false); // wave_shr:1
}
__device__ __forceinline__ uint4 next_piece(uint4 own, uint4 nxt)
{
    return make_uint4(next_lane(own.x, nxt.x), next_lane(own.y, nxt.y), next_lane(own.z, nxt.z), next_lane(own.w, nxt.w));
}
template <bool FIRST> __device__ __forceinline__ uint4 prev_piece(uint4 own, uint4 prv)
{
    if constexpr (FIRST)
        prv = make_uint4(0, 0, 0, 0);
    return make_uint4(prev_lane(own.x, prv.x), prev_lane(own.y, prv.y), prev_lane(own.z, prv.z), prev_lane(own.w, prv.w));
}

struct ParFast {
    uint32_t bs;
    uint64_t data_bytes;
};

template <int NP, int WV>
__global__ __launch_bounds__(64 * WV) void parity_fast_encode_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, const uint8_t* __restrict__ skip, uint64_t nblocks_all, ParFast a)
{
    const uint32_t lane = lane_id(), wave = wave_id();
    const uint32_t ds = a.bs - 1;
    const HamFast ha { a.bs, ds, 0, a.data_bytes };
    const uint64_t wg0 = (uint64_t)bf_wg<true>() * (WV * BF_BPW);
    const uint64_t nblocks = nblocks_all < wg0 + WV * BF_BPW ? nblocks_all : wg0 + WV * BF_BPW;
    const uint64_t stride = WV;
    uint64_t blk = wg0 + wave;
    HamEncStage<NP> cur;
    if (blk < nblocks)
        ham_stage_load<NP, PAR_ENC_NTLD>(cur, data, blk, ha, lane);
    for (; blk < nblocks; blk += stride) {
        const uint64_t nx = blk + stride;
        const uint32_t m = (uint32_t)((blk * ds) & 15u);
        uint8_t* rb = raw + blk * a.bs;
        const uint32_t old_last = (lane == 63 && PPFS_DBG_OK(rb + a.bs - 1, 1, raw, nblocks_all * a.bs)) ? rb[a.bs - 1] : 0u;
        uint4 O[NP];
        uint32_t ones = 0;
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            // next piece: lane + 1 of this group, or lane 0 of the next group (or the extra piece)
            const uint4 nb = next_piece(cur.v[k], cur.v[k + 1]);
            uint4 o = shift_pieces(cur.v[k], nb, m);
            if (k == NP - 1 && lane == 63)
                o.w = (o.w & 0x00FFFFFFu) | (old_last << 24); // raw byte bs-1: old contents
            ones += __builtin_popcount(o.x) + __builtin_popcount(o.y) + __builtin_popcount(o.z) + __builtin_popcount(o.w);
            O[k] = o;
        }
        const uint32_t odd = wave_xor(ones & 1u);
        if (!(skip && PPFS_DBG_OK(skip + blk, 1, skip, nblocks_all) && skip[blk] == 5)) {
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                uint4 o = O[k];
                if (k == NP - 1 && lane == 63)
                    o.w ^= odd << 24; // LSB of the last byte fixes the parity
                if (PPFS_DBG_OK(rb + 16u * (64u * k + lane), 16, raw, nblocks_all * a.bs))
                    gst16_raw(rb + 16u * (64u * k + lane), o);
            }
        }
        if (nx < nblocks)
            ham_stage_load<NP, PAR_ENC_NTLD>(cur, data, nx, ha, lane);
    }
}

// Parity check (the payload output stored before the parity reduction: 1.633-1.637 vs 1.447-1.450 ms,
// r5est)
template <int NP, int WV>
__global__ __launch_bounds__(64 * WV) void parity_fast_check_kernel(const uint8_t* __restrict__ raw,
    uint8_t* __restrict__ data, uint8_t* __restrict__ status, uint64_t nblocks_all, ParFast a)
{
    const uint32_t lane = lane_id(), wave = wave_id();
    const uint32_t ds = a.bs - 1;
    const uint64_t wg0 = (uint64_t)bf_wg<true>() * (WV * BF_BPW);
    const uint64_t nblocks = nblocks_all < wg0 + WV * BF_BPW ? nblocks_all : wg0 + WV * BF_BPW;
    const uint64_t stride = WV;
    uint64_t blk = wg0 + wave;
    uint4 R[NP];
    if (blk < nblocks)
#pragma unroll
        for (int k = 0; k < NP; ++k)
            R[k] = gld16c(raw + blk * a.bs + 16u * (64u * k + lane), raw, nblocks_all * a.bs);
    for (; blk < nblocks; blk += stride) {
        const uint64_t nx = blk + stride;
        auto emit = [&]() {
            if (data) {
                // payload byte x = raw byte x; output pieces on the payload's global 16-byte grid:
                // piece p holds raw bytes [16 p - m, +16) = tail of raw piece p-1 + head of raw piece p
                const uint64_t start = blk * ds, a0 = start & ~15ull;
                const uint32_t m = (uint32_t)(start - a0);
#pragma unroll
                for (int k = 0; k <= NP; ++k) {
                    const uint32_t p = 64u * k + lane;
                    const uint4 own = k < NP ? R[k] : make_uint4(0, 0, 0, 0);
                    const uint4 prev = k == 0 ? prev_piece<true>(own, own) : prev_piece<false>(own, R[k > 0 ? k - 1 : 0]);
                    // bytes [16 - m, 16) of prev then [0, 16 - m) of own
                    const uint4 o = shift_pieces(prev, own, (16u - m) & 15u);
                    const uint4 oo = m == 0 ? own : o;
                    const int32_t b0 = (int32_t)(16 * p) - (int32_t)m;
                    uint8_t* dst = data + a0 + 16ull * p;
                    if (b0 >= 0 && b0 + 16 <= (int32_t)ds) {
                        if (PPFS_DBG_OK(dst, 16, data, nblocks_all * ds))
                            gst16(dst, oo);
                    } else if (b0 < (int32_t)ds && b0 + 16 > 0
                        && PPFS_DBG_OK(dst + (b0 < 0 ? -b0 : 0), (b0 + 16 > (int32_t)ds ? (int32_t)ds - b0 : 16) - (b0 < 0 ? -b0 : 0),
                            data, nblocks_all * ds)) {
                        const uint32_t w[4] = { oo.x, oo.y, oo.z, oo.w };
                        store_piece_part(dst, w, b0 < 0 ? (uint32_t)(-b0) : 0u,
                            b0 + 16 > (int32_t)ds ? (uint32_t)((int32_t)ds - b0) : 16u);
                    }
                }
            }
        };
        uint32_t ones = 0;
#pragma unroll
        for (int k = 0; k < NP; ++k)
            ones += __builtin_popcount(R[k].x) + __builtin_popcount(R[k].y) + __builtin_popcount(R[k].z)
                + __builtin_popcount(R[k].w);
        const uint32_t odd = wave_xor(ones & 1u);
        emit();
        if (status && lane == 0 && PPFS_DBG_OK(status + blk, 1, status, nblocks_all))
            status[blk] = odd ? 5 : 0;
        if (nx < nblocks) {
#pragma unroll
            for (int k = 0; k < NP; ++k)
                R[k] = gld16c(raw + nx * a.bs + 16u * (64u * k + lane), raw, nblocks_all * a.bs);
        }
    }
}


// ------------------------------------------------------------------------------------
// CRC (n <= 32): V = D(x) x^(n-1) mod P over the payload D (MSB first), stored = (V << 1) & mask
// written MSB first after the payload (crc_polynomial.cpp:56-76 stops one reduction step early;
// closed form in DESIGN.md / SURVEY.md §0.4).  Everything is a linear map of 32-bit values mod P,
// done with nibble tables ("cmap": 8 LDS lookups of u32, every lane reading the same table):
//   piece (16 B = dwords D0..D3, big-endian) -> D0 x^96 + D1 x^64 + D2 x^32 + D3 mod P;
//   a lane's pieces (1 KiB apart) by Horner with x^8192; the 64 lanes: lane l by its own map
//   x^(128 (15 - l % 16)), an XOR over each row of 16 lanes (DPP), then two tree levels x^2048,
//   x^4096 over the 4 rows; then one block-uniform factor x^e that places the zero-padded 16-byte
//   grid at the payload's real position (e < 0 uses x^-1: P(0) = 1).
// ------------------------------------------------------------------------------------
constexpr int CF_MAP = 512;                      // 8 nibbles x 16 entries x u32
constexpr int CF_M0 = 0, CF_K = 4, CF_L = 5, CF_FENC = 11, CF_FCHK = 27, CF_NMAPS = 28;
// The 16 lane maps sit transposed after the CF_NMAPS maps: dword (16 i + v) x 16 + (lane % 16) =
// entry v of nibble table i, so the lanes of a row read 16 different banks.  (Round 3, r3z: the lane
// tree's 6 dependent maps become 1 + 2; 64 per-lane maps, 32 KiB, cost a workgroup per CU.)
constexpr int CF_LANES = 16;
constexpr int CF_LANE_OFF = CF_NMAPS * CF_MAP;
// The two lane-tree maps (x^2048, x^4096) also as 6-bit tables (5 x 64 entries + 4): 6 LDS lookups
// per map instead of 8 (a 64-entry table is 2-way conflicted for ds_read_b32 and still wins, r3zc).
constexpr int CF_MAP6 = 5 * 256 + 16;
constexpr int CF_NSIX = 2;
constexpr int CF_SIX_OFF = CF_NMAPS * CF_MAP + CF_LANES * CF_MAP;
// 8-bit tables of the encode's hot maps (round 4): M0..M3, K as 4 x 256 u32 entries each: table k
// (entries v << 2 at byte k of the input word).  The piece maps M0..M3 take the payload dword in
// memory order (table k = (v << 8 (3 - k)) C, no byte swap), K takes values (table k = (v << 8k) C).
// 4 lookups per map, each address one SDWA shift of a byte; 1 KiB tables put 32 random lanes on
// 32 banks with ~3.5-way worst groups, about what the 6-bit tables' 2-way aliasing costs over 6
// lookups, for a third of the VALU (r4z: encode 1.603 vs 1.625 ms against the 6-bit maps).
constexpr int CF_EIGHT = 4096, CF_NEIGHT = 5;
constexpr int CF_EIGHT_OFF = CF_SIX_OFF + CF_NSIX * CF_MAP6;
constexpr int CF_BYTES = CF_EIGHT_OFF + CF_NEIGHT * CF_EIGHT; // 22 KiB + 2.5 KiB + 20 KiB
// The encode's LDS image: the 16 placement maps FENC (one per payload misalignment), the lane maps,
// the 6-bit tree maps, the 8-bit maps -- 39,456 B, 4 workgroups per CU.  (The check keeps the nibble
// maps: on the 8-bit maps it ran the same, r4za.)
template <int NPLACE> struct CrcLds {
    static constexpr int PLACE = 0, LANE = NPLACE * CF_MAP, SIX = LANE + CF_LANES * CF_MAP, EIGHT = SIX + CF_NSIX * CF_MAP6;
    static constexpr int BYTES = EIGHT + CF_NEIGHT * CF_EIGHT;
    static_assert(SIX % 16 == 0 && EIGHT % 16 == 0 && CF_EIGHT_OFF % 16 == 0, "16-byte staging");
    // copy the image's parts from the blob (placement maps from blob map `place0`)
    __device__ static void stage(uint8_t* tbl, const uint8_t* __restrict__ tables, int place0, uint32_t nthreads)
    {
        auto part = [&](int dst, int src, int bytes) {
            for (uint32_t p = threadIdx.x; p < (uint32_t)bytes / 16; p += nthreads)
                *(uint4*)(tbl + dst + 16 * p) = *(const uint4*)(tables + src + 16 * p);
        };
        part(PLACE, place0 * CF_MAP, NPLACE * CF_MAP);
        part(LANE, CF_LANE_OFF, CF_LANES * CF_MAP);
        part(SIX, CF_SIX_OFF, CF_NSIX * CF_MAP6);
        part(EIGHT, CF_EIGHT_OFF, CF_NEIGHT * CF_EIGHT);
    }
};
using CE = CrcLds<16>;
// Blocks per wave of the CRC kernels: a workgroup stages its maps once and then walks CRC_BPW
// consecutive WV-block groups (one contiguous range, so the full grid keeps its address order); with
// one group per workgroup the map staging read as much L2 as the blocks themselves.  Round 5 (r5crc*,
// configs leg, 2 rounds each): the encode in 6-wave workgroups x 4 blocks per wave (24 waves per CU,
// the 39 KiB map image allows 4 workgroups) 1.537-1.546 vs 1.583-1.593 ms for round 4's 4 x 8
// (12 x 2: 1.545-1.549, 8 x 4: 1.551-1.556, 5 x 4: 1.567-1.573, 4 x 4: 1.570-1.593, 6 x 8: 1.627);
// the check on its 14 KiB image in 2-wave workgroups x 4: 1.586-1.605 vs 1.603-1.628 ms for 4 x 4
// (2 x 2: 1.70, 2 x 1: 1.89, 1-wave workgroups: 1.77-2.12 -- the image then caps a CU at 11 waves).
// Round 6, with the XCD-local block ranges (r6s / r6t, configs leg, 3 interleaved rounds): the check
// in 4-wave workgroups x 4 1.594-1.606 vs 1.609-1.613 ms for 2 x 4 (8 x 4: 1.602-1.608, 3 x 4:
// 1.610-1.621, 4 x 2: 1.620-1.628, 4 x 8: 1.635-1.639, 6 x 4: 1.757-1.762); the encode's shapes
// with the XCD-local ranges (6 x 2 / 4 x 4 / 6 x 8) and 8 x 4 all ran at or above its 6 x 4.
// (Register prefetch of a wave's next block and output stores issued before the lookups: slower,
// DESIGN.md Appendix A, r5cpf / r5est.)
constexpr int CRC_BPW = 4, CRC_CHK_BPW = 4;

// (x >> 8k) & 0x3C (a nibble * 4, the entry's byte offset): one v_and_b32_sdwa for k > 0
__device__ __forceinline__ uint32_t sel3c(uint32_t x, int k)
{
    uint32_t r;
    switch (k & 3) {
    case 0:
        return x & 0x3Cu;
    case 1:
        asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
            : "=v"(r) : "v"(x), "s"(0x3Cu));
        return r;
    case 2:
        asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
            : "=v"(r) : "v"(x), "s"(0x3Cu));
        return r;
    default:
        asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
            : "=v"(r) : "v"(x), "s"(0x3Cu));
        return r;
    }
}

// v(x) * C mod P, C given by its map (tb: LDS byte address of 8 nibble tables)
__device__ __forceinline__ uint32_t cmap(const uint8_t* tb, uint32_t v)
{
    const uint32_t lo = v << 2, hi = v >> 2; // low / high nibble of byte b at bits 8b+2..8b+5
    uint32_t e[8];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        e[2 * b] = *(const uint32_t*)(tb + (2 * b) * 64 + sel3c(lo, b));
        e[2 * b + 1] = *(const uint32_t*)(tb + (2 * b + 1) * 64 + sel3c(hi, b));
    }
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(e[0], e[1], e[2], 0x96),
        __builtin_amdgcn_bitop3_b32(e[3], e[4], e[5], 0x96), e[6] ^ e[7], 0x96);
}

// v(x) * C mod P from C's 6-bit tables (the lane-tree maps)
__device__ __forceinline__ uint32_t cmap6(const uint8_t* tb, uint32_t v)
{
    uint32_t e[6];
#pragma unroll
    for (int j = 0; j < 5; ++j)
        e[j] = *(const uint32_t*)(tb + j * 256 + (__builtin_amdgcn_ubfe(v, 6 * j, 6) << 2));
    e[5] = *(const uint32_t*)(tb + 1280 + ((v >> 30) << 2));
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(e[0], e[1], e[2], 0x96), e[3], e[4] ^ e[5], 0x96);
}
// byte K of w, times 4 (a table entry's byte offset): one SDWA shift
template <int K> __device__ __forceinline__ uint32_t byte4(uint32_t w)
{
    uint32_t r;
    if constexpr (K == 0)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(w));
    else if constexpr (K == 1)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(w));
    else if constexpr (K == 2)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(w));
    else
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(w));
    return r;
}
// w * C mod P from C's 8-bit tables at tb (memory-order or value-order input, see CF_EIGHT)
__device__ __forceinline__ uint32_t cmap8(const uint8_t* tb, uint32_t w)
{
    const uint32_t e0 = *(const uint32_t*)(tb + byte4<0>(w)), e1 = *(const uint32_t*)(tb + 1024 + byte4<1>(w));
    const uint32_t e2 = *(const uint32_t*)(tb + 2048 + byte4<2>(w)), e3 = *(const uint32_t*)(tb + 3072 + byte4<3>(w));
    return __builtin_amdgcn_bitop3_b32(e0, e1, e2, 0x96) ^ e3;
}

struct CrcFast {
    uint32_t bs, ds, n, nbc, mask;
    uint64_t data_bytes;
};

// 16 payload bytes (memory order) -> piece value mod P; bytes outside [lo, hi) count as zero
__device__ __forceinline__ uint32_t crc_piece(const uint8_t* tbl, uint4 v, uint32_t lo, uint32_t hi, bool n32)
{
    uint32_t w[4] = { v.x, v.y, v.z, v.w };
    if (lo > 0 || hi < 16) {
        // bytes [lo, hi) as two 64-bit masks (a handful of shifts instead of 16 byte compares)
        auto ge = [](uint32_t b) { return b >= 8u ? 0ull : (~0ull << (8u * b)); }; // bytes >= b of 8
        const uint64_t m0 = ge(lo) & ~ge(hi);
        const uint64_t m1 = ge(lo > 8u ? lo - 8u : 0u) & ~ge(hi > 8u ? hi - 8u : 0u);
        w[0] &= (uint32_t)m0;
        w[1] &= (uint32_t)(m0 >> 32);
        w[2] &= (uint32_t)m1;
        w[3] &= (uint32_t)(m1 >> 32);
    }
    const uint32_t d3 = bswap(w[3]);
    return __builtin_amdgcn_bitop3_b32(cmap(tbl + (CF_M0 + 3) * CF_MAP, bswap(w[0])),
               cmap(tbl + (CF_M0 + 2) * CF_MAP, bswap(w[1])), cmap(tbl + (CF_M0 + 1) * CF_MAP, bswap(w[2])), 0x96)
        ^ (n32 ? d3 : cmap(tbl + CF_M0 * CF_MAP, d3));
}

// crc_piece through the 8-bit maps (te: the LDS image's CE_EIGHT): the dwords in memory order
__device__ __forceinline__ uint32_t crc_piece8(const uint8_t* te, uint4 v, uint32_t lo, uint32_t hi, bool n32)
{
    uint32_t w[4] = { v.x, v.y, v.z, v.w };
    if (lo > 0 || hi < 16) {
        auto ge = [](uint32_t b) { return b >= 8u ? 0ull : (~0ull << (8u * b)); };
        const uint64_t m0 = ge(lo) & ~ge(hi);
        const uint64_t m1 = ge(lo > 8u ? lo - 8u : 0u) & ~ge(hi > 8u ? hi - 8u : 0u);
        w[0] &= (uint32_t)m0;
        w[1] &= (uint32_t)(m0 >> 32);
        w[2] &= (uint32_t)m1;
        w[3] &= (uint32_t)(m1 >> 32);
    }
    return __builtin_amdgcn_bitop3_b32(cmap8(te + 3 * CF_EIGHT, w[0]), cmap8(te + 2 * CF_EIGHT, w[1]),
               cmap8(te + CF_EIGHT, w[2]), 0x96)
        ^ (n32 ? bswap(w[3]) : cmap8(te, w[3]));
}

// value * x^(128 (15 - lane % 16)) mod P from the transposed lane maps (at tbl + LOFF)
template <int LOFF = CF_LANE_OFF>
__device__ __forceinline__ uint32_t lane_cmap(const uint8_t* tbl, uint32_t v, uint32_t lane)
{
    const uint8_t* tb = tbl + LOFF + 4u * (lane & (CF_LANES - 1));
    uint32_t e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        e[i] = *(const uint32_t*)(tb + i * 64 * CF_LANES + (__builtin_amdgcn_ubfe(v, 4 * i, 4) << 6));
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(e[0], e[1], e[2], 0x96),
        __builtin_amdgcn_bitop3_b32(e[3], e[4], e[5], 0x96), e[6] ^ e[7], 0x96);
}

// Sum over the wave of value_l * x^(128 (63 - l)) -> wave-uniform: each lane's row factor, the row
// XOR (DPP butterfly: every lane of row r ends with R_r), then R_0 x^6144 + R_1 x^4096 + R_2 x^2048 + R_3
// by two tree levels (the maps x^(128 2^j), j = 4, 5)
// LOFF: the lane maps; SOFF: the 6-bit tree maps, or < 0: the nibble maps CF_L + 4, CF_L + 5
template <int LOFF, int SOFF>
__device__ __forceinline__ uint32_t crc_lane_sum(const uint8_t* tbl, uint32_t acc, uint32_t lane)
{
    uint32_t v = lane_cmap<LOFF>(tbl, acc, lane);
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false); // row_half_mirror
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false); // row_mirror
#pragma unroll
    for (int j = 4; j < 6; ++j) {
        const uint32_t other = __shfl_down(v, 1 << j, 64);
        if constexpr (SOFF >= 0)
            v = cmap6(tbl + SOFF + (j - 4) * CF_MAP6, v) ^ other;
        else
            v = cmap(tbl + (CF_L + j) * CF_MAP, v) ^ other;
    }
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// The lane maps put the encode kernel at 131 VGPRs: the floor keeps 4 waves per SIMD (128, no
// spills; r3z A/B 1.64 vs 1.68 ms encode, 1.660 vs 1.668 check)
#ifndef PPFS_CRC_CHK_WPE
#define PPFS_CRC_CHK_WPE 4
#endif
#define PPFS_CRC_ATTR __attribute__((amdgpu_waves_per_eu(PPFS_CRC_CHK_WPE)))
#ifndef PPFS_CRC_ENC_WPE
#define PPFS_CRC_ENC_WPE 4
#endif
#define PPFS_CRC_ENC_ATTR __attribute__((amdgpu_waves_per_eu(PPFS_CRC_ENC_WPE)))

template <int NP, int WV, int BPW>
__global__ __launch_bounds__(64 * WV) PPFS_CRC_ENC_ATTR void crc_fast_encode_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, const uint8_t* __restrict__ skip, uint64_t nblocks_all, CrcFast a,
    const uint8_t* __restrict__ tables)
{
    __shared__ __attribute__((aligned(16))) uint8_t tbl[CE::BYTES];
    CE::stage(tbl, tables, CF_FENC, 64 * WV);
    if constexpr (WV > 1) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const uint32_t lane = lane_id(), wave = WV > 1 ? wave_id() : 0u;
    const HamFast ha { a.bs, a.ds, 0, a.data_bytes };
    const bool n32 = a.n == 32;
    const uint64_t wg0 = (uint64_t)bf_wg<false>() * (WV * BPW);
    const uint64_t nblocks = nblocks_all < wg0 + WV * BPW ? nblocks_all : wg0 + WV * BPW;
    const uint64_t stride = WV;
    uint64_t blk = wg0 + wave;
    HamEncStage<NP> cur;
    if (blk < nblocks)
        ham_stage_load<NP>(cur, data, blk, ha, lane);
    for (; blk < nblocks; blk += stride) {
        const uint64_t nx = blk + stride;
        const uint32_t m = (uint32_t)((blk * a.ds) & 15u); // payload byte 0 = superset byte m
        uint8_t* rb = raw + blk * a.bs;
        // superset piece q = 64 k + lane holds superset bytes [16 q, +16); payload = [m, m + ds)
        const bool store_blk = !(skip && PPFS_DBG_OK(skip + blk, 1, skip, nblocks_all) && skip[blk] == 5);
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k <= NP; ++k) {
            const int32_t q16 = 16 * (64 * k + (int32_t)lane);
            const int32_t lo = (int32_t)m - q16, hi = (int32_t)(m + a.ds) - q16;
            const uint32_t lo_c = lo < 0 ? 0u : (lo > 16 ? 16u : (uint32_t)lo);
            const uint32_t hi_c = hi < 0 ? 0u : (hi > 16 ? 16u : (uint32_t)hi);
            const uint32_t pv = crc_piece8(tbl + CE::EIGHT, cur.v[k], lo_c, hi_c > lo_c ? hi_c : lo_c, n32);
            acc = k == 0 ? pv : (cmap8(tbl + CE::EIGHT + 4 * CF_EIGHT, acc) ^ pv);
        }
        const uint32_t Vs = crc_lane_sum<CE::LANE, CE::SIX>(tbl, acc, lane);
        const uint32_t V = cmap(tbl + CE::PLACE + m * CF_MAP, Vs);
        const uint32_t st = (V << 1) & a.mask;
        if (store_blk) {
            // raw bytes [ds, ds + nbc): the n CRC bits MSB first (a partial last byte keeps its old
            // low bits); all in the row's last raw piece (lane 63, k = NP - 1)
            uint32_t old_last = 0;
            if (lane == 63 && (a.n & 7u) && PPFS_DBG_OK(rb + a.ds + a.nbc - 1, 1, raw, nblocks_all * a.bs))
                old_last = rb[a.ds + a.nbc - 1];
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                const uint4 nb = next_piece(cur.v[k], cur.v[k + 1]);
                uint4 o = shift_pieces(cur.v[k], nb, m);
                if (k == NP - 1 && lane == 63) {
                    // the field is the block's last nbc (<= 4) bytes (bs = ds + nbc), i.e. the top nbc
                    // bytes of the last dword: the n CRC bits left-aligned, MSB first, a partial last
                    // byte keeping its old low bits (round 4: byte by byte, ~100 VALU per block)
                    const uint32_t sh = 8u * (4u - a.nbc), rbits = a.n & 7u;
                    const uint32_t field = bswap(st << (32u - a.n)) << sh;
                    const uint32_t fmask = 0xFFFFFFFFu << sh;
                    const uint32_t keep = rbits ? ((1u << (8u - rbits)) - 1u) << 24 : 0u; // old low bits
                    o.w = (o.w & ~fmask) | field | ((old_last << 24) & keep);
                }
                if (PPFS_DBG_OK(rb + 16u * (64u * k + lane), 16, raw, nblocks_all * a.bs))
                    gst16_raw(rb + 16u * (64u * k + lane), o);
            }
        }
        if (nx < nblocks)
            ham_stage_load<NP>(cur, data, nx, ha, lane);
    }
}

// The check's LDS image (round 5): only the maps it reads -- M0..M3, K, the lane tree L..L+5
// (blob maps 0-10), FCHK (blob map 27, here map 11) and the lane maps: 14 KiB where it used to
// stage the blob's first 22.5 KiB (the encode's 16 placement maps included).  (The encode's 8-bit
// piece and Horner maps here instead, a 31 KiB image: same or +2 %, r4za / r4zb.)
constexpr int CK_FCHK = 11, CK_LANE_OFF = 12 * CF_MAP, CK_BYTES = CK_LANE_OFF + CF_LANES * CF_MAP;
template <int NP, int WV, int BPW>
__global__ __launch_bounds__(64 * WV) PPFS_CRC_ATTR void crc_fast_check_kernel(const uint8_t* __restrict__ raw,
    uint8_t* __restrict__ data, uint8_t* __restrict__ status, uint64_t nblocks_all, CrcFast a,
    const uint8_t* __restrict__ tables)
{
    __shared__ __attribute__((aligned(16))) uint8_t tbl[CK_BYTES];
    for (uint32_t p = threadIdx.x; p < CK_BYTES / 16; p += 64 * WV) {
        const uint32_t o = 16 * p;
        // maps 0-10 in place, then FCHK, then the lane maps
        const uint32_t src = o < CK_FCHK * CF_MAP ? o : (o < CK_LANE_OFF ? CF_FCHK * CF_MAP + (o - CK_FCHK * CF_MAP) : CF_LANE_OFF + (o - CK_LANE_OFF));
        *(uint4*)(tbl + o) = *(const uint4*)(tables + src);
    }
    if constexpr (WV > 1) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const uint32_t lane = lane_id(), wave = WV > 1 ? wave_id() : 0u;
    const bool n32 = a.n == 32;
    const uint32_t ds = a.ds;
    const uint64_t wg0 = (uint64_t)bf_wg<true>() * (WV * BPW);
    const uint64_t nblocks = nblocks_all < wg0 + WV * BPW ? nblocks_all : wg0 + WV * BPW;
    const uint64_t stride = WV;
    uint64_t blk = wg0 + wave;
    uint4 R[NP];
    if (blk < nblocks)
#pragma unroll
        for (int k = 0; k < NP; ++k)
            R[k] = gld16c(raw + blk * a.bs + 16u * (64u * k + lane), raw, nblocks_all * a.bs);
    for (; blk < nblocks; blk += stride) {
        const uint64_t nx = blk + stride;
        auto emit = [&]() {
            if (data) {
                const uint64_t start = blk * ds, a0 = start & ~15ull;
                const uint32_t m = (uint32_t)(start - a0);
#pragma unroll
                for (int k = 0; k <= NP; ++k) {
                    const uint32_t p = 64u * k + lane;
                    const uint4 own = k < NP ? R[k] : make_uint4(0, 0, 0, 0);
                    const uint4 prev = k == 0 ? prev_piece<true>(own, own) : prev_piece<false>(own, R[k > 0 ? k - 1 : 0]);
                    const uint4 oo = m == 0 ? own : shift_pieces(prev, own, (16u - m) & 15u);
                    const int32_t b0 = (int32_t)(16 * p) - (int32_t)m;
                    uint8_t* dst = data + a0 + 16ull * p;
                    if (b0 >= 0 && b0 + 16 <= (int32_t)ds) {
                        if (PPFS_DBG_OK(dst, 16, data, nblocks_all * ds))
                            gst16(dst, oo);
                    } else if (b0 < (int32_t)ds && b0 + 16 > 0
                        && PPFS_DBG_OK(dst + (b0 < 0 ? -b0 : 0), (b0 + 16 > (int32_t)ds ? (int32_t)ds - b0 : 16) - (b0 < 0 ? -b0 : 0),
                            data, nblocks_all * ds)) {
                        const uint32_t w[4] = { oo.x, oo.y, oo.z, oo.w };
                        store_piece_part(dst, w, b0 < 0 ? (uint32_t)(-b0) : 0u,
                            b0 + 16 > (int32_t)ds ? (uint32_t)((int32_t)ds - b0) : 16u);
                    }
                }
            }
        };
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const int32_t q16 = 16 * (64 * k + (int32_t)lane);
            const int32_t hi = (int32_t)ds - q16;
            const uint32_t hi_c = hi < 0 ? 0u : (hi > 16 ? 16u : (uint32_t)hi);
            const uint32_t pv = crc_piece(tbl, R[k], 0u, hi_c, n32);
            acc = k == 0 ? pv : (cmap(tbl + CF_K * CF_MAP, acc) ^ pv);
        }
        const uint32_t V = cmap(tbl + CK_FCHK * CF_MAP, crc_lane_sum<CK_LANE_OFF, -1>(tbl, acc, lane));
        const uint32_t st = (V << 1) & a.mask;
        // stored field: n bits MSB first from byte ds (in the last raw piece, lane 63)
        const uint4 last = make_uint4(__builtin_amdgcn_readlane(R[NP - 1].x, 63), __builtin_amdgcn_readlane(R[NP - 1].y, 63),
            __builtin_amdgcn_readlane(R[NP - 1].z, 63), __builtin_amdgcn_readlane(R[NP - 1].w, 63));
        const uint32_t lw[4] = { last.x, last.y, last.z, last.w };
        const uint32_t base = ds - 16u * (64u * (NP - 1) + 63u);
        uint64_t f = 0;
        for (uint32_t u = 0; u < a.nbc; ++u) {
            const uint32_t b = base + u;
            f = (f << 8) | ((lw[b >> 2] >> (8 * (b & 3))) & 0xFFu);
        }
        const uint32_t field = (uint32_t)(f >> (8 * a.nbc - a.n));
        emit();
        if (status && lane == 0 && PPFS_DBG_OK(status + blk, 1, status, nblocks_all))
            status[blk] = (st == field) ? 0 : 5;
        if (nx < nblocks) {
#pragma unroll
            for (int k = 0; k < NP; ++k)
                R[k] = gld16c(raw + nx * a.bs + 16u * (64u * k + lane), raw, nblocks_all * a.bs);
        }
    }
}

} // namespace bf
} // namespace ppfs

using namespace ppfs;

// Full grid: one wave per block, WV blocks per workgroup of WV waves (see BF_PREFETCH above); the
// entry points refuse batches whose grid would pass 2^30 workgroups.
template <typename K> static uint32_t bf_grid(K, uint64_t nb, int wv = bf::WAVES)
{
    const uint64_t want = (nb + (uint64_t)wv - 1) / (uint64_t)wv;
    const uint64_t cap = 1ull << 30;
    return (uint32_t)(want < cap ? (want ? want : 1) : cap);
}

// Waves per workgroup of the Hamming and parity kernels (each wave owns its blocks and its LDS
// buffer: no workgroup barrier).  Round 5: a wave-per-4-KiB-block copy with no coding work
// (tools/probes/stream_ceiling.hip, r5ce_*) moves 6.5-6.6 TB/s in one-wave workgroups at 6-8 waves per
// CU against 5.9-6.2 TB/s in 4-wave workgroups at any cap -- fewer bytes in flight, and a freed
// wave slot refills at once.  Measured on the kernels (configs leg, r5wv_* / r5wv2_*, two rounds):
// parity encode in one-wave workgroups at 12 waves per CU 1.323-1.325 vs 1.393-1.398 ms (10: 1.338,
// 14: 1.346-1.351, two-wave at 12: 1.346-1.349); parity check at 10 waves 1.462-1.463 vs 1.516-1.521
// (8: 1.60, 12: 1.471-1.477); Hamming encode one-wave, uncapped (16 waves by registers) 1.418-1.423
// vs 1.466-1.468 (two-wave 1.443-1.448, one-wave at 12: 1.494-1.497).  The Hamming decode keeps
// 4-wave workgroups (round 5 at 16 waves per CU, round 6 at 24, below): one-wave at 20 / 24 / 32 waves
// 1.545-1.561 / 1.611 vs 1.523-1.527 ms clean, at 6 / 8 waves 3.10 / 2.41 ms (its per-block chain
// needs the waves); round 6: 2- and 8-wave workgroups at 16 waves 1.504-1.515 / 1.538-1.552 ms.
#ifndef PPFS_BF_HAM_ENC_WV
#define PPFS_BF_HAM_ENC_WV 1
#endif
#ifndef PPFS_BF_HAM_DEC_WV
#define PPFS_BF_HAM_DEC_WV 4
#endif
#ifndef PPFS_BF_PAR_ENC_WV
#define PPFS_BF_PAR_ENC_WV 1
#endif
#ifndef PPFS_BF_PAR_CHK_WV
#define PPFS_BF_PAR_CHK_WV 1
#endif

// Workgroups per CU of the streaming kernels (PPFS_BF_*_WG), enforced by dynamic LDS (0 = as many as
// registers and static LDS allow).  One 4 KiB block per wave is in flight per wave.  Round 4 (cfg4,
// r4x / r4zc): parity encode 6 -> 4 -> 3 workgroups -2.5 % / -0.7 %, parity check at 3 -3.3 %
// (at 4 and 2 no gain), Hamming decode 9 -> 4 -1.5-2 % (3: +7 %), Hamming encode (4 by registers)
// and the CRC kernels: no gain at 4, slower at 3 (CRC encode +1 %, check +4 %, r4zh).
static constexpr uint32_t bf_occ_lds(int wg, uint32_t static_lds)
{
    return wg <= 0 ? 0u : (163840u / (uint32_t)(wg + 1) + 256u > static_lds ? 163840u / (uint32_t)(wg + 1) + 256u - static_lds : 0u);
}
// Hamming / parity: the cap in waves per CU (0 = none), i.e. WV-wave workgroups per CU x WV.
// Re-swept in round 6 with the XCD-local block ranges (r6u / r6v, configs leg, 3 interleaved
// rounds): the Hamming decode at 24 waves per CU clean 1.433-1.443 vs 1.487-1.497 ms at 16, 1-error
// 1.493-1.506 vs 1.551-1.556 (20: 1.449-1.456 / 1.502-1.505, 28: 1.444-1.450 / 1.508-1.516,
// uncapped: 1.463-1.465 / 1.534-1.536); the parity check at 12 1.371-1.374 vs 1.388-1.390 at 10
// (11 / 14: the same as 12, 16: 1.378-1.380, 8: 1.52); the parity encode at 10 / 16 and the
// Hamming encode at 12: the same or slower.
#ifndef PPFS_BF_PAR_ENC_WPC
#define PPFS_BF_PAR_ENC_WPC 12
#endif
#ifndef PPFS_BF_HAM_DEC_WPC
#define PPFS_BF_HAM_DEC_WPC 24
#endif
#ifndef PPFS_BF_HAM_ENC_WPC
#define PPFS_BF_HAM_ENC_WPC 0
#endif
#ifndef PPFS_BF_PAR_CHK_WPC
#define PPFS_BF_PAR_CHK_WPC 12
#endif
static constexpr int bf_wg_cap(int wpc, int wv) { return wpc <= 0 ? 0 : (wpc / wv > 0 ? wpc / wv : 1); }
template <int NP> static constexpr uint32_t par_enc_dyn_lds()
{
    return bf_occ_lds(bf_wg_cap(PPFS_BF_PAR_ENC_WPC, PPFS_BF_PAR_ENC_WV), 0);
}
template <int NP> static constexpr uint32_t ham_dec_dyn_lds()
{
    constexpr int wv = PPFS_BF_HAM_DEC_WV;
    return bf_occ_lds(bf_wg_cap(PPFS_BF_HAM_DEC_WPC, wv), wv * (NP * 1024 + 16)); // ham_fast_decode_kernel's lds[]
}
template <int NP> static constexpr uint32_t ham_enc_dyn_lds()
{
    constexpr int wv = PPFS_BF_HAM_ENC_WV;
    return bf_occ_lds(bf_wg_cap(PPFS_BF_HAM_ENC_WPC, wv), wv * ((NP + 1) * 1024 + 32)); // ham_fast_encode_kernel's lds[]
}
template <int NP> static constexpr uint32_t par_chk_dyn_lds()
{
    return bf_occ_lds(bf_wg_cap(PPFS_BF_PAR_CHK_WPC, PPFS_BF_PAR_CHK_WV), 0);
}
// CRC check: PPFS_BF_CRC_CHK_WV waves per workgroup, PPFS_CRC_CHK_BPW blocks per wave, at most
// PPFS_BF_CRC_CHK_WPC waves per CU (0: as registers allow)
#ifndef PPFS_BF_CRC_CHK_WV
#define PPFS_BF_CRC_CHK_WV 4
#endif
#ifndef PPFS_BF_CRC_CHK_WPC
#define PPFS_BF_CRC_CHK_WPC 0
#endif
template <int NP> static constexpr uint32_t crc_chk_dyn_lds()
{
    return bf_occ_lds(bf_wg_cap(PPFS_BF_CRC_CHK_WPC, PPFS_BF_CRC_CHK_WV), bf::CK_BYTES);
}
// CRC encode: PPFS_BF_CRC_ENC_WV waves per workgroup, PPFS_CRC_BPW blocks per wave, at most
// PPFS_BF_CRC_ENC_WPC waves per CU (0: as LDS and registers allow)
#ifndef PPFS_BF_CRC_ENC_WV
#define PPFS_BF_CRC_ENC_WV 6
#endif
#ifndef PPFS_BF_CRC_ENC_WPC
#define PPFS_BF_CRC_ENC_WPC 0
#endif
template <int NP> static constexpr uint32_t crc_enc_dyn_lds()
{
    return bf_occ_lds(bf_wg_cap(PPFS_BF_CRC_ENC_WPC, PPFS_BF_CRC_ENC_WV), bf::CE::BYTES);
}
template <int NP> static constexpr uint32_t no_dyn_lds() { return 0; }

extern "C" int ppfs_bitfast_supported(uint32_t bs) { return bs == 1024 || bs == 2048 || bs == 4096; }

#define PPFS_NP_DISPATCH_SH(bs, KERNEL, nb, SH, ...)                                                                  \
    switch (bs) {                                                                                                      \
    case 1024:                                                                                                         \
        PPFS_LAUNCH(KERNEL<1>, dim3(bf_grid(KERNEL<1>, nb)), dim3(256), SH<1>(), __VA_ARGS__);                  \
        break;                                                                                                         \
    case 2048:                                                                                                         \
        PPFS_LAUNCH(KERNEL<2>, dim3(bf_grid(KERNEL<2>, nb)), dim3(256), SH<2>(), __VA_ARGS__);                  \
        break;                                                                                                         \
    default:                                                                                                           \
        PPFS_LAUNCH(KERNEL<4>, dim3(bf_grid(KERNEL<4>, nb)), dim3(256), SH<4>(), __VA_ARGS__);                  \
        break;                                                                                                         \
    }
#define PPFS_NP_DISPATCH(bs, KERNEL, nb, ...) PPFS_NP_DISPATCH_SH(bs, KERNEL, nb, no_dyn_lds, __VA_ARGS__)
// the Hamming / parity kernels: WV waves per workgroup
#define PPFS_NP_DISPATCH_WV(bs, KERNEL, WV, nb, SH, ...)                                                               \
    switch (bs) {                                                                                                      \
    case 1024:                                                                                                         \
        PPFS_LAUNCH((KERNEL<1, WV>), dim3(bf_grid(KERNEL<1, WV>, nb, WV)), dim3(64 * WV), SH<1>(), __VA_ARGS__);       \
        break;                                                                                                         \
    case 2048:                                                                                                         \
        PPFS_LAUNCH((KERNEL<2, WV>), dim3(bf_grid(KERNEL<2, WV>, nb, WV)), dim3(64 * WV), SH<2>(), __VA_ARGS__);       \
        break;                                                                                                         \
    default:                                                                                                           \
        PPFS_LAUNCH((KERNEL<4, WV>), dim3(bf_grid(KERNEL<4, WV>, nb, WV)), dim3(64 * WV), SH<4>(), __VA_ARGS__);       \
        break;                                                                                                         \
    }

extern "C" hipError_t ppfs_ham_fast_encode(const uint8_t* d, uint8_t* r, const uint8_t* skip, uint64_t nb, uint32_t bs,
    uint32_t ds, uint32_t L, hipStream_t s)
{
    const bf::HamFast a { bs, ds, L, nb * (uint64_t)ds };
    if ((nb + (uint64_t)PPFS_BF_HAM_ENC_WV * bf::BF_BPW - 1) / ((uint64_t)PPFS_BF_HAM_ENC_WV * bf::BF_BPW) > (1ull << 30))
        return hipErrorInvalidValue;
    PPFS_NP_DISPATCH_WV(bs, bf::ham_fast_encode_kernel, PPFS_BF_HAM_ENC_WV, (nb + bf::BF_BPW - 1) / bf::BF_BPW, ham_enc_dyn_lds, s, d, r,
        skip, nb, a)
    return hipGetLastError();
}

extern "C" hipError_t ppfs_ham_fast_decode(uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb, int wb, uint32_t bs,
    uint32_t ds, uint32_t L, hipStream_t s)
{
    const bf::HamFast a { bs, ds, L, nb * (uint64_t)ds };
    if ((nb + (uint64_t)PPFS_BF_HAM_DEC_WV * bf::BF_BPW - 1) / ((uint64_t)PPFS_BF_HAM_DEC_WV * bf::BF_BPW) > (1ull << 30))
        return hipErrorInvalidValue;
    if (L < 32u * (bs / 4u - 1u) || L >= 8u * bs) // the kernel masks the last word only (true for 1-4 KiB)
        return hipErrorInvalidValue;
    PPFS_NP_DISPATCH_WV(bs, bf::ham_fast_decode_kernel, PPFS_BF_HAM_DEC_WV, (nb + bf::BF_BPW - 1) / bf::BF_BPW,
        ham_dec_dyn_lds, s, r, d, st, nb, wb, a)
    return hipGetLastError();
}

// The table blob's layout for the host builder (api.cpp build_crc_fast_tables), in this order:
// map bytes, maps, lane-map offset, lane maps, 6-bit offset, 6-bit maps, 6-bit map bytes, 8-bit
// offset, 8-bit maps, 8-bit map bytes, total bytes
extern "C" int ppfs_crc_fast_layout(int32_t* v, int n)
{
    const int32_t L[] = { bf::CF_MAP, bf::CF_NMAPS, bf::CF_LANE_OFF, bf::CF_LANES, bf::CF_SIX_OFF, bf::CF_NSIX, bf::CF_MAP6,
        bf::CF_EIGHT_OFF, bf::CF_NEIGHT, bf::CF_EIGHT, bf::CF_BYTES };
    const int m = (int)(sizeof(L) / sizeof(L[0]));
    for (int i = 0; i < m && i < n; ++i)
        v[i] = L[i];
    return m;
}

extern "C" hipError_t ppfs_crc_fast_encode(const uint8_t* d, uint8_t* r, const uint8_t* skip, uint64_t nb, uint32_t bs,
    uint32_t ds, uint32_t n, uint64_t mask, const uint8_t* tab, hipStream_t s)
{
    const bf::CrcFast a { bs, ds, n, bs - ds, (uint32_t)mask, nb * (uint64_t)ds };
    constexpr uint64_t per_wg = (uint64_t)PPFS_BF_CRC_ENC_WV * bf::CRC_BPW;
    if ((nb + per_wg - 1) / per_wg > (1ull << 30))
        return hipErrorInvalidValue;
    constexpr int wv = PPFS_BF_CRC_ENC_WV, bpw = bf::CRC_BPW;
    const uint64_t nw = (nb + bpw - 1) / bpw; // waves
    switch (bs) {
    case 1024:
        PPFS_LAUNCH((bf::crc_fast_encode_kernel<1, wv, bpw>), dim3(bf_grid(0, nw, wv)), dim3(64 * wv), crc_enc_dyn_lds<1>(), s, d,
            r, skip, nb, a, tab);
        break;
    case 2048:
        PPFS_LAUNCH((bf::crc_fast_encode_kernel<2, wv, bpw>), dim3(bf_grid(0, nw, wv)), dim3(64 * wv), crc_enc_dyn_lds<2>(), s, d,
            r, skip, nb, a, tab);
        break;
    default:
        PPFS_LAUNCH((bf::crc_fast_encode_kernel<4, wv, bpw>), dim3(bf_grid(0, nw, wv)), dim3(64 * wv), crc_enc_dyn_lds<4>(), s, d,
            r, skip, nb, a, tab);
        break;
    }
    return hipGetLastError();
}

extern "C" hipError_t ppfs_crc_fast_check(const uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb, uint32_t bs,
    uint32_t ds, uint32_t n, uint64_t mask, const uint8_t* tab, hipStream_t s)
{
    const bf::CrcFast a { bs, ds, n, bs - ds, (uint32_t)mask, nb * (uint64_t)ds };
    constexpr uint64_t per_wg = (uint64_t)PPFS_BF_CRC_CHK_WV * bf::CRC_CHK_BPW;
    if ((nb + per_wg - 1) / per_wg > (1ull << 30))
        return hipErrorInvalidValue;
    constexpr int wv = PPFS_BF_CRC_CHK_WV, bpw = bf::CRC_CHK_BPW;
    const uint64_t nw = (nb + bpw - 1) / bpw; // waves
    switch (bs) {
    case 1024:
        PPFS_LAUNCH((bf::crc_fast_check_kernel<1, wv, bpw>), dim3(bf_grid(0, nw, wv)), dim3(64 * wv), crc_chk_dyn_lds<1>(), s, r,
            d, st, nb, a, tab);
        break;
    case 2048:
        PPFS_LAUNCH((bf::crc_fast_check_kernel<2, wv, bpw>), dim3(bf_grid(0, nw, wv)), dim3(64 * wv), crc_chk_dyn_lds<2>(), s, r,
            d, st, nb, a, tab);
        break;
    default:
        PPFS_LAUNCH((bf::crc_fast_check_kernel<4, wv, bpw>), dim3(bf_grid(0, nw, wv)), dim3(64 * wv), crc_chk_dyn_lds<4>(), s, r,
            d, st, nb, a, tab);
        break;
    }
    return hipGetLastError();
}

extern "C" hipError_t ppfs_parity_fast_encode(const uint8_t* d, uint8_t* r, const uint8_t* skip, uint64_t nb,
    uint32_t bs, hipStream_t s)
{
    const bf::ParFast a { bs, nb * (uint64_t)(bs - 1) };
    if ((nb + (uint64_t)PPFS_BF_PAR_ENC_WV * bf::BF_BPW - 1) / ((uint64_t)PPFS_BF_PAR_ENC_WV * bf::BF_BPW) > (1ull << 30))
        return hipErrorInvalidValue;
    PPFS_NP_DISPATCH_WV(bs, bf::parity_fast_encode_kernel, PPFS_BF_PAR_ENC_WV, (nb + bf::BF_BPW - 1) / bf::BF_BPW,
        par_enc_dyn_lds, s, d, r, skip, nb, a)
    return hipGetLastError();
}

extern "C" hipError_t ppfs_parity_fast_check(const uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb, uint32_t bs,
    hipStream_t s)
{
    const bf::ParFast a { bs, nb * (uint64_t)(bs - 1) };
    if ((nb + (uint64_t)PPFS_BF_PAR_CHK_WV * bf::BF_BPW - 1) / ((uint64_t)PPFS_BF_PAR_CHK_WV * bf::BF_BPW) > (1ull << 30))
        return hipErrorInvalidValue;
    PPFS_NP_DISPATCH_WV(bs, bf::parity_fast_check_kernel, PPFS_BF_PAR_CHK_WV, (nb + bf::BF_BPW - 1) / bf::BF_BPW, par_chk_dyn_lds, s, r, d,
        st, nb, a)
    return hipGetLastError();
}

PPFS_DBG_ACCESSOR(ppfs_dbg_faults_bitfast)
