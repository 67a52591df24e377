// bit_kernels.hip -- CRC, extended Hamming (SECDED) and single-parity kernels for gfx950.
//
// One wave per filesystem block (a block is <= 4096 B = 64 lanes x 64 B), four waves per
// workgroup.  Blocks are packed in HBM at their reference strides (raw: rawBlockSize(),
// payload: dataSize()), so payload rows are generally not 4-byte aligned (Hamming 4091 B,
// parity 4095 B): rows are staged through a per-wave LDS buffer with funnel shifts.
//
// Reference semantics:
//   CRC      lib/ecc_helpers/src/crc_polynomial.cpp:56-76 (divide stops one step early),
//            lib/blockdevice/src/crc_block_device.cpp:12-67.  Closed form:
//            V = D(x) x^(n-1) mod P, stored = (V << 1) & (2^n - 1), written MSB first after
//            the payload; the ceil(n/8)*8 - n tail bits keep their old contents.
//   Hamming  lib/blockdevice/src/hamming_block_device.cpp:21-230 (MSB-first bit numbering,
//            payload bit i at the i-th integer >= 3 that is not a power of two, parity bits at
//            2^j, overall even parity at bit 0, unused tail bits untouched).
//   Parity   lib/blockdevice/src/parity_block_device.cpp:31-97.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dbg.hpp"
#include "srv_device.hpp"
#include "gf_common.hpp"

namespace ppfs {

constexpr int BK_WAVES = 4;
constexpr int BK_BUF = 4096 + 64; // per-wave LDS block buffer (with slack for funnel reads)

// ------------------------------------------------------------------------------------
// Wave-level copies with arbitrary global alignment.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_dw(const uint8_t* l, uint32_t off) { return *(const uint32_t*)(l + off); }

// LDS [0,n) <- global src[0,n); src may have any alignment; never reads outside [src, src+n).
__device__ __forceinline__ void wave_g2l(uint8_t* l, const uint8_t* __restrict__ src, uint32_t n, uint32_t lane)
{
    const uint32_t a = (uint32_t)((uintptr_t)src & 3u);
    if (a == 0) {
        const uint32_t nd = n >> 2;
        if (((uintptr_t)src & 15u) == 0) {
            const uint32_t nq = n >> 4;
            for (uint32_t i = lane; i < nq; i += 64)
                *(uint4*)(l + 16 * i) = *(const uint4*)(src + 16 * i);
            for (uint32_t i = nq * 4 + lane; i < nd; i += 64)
                *(uint32_t*)(l + 4 * i) = *(const uint32_t*)(src + 4 * i);
        } else {
            for (uint32_t i = lane; i < nd; i += 64)
                *(uint32_t*)(l + 4 * i) = *(const uint32_t*)(src + 4 * i);
        }
        for (uint32_t i = nd * 4 + lane; i < n; i += 64)
            l[i] = src[i];
    } else {
        // aligned dwords of [src - a, ...); output dword i = bytes src[4i, 4i+4)
        const uint32_t* base = (const uint32_t*)(src - a);
        const uint32_t nd = n >> 2;
        for (uint32_t i = lane; i < nd; i += 64) {
            uint32_t v;
            if (4 * i + 8 - a <= n) {
                v = __builtin_amdgcn_alignbit(base[i + 1], base[i], 8 * a);
            } else {
                v = (uint32_t)src[4 * i] | ((uint32_t)src[4 * i + 1] << 8) | ((uint32_t)src[4 * i + 2] << 16)
                    | ((uint32_t)src[4 * i + 3] << 24);
            }
            *(uint32_t*)(l + 4 * i) = v;
        }
        for (uint32_t i = nd * 4 + lane; i < n; i += 64)
            l[i] = src[i];
    }
}

// global dst[0,n) <- LDS [0,n); dst may have any alignment; writes only [dst, dst+n).
__device__ __forceinline__ void wave_l2g(uint8_t* __restrict__ dst, const uint8_t* l, uint32_t n, uint32_t lane)
{
    const uint32_t a = (uint32_t)((uintptr_t)dst & 3u);
    uint32_t head = (4u - a) & 3u;
    head = head > n ? n : head;
    if (lane < head)
        dst[lane] = l[lane];
    const uint32_t rem = n - head, nd = rem >> 2;
    uint8_t* d4 = dst + head;
    const uint32_t sh = head & 3u;
    if (sh == 0 && ((uintptr_t)d4 & 15u) == 0) {
        const uint32_t nq = rem >> 4;
        for (uint32_t i = lane; i < nq; i += 64)
            *(uint4*)(d4 + 16 * i) = *(const uint4*)(l + head + 16 * i);
        for (uint32_t i = nq * 4 + lane; i < nd; i += 64)
            *(uint32_t*)(d4 + 4 * i) = lds_dw(l, head + 4 * i);
    } else {
        for (uint32_t i = lane; i < nd; i += 64) {
            const uint32_t o = head + 4 * i; // LDS offset of the 4 output bytes
            const uint32_t o4 = o & ~3u;
            const uint32_t v = sh ? __builtin_amdgcn_alignbit(lds_dw(l, o4 + 4), lds_dw(l, o4), 8 * sh) : lds_dw(l, o);
            *(uint32_t*)(d4 + 4 * i) = v;
        }
    }
    for (uint32_t i = head + nd * 4 + lane; i < n; i += 64)
        dst[i] = l[i];
}

__device__ __forceinline__ void wave_zero(uint8_t* l, uint32_t from, uint32_t to, uint32_t lane)
{
    for (uint32_t i = from + lane; i < to; i += 64)
        l[i] = 0;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m)
{
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = __shfl_xor(lo, m, 64);
    hi = __shfl_xor(hi, m, 64);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_xor64(uint64_t v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1)
        v ^= shfl_xor64(v, m);
    return v;
}

__device__ __forceinline__ uint32_t wave_xor32(uint32_t v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1)
        v ^= __shfl_xor(v, m, 64);
    return v;
}

__device__ __forceinline__ uint32_t wave_add32(uint32_t v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1)
        v += __shfl_xor(v, m, 64);
    return v;
}

// ------------------------------------------------------------------------------------
// CRC
// Tables (built on the host, api.cpp): PT[64 pos][2 nibble][16] u64 =
//   (v << 4h) * x^(8(63-pos) + n - 8z - 1) mod P   (z = 64*G - ds zero bytes appended)
// and LV[6 level][16 nibble][16] u64 = (v << 4k) * x^(512 * 2^level) mod P.
// Lane s owns payload bytes [64s, 64s+64) (zero past ds); its contribution is shifted by
// x^(512 (G-1-s)); the XOR over lanes is V = D(x) x^(n-1) mod P.
// ------------------------------------------------------------------------------------
constexpr int CRC_PT_BYTES = 64 * 2 * 16 * 8;     // 16 KiB
constexpr int CRC_LV_BYTES = 6 * 16 * 16 * 8;     // 12 KiB
constexpr int CRC_TBL_BYTES = CRC_PT_BYTES + CRC_LV_BYTES;

struct CrcArgs {
    uint32_t bs, ds, n, G, nnib; // nnib = ceil(n/4)
    uint64_t mask;
};

__device__ __forceinline__ uint64_t crc_apply_level(const uint8_t* lv, uint64_t v, uint32_t nnib)
{
    uint64_t acc = 0;
    for (uint32_t k = 0; k < nnib; ++k)
        acc ^= *(const uint64_t*)(lv + ((k * 16 + ((v >> (4 * k)) & 15u)) << 3));
    return acc;
}

// V for the payload held in LDS [0, 64G) (zero padded past ds)
__device__ __forceinline__ uint64_t crc_wave_value(const uint8_t* buf, const uint8_t* tbl, const CrcArgs& a, uint32_t lane)
{
    uint64_t acc = 0;
    if (lane < a.G) {
        const uint8_t* seg = buf + 64 * lane;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint32_t w = *(const uint32_t*)(seg + 4 * q);
            const uint32_t l8 = (w << 3) & 0x78787878u, h8 = (w >> 1) & 0x78787878u;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int pos = 4 * q + p;
                acc ^= *(const uint64_t*)(tbl + (((pos * 2 + 0) * 16) << 3) + ((l8 >> (8 * p)) & 0xFFu));
                acc ^= *(const uint64_t*)(tbl + (((pos * 2 + 1) * 16) << 3) + ((h8 >> (8 * p)) & 0xFFu));
            }
        }
        const uint32_t sh = a.G - 1 - lane;
        for (int j = 0; j < 6; ++j)
            if (sh & (1u << j))
                acc = crc_apply_level(tbl + CRC_PT_BYTES + j * 2048, acc, a.nnib);
    }
    return wave_xor64(acc);
}

__device__ __forceinline__ uint64_t crc_stored_from_v(uint64_t V, const CrcArgs& a) { return (V << 1) & a.mask; }

// n CRC bits MSB first from bit ds*8 of the block (the stored field)
__device__ __forceinline__ uint64_t crc_read_field(const uint8_t* blk, const CrcArgs& a)
{
    uint64_t f = 0;
    const uint32_t nbc = (a.n + 7) / 8;
    for (uint32_t u = 0; u < nbc; ++u)
        f = (f << 8) | blk[a.ds + u];
    return f >> (8 * nbc - a.n);
}

// encode: raw[i] <- data[i] ++ CRC bits (+ old tail bits); skip blocks whose status is 5
// per-wave body of crc_encode_kernel (also run by bit_server_kernel): blocks first, first + stride, ...
__device__ __forceinline__ void crc_encode_blocks(const uint8_t* __restrict__ data, uint8_t* __restrict__ raw,
    const uint8_t* __restrict__ skip, uint64_t nblocks, CrcArgs a, const uint8_t* __restrict__ tables,
    uint8_t* lds, uint64_t first, uint64_t stride)
{
    const uint32_t lane = lane_id(), wave = wave_id();
    uint8_t* buf = lds + CRC_TBL_BYTES + wave * BK_BUF;
    for (uint64_t blk = first; blk < nblocks; blk += stride) {
        if (!PPFS_DBG_OK(data + blk * a.ds, a.ds, data, nblocks * a.ds) || !PPFS_DBG_OK(raw + blk * a.bs, a.bs, raw, nblocks * a.bs)
            || (skip && !PPFS_DBG_OK(skip + blk, 1, skip, nblocks)))
            continue; // PPFS_ECC_DEBUG: the block's rows (wave_g2l may also read the aligned dword holding a row's first byte)
        if (skip && skip[blk] == 5)
            continue;
        wave_g2l(buf, data + blk * a.ds, a.ds, lane);
        wave_zero(buf, a.ds, 64 * a.G + 8, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        const uint64_t V = crc_wave_value(buf, lds, a, lane);
        const uint64_t st = crc_stored_from_v(V, a);
        uint8_t* rb = raw + blk * a.bs;
        if (lane == 0) {
            const uint32_t nbc = (a.n + 7) / 8, rbits = a.n & 7u;
            for (uint32_t u = 0; u < nbc; ++u) {
                uint32_t byte;
                if (8 * (u + 1) <= a.n) {
                    byte = (uint32_t)(st >> (a.n - 8 * (u + 1))) & 0xFFu;
                } else {
                    const uint32_t hi = (uint32_t)(st & ((1u << rbits) - 1u)) << (8 - rbits);
                    byte = hi | (rb[a.ds + u] & ((1u << (8 - rbits)) - 1u));
                }
                buf[a.ds + u] = (uint8_t)byte;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        wave_l2g(rb, buf, a.bs, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
}

__global__ __launch_bounds__(256) void crc_encode_kernel(const uint8_t* __restrict__ data, uint8_t* __restrict__ raw,
    const uint8_t* __restrict__ skip, uint64_t nblocks, CrcArgs a, const uint8_t* __restrict__ tables)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[CRC_TBL_BYTES + BK_WAVES * BK_BUF];
    for (uint32_t p = threadIdx.x; p < CRC_TBL_BYTES / 16; p += 256)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    __syncthreads();
    crc_encode_blocks(data, raw, skip, nblocks, a, tables, lds, (uint64_t)blockIdx.x * BK_WAVES + wave_id(),
        (uint64_t)gridDim.x * BK_WAVES);
}

// check: status 0 / 5; optional payload copy
// per-wave body of crc_check_kernel (also run by bit_server_kernel): blocks first, first + stride, ...
__device__ __forceinline__ void crc_check_blocks(const uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks, CrcArgs a, const uint8_t* __restrict__ tables,
    uint8_t* lds, uint64_t first, uint64_t stride)
{
    const uint32_t lane = lane_id(), wave = wave_id();
    uint8_t* buf = lds + CRC_TBL_BYTES + wave * BK_BUF;
    for (uint64_t blk = first; blk < nblocks; blk += stride) {
        const uint8_t* rb = raw + blk * a.bs;
        if (!PPFS_DBG_OK(rb, a.bs, raw, nblocks * a.bs) || (data && !PPFS_DBG_OK(data + blk * a.ds, a.ds, data, nblocks * a.ds))
            || (status && !PPFS_DBG_OK(status + blk, 1, status, nblocks)))
            continue;
        wave_g2l(buf, rb, a.bs, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        const uint64_t field = crc_read_field(buf, a);
        if (data)
            wave_l2g(data + blk * a.ds, buf, a.ds, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        wave_zero(buf, a.ds, 64 * a.G + 8, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        const uint64_t V = crc_wave_value(buf, lds, a, lane);
        const uint64_t st = crc_stored_from_v(V, a);
        if (lane == 0 && status)
            status[blk] = (st == field) ? 0 : 5;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
}

__global__ __launch_bounds__(256) void crc_check_kernel(const uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks, CrcArgs a, const uint8_t* __restrict__ tables)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[CRC_TBL_BYTES + BK_WAVES * BK_BUF];
    for (uint32_t p = threadIdx.x; p < CRC_TBL_BYTES / 16; p += 256)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    __syncthreads();
    crc_check_blocks(raw, data, status, nblocks, a, tables, lds, (uint64_t)blockIdx.x * BK_WAVES + wave_id(),
        (uint64_t)gridDim.x * BK_WAVES);
}

// ------------------------------------------------------------------------------------
// Hamming
// ------------------------------------------------------------------------------------
struct HamArgs {
    uint32_t bs, ds, bits, L; // L = raw index of the last payload bit
};

__device__ __forceinline__ bool is_pow2(uint32_t x) { return x && !(x & (x - 1)); }
__device__ __forceinline__ uint32_t ilog2(uint32_t x) { return 31u - __builtin_clz(x); }

// 32 bits of a big-endian bit stream held in LDS starting at bit offset o
__device__ __forceinline__ uint32_t be_window(const uint8_t* l, uint32_t o)
{
    const uint32_t byte = o >> 3, a4 = byte & ~3u;
    const uint32_t k = 8 * (byte - a4) + (o & 7u); // 0..31
    const uint64_t e = ((uint64_t)__builtin_bswap32(lds_dw(l, a4)) << 32) | __builtin_bswap32(lds_dw(l, a4 + 4));
    return (uint32_t)(e >> (32 - k));
}


// XOR of (r0 + q) over set bits q of a big-endian word X (bit q = MSB-first position q)
__device__ __forceinline__ uint32_t word_index_xor(uint32_t X, uint32_t r0)
{
    uint32_t x = (__builtin_popcount(X) & 1u) ? r0 : 0u;
    x |= (__builtin_popcount(X & 0x55555555u) & 1u);
    x |= (__builtin_popcount(X & 0x33333333u) & 1u) << 1;
    x |= (__builtin_popcount(X & 0x0F0F0F0Fu) & 1u) << 2;
    x |= (__builtin_popcount(X & 0x00FF00FFu) & 1u) << 3;
    x |= (__builtin_popcount(X & 0x0000FFFFu) & 1u) << 4;
    return x;
}

// mask of MSB-first positions q in [lo, hi] (inclusive), clamped to [0,31]
__device__ __forceinline__ uint32_t qmask(int lo, int hi)
{
    if (hi < 0 || lo > 31 || hi < lo)
        return 0u;
    lo = lo < 0 ? 0 : lo;
    hi = hi > 31 ? 31 : hi;
    const uint32_t top = 0xFFFFFFFFu >> lo;               // positions >= lo
    const uint32_t bot = hi >= 31 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (hi + 1)); // positions <= hi
    return top & bot;
}

// used-bit mask of raw word w (positions 0..L plus parity positions above L)
__device__ __forceinline__ uint32_t ham_used_mask(uint32_t r0, const HamArgs& a)
{
    uint32_t m = qmask(0, (int)a.L - (int)r0);
    if (r0 + 31 > a.L) {
        // parity positions 2^j > L inside this word (at most one per word for r0 >= 32)
        if (r0 == 0) {
            for (uint32_t p = 1; p < 32 && p < a.bits; p <<= 1)
                if (p > a.L)
                    m |= 0x80000000u >> p;
        } else {
            const uint32_t p = 1u << ilog2(r0 + 31);
            if (p >= r0 && p > a.L && p < a.bits)
                m |= 0x80000000u >> (p - r0);
        }
    }
    return m;
}

// Raw word w (big-endian value) built from the payload bits (parity bits and tail zero).
__device__ __forceinline__ uint32_t ham_place_word(const uint8_t* dbuf, uint32_t w, const HamArgs& a)
{
    const uint32_t r0 = 32 * w;
    if (r0 > a.L)
        return 0;
    uint32_t X;
    if (w == 0) {
        // payload bits 0, 1-3, 4-10, 11-25 sit at raw positions 3, 5-7, 9-15, 17-31
        const uint32_t D = be_window(dbuf, 0);
        X = ((D >> 31) << 28) | (((D >> 28) & 0x7u) << 24) | (((D >> 21) & 0x7Fu) << 16) | ((D >> 6) & 0x7FFFu);
        return X & qmask(0, (int)a.L);
    }
    const uint32_t j1 = ilog2(r0), j2 = ilog2(r0 + 31);
    const int k = (j1 == j2 && !is_pow2(r0)) ? 32 : (int)((1u << j2) - r0);
    const uint32_t wa = be_window(dbuf, r0 - j1 - 2);
    const uint32_t wb = be_window(dbuf, r0 - j2 - 2);
    X = (wa & qmask(0, k - 1)) | (wb & qmask(k + 1, 31));
    return X & qmask(0, (int)a.L - (int)r0);
}

// encode: per lane 16 raw words (64 B); tail bits from the old raw block
// per-wave body of ham_encode_kernel (also run by bit_server_kernel): blocks first, first + stride, ...
__device__ __forceinline__ void ham_encode_blocks(const uint8_t* __restrict__ data, uint8_t* __restrict__ raw,
    const uint8_t* __restrict__ skip, uint64_t nblocks, HamArgs a,
    uint8_t* lds, uint64_t first, uint64_t stride)
{
    const uint32_t lane = lane_id(), wave = wave_id();
    uint8_t* buf = lds + wave * BK_BUF;
    const uint32_t nwords = a.bits / 32;
    for (uint64_t blk = first; blk < nblocks; blk += stride) {
        if (!PPFS_DBG_OK(data + blk * a.ds, a.ds, data, nblocks * a.ds) || !PPFS_DBG_OK(raw + blk * a.bs, a.bs, raw, nblocks * a.bs)
            || (skip && !PPFS_DBG_OK(skip + blk, 1, skip, nblocks)))
            continue;
        if (skip && skip[blk] == 5)
            continue;
        wave_g2l(buf, data + blk * a.ds, a.ds, lane);
        wave_zero(buf, a.ds, a.bs + 16, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        uint8_t* rb = raw + blk * a.bs;
        uint32_t X[16];
        uint32_t syn = 0, dpar = 0;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint32_t w = 16 * lane + u;
            uint32_t x = 0;
            if (w < nwords) {
                x = ham_place_word(buf, w, a);
                syn ^= word_index_xor(x, 32 * w);
                dpar ^= __builtin_popcount(x) & 1u;
            }
            X[u] = x;
        }
        syn = wave_xor32(syn);
        dpar = wave_xor32(dpar) & 1u;
        const uint32_t bit0 = (dpar ^ (__builtin_popcount(syn) & 1u)) & 1u;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint32_t w = 16 * lane + u;
            if (w >= nwords)
                continue;
            const uint32_t r0 = 32 * w;
            uint32_t x = X[u];
            // parity bits 2^j inside this word, overall parity at bit 0
            if (w == 0) {
                for (uint32_t j = 0; j < 5 && (1u << j) < a.bits; ++j)
                    if ((syn >> j) & 1u)
                        x |= 0x80000000u >> (1u << j);
                if (bit0)
                    x |= 0x80000000u;
            } else {
                const uint32_t j = ilog2(r0 + 31), p = 1u << j;
                if (p >= r0 && p < a.bits && ((syn >> j) & 1u))
                    x |= 0x80000000u >> (p - r0);
            }
            // unused tail bits keep the old raw contents
            const uint32_t keep = ~ham_used_mask(r0, a);
            if (keep && r0 + 31 > a.L) {
                const uint32_t old = __builtin_bswap32(*(const uint32_t*)(rb + 4 * w));
                x = (x & ~keep) | (old & keep);
            }
            X[u] = __builtin_bswap32(x);
        }
#pragma unroll
        for (int u = 0; u < 16; u += 4) {
            const uint32_t w = 16 * lane + u;
            if (w + 3 < nwords) {
                *(uint4*)(rb + 4 * w) = make_uint4(X[u], X[u + 1], X[u + 2], X[u + 3]);
            } else {
                for (int v = 0; v < 4; ++v)
                    if (w + v < nwords)
                        *(uint32_t*)(rb + 4 * (w + v)) = X[u + v];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
}

__global__ __launch_bounds__(256) void ham_encode_kernel(const uint8_t* __restrict__ data, uint8_t* __restrict__ raw,
    const uint8_t* __restrict__ skip, uint64_t nblocks, HamArgs a)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[BK_WAVES * BK_BUF];
    ham_encode_blocks(data, raw, skip, nblocks, a, lds, (uint64_t)blockIdx.x * BK_WAVES + wave_id(),
        (uint64_t)gridDim.x * BK_WAVES);
}

// decode: status 0/1/5, one-byte write-back, payload extraction
// per-wave body of ham_decode_kernel (also run by bit_server_kernel): blocks first, first + stride, ...
__device__ __forceinline__ void ham_decode_blocks(uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks, int write_back, HamArgs a,
    uint8_t* lds, uint64_t first, uint64_t stride)
{
    const uint32_t lane = lane_id(), wave = wave_id();
    uint8_t* buf = lds + wave * BK_BUF;
    const uint32_t nwords = a.bits / 32;
    for (uint64_t blk = first; blk < nblocks; blk += stride) {
        uint8_t* rb = raw + blk * a.bs;
        if (!PPFS_DBG_OK(rb, a.bs, raw, nblocks * a.bs) || (data && !PPFS_DBG_OK(data + blk * a.ds, a.ds, data, nblocks * a.ds))
            || (status && !PPFS_DBG_OK(status + blk, 1, status, nblocks)))
            continue;
        uint32_t X[16];
        uint32_t syn = 0, par = 0;
#pragma unroll
        for (int u = 0; u < 16; u += 4) {
            const uint32_t w = 16 * lane + u;
            if (w + 3 < nwords) {
                const uint4 v = *(const uint4*)(rb + 4 * w);
                X[u] = v.x;
                X[u + 1] = v.y;
                X[u + 2] = v.z;
                X[u + 3] = v.w;
            } else {
                for (int q = 0; q < 4; ++q)
                    X[u + q] = (w + q < nwords) ? *(const uint32_t*)(rb + 4 * (w + q)) : 0u;
            }
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint32_t w = 16 * lane + u;
            if (w < nwords) {
                const uint32_t x = __builtin_bswap32(X[u]) & ham_used_mask(32 * w, a);
                syn ^= word_index_xor(x, 32 * w);
                par ^= __builtin_popcount(x) & 1u;
            }
        }
        syn = wave_xor32(syn);
        par = wave_xor32(par) & 1u;
        uint32_t st = 0;
        if (par) {
            st = 1;
            const uint32_t wf = syn >> 5; // word holding the flipped bit
            if (wf >= 16 * lane && wf < 16 * lane + 16) {
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (16 * lane + u == wf)
                        X[u] ^= __builtin_bswap32(0x80000000u >> (syn & 31u));
                if (write_back) {
                    const uint32_t byte = syn >> 3;
                    rb[byte] = (uint8_t)(rb[byte] ^ (0x80u >> (syn & 7u)));
                }
            }
        } else if (syn != 0) {
            st = 5;
        }
        if (lane == 0 && status)
            status[blk] = (uint8_t)st;
        if (data && st != 5) {
            // fixed raw block -> LDS, then extract payload words into the second half of buf
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const uint32_t w = 16 * lane + u;
                if (w < nwords)
                    *(uint32_t*)(buf + 4 * w) = X[u];
            }
            *(uint32_t*)(buf + a.bs + 4 * (lane & 3)) = 0; // slack for window reads
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            uint8_t* dbuf = buf; // payload is written over the raw image only after all reads
            const uint32_t ndw = (8 * a.ds + 31) / 32;
            uint32_t Y[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const uint32_t v = 16 * lane + u;
                uint32_t y = 0;
                if (v < ndw) {
                    const uint32_t i0 = 32 * v;
                    if (v == 0) {
                        // payload bits 0, 1-3, 4-10, 11-25, 26-31 from raw positions 3, 5-7, 9-15,
                        // 17-31, 33-38 (the inverse of ham_place_word's head word)
                        const uint32_t R0 = be_window(buf, 0), R1 = be_window(buf, 32);
                        y = (((R0 >> 28) & 1u) << 31) | (((R0 >> 24) & 0x7u) << 28) | (((R0 >> 16) & 0x7Fu) << 21)
                            | ((R0 & 0x7FFFu) << 6) | ((R1 >> 25) & 0x3Fu);
                    } else {
                        uint32_t j1 = ilog2(i0 + 2);
                        if (i0 > (2u << j1) - j1 - 3)
                            j1++;
                        const uint32_t nxt = (2u << j1) - j1 - 2; // first payload bit of segment j1+1
                        const int qb = (int)nxt - (int)i0;          // boundary position in the word
                        const uint32_t wa = be_window(buf, i0 + j1 + 2);
                        y = wa & qmask(0, qb - 1);
                        if (qb <= 31)
                            y |= be_window(buf, i0 + j1 + 3) & qmask(qb, 31);
                    }
                }
                Y[u] = __builtin_bswap32(y);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const uint32_t v = 16 * lane + u;
                if (v < ndw)
                    *(uint32_t*)(dbuf + 4 * v) = Y[u];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            wave_l2g(data + blk * a.ds, dbuf, a.ds, lane);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
}

__global__ __launch_bounds__(256) void ham_decode_kernel(uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks, int write_back, HamArgs a)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[BK_WAVES * BK_BUF];
    ham_decode_blocks(raw, data, status, nblocks, write_back, a, lds, (uint64_t)blockIdx.x * BK_WAVES + wave_id(),
        (uint64_t)gridDim.x * BK_WAVES);
}

// ------------------------------------------------------------------------------------
// Hamming blocks of 1, 2 and 4 bytes (block_size_power 0-2; hamming_block_device.cpp:11-19 takes
// any power): one thread per block over a 32-bit register image of the block (MSB-first bit q at
// register bit 31 - q), walking the reference's iterators literally.  Power 0 has no payload, and
// its used bits are the parity positions 1, 2, 4 only (HammingUsedBitsIterator :209-219 starts in
// its parity branch), not bit 0.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t tiny_load(const uint8_t* __restrict__ p, uint32_t n)
{
    uint32_t v = 0;
    for (uint32_t i = 0; i < n; ++i)
        v |= (uint32_t)p[i] << (24 - 8 * i);
    return v;
}

__device__ __forceinline__ void tiny_store(uint8_t* __restrict__ p, uint32_t n, uint32_t v)
{
    for (uint32_t i = 0; i < n; ++i)
        p[i] = (uint8_t)(v >> (24 - 8 * i));
}

__device__ __forceinline__ uint32_t qbit(uint32_t q) { return 0x80000000u >> q; }

// HammingDataBitsIterator::next (:188-198): the next integer that is neither 0 nor a power of two
__device__ __forceinline__ uint32_t tiny_next_data(uint32_t& cur)
{
    while ((cur & (cur - 1)) == 0)
        cur++;
    return cur++;
}

__global__ __launch_bounds__(256) void ham_tiny_encode_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, const uint8_t* __restrict__ skip, uint64_t nblocks, uint32_t bs, uint32_t ds)
{
    for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < nblocks; b += (uint64_t)gridDim.x * 256) {
        if (skip && skip[b] == 5)
            continue;
        const uint32_t D = ds ? tiny_load(data + b * ds, ds) : 0u;
        uint32_t R = tiny_load(raw + b * bs, bs); // unused tail bits keep their contents
        uint32_t parity = 1, pxor = 0, cur = 0;
        for (uint32_t i = 0; i < 8 * ds; ++i) { // _encodeData :85-94
            const uint32_t idx = tiny_next_data(cur);
            const uint32_t v = (D >> (31 - i)) & 1u;
            parity ^= v;
            pxor ^= v ? idx : 0u;
            R = v ? (R | qbit(idx)) : (R & ~qbit(idx));
        }
        for (uint32_t pi = 1; pi < 8 * bs; pi <<= 1) { // :96-105
            const bool pv = (pxor & pi) != 0;
            parity ^= pv ? 1u : 0u;
            R = pv ? (R | qbit(pi)) : (R & ~qbit(pi));
        }
        R = parity ? (R & ~qbit(0)) : (R | qbit(0)); // bit 0 = !parity (:107-108)
        tiny_store(raw + b * bs, bs, R);
    }
}

__global__ __launch_bounds__(256) void ham_tiny_decode_kernel(uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks, int write_back, uint32_t bs, uint32_t ds)
{
    for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < nblocks; b += (uint64_t)gridDim.x * 256) {
        uint32_t R = tiny_load(raw + b * bs, bs);
        // HammingUsedBitsIterator (:209-230) over the block, _readAndFixBlock :30-39
        const uint32_t lim = 8 * ds, bits = 8 * bs;
        uint32_t cur = 0, next_par = 1, ret = 0, epos = 0, parity = 1;
        for (;;) {
            uint32_t idx;
            if (ret >= lim && next_par >= bits)
                break;
            if (ret >= lim) {
                idx = next_par;
                next_par <<= 1;
            } else {
                const bool pow2 = cur && (cur & (cur - 1)) == 0;
                if (pow2)
                    next_par = cur << 1;
                if (cur && !pow2)
                    ret++;
                idx = cur++;
            }
            if (R & qbit(idx)) {
                epos ^= idx;
                parity ^= 1u;
            }
        }
        uint32_t st = 0;
        if (!parity) { // :41-57: flip, write back only that byte
            R ^= qbit(epos);
            st = 1;
            if (write_back)
                raw[b * bs + epos / 8] = (uint8_t)(R >> (24 - 8 * (epos / 8)));
        } else if (epos != 0) {
            st = 5; // :58-61
        }
        if (status)
            status[b] = (uint8_t)st;
        if (data && ds && st != 5) { // _extractData :67-74
            uint32_t D = 0, c2 = 0;
            for (uint32_t i = 0; i < 8 * ds; ++i)
                D |= (R & qbit(tiny_next_data(c2))) ? qbit(i) : 0u;
            tiny_store(data + b * ds, ds, D);
        }
    }
}

// ------------------------------------------------------------------------------------
// Parity (even parity over the whole raw block; the LSB of the last byte is the fix bit)
// ------------------------------------------------------------------------------------
// per-wave body of parity_encode_kernel (also run by bit_server_kernel): blocks first, first + stride, ...
__device__ __forceinline__ void parity_encode_blocks(const uint8_t* __restrict__ data, uint8_t* __restrict__ raw,
    const uint8_t* __restrict__ skip, uint64_t nblocks, uint32_t bs,
    uint8_t* lds, uint64_t first, uint64_t stride)
{
    const uint32_t lane = lane_id(), wave = wave_id();
    uint8_t* buf = lds + wave * BK_BUF;
    const uint32_t ds = bs - 1;
    for (uint64_t blk = first; blk < nblocks; blk += stride) {
        if (!PPFS_DBG_OK(data + blk * ds, ds, data, nblocks * ds) || !PPFS_DBG_OK(raw + blk * bs, bs, raw, nblocks * bs)
            || (skip && !PPFS_DBG_OK(skip + blk, 1, skip, nblocks)))
            continue;
        if (skip && skip[blk] == 5)
            continue;
        uint8_t* rb = raw + blk * bs;
        wave_g2l(buf, data + blk * ds, ds, lane);
        const uint32_t last = rb[bs - 1];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        uint32_t ones = 0;
        for (uint32_t i = lane; i < ds; i += 64)
            ones += __builtin_popcount(buf[i]);
        ones = wave_add32(ones) + __builtin_popcount(last);
        if (lane == 0)
            buf[ds] = (uint8_t)(last ^ (ones & 1u));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        wave_l2g(rb, buf, bs, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
}

__global__ __launch_bounds__(256) void parity_encode_kernel(const uint8_t* __restrict__ data, uint8_t* __restrict__ raw,
    const uint8_t* __restrict__ skip, uint64_t nblocks, uint32_t bs)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[BK_WAVES * BK_BUF];
    parity_encode_blocks(data, raw, skip, nblocks, bs, lds, (uint64_t)blockIdx.x * BK_WAVES + wave_id(),
        (uint64_t)gridDim.x * BK_WAVES);
}

// per-wave body of parity_check_kernel (also run by bit_server_kernel): blocks first, first + stride, ...
__device__ __forceinline__ void parity_check_blocks(const uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks, uint32_t bs,
    uint8_t* lds, uint64_t first, uint64_t stride)
{
    const uint32_t lane = lane_id(), wave = wave_id();
    uint8_t* buf = lds + wave * BK_BUF;
    for (uint64_t blk = first; blk < nblocks; blk += stride) {
        const uint8_t* rb = raw + blk * bs;
        if (!PPFS_DBG_OK(rb, bs, raw, nblocks * bs) || (data && !PPFS_DBG_OK(data + blk * (bs - 1), bs - 1, data, nblocks * (bs - 1)))
            || (status && !PPFS_DBG_OK(status + blk, 1, status, nblocks)))
            continue;
        wave_g2l(buf, rb, bs, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        uint32_t ones = 0;
        for (uint32_t i = lane; i < bs; i += 64)
            ones += __builtin_popcount(buf[i]);
        ones = wave_add32(ones);
        if (lane == 0 && status)
            status[blk] = (ones & 1u) ? 5 : 0;
        if (data)
            wave_l2g(data + blk * (bs - 1), buf, bs - 1, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
}

__global__ __launch_bounds__(256) void parity_check_kernel(const uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks, uint32_t bs)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[BK_WAVES * BK_BUF];
    parity_check_blocks(raw, data, status, nblocks, bs, lds, (uint64_t)blockIdx.x * BK_WAVES + wave_id(),
        (uint64_t)gridDim.x * BK_WAVES);
}

// ------------------------------------------------------------------------------------
// Resident small-batch server for CRC / Hamming / parity (server_box.hpp protocol; the RS twins
// are rs_wg_server_kernel and rs_pair_server_kernel): one 256-thread workgroup, wave w takes the
// request's blocks w, w + 4, ... through the per-wave bodies above (every block size: the CRC
// context always carries these generic tables, the fast ones follow them).  A write is the check
// (Hamming: decode with write-back) then the encode that skips status-5 blocks, as
// ppfs_ecc_write_device queues them.
// ------------------------------------------------------------------------------------
struct BitSrv {
    CrcArgs crc;
    HamArgs ham;
    uint32_t bs, ds;
};

template <int CODEC> // PPFS_ECC_CRC 1, PPFS_ECC_HAMMING 2, PPFS_ECC_PARITY 3
__global__ __launch_bounds__(256, 1) void bit_server_kernel(SrvBox* box, uint8_t* zc, uint64_t zc_bytes, BitSrv a,
    const uint8_t* __restrict__ tables, uint32_t gen, uint32_t idle_us)
{
    constexpr int TBL = CODEC == 1 ? CRC_TBL_BYTES : 0;
    __shared__ __attribute__((aligned(16))) uint8_t lds[TBL + BK_WAVES * BK_BUF];
    __shared__ uint32_t s_cmd[2];
    for (uint32_t p = threadIdx.x; p < (uint32_t)TBL / 16; p += 256)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    const uint64_t w0 = wave_id(), W = BK_WAVES;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t last = t0;
    uint32_t seen = srv::ld_sys(&box->done), served = 0;
    if (threadIdx.x == 0)
        srv::st_sys(&box->alive, gen);
    for (;;) {
        const uint32_t r = srv::next_request(box, seen, last, t0, idle_us, s_cmd);
        if (r == 0)
            break;
        const SrvCmd cmd = srv_cmd_unpack(r);
        const uint32_t nb = cmd.nb;
        const SrvLayout lay = srv_layout(nb, a.ds, a.bs);
        uint8_t* data = zc + lay.data;
        uint8_t* raw = zc + lay.raw;
        uint8_t* status = zc + lay.status;
        const bool ok = nb >= 1 && nb <= SRV_MAX_BLOCKS && PPFS_DBG_OK(data, nb * a.ds, zc, zc_bytes)
            && PPFS_DBG_OK(raw, nb * a.bs, zc, zc_bytes) && PPFS_DBG_OK(status, nb, zc, zc_bytes);
        uint8_t* want = cmd.want_data ? data : nullptr;
        if (ok && cmd.op == SRV_DECODE) {
            if constexpr (CODEC == 1)
                crc_check_blocks(raw, want, status, nb, a.crc, tables, lds, w0, W);
            else if constexpr (CODEC == 2)
                ham_decode_blocks(raw, want, status, nb, cmd.write_back ? 1 : 0, a.ham, lds, w0, W);
            else
                parity_check_blocks(raw, want, status, nb, a.bs, lds, w0, W);
        }
        if (ok && cmd.op == SRV_WRITE) { // the old blocks' check: status, Hamming's write-back
            if constexpr (CODEC == 1)
                crc_check_blocks(raw, nullptr, status, nb, a.crc, tables, lds, w0, W);
            else if constexpr (CODEC == 2)
                ham_decode_blocks(raw, nullptr, status, nb, 1, a.ham, lds, w0, W);
            else
                parity_check_blocks(raw, nullptr, status, nb, a.bs, lds, w0, W);
            __threadfence_system(); // status and write-back bytes before the encode reads them
            __syncthreads();
        }
        if (ok && (cmd.op == SRV_ENCODE || cmd.op == SRV_WRITE)) {
            const uint8_t* skip = cmd.op == SRV_WRITE ? status : nullptr;
            if constexpr (CODEC == 1)
                crc_encode_blocks(data, raw, skip, nb, a.crc, tables, lds, w0, W);
            else if constexpr (CODEC == 2)
                ham_encode_blocks(data, raw, skip, nb, a.ham, lds, w0, W);
            else
                parity_encode_blocks(data, raw, skip, nb, a.bs, lds, w0, W);
        }
        seen = r;
        srv::finish_request(box, r, ++served);
    }
    if (threadIdx.x == 0)
        srv::st_sys(&box->alive, gen | SRV_EXITED);
}

} // namespace ppfs

using namespace ppfs;

// 1, 2 and 4 KiB blocks: the streaming kernels of bit_fast.hip
extern "C" int ppfs_bitfast_supported(uint32_t bs);
extern "C" hipError_t ppfs_ham_fast_encode(const uint8_t*, uint8_t*, const uint8_t*, uint64_t, uint32_t, uint32_t,
    uint32_t, hipStream_t);
extern "C" hipError_t ppfs_ham_fast_decode(uint8_t*, uint8_t*, uint8_t*, uint64_t, int, uint32_t, uint32_t, uint32_t,
    hipStream_t);
extern "C" hipError_t ppfs_parity_fast_encode(const uint8_t*, uint8_t*, const uint8_t*, uint64_t, uint32_t, hipStream_t);
extern "C" hipError_t ppfs_parity_fast_check(const uint8_t*, uint8_t*, uint8_t*, uint64_t, uint32_t, hipStream_t);
extern "C" hipError_t ppfs_crc_fast_encode(const uint8_t*, uint8_t*, const uint8_t*, uint64_t, uint32_t, uint32_t,
    uint32_t, uint64_t, const uint8_t*, hipStream_t);
extern "C" hipError_t ppfs_crc_fast_check(const uint8_t*, uint8_t*, uint8_t*, uint64_t, uint32_t, uint32_t, uint32_t,
    uint64_t, const uint8_t*, hipStream_t);

// the CRC fast path (n <= 32, 1-4 KiB blocks) reads its tables after the generic ones
extern "C" int ppfs_crc_fast_supported(uint32_t bs, uint32_t n) { return ppfs_bitfast_supported(bs) && n <= 32; }

static uint32_t bk_grid(uint64_t nb)
{
    uint64_t g = (nb + BK_WAVES - 1) / BK_WAVES;
    return (uint32_t)(g > 8192 ? 8192 : (g ? g : 1));
}

// thread-per-block kernels (Hamming blocks < 8 bytes)
static uint32_t tiny_grid(uint64_t nb)
{
    uint64_t g = (nb + 255) / 256;
    return (uint32_t)(g > 8192 ? 8192 : (g ? g : 1));
}

extern "C" int ppfs_crc_tables_bytes(void) { return CRC_TBL_BYTES; }

extern "C" hipError_t ppfs_crc_encode(const uint8_t* d, uint8_t* r, const uint8_t* skip, uint64_t nb, uint32_t bs,
    uint32_t ds, uint32_t n, uint64_t mask, const uint8_t* tab, hipStream_t s)
{
    if (ppfs_crc_fast_supported(bs, n))
        return ppfs_crc_fast_encode(d, r, skip, nb, bs, ds, n, mask, tab + CRC_TBL_BYTES, s);
    CrcArgs a { bs, ds, n, (ds + 63) / 64, (n + 3) / 4, mask };
    hipLaunchKernelGGL(crc_encode_kernel, dim3(bk_grid(nb)), dim3(256), 0, s, d, r, skip, nb, a, tab);
    return hipGetLastError();
}

extern "C" hipError_t ppfs_crc_check(const uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb, uint32_t bs, uint32_t ds,
    uint32_t n, uint64_t mask, const uint8_t* tab, hipStream_t s)
{
    if (ppfs_crc_fast_supported(bs, n))
        return ppfs_crc_fast_check(r, d, st, nb, bs, ds, n, mask, tab + CRC_TBL_BYTES, s);
    CrcArgs a { bs, ds, n, (ds + 63) / 64, (n + 3) / 4, mask };
    hipLaunchKernelGGL(crc_check_kernel, dim3(bk_grid(nb)), dim3(256), 0, s, r, d, st, nb, a, tab);
    return hipGetLastError();
}

extern "C" hipError_t ppfs_ham_encode(const uint8_t* d, uint8_t* r, const uint8_t* skip, uint64_t nb, uint32_t bs,
    uint32_t ds, uint32_t L, hipStream_t s)
{
    if (ppfs_bitfast_supported(bs))
        return ppfs_ham_fast_encode(d, r, skip, nb, bs, ds, L, s);
    if (bs < 8) {
        hipLaunchKernelGGL(ham_tiny_encode_kernel, dim3(tiny_grid(nb)), dim3(256), 0, s, d, r, skip, nb, bs, ds);
        return hipGetLastError();
    }
    HamArgs a { bs, ds, 8 * bs, L };
    hipLaunchKernelGGL(ham_encode_kernel, dim3(bk_grid(nb)), dim3(256), 0, s, d, r, skip, nb, a);
    return hipGetLastError();
}

extern "C" hipError_t ppfs_ham_decode(uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb, int wb, uint32_t bs,
    uint32_t ds, uint32_t L, hipStream_t s)
{
    if (ppfs_bitfast_supported(bs))
        return ppfs_ham_fast_decode(r, d, st, nb, wb, bs, ds, L, s);
    if (bs < 8) {
        hipLaunchKernelGGL(ham_tiny_decode_kernel, dim3(tiny_grid(nb)), dim3(256), 0, s, r, d, st, nb, wb, bs, ds);
        return hipGetLastError();
    }
    HamArgs a { bs, ds, 8 * bs, L };
    hipLaunchKernelGGL(ham_decode_kernel, dim3(bk_grid(nb)), dim3(256), 0, s, r, d, st, nb, wb, a);
    return hipGetLastError();
}

extern "C" hipError_t ppfs_parity_encode(const uint8_t* d, uint8_t* r, const uint8_t* skip, uint64_t nb, uint32_t bs,
    hipStream_t s)
{
    if (ppfs_bitfast_supported(bs))
        return ppfs_parity_fast_encode(d, r, skip, nb, bs, s);
    hipLaunchKernelGGL(parity_encode_kernel, dim3(bk_grid(nb)), dim3(256), 0, s, d, r, skip, nb, bs);
    return hipGetLastError();
}

extern "C" hipError_t ppfs_parity_check(const uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb, uint32_t bs,
    hipStream_t s)
{
    if (ppfs_bitfast_supported(bs))
        return ppfs_parity_fast_check(r, d, st, nb, bs, s);
    hipLaunchKernelGGL(parity_check_kernel, dim3(bk_grid(nb)), dim3(256), 0, s, r, d, st, nb, bs);
    return hipGetLastError();
}

// resident small-batch server for CRC / Hamming / parity contexts (api.cpp server_call)
extern "C" hipError_t ppfs_bit_server_launch(int ecc_type, uint32_t bs, uint32_t ds, uint32_t crc_n, uint64_t crc_mask,
    uint32_t ham_L, SrvBox* box, uint8_t* zc, uint64_t zc_bytes, const uint8_t* tab, uint32_t gen, uint32_t idle_us,
    hipStream_t s)
{
    BitSrv a {};
    a.crc = CrcArgs { bs, ds, crc_n, (ds + 63) / 64, (crc_n + 3) / 4, crc_mask };
    a.ham = HamArgs { bs, ds, 8 * bs, ham_L };
    a.bs = bs;
    a.ds = ds;
    switch (ecc_type) {
    case 1:
        hipLaunchKernelGGL(bit_server_kernel<1>, dim3(1), dim3(256), 0, s, box, zc, zc_bytes, a, tab, gen, idle_us);
        break;
    case 2:
        hipLaunchKernelGGL(bit_server_kernel<2>, dim3(1), dim3(256), 0, s, box, zc, zc_bytes, a, tab, gen, idle_us);
        break;
    case 3:
        hipLaunchKernelGGL(bit_server_kernel<3>, dim3(1), dim3(256), 0, s, box, zc, zc_bytes, a, tab, gen, idle_us);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

PPFS_DBG_ACCESSOR(ppfs_dbg_faults_bit)
