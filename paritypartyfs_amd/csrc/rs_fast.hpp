#pragma once
// rs_fast.hpp -- Reed-Solomon GF(2^8) encode / syndrome / correct kernels for gfx950.
//
// Reference semantics: lib/blockdevice/src/rs_block_device.cpp
//   encode  _encodeBlock :95-117   c(x) = m(x) x^2t + (m(x) x^2t mod g(x)); byte i = coeff of x^i,
//                                  parity in bytes [0,2t), payload in [2t,n)
//   decode  _fixBlockAndExtract :119-183, _berlekampMassey :234-269, _errorLocations :271-280,
//           _calculateOmega :224-232, _forney :210-222
//
// Fast path (n = 255, 2t in {2,4,...,32}): one workgroup = 4 waves = a tile of 256 blocks.
//   - The tile's packed bytes are staged into LDS with LDS-DMA (global_load_lds_dwordx4).
//   - Lane l of wave c owns block 4l+c, so every block of a wave has the same byte alignment
//     in LDS; the wave's code is specialised on c (template) and every register index and
//     funnel shift is a compile-time constant.
//   - The parity / remainder is computed slicing-by-8 from the top: for 8 payload bytes e_i
//     (XORed with the top of the running remainder), the new remainder is the XOR of 16 LDS
//     table entries T[i][nibble] = nibble * (x^(2t+i) mod g), no dependency inside a chunk.
//   - Decode recomputes the parity of the payload and compares it with the stored parity
//     (c mod g == 0  <=>  all syndromes are zero).  Lanes with a non-zero remainder run the
//     exact reference correction (syndromes -> Berlekamp-Massey -> roots over all 255 field
//     values -> Omega -> Forney) in registers.
//   - Output is rebuilt in place in the same LDS tile and streamed out with 16-byte stores.
// Generic path (any n <= 255, any t): one thread per block, bytewise LFSR, private arrays.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf_common.hpp"

namespace ppfs {

constexpr int RS_TILE = 256;                // blocks per workgroup tile
constexpr int RS_N = 255;                   // fast-path codeword length
constexpr int RS_TILE_BYTES = RS_TILE * RS_N; // 65280

template <int T2> struct RsCfg {
    static constexpr int K = RS_N - T2;
    static constexpr int W = T2 <= 8 ? 2 : (T2 <= 16 ? 4 : 8); // remainder words (top aligned)
    static constexpr int TBL_BYTES = W <= 4 ? 4096 : 8192;      // 16 nibble tables x 16 x 16 B (x2)
    static constexpr int OFF_GF = TBL_BYTES;
    static constexpr int OFF_STATUS = OFF_GF + GF_BYTES;
    static constexpr int OFF_TILE = OFF_STATUS + RS_TILE;
    static constexpr int LDS_BYTES = OFF_TILE + RS_TILE_BYTES + 16;
    static constexpr int NCHUNK = (K + 7) / 8;
};

// ------------------------------------------------------------------------------------
// Tile staging: global <-> LDS
// ------------------------------------------------------------------------------------

// Copy `bytes` bytes from global src (16-byte aligned) into LDS [dst, dst+bytes) using
// LDS-DMA for whole 16-byte pieces (each wave-instruction moves one contiguous KiB) and
// byte loads for the tail.  All 256 threads call it.
__device__ __forceinline__ void stage_in(uint8_t* lds_dst, const uint8_t* __restrict__ src, uint32_t bytes)
{
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = wave_id();
    const uint32_t npiece = bytes >> 4;     // whole 16-byte pieces
    const uint32_t ngroup = (npiece + 63) >> 6; // 1 KiB groups
    for (uint32_t g = wave; g < ngroup; g += 4) {
        uint32_t piece = g * 64 + lane;
        if (piece < npiece) {
            __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)piece * 16),
                (__attribute__((address_space(3))) void*)(lds_dst + g * 1024), 16, 0, 0);
        }
    }
    uint32_t tail = bytes & 15u;
    if (tid < tail)
        lds_dst[npiece * 16 + tid] = src[npiece * 16 + tid];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// Copy LDS [src, src+bytes) to global dst (16-byte aligned): 16-byte stores + byte tail.
__device__ __forceinline__ void stage_out(uint8_t* __restrict__ dst, const uint8_t* lds_src, uint32_t bytes)
{
    const uint32_t tid = threadIdx.x;
    const uint32_t npiece = bytes >> 4;
    for (uint32_t p = tid; p < npiece; p += 256) {
        uint4 v = *(const uint4*)(lds_src + p * 16);
        *(uint4*)(dst + (size_t)p * 16) = v;
    }
    uint32_t tail = bytes & 15u;
    if (tid < tail)
        dst[npiece * 16 + tid] = lds_src[npiece * 16 + tid];
}

// Copy the context's tables (global, 16-byte multiple) into LDS.
__device__ __forceinline__ void load_tables(uint8_t* lds_dst, const uint8_t* __restrict__ src, uint32_t bytes)
{
    for (uint32_t p = threadIdx.x; p < (bytes >> 4); p += 256)
        *(uint4*)(lds_dst + p * 16) = *(const uint4*)(src + (size_t)p * 16);
}

// ------------------------------------------------------------------------------------
// Slicing-by-8 remainder step
// ------------------------------------------------------------------------------------
template <int W>
__device__ __forceinline__ void tbl_acc(uint32_t (&acc)[W], const uint8_t* lds, uint32_t addr)
{
    if constexpr (W == 2) {
        uint2 v = *(const uint2*)(lds + addr);
        acc[0] ^= v.x;
        acc[1] ^= v.y;
    } else if constexpr (W == 4) {
        uint4 v = *(const uint4*)(lds + addr);
        acc[0] ^= v.x;
        acc[1] ^= v.y;
        acc[2] ^= v.z;
        acc[3] ^= v.w;
    } else {
        uint4 v = *(const uint4*)(lds + addr);
        uint4 u = *(const uint4*)(lds + addr + 4096);
        acc[0] ^= v.x;
        acc[1] ^= v.y;
        acc[2] ^= v.z;
        acc[3] ^= v.w;
        acc[4] ^= u.x;
        acc[5] ^= u.y;
        acc[6] ^= u.z;
        acc[7] ^= u.w;
    }
}

// One 8-byte chunk: st <- (st * x^8 + sum_i chunk_i x^(2t+i)) mod g, state top-aligned.
// NB = number of chunk bytes that can be non-zero when FIRST (state still zero).
template <int W, bool FIRST, int NB>
__device__ __forceinline__ void slice8(uint32_t (&st)[W], uint32_t lo, uint32_t hi, const uint8_t* lds)
{
    if constexpr (!FIRST) {
        lo ^= st[W - 2];
        hi ^= st[W - 1];
    }
    uint32_t acc[W];
    acc[0] = 0;
    acc[1] = 0;
#pragma unroll
    for (int w = 2; w < W; ++w)
        acc[w] = FIRST ? 0u : st[w - 2];
    const uint32_t ll = (lo << 4) & 0xF0F0F0F0u, lh = lo & 0xF0F0F0F0u;
    const uint32_t hl = (hi << 4) & 0xF0F0F0F0u, hh = hi & 0xF0F0F0F0u;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        if (!FIRST || p < NB) {
            tbl_acc<W>(acc, lds, ((ll >> (8 * p)) & 0xFFu) + (2 * p) * 256);
            tbl_acc<W>(acc, lds, ((lh >> (8 * p)) & 0xFFu) + (2 * p + 1) * 256);
        }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        if (!FIRST || 4 + p < NB) {
            tbl_acc<W>(acc, lds, ((hl >> (8 * p)) & 0xFFu) + (2 * (4 + p)) * 256);
            tbl_acc<W>(acc, lds, ((hh >> (8 * p)) & 0xFFu) + (2 * (4 + p) + 1) * 256);
        }
    }
#pragma unroll
    for (int w = 0; w < W; ++w)
        st[w] = acc[w];
}

// 4 bytes starting at register-byte position s of the lane's register image R[0..NR).
template <int NR>
__device__ __forceinline__ uint32_t rdw(const uint32_t (&R)[NR], int s)
{
    const int q = s >> 2, sh = s & 3;
    const uint32_t lo = (q < NR) ? R[q] : 0u;
    if (sh == 0)
        return lo;
    const uint32_t hi = (q + 1 < NR) ? R[q + 1] : 0u;
    return __builtin_amdgcn_alignbit(hi, lo, 8 * sh);
}

template <int NR> __device__ __forceinline__ uint32_t rbyte(const uint32_t (&R)[NR], int s)
{
    return (R[s >> 2] >> (8 * (s & 3))) & 0xFFu;
}

// Remainder of the K payload bytes held at register-byte offset BASE (payload byte j at
// register byte BASE + j), processed from the top chunk down.
template <int T2, int NR, int BASE>
__device__ __forceinline__ void rs_remainder(uint32_t (&st)[RsCfg<T2>::W], const uint32_t (&R)[NR], const uint8_t* lds)
{
    using C = RsCfg<T2>;
    constexpr int W = C::W, K = C::K, NC = C::NCHUNK;
    constexpr int TOPN = K - 8 * (NC - 1); // valid bytes in the top chunk (1..8)
#pragma unroll
    for (int w = 0; w < W; ++w)
        st[w] = 0;
    {
        constexpr int J = 8 * (NC - 1);
        uint32_t lo = rdw<NR>(R, BASE + J), hi = rdw<NR>(R, BASE + J + 4);
        if constexpr (TOPN < 4) {
            lo &= (1u << (8 * TOPN)) - 1u;
            hi = 0;
        } else if constexpr (TOPN == 4) {
            hi = 0;
        } else if constexpr (TOPN < 8) {
            hi &= (1u << (8 * (TOPN - 4))) - 1u;
        }
        slice8<W, true, TOPN>(st, lo, hi, lds);
    }
#pragma unroll
    for (int c = NC - 2; c >= 0; --c) {
        const int J = 8 * c;
        uint32_t lo = rdw<NR>(R, BASE + J), hi = rdw<NR>(R, BASE + J + 4);
        slice8<W, false, 8>(st, lo, hi, lds);
    }
}

// Byte q (0..2t-1) of a top-aligned remainder.
template <int T2, int W> __device__ __forceinline__ uint32_t st_byte(const uint32_t (&st)[W], int q)
{
    const int P = 4 * W - T2 + q;
    return (st[P >> 2] >> (8 * (P & 3))) & 0xFFu;
}

// ------------------------------------------------------------------------------------
// Exact reference correction for one block from its remainder r = c mod g.
// Calls fix(pos, e) for every root of sigma found over all 255 field values.
// ------------------------------------------------------------------------------------
template <int T2, typename Fix>
__device__ __forceinline__ void rs_correct(const uint32_t (&r)[T2], const Gf& gf, Fix&& fix)
{
    // syndromes S_i = c(alpha^i) = r(alpha^i), i = 1..2t   (rs_block_device.cpp:131-141)
    uint32_t lr[T2];
#pragma unroll
    for (int q = 0; q < T2; ++q)
        lr[q] = gf.log(r[q]);
    uint32_t S[T2];
#pragma unroll
    for (int i = 1; i <= T2; ++i) {
        uint32_t s = 0;
#pragma unroll
        for (int q = 0; q < T2; ++q) {
            uint32_t v = gf.exp(lr[q] + (uint32_t)((i * q) % 255));
            s ^= r[q] ? v : 0u;
        }
        S[i - 1] = s;
    }
    // Berlekamp-Massey (rs_block_device.cpp:234-269) with Bs = x^m * B kept pre-shifted.
    uint32_t sig[T2 + 1], Bs[T2 + 1];
#pragma unroll
    for (int i = 0; i <= T2; ++i) {
        sig[i] = i == 0 ? 1u : 0u;
        Bs[i] = i == 1 ? 1u : 0u;
    }
    uint32_t b = 1;
    int L = 0;
#pragma unroll
    for (int n = 0; n < T2; ++n) {
        uint32_t d = S[n];
#pragma unroll
        for (int i = 1; i <= n; ++i) {
            uint32_t p = gf.mul(sig[i], S[n - i]);
            d ^= (i <= L) ? p : 0u;
        }
        if (d != 0) {
            const uint32_t coef = gf.div(d, b);
            const uint32_t lc = gf.log(coef);
            uint32_t T[T2 + 1];
#pragma unroll
            for (int i = 0; i <= T2; ++i) {
                T[i] = sig[i];
                sig[i] ^= gf.mul_log(lc, Bs[i]);
            }
            if (2 * L <= n) {
                L = n + 1 - L;
#pragma unroll
                for (int i = T2; i >= 1; --i)
                    Bs[i] = T[i - 1];
                Bs[0] = 0;
                b = d;
            } else {
#pragma unroll
                for (int i = T2; i >= 1; --i)
                    Bs[i] = Bs[i - 1];
                Bs[0] = 0;
            }
        } else {
#pragma unroll
            for (int i = T2; i >= 1; --i)
                Bs[i] = Bs[i - 1];
            Bs[0] = 0;
        }
    }
    // Omega = (S(x) sigma(x)) mod x^2t   (:224-232)
    uint32_t om[T2];
#pragma unroll
    for (int j = 0; j < T2; ++j) {
        uint32_t o = 0;
#pragma unroll
        for (int a = 0; a <= j; ++a)
            o ^= gf.mul(S[a], sig[j - a]);
        om[j] = o;
    }
    int deg = 0;
#pragma unroll
    for (int i = 1; i <= T2; ++i)
        deg = sig[i] ? i : deg;

    // Omega(v) / sigma'(v) for a root v (given with its log)  (:210-222)
    auto forney = [&](uint32_t lv, uint32_t dsig) -> uint32_t {
        uint32_t acc = om[T2 - 1];
#pragma unroll
        for (int j = T2 - 2; j >= 0; --j)
            acc = gf.mul_log(lv, acc) ^ om[j];
        return gf.div(acc, dsig);
    };
    // position of the error for root v = alpha^lv : LOG[inv(v)]
    auto pos_of = [](uint32_t lv) -> uint32_t { return lv == 0 ? 0u : 255u - lv; };

    if (deg == 1) {
        // sigma = 1 + s1 x: single root v = 1/s1; sigma' = s1
        const uint32_t ls1 = gf.log(sig[1]);
        const uint32_t lv = ls1 == 0 ? 0u : 255u - ls1;
        fix(pos_of(lv), forney(lv, sig[1]));
    } else if (deg == 2) {
        if (sig[1] == 0) {
            // x^2 = 1/s2: one (double) root, sigma' == 0 -> e = 0 (division by zero is 0)
            const uint32_t u = (255u - gf.log(sig[2])) % 255u;
            const uint32_t lv = (u & 1u) ? (u + 255u) >> 1 : u >> 1;
            fix(pos_of(lv), 0u);
        } else {
            // x = (s1/s2) y,  y^2 + y = s2 / s1^2
            const uint32_t c = gf.div(sig[2], gf.mul(sig[1], sig[1]));
            const uint32_t y0 = gf.qs(c);
            if (y0 != 0) {
                const uint32_t k = gf.div(sig[1], sig[2]);
                const uint32_t v1 = gf.mul(k, y0), v2 = gf.mul(k, y0 ^ 1u);
                const uint32_t l1 = gf.log(v1), l2 = gf.log(v2);
                fix(pos_of(l1), forney(l1, sig[1]));
                fix(pos_of(l2), forney(l2, sig[1]));
            }
        }
    } else if (deg >= 3) {
        // exhaustive Chien over every v = alpha^m, m = 0..254 (:271-280)
        uint32_t ls[T2 + 1];
#pragma unroll
        for (int i = 0; i <= T2; ++i)
            ls[i] = gf.log(sig[i]);
        for (uint32_t m = 0; m < 255; ++m) {
            uint32_t s = 0, ds = 0;
#pragma unroll
            for (int i = 0; i <= T2; ++i) {
                const uint32_t e = (ls[i] + (uint32_t)i * m) % 255u;
                const uint32_t term = sig[i] ? gf.exp(e) : 0u; // sigma_i v^i
                s ^= term;
                if (i & 1) {
                    // derivative term sigma_i v^(i-1) = term / v
                    const uint32_t td = sig[i] ? gf.exp((e + 255u - m) % 255u) : 0u;
                    ds ^= td;
                }
            }
            if (s == 0)
                fix(pos_of(m), forney(m, ds));
        }
    }
}

// ------------------------------------------------------------------------------------
// Per-wave bodies (C = wave index in the workgroup; the wave owns blocks 4*lane + C).
// ------------------------------------------------------------------------------------
template <int T2, int C>
__device__ __forceinline__ void rs_encode_wave(uint8_t* lds, uint32_t lane)
{
    using Cf = RsCfg<T2>;
    constexpr int K = Cf::K, W = Cf::W;
    constexpr int A = (K * C) % 4;          // input alignment of this wave's blocks
    constexpr int NR = (A + K + 3) / 4;
    const uint32_t b = 4 * lane + C;
    uint8_t* tile = lds + Cf::OFF_TILE;

    uint32_t R[NR];
    const uint32_t inb = K * b - A;
#pragma unroll
    for (int q = 0; q < NR; ++q)
        R[q] = *(const uint32_t*)(tile + inb + 4 * q);

    uint32_t st[W];
    rs_remainder<T2, NR, A>(st, R, lds);

    __syncthreads(); // every lane of every wave has its block in registers

    // codeword byte m: parity m < 2t, payload byte m-2t otherwise
    auto cw_byte = [&](int m) -> uint32_t { return m < T2 ? st_byte<T2, W>(st, m) : rbyte<NR>(R, A + m - T2); };
    constexpr int OB = (RS_N * C) % 4;
    constexpr int M0 = (4 - OB) % 4;
    constexpr int NU = (RS_N - M0) / 4;
    const uint32_t ob = RS_N * b;
#pragma unroll
    for (int m = 0; m < M0; ++m)
        tile[ob + m] = (uint8_t)cw_byte(m);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int m = M0 + 4 * u;
        uint32_t v;
        if (m >= T2) {
            v = rdw<NR>(R, A + m - T2);
        } else {
            v = cw_byte(m) | (cw_byte(m + 1) << 8) | (cw_byte(m + 2) << 16) | (cw_byte(m + 3) << 24);
        }
        *(uint32_t*)(tile + ob + m) = v;
    }
#pragma unroll
    for (int m = M0 + 4 * NU; m < RS_N; ++m)
        tile[ob + m] = (uint8_t)cw_byte(m);
}

template <int T2, int C>
__device__ __forceinline__ void rs_decode_wave(uint8_t* lds, uint32_t lane, uint32_t nb, uint8_t* __restrict__ raw_g,
    size_t tile_block0, bool write_back, bool want_data)
{
    using Cf = RsCfg<T2>;
    constexpr int K = Cf::K, W = Cf::W;
    constexpr int A = (RS_N * C) % 4;
    constexpr int NR = (A + RS_N + 3) / 4;
    const uint32_t b = 4 * lane + C;
    const bool valid = b < nb;
    uint8_t* tile = lds + Cf::OFF_TILE;

    uint32_t R[NR];
    const uint32_t inb = RS_N * b - A;
#pragma unroll
    for (int q = 0; q < NR; ++q)
        R[q] = *(const uint32_t*)(tile + inb + 4 * q);

    // remainder of the payload, then r = c mod g = parity(payload) ^ stored parity
    uint32_t st[W];
    rs_remainder<T2, NR, A + T2>(st, R, lds);
    uint32_t any = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const int s = A + 4 * w - (4 * W - T2); // register byte of stored-parity byte (4w - pad)
        uint32_t v;
        if (s >= A) {
            v = rdw<NR>(R, s);
        } else if (s + 4 > A) {
            // partially padding: keep the bytes >= A
            const int keep = s + 4 - A;
            v = (rdw<NR>(R, A) << (8 * (4 - keep)));
        } else {
            v = 0;
        }
        st[w] ^= v;
        any |= st[w];
    }
    const bool err = valid && any != 0;

    if (__builtin_amdgcn_ballot_w64(err)) {
        if (err) {
            uint32_t r[T2];
#pragma unroll
            for (int q = 0; q < T2; ++q)
                r[q] = st_byte<T2, W>(st, q);
            const Gf gf { lds + Cf::OFF_GF };
            const size_t gblk = tile_block0 + b;
            rs_correct<T2>(r, gf, [&](uint32_t pos, uint32_t e) {
                if (e == 0)
                    return;
                const uint32_t orig = tile[RS_N * b + pos];
                if (write_back)
                    raw_g[gblk * RS_N + pos] = (uint8_t)(orig ^ e);
                const uint32_t idx = A + pos, q = idx >> 2, msk = e << (8 * (idx & 3));
#pragma unroll
                for (int qq = 0; qq < NR; ++qq)
                    R[qq] ^= ((uint32_t)qq == q) ? msk : 0u;
            });
        }
    }
    lds[Cf::OFF_STATUS + b] = err ? 1 : 0;
    if (!want_data)
        return;

    __syncthreads();
    constexpr int OB = (K * C) % 4;
    constexpr int M0 = (4 - OB) % 4;
    constexpr int NU = (K - M0) / 4;
    const uint32_t ob = K * b;
    constexpr int D = A + T2; // register byte of payload byte 0
#pragma unroll
    for (int m = 0; m < M0; ++m)
        tile[ob + m] = (uint8_t)rbyte<NR>(R, D + m);
#pragma unroll
    for (int u = 0; u < NU; ++u)
        *(uint32_t*)(tile + ob + M0 + 4 * u) = rdw<NR>(R, D + M0 + 4 * u);
#pragma unroll
    for (int m = M0 + 4 * NU; m < K; ++m)
        tile[ob + m] = (uint8_t)rbyte<NR>(R, D + m);
}

// ------------------------------------------------------------------------------------
// Kernels
// ------------------------------------------------------------------------------------
template <int T2>
__global__ __launch_bounds__(256, 2) void rs255_encode_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables)
{
    using Cf = RsCfg<T2>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[Cf::LDS_BYTES];
    const uint64_t tile0 = (uint64_t)blockIdx.x * RS_TILE;
    const uint32_t nb = (uint32_t)min((uint64_t)RS_TILE, nblocks - tile0);
    load_tables(lds, tables, Cf::TBL_BYTES);
    stage_in(lds + Cf::OFF_TILE, data + tile0 * Cf::K, nb * Cf::K);
    const uint32_t lane = lane_id();
    switch (wave_id()) {
    case 0: rs_encode_wave<T2, 0>(lds, lane); break;
    case 1: rs_encode_wave<T2, 1>(lds, lane); break;
    case 2: rs_encode_wave<T2, 2>(lds, lane); break;
    default: rs_encode_wave<T2, 3>(lds, lane); break;
    }
    __syncthreads();
    stage_out(raw + tile0 * RS_N, lds + Cf::OFF_TILE, nb * RS_N);
}

template <int T2>
__global__ __launch_bounds__(256, 2) void rs255_decode_kernel(uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks, const uint8_t* __restrict__ tables, int write_back)
{
    using Cf = RsCfg<T2>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[Cf::LDS_BYTES];
    const uint64_t tile0 = (uint64_t)blockIdx.x * RS_TILE;
    const uint32_t nb = (uint32_t)min((uint64_t)RS_TILE, nblocks - tile0);
    load_tables(lds, tables, Cf::TBL_BYTES + GF_BYTES);
    stage_in(lds + Cf::OFF_TILE, raw + tile0 * RS_N, nb * RS_N);
    const uint32_t lane = lane_id();
    const bool wb = write_back != 0, want = data != nullptr;
    switch (wave_id()) {
    case 0: rs_decode_wave<T2, 0>(lds, lane, nb, raw, tile0, wb, want); break;
    case 1: rs_decode_wave<T2, 1>(lds, lane, nb, raw, tile0, wb, want); break;
    case 2: rs_decode_wave<T2, 2>(lds, lane, nb, raw, tile0, wb, want); break;
    default: rs_decode_wave<T2, 3>(lds, lane, nb, raw, tile0, wb, want); break;
    }
    __syncthreads();
    if (want)
        stage_out(data + tile0 * Cf::K, lds + Cf::OFF_TILE, nb * Cf::K);
    if (status)
        stage_out(status + tile0, lds + Cf::OFF_STATUS, nb);
}


} // namespace ppfs
