#pragma once
// rs_fast.hpp -- Reed-Solomon GF(2^8) encode / syndrome / correct kernels for gfx950 (n = 255).
//
// Reference semantics: lib/blockdevice/src/rs_block_device.cpp
//   encode  _encodeBlock :95-117   c(x) = m(x) x^2t + (m(x) x^2t mod g(x)); byte i = coeff of x^i,
//                                  parity in bytes [0,2t), payload in [2t,n)
//   decode  _fixBlockAndExtract :119-183, _berlekampMassey :234-269, _errorLocations :271-280,
//           _calculateOmega :224-232, _forney :210-222
//
// Work decomposition (gfx950: 64-lane waves, 160 KiB LDS per CU):
//   - A wave-tile is 64 consecutive blocks; lane l owns block l of the tile.  Each wave of a
//     persistent 256-thread workgroup streams its own wave-tiles through a private 16 KiB LDS
//     buffer -- no workgroup barriers on the hot path, so the 8 waves resident on a CU run
//     their load / compute / store phases independently.  The codec tables (slicing tables,
//     GF log/antilog) are loaded into LDS once per workgroup.
//   - Packed input rows (249 B payloads, 255 B codewords) arrive by LDS-DMA
//     (global_load_lds_dwordx4: one contiguous KiB per wave-instruction).  Each lane then
//     reads its block as aligned dwords R[0..NR) and funnel-shifts (v_alignbit) by its own
//     byte misalignment, so every register index is a compile-time constant.
//   - Remainder: slicing-by-8 from the top chunk down.  For 8 bytes e_i (XORed with the top
//     of the running remainder) the new remainder is the XOR of 16 LDS table entries
//     T[i][nibble] = nibble * (x^(2t+i) mod g) -- no serial dependency inside a chunk.
//   - Decode runs the same slicing over all 255 codeword bytes: r' = x^2t c(x) mod g, which is
//     zero iff every syndrome is zero (g(0) != 0).  Lanes with r' != 0 run the reference's
//     correction exactly (syndromes S_i = r'(a^i) a^(-2t i), Berlekamp-Massey, roots over all
//     255 field values, Omega, Forney) in registers.
//   - Output rows are rebuilt in place in the same LDS buffer (interior dwords + byte-wise
//     row ends) and streamed out with 16-byte stores.
#include <hip/hip_runtime.h>

#include "dbg.hpp"
#include "srv_device.hpp"
#include <stdint.h>

#include "gf_common.hpp"

namespace ppfs {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int RS_N = 255;   // fast-path codeword length
constexpr int RS_WT = 64;   // blocks per wave-tile (one per lane)
constexpr int RS_WAVES = 4; // waves per workgroup

// Variant knobs: NSEG_ = independent remainder chains per lane (0 = default policy),
// PF = prefetch the next tile into VGPRs while computing (1) or not (0).
template <int T2, int NSEG_ = 0> struct RsCfg {
    static constexpr int K = RS_N - T2;
    static constexpr int W = T2 <= 8 ? 2 : (T2 <= 16 ? 4 : 8); // remainder words (top aligned)
    // independent remainder chains per lane (segments of 256/NSEG bytes), combined with
    // x^64 / x^128 map tables: more LDS reads in flight per wave
    // measured on MI355X (tools/probes/rs_ablate.hip): one chain per lane is fastest at 2 waves/SIMD
    static constexpr int NSEG = NSEG_ ? NSEG_ : 1;
    static constexpr int SEGL = 256 / NSEG;
    static constexpr int SLICE_BYTES = W <= 4 ? 4096 : 8192;    // 16 nibble tables x 16 x 16 B (x2)
    static constexpr int NMAP = NSEG == 4 ? 2 : (NSEG == 2 ? 1 : 0);
    static constexpr int MAP_BYTES = NMAP * T2 * 512;           // per map: 2t x 2 nibble tables x 16 x 16 B
    static constexpr int OFF_MAP = SLICE_BYTES;
    static constexpr int TBL_BYTES = SLICE_BYTES + MAP_BYTES;   // what encode loads
    static constexpr int OFF_GF = TBL_BYTES;
    static constexpr int OFF_WAVES = OFF_GF + GF_BYTES;
    static constexpr int WAVE_BUF = RS_WT * RS_N + 16;          // 16336: codeword tile + slack
    static constexpr int WAVE_STATUS = 64;
    static constexpr int WAVE_BYTES = WAVE_BUF + WAVE_STATUS;   // 16400 (16-byte multiple)
    static constexpr int LDS_BYTES = OFF_WAVES + RS_WAVES * WAVE_BYTES;
    static_assert(2 * LDS_BYTES <= 163840, "two workgroups per CU");
};

// ------------------------------------------------------------------------------------
// Wave-level staging: global <-> the wave's LDS buffer
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_stage_in(uint8_t* buf, const uint8_t* __restrict__ src, uint32_t bytes,
    uint32_t lane)
{
    const uint32_t npiece = bytes >> 4;
    const uint32_t ngroup = (npiece + 63) >> 6;
    for (uint32_t g = 0; g < ngroup; ++g) {
        const uint32_t piece = g * 64 + lane;
        if (piece < npiece)
            __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)piece * 16),
                (__attribute__((address_space(3))) void*)(buf + g * 1024), 16, 0, 0);
    }
    const uint32_t tail = bytes & 15u;
    if (lane < tail)
        buf[npiece * 16 + lane] = src[npiece * 16 + lane];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void wave_stage_out(uint8_t* __restrict__ dst, const uint8_t* buf, uint32_t bytes,
    uint32_t lane)
{
    const uint32_t npiece = bytes >> 4;
    for (uint32_t p = lane; p < npiece; p += 64)
        *(uint4*)(dst + (size_t)p * 16) = *(const uint4*)(buf + p * 16);
    const uint32_t tail = bytes & 15u;
    if (lane < tail)
        dst[npiece * 16 + lane] = buf[npiece * 16 + lane];
}

__device__ __forceinline__ void load_tables(uint8_t* lds_dst, const uint8_t* __restrict__ src, uint32_t bytes)
{
    for (uint32_t p = threadIdx.x; p < (bytes >> 4); p += blockDim.x)
        *(uint4*)(lds_dst + p * 16) = *(const uint4*)(src + (size_t)p * 16);
}

// compiler + wave-level ordering point between LDS phases of one wave
__device__ __forceinline__ void wave_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------------------------
// Slicing-by-8 remainder step
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); // v_bitop3_b32: a ^ b ^ c
}

template <int W> struct Ent {
    uint32_t w[W];
};

template <int W> __device__ __forceinline__ Ent<W> tbl_ld(const uint8_t* lds, uint32_t addr)
{
    Ent<W> e;
    if constexpr (W == 2) {
        const uint2 v = *(const uint2*)(lds + addr);
        e.w[0] = v.x;
        e.w[1] = v.y;
    } else if constexpr (W == 4) {
        const uint4 v = *(const uint4*)(lds + addr);
        e.w[0] = v.x;
        e.w[1] = v.y;
        e.w[2] = v.z;
        e.w[3] = v.w;
    } else {
        const uint4 v = *(const uint4*)(lds + addr);
        const uint4 u = *(const uint4*)(lds + addr + 4096);
        e.w[0] = v.x;
        e.w[1] = v.y;
        e.w[2] = v.z;
        e.w[3] = v.w;
        e.w[4] = u.x;
        e.w[5] = u.y;
        e.w[6] = u.z;
        e.w[7] = u.w;
    }
    return e;
}

// acc ^= XOR of N entries, three inputs per v_bitop3
template <int W, int N> __device__ __forceinline__ void xor_into(uint32_t (&acc)[W], const Ent<W> (&e)[N])
{
#pragma unroll
    for (int w = 0; w < W; ++w) {
        uint32_t a = acc[w];
        int i = 0;
#pragma unroll
        for (; i + 1 < N; i += 2)
            a = xor3(a, e[i].w[w], e[i + 1].w[w]);
        if (i < N)
            a ^= e[i].w[w];
        acc[w] = a;
    }
}

// (x >> 8K) & 0xF0 in one VALU op (SDWA byte select; LLVM only forms it for K = 2, 3)
template <int K> __device__ __forceinline__ uint32_t nib16(uint32_t x)
{
    if constexpr (K == 0) {
        return x & 0xF0u;
    } else {
        uint32_t r;
        if constexpr (K == 1)
            asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
                : "=v"(r) : "v"(x), "s"(0xF0u));
        else if constexpr (K == 2)
            asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
                : "=v"(r) : "v"(x), "s"(0xF0u));
        else
            asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
                : "=v"(r) : "v"(x), "s"(0xF0u));
        return r;
    }
}

// the 2 NL table reads of one slicing step (compile-time byte positions P..NL-1)
template <int W, int NL, int P>
__device__ __forceinline__ void slice_lookups(Ent<W> (&e)[2 * NL], uint32_t lo, uint32_t hi, uint32_t lo4, uint32_t hi4,
    const uint8_t* lds)
{
    if constexpr (P < NL) {
        const uint32_t x = P < 4 ? lo : hi, x4 = P < 4 ? lo4 : hi4;
        e[2 * P] = tbl_ld<W>(lds, nib16<P & 3>(x4) + (2 * P) * 256);
        e[2 * P + 1] = tbl_ld<W>(lds, nib16<P & 3>(x) + (2 * P + 1) * 256);
        slice_lookups<W, NL, P + 1>(e, lo, hi, lo4, hi4, lds);
    }
}

// st <- (st * x^8 + sum_i chunk_i x^(2t+i)) mod g, top-aligned state.
// NB = number of chunk bytes that may be non-zero when FIRST (state still zero).
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
    constexpr int NL = FIRST ? (NB < 8 ? NB : 8) : 8;
    Ent<W> e[2 * NL];
    // slot address of a nibble = nibble * 16: the high nibble of byte k is (x >> 8k) & 0xF0,
    // the low one (x << 4 >> 8k) & 0xF0 -- one v_and_b32_sdwa (byte select) each
    slice_lookups<W, NL, 0>(e, lo, hi, lo << 4, hi << 4, lds);
    xor_into<W, 2 * NL>(acc, e);
#pragma unroll
    for (int w = 0; w < W; ++w)
        st[w] = acc[w];
}

// out = (r(x) x^E) mod g for a top-aligned remainder r, via the 2t x 2 nibble map tables at mapb
template <int T2, int W>
__device__ __forceinline__ void map_apply(uint32_t (&out)[W], const uint32_t (&r)[W], const uint8_t* lds, uint32_t mapb)
{
    Ent<W> e[2 * T2];
#pragma unroll
    for (int i = 0; i < T2; ++i) {
        const int P = 4 * W - T2 + i;
        const uint32_t w = r[P >> 2] >> (8 * (P & 3));
        e[2 * i] = tbl_ld<W>(lds, mapb + (2 * i) * 256 + ((w << 4) & 0xF0u));
        e[2 * i + 1] = tbl_ld<W>(lds, mapb + (2 * i + 1) * 256 + (w & 0xF0u));
    }
#pragma unroll
    for (int w = 0; w < W; ++w)
        out[w] = 0;
    xor_into<W, 2 * T2>(out, e);
}

template <int NR> __device__ __forceinline__ uint32_t rget(const uint32_t (&R)[NR], int q)
{
    return (q >= 0 && q < NR) ? R[q] : 0u;
}

// 4 bytes at register-byte position 4q + sh (sh = the lane's runtime misalignment 0..3)
template <int NR> __device__ __forceinline__ uint32_t rdw(const uint32_t (&R)[NR], int q, uint32_t sh)
{
    return __builtin_amdgcn_alignbit(rget<NR>(R, q + 1), rget<NR>(R, q), 8 * sh);
}

template <int LEN, int SEGL, int S> struct SegInfo {
    static constexpr int LO = SEGL * S;
    static constexpr int LENS = (LEN - LO) < SEGL ? (LEN - LO) : SEGL;
    static constexpr int NC = LENS > 0 ? (LENS + 7) / 8 : 0;
    static constexpr int TOPN = LENS - 8 * (NC - 1);
};

// one chunk (index c, counted from the segment start) of segment S
template <int T2, int NR, int LEN, int SEGL, int S, int C>
__device__ __forceinline__ void seg_step(uint32_t (&st)[RsCfg<T2>::W], const uint32_t (&R)[NR], uint32_t sh,
    const uint8_t* lds)
{
    using SI = SegInfo<LEN, SEGL, S>;
    constexpr int W = RsCfg<T2>::W;
    if constexpr (C < SI::NC) {
        constexpr int J = SI::LO + 8 * C;
        uint32_t lo = rdw<NR>(R, J / 4, sh), hi = rdw<NR>(R, J / 4 + 1, sh);
        if constexpr (C == SI::NC - 1) {
            constexpr int TOPN = SI::TOPN;
            if constexpr (TOPN < 4) {
                lo &= (1u << (8 * TOPN)) - 1u;
                hi = 0;
            } else if constexpr (TOPN == 4) {
                hi = 0;
            } else if constexpr (TOPN < 8) {
                hi &= (1u << (8 * (TOPN - 4))) - 1u;
            }
            slice8<W, true, TOPN>(st, lo, hi, lds);
        } else {
            slice8<W, false, 8>(st, lo, hi, lds);
        }
    }
}

template <int T2, int NR, int LEN, int SEGL, int C>
__device__ __forceinline__ void seg_round(uint32_t (&s0)[RsCfg<T2>::W], uint32_t (&s1)[RsCfg<T2>::W],
    uint32_t (&s2)[RsCfg<T2>::W], uint32_t (&s3)[RsCfg<T2>::W], const uint32_t (&R)[NR], uint32_t sh,
    const uint8_t* lds)
{
    seg_step<T2, NR, LEN, SEGL, 0, C>(s0, R, sh, lds);
    if constexpr (256 / SEGL > 1)
        seg_step<T2, NR, LEN, SEGL, 1, C>(s1, R, sh, lds);
    if constexpr (256 / SEGL > 2) {
        seg_step<T2, NR, LEN, SEGL, 2, C>(s2, R, sh, lds);
        seg_step<T2, NR, LEN, SEGL, 3, C>(s3, R, sh, lds);
    }
    if constexpr (C > 0)
        seg_round<T2, NR, LEN, SEGL, C - 1>(s0, s1, s2, s3, R, sh, lds);
}

// Remainder of LEN bytes (byte j at register byte sh + j), as NSEG independent chains.
template <int T2, int NR, int LEN, int NS = 0>
__device__ __forceinline__ void rs_remainder(uint32_t (&st)[RsCfg<T2>::W], const uint32_t (&R)[NR], uint32_t sh,
    const uint8_t* lds)
{
    using Cf = RsCfg<T2, NS>;
    constexpr int W = Cf::W, SEGL = Cf::SEGL;
    uint32_t s0[W], s1[W], s2[W], s3[W];
#pragma unroll
    for (int w = 0; w < W; ++w)
        s0[w] = s1[w] = s2[w] = s3[w] = 0;
    seg_round<T2, NR, LEN, SEGL, SEGL / 8 - 1>(s0, s1, s2, s3, R, sh, lds);
    if constexpr (Cf::NSEG == 4) {
        uint32_t m1[W], m3[W], b[W], mb[W];
        map_apply<T2, W>(m1, s1, lds, Cf::OFF_MAP);      // x^64
        map_apply<T2, W>(m3, s3, lds, Cf::OFF_MAP);      // x^64
#pragma unroll
        for (int w = 0; w < W; ++w)
            b[w] = s2[w] ^ m3[w];
        map_apply<T2, W>(mb, b, lds, Cf::OFF_MAP + T2 * 512); // x^128
#pragma unroll
        for (int w = 0; w < W; ++w)
            st[w] = xor3(s0[w], m1[w], mb[w]);
    } else if constexpr (Cf::NSEG == 2) {
        uint32_t m1[W];
        map_apply<T2, W>(m1, s1, lds, Cf::OFF_MAP);      // x^128
#pragma unroll
        for (int w = 0; w < W; ++w)
            st[w] = s0[w] ^ m1[w];
    } else {
#pragma unroll
        for (int w = 0; w < W; ++w)
            st[w] = s0[w];
    }
}

// ------------------------------------------------------------------------------------
// Row emission: write LEN stream bytes to LDS [out, out+LEN) (any alignment), in place.
// Stream byte p comes from register byte (cbase + p) of R, except bytes p < NPAR which come
// from the parity function par(u, p_u) (only called for dwords that contain them).
// Interior dwords are written whole; the first/last partial dwords byte by byte, so lanes
// never write each other's bytes.
// ------------------------------------------------------------------------------------
template <int NR, int LEN, int CMIN, int CMAX, int NPAR, typename Par>
__device__ __forceinline__ void emit_row(uint8_t* tile, uint32_t out, int cbase, const uint32_t (&R)[NR], Par&& par)
{
    const uint32_t m0 = (4u - (out & 3u)) & 3u;      // first stream byte of the first whole dword
    const int cb = cbase + (int)m0;                  // register byte of stream byte m0
    const int qoff = cb >> 2;                        // arithmetic: floor
    const uint32_t sh = (uint32_t)cb & 3u;
    constexpr int DMIN = (CMIN >= 0) ? CMIN / 4 : -((-CMIN + 3) / 4);
    constexpr int DMAX = (CMAX + 3) / 4;
    constexpr int UMAX = LEN / 4; // u in [-1, UMAX]
    // X(u) = R[u + qoff] selected over the possible offsets
    auto X = [&](int u) -> uint32_t {
        uint32_t v = 0;
#pragma unroll
        for (int d = DMIN; d <= DMAX; ++d)
            v = (qoff == d) ? rget<NR>(R, u + d) : v;
        return v;
    };
    uint32_t xcur = X(-1);
#pragma unroll
    for (int u = -1; u <= UMAX; ++u) {
        const uint32_t xnext = X(u + 1);
        uint32_t v = __builtin_amdgcn_alignbit(xnext, xcur, 8 * sh);
        xcur = xnext;
        const int p = (int)m0 + 4 * u; // stream position of byte 0 of this dword
        if constexpr (NPAR > 0) {
            if (4 * u <= NPAR + 3) // only the first few dwords can hold parity bytes
                v = par(v, p);
        }
        const bool full = p >= 0 && p + 4 <= LEN;
        if (u >= 0 && 4 * u + 7 <= LEN) {
            // always whole for every m0 in [0,3]
            *(uint32_t*)(tile + out + m0 + 4 * u) = v;
        } else if (full) {
            *(uint32_t*)(tile + out + m0 + 4 * u) = v;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int pk = p + k;
                if (pk >= 0 && pk < LEN)
                    tile[out + (uint32_t)pk] = (uint8_t)(v >> (8 * k));
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// Exact reference correction from r' = x^2t c(x) mod g.  Calls fix(pos, e) for every root of
// sigma over all 255 field values.
// ------------------------------------------------------------------------------------
// S_i = c(a^i) = r'(a^i) * a^(-2t i), i = 1..2t   (rs_block_device.cpp:131-141)
template <int T2>
__device__ __forceinline__ void rs_syndromes(const uint32_t (&r)[T2], const Gf& gf, uint32_t (&S)[T2])
{
    uint32_t lr[T2];
#pragma unroll
    for (int q = 0; q < T2; ++q)
        lr[q] = gf.log(r[q]);
#pragma unroll
    for (int i = 1; i <= T2; ++i) {
        uint32_t s = 0;
#pragma unroll
        for (int q = 0; q < T2; ++q) {
            const uint32_t e = (uint32_t)(((i * q - i * T2) % 255 + 255) % 255);
            const uint32_t v = gf.exp(lr[q] + e);
            s ^= r[q] ? v : 0u;
        }
        S[i - 1] = s;
    }
}

// Geometric syndromes S_i = S_1 X^(i-1) (all non-zero): the shortest LFSR of the sequence is
// 1 + X x, which is what Berlekamp-Massey returns for it (its output depends on S only), so
// the reference corrects exactly one byte: root v = 1/X -> pos = LOG[X],
// Omega = S_1 (higher terms cancel), e = Omega(v) / sigma'(v) = S_1 / X.
// This is the single-error case; it skips BM / Omega / Forney.
template <int T2>
__device__ __forceinline__ bool rs_geometric(const uint32_t (&S)[T2], const Gf& gf, uint32_t& pos, uint32_t& e)
{
    uint32_t ls[T2];
    bool geo = true;
#pragma unroll
    for (int i = 0; i < T2; ++i) {
        ls[i] = gf.log(S[i]);
        geo = geo && S[i] != 0;
    }
    const uint32_t lx = (ls[1] + 255u - ls[0]) % 255u;
#pragma unroll
    for (int i = 1; i + 1 < T2; ++i)
        geo = geo && (ls[i + 1] + 255u - ls[i]) % 255u == lx;
    pos = lx;
    e = gf.exp(ls[0] + 255u - lx);
    return geo;
}

// ------------------------------------------------------------------------------------
// Exact reference correction from the syndromes (general case).  Calls fix(pos, e) for every
// root of sigma over all 255 field values.
// ------------------------------------------------------------------------------------
template <int T2, typename Fix>
__device__ __forceinline__ void rs_correct_general(const uint32_t (&S)[T2], const Gf& gf, Fix&& fix)
{
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
            const uint32_t p = gf.mul(sig[i], S[n - i]);
            d ^= (i <= L) ? p : 0u;
        }
        if (d != 0) {
            const uint32_t lc = gf.log(gf.div(d, b));
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

    // Omega(v) / sigma'(v) for a root v given by its log  (:210-222)
    auto forney = [&](uint32_t lv, uint32_t dsig) -> uint32_t {
        uint32_t acc = om[T2 - 1];
#pragma unroll
        for (int j = T2 - 2; j >= 0; --j)
            acc = gf.mul_log(lv, acc) ^ om[j];
        return gf.div(acc, dsig);
    };
    // error position for root v = a^lv:  LOG[inv(v)]
    auto pos_of = [](uint32_t lv) -> uint32_t { return lv == 0 ? 0u : 255u - lv; };

    if (deg == 1) {
        // sigma = 1 + s1 x: the single root v = 1/s1, sigma' = s1
        const uint32_t ls1 = gf.log(sig[1]);
        const uint32_t lv = ls1 == 0 ? 0u : 255u - ls1;
        fix(pos_of(lv), forney(lv, sig[1]));
    } else if (deg == 2) {
        if (sig[1] == 0) {
            // x^2 = 1/s2: one root, sigma' == 0 -> e = 0 (division by zero is 0 in GF256)
            const uint32_t u = (255u - gf.log(sig[2])) % 255u;
            const uint32_t lv = (u & 1u) ? (u + 255u) >> 1 : u >> 1;
            fix(pos_of(lv), 0u);
        } else {
            // x = (s1/s2) y with y^2 + y = s2 / s1^2: two roots or none
            const uint32_t c = gf.div(sig[2], gf.mul(sig[1], sig[1]));
            const uint32_t y0 = gf.qs(c);
            if (y0 != 0) {
                const uint32_t k = gf.div(sig[1], sig[2]);
                const uint32_t l1 = gf.log(gf.mul(k, y0)), l2 = gf.log(gf.mul(k, y0 ^ 1u));
                fix(pos_of(l1), forney(l1, sig[1]));
                fix(pos_of(l2), forney(l2, sig[1]));
            }
        }
    } else if (deg >= 3) {
        // exhaustive search over every v = a^m, m = 0..254 (:271-280)
        uint32_t ls[T2 + 1];
#pragma unroll
        for (int i = 0; i <= T2; ++i)
            ls[i] = gf.log(sig[i]);
        for (uint32_t m = 0; m < 255; ++m) {
            uint32_t s = 0, ds = 0;
#pragma unroll
            for (int i = 0; i <= T2; ++i) {
                const uint32_t e = (ls[i] + (uint32_t)i * m) % 255u;
                s ^= sig[i] ? gf.exp(e) : 0u;
                if (i & 1)
                    ds ^= sig[i] ? gf.exp((e + 255u - m) % 255u) : 0u;
            }
            if (s == 0)
                fix(pos_of(m), forney(m, ds));
        }
    }
}

// ------------------------------------------------------------------------------------
// Per-lane bodies
// ------------------------------------------------------------------------------------
template <int T2, int NS, typename Pre>
__device__ __forceinline__ void rs_encode_lane(uint8_t* tile, const uint8_t* lds, uint32_t l, Pre&& prefetch)
{
    using Cf = RsCfg<T2, NS>;
    constexpr int K = Cf::K, W = Cf::W;
    constexpr int NR = (3 + K + 3) / 4;
    const uint32_t ib = K * l, a = ib & 3u;
    const uint32_t* tw = (const uint32_t*)(tile + (ib & ~3u));
    uint32_t R[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q)
        R[q] = tw[q];
    prefetch();
    uint32_t st[W];
    rs_remainder<T2, NR, K, NS>(st, R, a, lds);
    wave_fence(); // every lane's block is in registers before the in-place rewrite

    // codeword stream: byte p < 2t parity (top-aligned state byte 4W-2t+p), else payload p-2t
    auto par = [&](uint32_t v, int p) -> uint32_t {
        // 4 parity-stream bytes at positions p..p+3 merged over the payload bytes
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int pk = p + k;
            uint32_t pb = 0;
#pragma unroll
            for (int q = 0; q < T2; ++q) {
                const int P = 4 * W - T2 + q;
                pb = (pk == q) ? ((st[P >> 2] >> (8 * (P & 3))) & 0xFFu) : pb;
            }
            const bool isp = pk >= 0 && pk < T2;
            v = isp ? ((v & ~(0xFFu << (8 * k))) | (pb << (8 * k))) : v;
        }
        return v;
    };
    if constexpr (T2 >= 4) {
        // Direct emission: v_q = funnel(R[q+1], R[q]) by sh = 8 * ((2a - 2t) mod 4) bits holds
        // payload bytes 4q + sh/8 - a .. +3, whose output position ob + 2t + 4q + sh/8 - a is
        // 4-aligned (ob = 255 l = -a mod 4, and 2t is even): one v_alignbit + one ds_write_b32
        // per dword, no per-lane register selection.  The first and last dwords may carry up to
        // 3 stray bytes into this row's / the next row's parity field (2t >= 4 >= 3 bytes);
        // the parity bytes are written after every lane's payload dwords, over them.
        const uint32_t ob = RS_N * l;
        const uint32_t sb = ((2u * a) - (uint32_t)T2) & 3u; // sh / 8, 0 or 2
        const uint32_t shb = 8u * sb;
        const int qlo = (int)sb > (int)a ? -1 : 0;         // 4q + sb - a <= 0
        uint8_t* dst = tile + ob + T2 + sb - a;            // + 4q
        if (qlo < 0)
            *(uint32_t*)(dst - 4) = __builtin_amdgcn_alignbit(R[0], 0u, shb);
#pragma unroll
        for (int q = 0; q < NR; ++q) {
            // dword q starts at payload byte 4q + sb - a: written iff that is <= K - 1, so a
            // row's last dword reaches at most 3 bytes past the row (into the next parity field)
            const uint32_t v = __builtin_amdgcn_alignbit(rget<NR>(R, q + 1), R[q], shb);
            if (4 * q + 3 <= K - 1)
                *(uint32_t*)(dst + 4 * q) = v;
            else if (4 * q + (int)sb - (int)a <= K - 1)
                *(uint32_t*)(dst + 4 * q) = v;
        }
        asm volatile("" ::: "memory"); // every lane's payload dwords precede any parity byte
#pragma unroll
        for (int q = 0; q < T2; ++q) {
            const int P = 4 * W - T2 + q;
            tile[ob + q] = (uint8_t)(st[P >> 2] >> (8 * (P & 3)));
        }
        return;
    }
    // payload byte j at register byte a + j -> stream byte p at register byte a + p - 2t
    emit_row<NR, RS_N, -T2, 3 - T2, T2>(tile, RS_N * l, (int)a - T2, R, par);
}

// Decode emission: payload row of lane l at ob = K l from the codeword dwords R (codeword byte c
// at register byte a + c).  v_q = funnel(R[q+1], R[q]) by sb bytes holds payload bytes
// 4q + sb - 2t - a .. +3 at ob + 4q + sb - 2t - a, 4-aligned for sb = 2t (1 - a) mod 4.  Dwords
// inside the row for every lane are plain ds_write_b32; the few that may straddle a row end
// (classified at compile time) write only their in-row bytes.
template <int T2, int NR>
__device__ __forceinline__ void emit_payload_direct(uint8_t* tile, uint32_t l, uint32_t a, const uint32_t (&R)[NR])
{
    constexpr int K = RS_N - T2;
    const uint32_t ob = (uint32_t)K * l;
    const uint32_t sb = ((uint32_t)T2 * (1u - a)) & 3u;
    const uint32_t shb = 8u * sb;
    const int off = (int)sb - T2 - (int)a; // dest(q) - ob = 4q + off, off in [-T2-3, -T2+2]
    uint8_t* dst = tile + (int)ob + off;
#pragma unroll
    for (int q = 0; q < NR; ++q) {
        constexpr int dummy = 0;
        (void)dummy;
        const int lo = 4 * q - T2 - 3, hi = 4 * q - T2 + 2; // range of 4q + off over lanes
        if (hi + 3 < 0 || lo > K - 1)
            continue; // never touches the row
        const uint32_t v = __builtin_amdgcn_alignbit(rget<NR>(R, q + 1), R[q], shb);
        if (lo >= 0 && hi + 3 <= K - 1) {
            *(uint32_t*)(dst + 4 * q) = v;
        } else {
            const int d0 = 4 * q + off; // row offset of byte 0 of v
            if (d0 >= 0 && d0 + 3 <= K - 1) {
                *(uint32_t*)(dst + 4 * q) = v;
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (d0 + k >= 0 && d0 + k <= K - 1)
                        dst[4 * q + k] = (uint8_t)(v >> (8 * k));
            }
        }
    }
}


template <int T2, int NS, typename Pre>
__device__ __forceinline__ void rs_decode_lane(uint8_t* tile, const uint8_t* lds, uint32_t l, bool valid,
    uint8_t* __restrict__ raw_g, size_t blk, bool write_back, bool want_data, uint8_t* status_lds, Pre&& prefetch,
    [[maybe_unused]] uint64_t raw_bytes)
{
    using Cf = RsCfg<T2, NS>;
    constexpr int K = Cf::K, W = Cf::W;
    constexpr int NR = (3 + RS_N + 3) / 4;
    const uint32_t ib = RS_N * l, a = ib & 3u;
    const uint32_t* tw = (const uint32_t*)(tile + (ib & ~3u));
    uint32_t R[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q)
        R[q] = tw[q];
    prefetch();
    // r' = x^2t c(x) mod g over all 255 codeword bytes
    uint32_t st[W];
    rs_remainder<T2, NR, RS_N, NS>(st, R, a, lds);
    uint32_t any = 0;
#pragma unroll
    for (int w = 0; w < W; ++w)
        any |= st[w];
    const bool err = valid && any != 0;
    // a single corrected payload byte, applied to the output row after emission
    uint32_t fpos = 0xFFFFFFFFu, fval = 0;
    if (__builtin_amdgcn_ballot_w64(err)) {
        const Gf gf { lds + Cf::OFF_GF };
        uint32_t S[T2];
        bool geo = false;
        uint32_t gpos = 0, ge = 0;
        if (err) {
            uint32_t r[T2];
#pragma unroll
            for (int q = 0; q < T2; ++q) {
                const int P = 4 * W - T2 + q;
                r[q] = (st[P >> 2] >> (8 * (P & 3))) & 0xFFu;
            }
            rs_syndromes<T2>(r, gf, S);
            geo = rs_geometric<T2>(S, gf, gpos, ge);
        }
        if (__builtin_amdgcn_ballot_w64(err && !geo)) {
            // general path somewhere in the wave: corrections patch each lane's own row of the
            // LDS tile (other lanes only use their own bytes of shared words), then the whole
            // wave reloads R, which is therefore dead through the register-hungry BM code
            auto fix = [&](uint32_t pos, uint32_t e) {
                if (e == 0)
                    return;
                const uint8_t fixed = (uint8_t)(tile[ib + pos] ^ e);
                tile[ib + pos] = fixed;
                if (write_back && PPFS_DBG_OK(raw_g + blk * RS_N + pos, 1, raw_g, raw_bytes))
                    raw_g[blk * RS_N + pos] = fixed;
            };
            if (err) {
                if (geo)
                    fix(gpos, ge);
                else
                    rs_correct_general<T2>(S, gf, fix);
            }
#pragma unroll
            for (int q = 0; q < NR; ++q)
                R[q] = tw[q];
        } else if (geo && ge != 0) {
            // single-error lanes only: R stays as read; the byte is patched after emission
            const uint8_t fixed = (uint8_t)(tile[ib + gpos] ^ ge);
            if (write_back && PPFS_DBG_OK(raw_g + blk * RS_N + gpos, 1, raw_g, raw_bytes))
                raw_g[blk * RS_N + gpos] = fixed;
            fpos = gpos;
            fval = fixed;
        }
    }
    status_lds[l] = err ? 1 : 0;
    if (!want_data)
        return;
    wave_fence();
    emit_payload_direct<T2, NR>(tile, l, a, R);
    // the row's own bytes only: ordered after this lane's emission stores
    if (fpos >= (uint32_t)T2 && fpos != 0xFFFFFFFFu)
        tile[K * l + fpos - T2] = (uint8_t)fval;
}

// ------------------------------------------------------------------------------------
// Kernels (persistent: each wave walks wave-tiles wt = global_wave, += total waves).
// Pipelining per wave: the out-tile is read into VGPRs, then the NEXT tile's LDS-DMA is issued
// into the (now free) buffer, then the global stores -- so the wait for the next tile's data
// (a counted vmcnt) does not wait for this tile's stores.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_dma_issue(uint8_t* buf, const uint8_t* __restrict__ src, uint32_t npiece,
    uint32_t lane)
{
    const uint32_t ngroup = (npiece + 63) >> 6;
    for (uint32_t g = 0; g < ngroup; ++g) {
        const uint32_t piece = g * 64 + lane;
        if (piece < npiece)
            __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)piece * 16),
                (__attribute__((address_space(3))) void*)(buf + g * 1024), 16, 0, 0);
    }
}

// s_waitcnt vmcnt(n) (gfx9 simm16: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt[5:4] at [15:14]).
// The builtin form is visible to the compiler's waitcnt pass, unlike inline asm.
#define PPFS_VMCNT(n) (((n)&15) | (((n) >> 4) << 14) | 0x70 | 0xF00)
__device__ __forceinline__ void wait_vmcnt(int n)
{
    switch (n) {
    case 0: __builtin_amdgcn_s_waitcnt(PPFS_VMCNT(0)); break;
    case 1: __builtin_amdgcn_s_waitcnt(PPFS_VMCNT(1)); break;
    case 16: __builtin_amdgcn_s_waitcnt(PPFS_VMCNT(16)); break;
    case 17: __builtin_amdgcn_s_waitcnt(PPFS_VMCNT(17)); break;
    default: __builtin_amdgcn_s_waitcnt(PPFS_VMCNT(0)); break;
    }
}

// stores of one full out-tile region from VGPRs: returns the number of store instructions
template <int NPIECE, int NT = 0>
__device__ __forceinline__ void store_tile(uint8_t* __restrict__ dst, const uint4 (&o)[(NPIECE + 63) / 64], uint32_t lane)
{
#pragma unroll
    for (int k = 0; k < (NPIECE + 63) / 64; ++k) {
        const uint32_t p = lane + 64 * k;
        if (k < NPIECE / 64 || p < NPIECE) {
            uint4* q = (uint4*)(dst + (size_t)p * 16);
            if constexpr (NT) {
                const u32x4 v = { o[k].x, o[k].y, o[k].z, o[k].w };
                __builtin_nontemporal_store(v, (u32x4*)q);
            } else {
                *q = o[k];
            }
        }
    }
}

template <int NPIECE>
__device__ __forceinline__ void read_tile(uint4 (&o)[(NPIECE + 63) / 64], const uint8_t* buf, uint32_t lane)
{
#pragma unroll
    for (int k = 0; k < (NPIECE + 63) / 64; ++k) {
        const uint32_t p = lane + 64 * k;
        o[k] = (k < NPIECE / 64 || p < NPIECE) ? *(const uint4*)(buf + p * 16) : make_uint4(0, 0, 0, 0);
    }
}

// next-tile prefetch into VGPRs (register staging): 16-byte coalesced loads
template <int NPIECE, int NT = 0>
__device__ __forceinline__ void load_regs(uint4 (&L)[(NPIECE + 63) / 64], const uint8_t* __restrict__ src, uint32_t lane)
{
#pragma unroll
    for (int k = 0; k < (NPIECE + 63) / 64; ++k) {
        const uint32_t p = lane + 64 * k;
        const uint4* q = (const uint4*)(src + (size_t)p * 16);
        if (k < NPIECE / 64 || p < NPIECE) {
            if constexpr (NT) {
                const u32x4 v = __builtin_nontemporal_load((const u32x4*)q);
                L[k] = make_uint4(v.x, v.y, v.z, v.w);
            } else {
                L[k] = *q;
            }
        } else {
            L[k] = make_uint4(0, 0, 0, 0);
        }
    }
}

// conditional prefetch that defines L on both paths: a conditionally-kept L would stay live
// (and be spilled) through the whole loop body
template <int NPIECE, int NT = 0>
__device__ __forceinline__ void load_regs_if(bool cond, uint4 (&L)[(NPIECE + 63) / 64], const uint8_t* __restrict__ src,
    uint32_t lane, const uint8_t* __restrict__ dummy = nullptr)
{
    if (dummy) {
        // branch-free: without a next tile the loads re-read a 1 KiB L2-resident region, so the
        // loads are unconditional and the waitcnt pass can count them (a branch around them
        // makes it fall back to vmcnt(0), which also waits for this tile's stores)
        const uint8_t* base = cond ? src : dummy;
        const uint32_t wrap = cond ? 0xFFFFFFFFu : 1023u;
#pragma unroll
        for (int k = 0; k < (NPIECE + 63) / 64; ++k) {
            const uint32_t p = lane + 64 * k;
            const uint32_t off = ((k < NPIECE / 64 || p < NPIECE) ? p * 16u : 0u) & wrap;
            const uint4* q = (const uint4*)(base + off);
            if constexpr (NT) {
                const u32x4 v = __builtin_nontemporal_load((const u32x4*)q);
                L[k] = make_uint4(v.x, v.y, v.z, v.w);
            } else {
                L[k] = *q;
            }
        }
        return;
    }
    if (cond) {
        load_regs<NPIECE, NT>(L, src, lane);
    } else {
#pragma unroll
        for (int k = 0; k < (NPIECE + 63) / 64; ++k)
            L[k] = make_uint4(0, 0, 0, 0);
    }
}

template <int NPIECE>
__device__ __forceinline__ void write_regs(uint8_t* buf, const uint4 (&L)[(NPIECE + 63) / 64], uint32_t lane)
{
#pragma unroll
    for (int k = 0; k < (NPIECE + 63) / 64; ++k) {
        const uint32_t p = lane + 64 * k;
        if (k < NPIECE / 64 || p < NPIECE)
            *(uint4*)(buf + p * 16) = L[k];
    }
}

// Defaults = fastest measured variant: one chain, next-tile prefetch during compute,
// non-temporal (streaming) global loads and stores.
template <int T2, int NS = 0, int PF = 1, int NT = 1, int MEMONLY = 0>
__global__ __launch_bounds__(256, 2) void rs255_encode_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables)
{
    using Cf = RsCfg<T2, NS>;
    constexpr int K = Cf::K;
    constexpr int IN_PIECES = RS_WT * K / 16;     // full tile: 64*K bytes (multiple of 16)
    constexpr int OUT_PIECES = RS_WT * RS_N / 16; // 1020
    static_assert((RS_WT * K) % 16 == 0, "full input tiles are whole 16-byte pieces");
    __shared__ __attribute__((aligned(16))) uint8_t lds[Cf::LDS_BYTES];
    load_tables(lds, tables, Cf::TBL_BYTES);
    __syncthreads();
    const uint32_t lane = lane_id(), wave = wave_id();
    uint8_t* tile = lds + Cf::OFF_WAVES + wave * Cf::WAVE_BYTES;
    const uint64_t ntiles = (nblocks + RS_WT - 1) / RS_WT;
    const uint64_t nfull = nblocks / RS_WT;
    const uint64_t stride = (uint64_t)gridDim.x * RS_WAVES;
    uint64_t wt = (uint64_t)blockIdx.x * RS_WAVES + wave;
    // Full tiles: a straight-line body (fixed numbers of loads and stores), so the compiler's
    // waitcnt pass counts the in-flight prefetch instead of draining this tile's stores.
    // PF = 2: one-shot (grid covers every tile, no prefetch: other waves hide the latency)
    uint4 L[(IN_PIECES + 63) / 64];
    if (PF != 2)
        load_regs_if<IN_PIECES, NT>(wt < nfull && PPFS_DBG_OK(data + wt * RS_WT * K, RS_WT * K, data, nblocks * K), L,
            data + wt * RS_WT * K, lane, tables);
    for (; wt < nfull; wt += stride) {
        const uint64_t b0 = wt * RS_WT;
        if (PF == 2)
            load_regs<IN_PIECES, NT>(L, data + b0 * K, lane);
        write_regs<IN_PIECES>(tile, L, lane); // loads issued one tile earlier
        wave_fence();
        const uint64_t nx = wt + stride;
        if constexpr (!MEMONLY) {
            rs_encode_lane<T2, NS>(tile, lds, lane, [&]() {
                // block is in registers: prefetch the next tile now, its latency hides under compute
                if (PF == 1)
                    load_regs_if<IN_PIECES, NT>(nx < nfull && PPFS_DBG_OK(data + nx * RS_WT * K, RS_WT * K, data, nblocks * K), L,
                        data + nx * RS_WT * K, lane, tables);
            });
        } else {
            if (PF == 1)
                load_regs_if<IN_PIECES, NT>(nx < nfull && PPFS_DBG_OK(data + nx * RS_WT * K, RS_WT * K, data, nblocks * K), L,
                        data + nx * RS_WT * K, lane, tables);
        }
        wave_fence();
        uint4 o[(OUT_PIECES + 63) / 64];
        read_tile<OUT_PIECES>(o, tile, lane);
        if (PF == 0)
            load_regs_if<IN_PIECES, NT>(nx < nfull && PPFS_DBG_OK(data + nx * RS_WT * K, RS_WT * K, data, nblocks * K), L,
                        data + nx * RS_WT * K, lane, tables);
        if (PPFS_DBG_OK(raw + b0 * RS_N, RS_WT * RS_N, raw, nblocks * RS_N))
            store_tile<OUT_PIECES, NT>(raw + b0 * RS_N, o, lane);
        wave_fence();
    }
    // the one partial tile (nblocks % 64 blocks), by the wave whose walk reaches it
    if (wt == nfull && nfull < ntiles) {
        const uint64_t b0 = wt * RS_WT;
        const uint32_t nb = (uint32_t)(nblocks - b0);
        if (!PPFS_DBG_OK(data + b0 * K, nb * K, data, nblocks * K) || !PPFS_DBG_OK(raw + b0 * RS_N, nb * RS_N, raw, nblocks * RS_N))
            return;
        wave_stage_in(tile, data + b0 * K, nb * K, lane);
        wave_fence();
        rs_encode_lane<T2, NS>(tile, lds, lane, []() {});
        wave_fence();
        wave_stage_out(raw + b0 * RS_N, tile, nb * RS_N, lane);
    }
}

// Input staging of the decode kernel (STAGE):
//   0  next tile -> VGPRs after this tile's out-tile is read, before its stores
//   1  next tile -> VGPRs after this tile's stores
//   2  next tile -> VGPRs during the syndrome pass (prefetch, as encode)
//   3  next tile -> LDS by DMA after this tile's stores
//   4  one-shot: no prefetch (launch one wave per tile; other waves hide the load latency)
// NT: bit 0 = non-temporal codeword loads, bit 1 = non-temporal payload stores.  Codeword
// loads stay temporal by default: the write-back RMWs bytes of lines just read.
template <int T2, int NS = 0, int STAGE = 1, int NT = 0>
__global__ __launch_bounds__(256, 2) void rs255_decode_kernel(uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks, const uint8_t* __restrict__ tables, int write_back)
{
    using Cf = RsCfg<T2, NS>;
    constexpr int K = Cf::K;
    constexpr int IN_PIECES = RS_WT * RS_N / 16; // 1020
    constexpr int OUT_PIECES = RS_WT * K / 16;
    constexpr bool REGS = STAGE != 3;
    static_assert((RS_WT * K) % 16 == 0, "full output tiles are whole 16-byte pieces");
    __shared__ __attribute__((aligned(16))) uint8_t lds[Cf::LDS_BYTES];
    load_tables(lds, tables, Cf::TBL_BYTES + GF_BYTES);
    __syncthreads();
    const uint32_t lane = lane_id(), wave = wave_id();
    uint8_t* tile = lds + Cf::OFF_WAVES + wave * Cf::WAVE_BYTES;
    uint8_t* st_lds = tile + Cf::WAVE_BUF;
    const bool wb = write_back != 0, want = data != nullptr;
    const uint64_t ntiles = (nblocks + RS_WT - 1) / RS_WT;
    const uint64_t nfull = nblocks / RS_WT;
    const uint64_t stride = (uint64_t)gridDim.x * RS_WAVES;
    uint64_t wt = (uint64_t)blockIdx.x * RS_WAVES + wave;
    uint4 L[REGS ? (IN_PIECES + 63) / 64 : 1];
    if constexpr (STAGE == 4) {
        // one-shot: loaded at the loop top
    } else if constexpr (REGS) {
        load_regs_if<IN_PIECES, NT & 1>(wt < nfull && PPFS_DBG_OK(raw + wt * RS_WT * RS_N, RS_WT * RS_N, raw, nblocks * RS_N),
            L, raw + wt * RS_WT * RS_N, lane, tables);
    } else if (wt < nfull) {
        wave_dma_issue(tile, raw + wt * RS_WT * RS_N, IN_PIECES, lane);
    }
    for (; wt < nfull; wt += stride) {
        const uint64_t b0 = wt * RS_WT;
        if constexpr (STAGE == 4)
            load_regs<IN_PIECES, NT & 1>(L, raw + b0 * RS_N, lane);
        if constexpr (REGS)
            write_regs<IN_PIECES>(tile, L, lane);
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wave_fence();
        const uint64_t nx = wt + stride;
        const bool nfullx = nx < nfull;
        rs_decode_lane<T2, NS>(tile, lds, lane, true, raw, b0 + lane, wb, want, st_lds,
            [&]() {
            if constexpr (STAGE == 2)
                load_regs_if<IN_PIECES, NT & 1>(nfullx && PPFS_DBG_OK(raw + nx * RS_WT * RS_N, RS_WT * RS_N, raw, nblocks * RS_N),
                L, raw + nx * RS_WT * RS_N, lane, tables);
            },
            nblocks * RS_N);
        wave_fence();
        uint4 o[(OUT_PIECES + 63) / 64];
        if (want)
            read_tile<OUT_PIECES>(o, tile, lane);
        const uint4 sv = (lane < 4) ? *(const uint4*)(st_lds + 16 * lane) : make_uint4(0, 0, 0, 0);
        if constexpr (STAGE == 0)
            load_regs_if<IN_PIECES, NT & 1>(nfullx && PPFS_DBG_OK(raw + nx * RS_WT * RS_N, RS_WT * RS_N, raw, nblocks * RS_N),
                L, raw + nx * RS_WT * RS_N, lane, tables);
        if (want && PPFS_DBG_OK(data + b0 * K, RS_WT * K, data, nblocks * K))
            store_tile<OUT_PIECES, (NT >> 1) & 1>(data + b0 * K, o, lane);
        if (status && lane < 4 && PPFS_DBG_OK(status + b0 + 16 * lane, 16, status, nblocks))
            *(uint4*)(status + b0 + 16 * lane) = sv;
        if constexpr (STAGE == 1)
            load_regs_if<IN_PIECES, NT & 1>(nfullx && PPFS_DBG_OK(raw + nx * RS_WT * RS_N, RS_WT * RS_N, raw, nblocks * RS_N),
                L, raw + nx * RS_WT * RS_N, lane, tables);
        wave_fence();
        if constexpr (STAGE == 3)
            if (nfullx)
                wave_dma_issue(tile, raw + nx * RS_WT * RS_N, IN_PIECES, lane);
    }
    if (wt == nfull && nfull < ntiles) {
        const uint64_t b0 = wt * RS_WT;
        const uint32_t nb = (uint32_t)(nblocks - b0);
        if (!PPFS_DBG_OK(raw + b0 * RS_N, nb * RS_N, raw, nblocks * RS_N) || (want && !PPFS_DBG_OK(data + b0 * K, nb * K, data, nblocks * K))
            || (status && !PPFS_DBG_OK(status + b0, nb, status, nblocks)))
            return;
        wave_stage_in(tile, raw + b0 * RS_N, nb * RS_N, lane);
        wave_fence();
        rs_decode_lane<T2, NS>(tile, lds, lane, lane < nb, raw, b0 + lane, wb, want, st_lds, []() {}, nblocks * RS_N);
        wave_fence();
        if (want)
            wave_stage_out(data + b0 * K, tile, nb * K, lane);
        if (status)
            wave_stage_out(status + b0, st_lds, nb, lane);
    }
}

// Resident small-batch server for 8 < 2t <= 16 (server_box.hpp protocol): one wave runs a request
// of <= 64 blocks as the partial-tile path of the kernels above (lane = block).  A write is the
// old blocks' decode for their status, then the encode.
template <int T2, int NS = 0>
__global__ __launch_bounds__(64, 1) void rs255_server_kernel(SrvBox* box, uint8_t* zc, uint64_t zc_bytes,
    const uint8_t* __restrict__ tables, uint32_t gen, uint32_t idle_us)
{
    using Cf = RsCfg<T2, NS>;
    constexpr int K = Cf::K;
    __shared__ __attribute__((aligned(16))) uint8_t lds[Cf::OFF_WAVES + Cf::WAVE_BYTES];
    __shared__ uint32_t s_cmd[2];
    load_tables(lds, tables, Cf::TBL_BYTES + GF_BYTES);
    __syncthreads();
    const uint32_t lane = lane_id();
    uint8_t* tile = lds + Cf::OFF_WAVES;
    uint8_t* st_lds = tile + Cf::WAVE_BUF;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t last = t0;
    uint32_t seen = srv::ld_sys(&box->done), served = 0;
    if (lane == 0)
        srv::st_sys(&box->alive, gen);
    for (;;) {
        const uint32_t r = srv::next_request(box, seen, last, t0, idle_us, s_cmd);
        if (r == 0)
            break;
        const SrvCmd cmd = srv_cmd_unpack(r);
        const uint32_t nb = cmd.nb;
        const SrvLayout lay = srv_layout(nb, (uint32_t)K, (uint32_t)RS_N);
        uint8_t* data = zc + lay.data;
        uint8_t* raw = zc + lay.raw;
        uint8_t* status = zc + lay.status;
        const bool ok = nb >= 1 && nb <= (uint32_t)RS_WT && PPFS_DBG_OK(data, nb * K, zc, zc_bytes)
            && PPFS_DBG_OK(raw, nb * RS_N, zc, zc_bytes) && PPFS_DBG_OK(status, nb, zc, zc_bytes);
        if (ok && (cmd.op == SRV_DECODE || cmd.op == SRV_WRITE)) {
            const bool dec = cmd.op == SRV_DECODE, want = dec && cmd.want_data;
            wave_stage_in(tile, raw, nb * RS_N, lane);
            wave_fence();
            rs_decode_lane<T2, NS>(tile, lds, lane, lane < nb, raw, lane, dec && cmd.write_back, want, st_lds, []() {},
                nb * RS_N);
            wave_fence();
            if (want)
                wave_stage_out(data, tile, nb * K, lane);
            wave_stage_out(status, st_lds, nb, lane);
            wave_fence();
        }
        if (ok && (cmd.op == SRV_ENCODE || cmd.op == SRV_WRITE)) {
            wave_stage_in(tile, data, nb * K, lane);
            wave_fence();
            rs_encode_lane<T2, NS>(tile, lds, lane, []() {});
            wave_fence();
            wave_stage_out(raw, tile, nb * RS_N, lane);
            wave_fence();
        }
        seen = r;
        srv::finish_request(box, r, ++served);
    }
    if (lane == 0)
        srv::st_sys(&box->alive, gen | SRV_EXITED);
}

} // namespace ppfs
