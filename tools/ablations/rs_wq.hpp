#pragma once
// rs_wq.hpp -- barrier-free t <= 4 RS encode for gfx950 ("wave quarters", round 3).  ABLATION, not
// shipped: correct (94 RS GPU tests, bounds-checked build clean) and 5-8 % faster cache-hot, but
// 10-12 % slower from HBM and in the bench step than the ticket encode (static walk), 25 % slower
// with per-wave tickets (65,536 atomics per launch); profiles/r3k_*, r3m_slx_wq_bench_ab.txt.
// Built by tools/build_alt.sh <name> -DPPFS_WG_WQ=1|2.
//
// Reference semantics: lib/blockdevice/src/rs_block_device.cpp _encodeBlock :95-117 (see rs_wg.hpp).
//
// rs_wg_tk.hpp's encode spends ~15 % of every 64-block tile in two workgroup barriers (the phase
// trace, profiles/r3h_phase_trace.jsonl: barrier B behind the slowest segment wave, barrier A behind
// the tile DMA and the ticket).  Here every wave works alone on 16-block tiles:
//   - lane = 4 j + s owns segment s (bytes [64 s, 64 s + 64)) of block j: the same 8-step slicing
//     chain per lane as rs_wg's segment waves, and the SLX last step (rs_layout.hpp) folds x^(64 s)
//     in, so the four segment remainders of a block just XOR together -- two DPP quad_perm XORs,
//     no LDS atomic, no barrier;
//   - the wave DMAs its own tiles (16 x K bytes, 4 LDS-DMA instructions) into its own ring of NBUF
//     buffers and emits its own 16 codewords (255 pieces of 16 B, rs_wg.hpp enc_piece), so the only
//     ordering is the wave's own vmcnt.
// Wave tiles are walked statically: wave g of the grid takes tiles g, g + W, g + 2 W, ... (W = waves
// in the grid), so the tiles in flight chip-wide advance as one window of the payload.
#include "rs_wg_tk.hpp"

namespace ppfs {
namespace wq {

using wg::dma16;
using wg::enc_piece;
using wg::lds_addr;
using wg::ld8;
using wg::PAD;
using wg::sel78;
using wg::st_bytes;
using wg::st_nt;

constexpr int QB = 16;           // blocks per wave tile
constexpr uint32_t XSTRIDE = 2176; // LDS stride of the last-step tables: SL at 0, SLX_s at 2176 s
                                   // (2176 = 2048 + 128: segments 0/2 and 1/3 use opposite 32-bank halves)
constexpr int TBL_BYTES = 3 * XSTRIDE + 2048;
constexpr int PARW = 144;        // per wave: 16 parity slots of 8 B + the over-read slot 16

template <int T2, int NBUF> struct WqLds {
    static constexpr int K = 255 - T2;
    static constexpr int OFF_PAR = TBL_BYTES;
    static constexpr int OFF_BUF = OFF_PAR + 4 * PARW;
    static constexpr int BUFQ = (PAD + QB * K + 32 + 15) / 16 * 16; // one wave tile (+ row over-read slack)
    static constexpr int BYTES = OFF_BUF + 4 * NBUF * BUFQ;
    static_assert(OFF_BUF % 16 == 0 && BUFQ % 16 == 0, "aligned tile buffers");
};

// The lane's segment remainder, already multiplied by x^(64 s): lane (j, s) of the wave, row = LDS
// byte of block j's payload row.  Every lane runs 8 steps of 16 nibble lookups; segment 3's bytes
// past the row (K - 192 of its 64 are real) are masked to zero (their lookups hit entry 0 = 0).
template <int T2>
__device__ __forceinline__ void wq_remainder(uint32_t (&s)[2], const uint8_t* lds, uint32_t row, uint32_t seg)
{
    constexpr int K = 255 - T2;
    constexpr int L3 = K - 192; // real bytes of segment 3 (55..61)
    const uint32_t a0 = row + 64u * seg;
    const uint32_t sh = (a0 & 3u) * 8u;
    const uint32_t* w = (const uint32_t*)(lds + (a0 & ~3u));
    uint32_t R[17];
#pragma unroll
    for (int q = 0; q < 17; ++q)
        R[q] = w[q];
    const bool s3 = seg == 3u;
    const uint32_t tlast = seg * XSTRIDE; // the last step's tables (segment 0: SL itself)
    s[0] = 0;
    s[1] = 0;
#pragma unroll
    for (int c = 7; c >= 0; --c) {
        uint32_t lo = __builtin_amdgcn_alignbit(R[2 * c + 1], R[2 * c], sh);
        uint32_t hi = __builtin_amdgcn_alignbit(R[2 * c + 2], R[2 * c + 1], sh);
        const int nb = L3 - 8 * c; // real bytes of segment 3 in this chunk (compile-time per c)
        if (nb < 8) {
            const uint32_t ml = nb >= 4 ? ~0u : (nb <= 0 ? 0u : (1u << (8 * nb)) - 1u);
            const uint32_t mh = nb >= 8 ? ~0u : (nb <= 4 ? 0u : (1u << (8 * (nb - 4))) - 1u);
            lo = s3 ? (lo & ml) : lo;
            hi = s3 ? (hi & mh) : hi;
        }
        if (c != 7) {
            lo ^= s[0];
            hi ^= s[1];
        }
        const uint32_t ll = lo << 3, lh = lo >> 1, hl = hi << 3, hh = hi >> 1;
        uint2 e[16];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t xl = i < 4 ? ll : hl, xh = i < 4 ? lh : hh;
            if (c == 0) {
                e[2 * i] = ld8(lds + tlast + (2 * i) * 128 + sel78(xl, i));
                e[2 * i + 1] = ld8(lds + tlast + (2 * i + 1) * 128 + sel78(xh, i));
            } else {
                e[2 * i] = ld8(lds + (2 * i) * 128 + sel78(xl, i));
                e[2 * i + 1] = ld8(lds + (2 * i + 1) * 128 + sel78(xh, i));
            }
        }
        s[0] = 0;
        s[1] = 0;
        wg::xor_entries<16>(s, e);
    }
}

// Ticket atomic issued from inline asm (lane 0; returns the old value): the compiler does not track
// it, so it never inserts its own (draining) wait for the result.  The caller guarantees completion
// with its counted vmcnt before the value is read, then ties the register (tk_ready).
__device__ __forceinline__ void tk_take(uint32_t& tk, uint32_t* ctr)
{
    asm volatile("global_atomic_inc %0, %1, %2, off sc0" : "=v"(tk) : "v"(ctr), "v"(0xFFFFFFFFu) : "memory");
}
__device__ __forceinline__ uint32_t tk_ready(uint32_t& tk)
{
    asm volatile("" : "+v"(tk)); // ordered after the caller's volatile wait: no read of tk moves above it
    return (uint32_t)__builtin_amdgcn_readfirstlane(tk);
}

// XOR over the 4 lanes of a quad (the four segments of one block): every lane gets the total
__device__ __forceinline__ uint32_t quad_xor(uint32_t v)
{
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false); // quad_perm [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false); // quad_perm [2,3,0,1]
    return v;
}

// LDS-DMA of wave tile u's payload (16 K bytes = IN_PIECES pieces) into the buffer at LDS byte dst
template <int IN_PIECES>
__device__ __forceinline__ void dma_qtile(uint32_t dst, const uint8_t* __restrict__ src, uint32_t lane,
    [[maybe_unused]] const uint8_t* gbase, [[maybe_unused]] uint64_t extent)
{
    constexpr int KI = (IN_PIECES + 63) / 64;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
        const uint32_t p = lane + 64u * (uint32_t)k;
        if (((k + 1) * 64 <= IN_PIECES || p < (uint32_t)IN_PIECES) && PPFS_DBG_OK(src + 16u * p, 16, gbase, extent))
            dma16(src + 16u * p, __builtin_amdgcn_readfirstlane(dst + 1024u * (uint32_t)k));
    }
}

// Vector-memory bookkeeping of one wave's ring (the waits must count the operations issued after
// a tile's DMA: a wave's vector-memory operations complete in issue order).  after[r] = operations
// issued since the DMA into ring slot r (while it is outstanding).
template <int NBUF> struct VmRing {
    uint32_t after[NBUF];
    __device__ __forceinline__ void init()
    {
#pragma unroll
        for (int r = 0; r < NBUF; ++r)
            after[r] = 0;
    }
    __device__ __forceinline__ void issued(uint32_t n) // n more operations (any kind) went out
    {
#pragma unroll
        for (int r = 0; r < NBUF; ++r)
            after[r] += n;
    }
    __device__ __forceinline__ void dma(uint32_t slot, uint32_t n) // the DMA into `slot` (n instructions)
    {
        issued(n);
#pragma unroll
        for (int r = 0; r < NBUF; ++r)
            if ((uint32_t)r == slot)
                after[r] = 0;
    }
    __device__ __forceinline__ uint32_t newer(uint32_t slot) const
    {
        uint32_t v = 0;
#pragma unroll
        for (int r = 0; r < NBUF; ++r)
            v = (uint32_t)r == slot ? after[r] : v;
        return v;
    }
};

// TK: wave tiles come from ticket counters (rs_wg_tk.hpp's scheme at wave granularity): 32
// counters, one per (XCD, wave slot), 64 B apart in the stream's set; local ticket k of counter
// (x, w) is wave tile 4 (k nx + x) + w, so the four quarters of a 64-block range go to the four
// wave slots of one XCD at about the same time and the tiles in flight stay one window of the
// payload.  Iterations 0 and 1 take static tickets (the workgroup's rank among its XCD's gx
// workgroups, and that + gx); the counters hand out the rest from 2 gx on.  The ticket of
// iteration m is taken (lane 0, an inline-asm atomic the compiler does not track, tk_take) at the
// top of iteration m - 4, right before the DMA of iteration m - 2's tile, and read at the top of
// iteration m - 2, after the counted wait for that tile: in-order completion means the ticket has
// arrived, and no wait drains the ring.  A launch zeroes ctr_clear, the set the previous launch of the same
// kind on this stream counted on (api.cpp ctr_for alternates them).
template <int T2, int WPC = 2, int NBUF = 3, int NTST = 1, bool TK = false>
__global__ __launch_bounds__(256, WPC) void rs_wq_encode_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables, uint32_t* __restrict__ ctr = nullptr,
    uint32_t* __restrict__ ctr_clear = nullptr)
{
    static_assert(NBUF >= 2 && NBUF <= 4, "ring of 2 to 4 wave-tile buffers");
    static_assert(!TK || NBUF == 3, "the ticket lead is sized for a ring of 3");
    using L = RsWgLayout<T2>;
    using D = WqLds<T2, NBUF>;
    constexpr int K = L::K;
    constexpr int IN_PIECES = QB * K / 16;   // 16 | QB K
    constexpr int OUT_PIECES = QB * 255 / 16; // 255
    constexpr int KI = (IN_PIECES + 63) / 64; // DMA instructions per wave tile
    constexpr int KO = (OUT_PIECES + 63) / 64; // store instructions per wave tile
    static_assert(KI == 4 && KO == 4, "vmcnt accounting assumes 4 + 4 per wave tile");
    constexpr int LDS_ALLOC = wg::lds_alloc<D::BYTES + 64, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t j = lane >> 2, seg = lane & 3u;
    const uint64_t nfull = nblocks / QB, ntiles = (nblocks + QB - 1) / QB;
    const uint64_t W = (uint64_t)gridDim.x * 4u;
    uint64_t u = (uint64_t)blockIdx.x * 4u + wave;
    // ticket geometry (TK): counter (xc, wave), this workgroup's rank among the gx of its counter
    const uint32_t nx = gridDim.x < 8u ? gridDim.x : 8u, xc = blockIdx.x % nx;
    const uint32_t gx = (gridDim.x - xc + nx - 1u) / nx, rank = blockIdx.x / nx;
    uint32_t* const my_ctr = TK ? ctr + 16u * (4u * xc + wave) : nullptr;
    auto tile_of = [&](uint64_t k) -> uint64_t { return 4u * (k * nx + xc) + wave; };
    uint64_t u1 = u + W;  // the tile of iteration 1
    uint32_t tka = 0, tkb = 0; // TK: tickets of the iterations two and three ahead (lane 0)
    if constexpr (TK) {
        u = tile_of(rank);
        u1 = tile_of(rank + gx);
        if (blockIdx.x == 0 && wave == 0 && lane < 32u)
            __hip_atomic_store(ctr_clear + 16u * lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 0)
            tk_take(tka, my_ctr); // iteration 2
    }
    const uint32_t par = D::OFF_PAR + wave * PARW;
    const uint32_t buf0 = D::OFF_BUF + wave * (NBUF * D::BUFQ);
    const uint32_t lbase = __builtin_amdgcn_readfirstlane(lds_addr(lds) + buf0 + PAD);
    const uint64_t ext = nblocks * K;
    VmRing<NBUF> vm;
    vm.init();

    // prologue: tile u into slot 0, the tables (SL at 0, SLX_s at 2176 s), then tiles u + W .. into
    // slots 1 .. NBUF - 2
    if (u < nfull)
        dma_qtile<IN_PIECES>(lbase, data + u * (QB * K), lane, data, ext);
    if constexpr (TK)
        if (lane == 0)
            tk_take(tkb, my_ctr); // iteration 3
    for (uint32_t p = tid; p < 2048u / 16u; p += 256u)
        *(uint4*)(lds + 16u * p) = *(const uint4*)(tables + L::OFF_SL + 16u * p);
    for (uint32_t p = tid; p < 3u * 2048u / 16u; p += 256u) {
        const uint32_t m = p >> 7, q = p & 127u; // SLX table m + 1, piece q
        *(uint4*)(lds + XSTRIDE * (m + 1u) + 16u * q) = *(const uint4*)(tables + L::OFF_SLX + 2048u * m + 16u * q);
    }
    // the table loads' wait covered tile u (issued before them: a wave's loads complete in order)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (TK) {
        if (u1 < nfull) {
            dma_qtile<IN_PIECES>(lbase + D::BUFQ, data + u1 * (QB * K), lane, data, ext);
            vm.dma(1u, KI);
        }
    } else {
#pragma unroll
        for (int r = 1; r <= NBUF - 2; ++r)
            if (u + (uint64_t)r * W < nfull) {
                dma_qtile<IN_PIECES>(lbase + (uint32_t)r * D::BUFQ, data + (u + (uint64_t)r * W) * (QB * K), lane, data, ext);
                vm.dma((uint32_t)r, KI);
            }
    }
    wg::barrier_lds(); // tables visible to every wave; the only workgroup barrier of the kernel

    uint32_t cur = 0;
    // one iteration; tk = the register holding this iteration's ticket two ahead, refilled with the
    // ticket four ahead (the loop runs two iterations per trip so that the two ticket registers keep
    // fixed roles: a register copy would make the compiler wait for the atomic one iteration early,
    // and that wait would also drain the newest tile DMA)
    auto iteration = [&](uint32_t& tk) {
        const uint32_t buf = buf0 + cur * D::BUFQ;
        uint64_t ua; // the tile NBUF - 1 iterations ahead
        if constexpr (TK) {
            // taken two iterations ago right before the DMA of this iteration's tile, so the wait
            // for that tile (end of the last iteration, or the prologue's) covered it
            ua = tile_of((uint64_t)tk_ready(tk) + 2u * gx);
            if (lane == 0)
                tk_take(tk, my_ctr); // the iteration four ahead
            vm.issued(1);
        } else {
            (void)tk;
            ua = u + (uint64_t)(NBUF - 1) * W;
        }
        const uint32_t sa = wg::ring_add(cur, NBUF - 1, NBUF);
        if (ua < nfull) {
            dma_qtile<IN_PIECES>(lbase + sa * D::BUFQ, data + ua * (QB * K), lane, data, ext);
            vm.dma(sa, KI);
        }
        uint32_t s[2];
        wq_remainder<T2>(s, lds, buf + PAD + (uint32_t)K * j, seg);
        s[0] = quad_xor(s[0]);
        s[1] = quad_xor(s[1]);
        if (seg == 0u)
            *(uint64_t*)(lds + par + 8u * j) = ((uint64_t)s[1] << 32) | s[0];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the slots are written (one wave: in order)
        uint8_t* dst = raw + u * (QB * 255);
#pragma unroll
        for (int k = 0; k < KO; ++k) {
            const uint32_t p = lane + 64u * (uint32_t)k;
            const uint4 o = enc_piece<T2>(lds, buf, par, p);
            if (((k + 1) * 64 <= OUT_PIECES || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, raw, nblocks * 255u))
                st_nt<NTST>(dst + 16u * p, o);
        }
        vm.issued(KO);
        cur = wg::ring_add(cur, 1, NBUF);
        const uint64_t un = TK ? u1 : u + W; // the next iteration's tile
        if (un < nfull)
            wg::vm_wait_exact(vm.newer(cur)); // the next tile landed
        u = un;
        if constexpr (TK)
            u1 = ua;
    };
    while (u < nfull) {
        iteration(tka);
        if (u >= nfull)
            break;
        iteration(tkb);
    }
    // tickets still in flight land in tka / tkb: drain them before those registers can be reused
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(tka), "+v"(tkb)::"memory");
    if (u == nfull && nfull < ntiles) { // the partial wave tile (nblocks % 16 blocks), staged bytewise
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t buf = buf0 + cur * D::BUFQ;
        const uint32_t nb = (uint32_t)(nblocks - u * QB);
        const uint8_t* src = data + u * (QB * K);
        if (!PPFS_DBG_OK(src, nb * (uint32_t)K, data, ext))
            return;
        for (uint32_t i = lane; i < nb * (uint32_t)K; i += 64u)
            lds[buf + PAD + i] = src[i];
        wave_fence();
        uint32_t s[2];
        wq_remainder<T2>(s, lds, buf + PAD + (uint32_t)K * j, seg);
        s[0] = quad_xor(s[0]);
        s[1] = quad_xor(s[1]);
        if (seg == 0u)
            *(uint64_t*)(lds + par + 8u * j) = ((uint64_t)s[1] << 32) | s[0];
        wave_fence();
        uint8_t* dst = raw + u * (QB * 255);
        const uint32_t nout = nb * 255u;
        for (uint32_t p = lane; 16u * p < nout; p += 64u) {
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

} // namespace wq
} // namespace ppfs
