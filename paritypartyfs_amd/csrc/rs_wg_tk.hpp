#pragma once
// rs_wg_tk.hpp -- the t <= 4 RS encode (rs_wg.hpp's ring of 3 LDS tile buffers, 2 workgroups per
// CU) and decode (double buffer, 3 per CU) with their tiles handed out dynamically: per-XCD ticket
// counters keep the tiles in flight one window of HBM and let fast workgroups take more tiles (the
// persistent static walk's copy skeleton measured 96 vs 91.6 us against dynamic tiles, DESIGN.md
// 4.1).  The counters live in a per-context buffer, one pair of sets per stream that runs them
// through the context (api.cpp ctr_for): launches on one stream are ordered.
//
// Launch bookkeeping without a tail (round 3): a launch counts on set `ctr` and zeroes `ctr_clear`,
// the set the previous launch of the same kind on the stream counted on (complete: same stream);
// the host alternates the two.  So no workgroup has to find out that it is the last one to reset
// the counters after the grid's final tiles (one more atomic round trip at the end of every launch).
//
// Startup (round 3): a workgroup's first tiles are static (its rank among the workgroups of its
// XCD, plus multiples of their number: encode 3, decode 1), so the DMA waves issue the first ones
// right away, before any table byte or ticket arrives; wave 0 brings the tables into LDS by LDS-DMA
// meanwhile and takes the first dynamic ticket.  Tickets continue after the static tiles of the XCD.
// A workgroup's tiles increase, so it stops at its first tile past the batch without skipping one.
#include "rs_wg.hpp"

namespace ppfs {
namespace wg {

// DMA instructions one wave of waves 1-3 issues for an NPIECE-piece tile (pieces p = w + 192 k,
// w = tid - 64): the last, partial round only in the waves whose first lane has a piece
template <int NPIECE> constexpr uint32_t dma_count(uint32_t wave)
{
    return (uint32_t)(NPIECE / 192) + ((NPIECE % 192) > (int)(64u * (wave - 1u)) ? 1u : 0u);
}

template <int NPIECE>
__device__ __forceinline__ void dma_tile192(uint8_t* dst, const uint8_t* __restrict__ src, uint32_t tid,
    [[maybe_unused]] const uint8_t* gbase, [[maybe_unused]] uint64_t extent)
{
    constexpr int KI = (NPIECE + 191) / 192;
    const uint32_t w = tid - 64u; // waves 1-3
    const uint32_t lbase = __builtin_amdgcn_readfirstlane(lds_addr(dst) + (w & ~63u) * 16u);
    // the last round is issued only by the waves that have pieces in it (wave-uniform branch), so
    // every wave's instruction count is exactly dma_count<NPIECE>(wave)
    const bool last_round = __builtin_amdgcn_readfirstlane(w & ~63u) < (uint32_t)(NPIECE - 192 * (KI - 1));
#pragma unroll
    for (int k = 0; k < KI; ++k) {
        const uint32_t p = w + 192u * (uint32_t)k;
        if ((k + 1) * 192 <= NPIECE) {
            if (PPFS_DBG_OK(src + (size_t)p * 16, 16, gbase, extent))
                dma16(src + (size_t)p * 16, __builtin_amdgcn_readfirstlane(lbase + 3072u * (uint32_t)k));
        } else if (last_round) {
            if (p < (uint32_t)NPIECE && PPFS_DBG_OK(src + (size_t)p * 16, 16, gbase, extent))
                dma16(src + (size_t)p * 16, __builtin_amdgcn_readfirstlane(lbase + 3072u * (uint32_t)k));
        }
    }
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 31] (exact: the counts below are known per wave)
__device__ __forceinline__ void vm_wait_exact(uint32_t n)
{
#ifdef PPFS_ECC_DEBUG
    // the checked build may skip a DMA (PPFS_DBG_OK), so fewer loads are in flight than counted and
    // an exact count would let an older tile's loads still fly: wait for everything
    (void)n;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
#endif
    switch (__builtin_amdgcn_readfirstlane(n)) {
#define PPFS_VMW(N)                                                                                                    \
    case N:                                                                                                            \
        asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory");                                                          \
        break;
        PPFS_VMW(1) PPFS_VMW(2) PPFS_VMW(3) PPFS_VMW(4) PPFS_VMW(5) PPFS_VMW(6) PPFS_VMW(7) PPFS_VMW(8)
        PPFS_VMW(9) PPFS_VMW(10) PPFS_VMW(11) PPFS_VMW(12) PPFS_VMW(13) PPFS_VMW(14) PPFS_VMW(15)
        PPFS_VMW(16) PPFS_VMW(17) PPFS_VMW(18) PPFS_VMW(19) PPFS_VMW(20) PPFS_VMW(21) PPFS_VMW(22) PPFS_VMW(23)
        PPFS_VMW(24) PPFS_VMW(25) PPFS_VMW(26) PPFS_VMW(27) PPFS_VMW(28) PPFS_VMW(29) PPFS_VMW(30) PPFS_VMW(31)
#undef PPFS_VMW
    default:
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        break;
    }
}

// Wave 0 (64 lanes) copies the first BYTES of the table blob into LDS at 0 by LDS-DMA: no register
// round trip, and its loads never share a queue with the DMA waves' tiles.  Caller: vmcnt(0).
template <int BYTES>
__device__ __forceinline__ void dma_tables_w0(uint8_t* dst, const uint8_t* __restrict__ tables, uint32_t lane)
{
    static_assert(BYTES % 16 == 0, "16-byte pieces");
    constexpr int NP = BYTES / 16, KI = (NP + 63) / 64;
    const uint32_t lbase = __builtin_amdgcn_readfirstlane(lds_addr(dst));
#pragma unroll
    for (int k = 0; k < KI; ++k) {
        const uint32_t p = lane + 64u * (uint32_t)k;
        if ((k + 1) * 64 <= NP || p < (uint32_t)NP)
            dma16(tables + 16u * p, lbase + 1024u * (uint32_t)k);
    }
}

// XCD-local tile numbering: workgroup b sits on counter xc = b % nx with rank b / nx among the gx
// workgroups of that counter; local ticket j is tile j * nx + xc
struct TkGeom {
    uint32_t nx, xc, gx, rank;
};
// One counter per XCD (8).  One chip-wide counter: its atomics serialize at ~80 per us and both t = 3
// kernels ran 2x slower, 2 counters +18 % (r5za).  Round 5 also measured cross-XCD stealing (a
// workgroup whose counter runs dry draws the next XCD's): no gain, the slow XCD's lag sits in its
// workgroups' already-drawn lookahead tiles (r5zb-r5zd).
constexpr uint32_t TK_NX = 8;
__device__ __forceinline__ TkGeom tk_geom()
{
    TkGeom g;
    g.nx = gridDim.x < TK_NX ? gridDim.x : TK_NX;
    g.xc = blockIdx.x % g.nx;
    g.gx = (gridDim.x - g.xc + g.nx - 1u) / g.nx;
    g.rank = blockIdx.x / g.nx;
    return g;
}

// the tile of local ticket j on this XCD: interleaved, j nx + xc (round 3 measured each XCD walking
// a contiguous range instead: no gain)
__device__ __forceinline__ uint64_t tk_tile(uint64_t j, const TkGeom& g, uint64_t /*nfull*/) { return j * g.nx + g.xc; }

// block 0, one lane: zero the counter set the previous launch on this stream used -- all 8 counter
// lines, whatever this launch's nx: the previous launch may have counted on more XCD counters than
// this (small) one does, and a counter left dirty would start a later large launch's tickets past
// tiles nobody then encodes
__device__ __forceinline__ void tk_clear(uint32_t* __restrict__ ctr_clear)
{
#pragma unroll
    for (uint32_t x = 0; x < 8u; ++x)
        __hip_atomic_store(ctr_clear + 32u * x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// PPFS_TK_TRACE (profiling builds only, tools/build_alt.sh --product trace -DPPFS_TK_TRACE=1): waves 0
// and 1 of every encode workgroup sum s_memtime cycles per loop phase into g_tk_trace, read back by
// ppfs_tk_trace_read_t<2t> (tools/tk_trace.py).  Normal builds: nothing.
#ifdef PPFS_TK_TRACE
constexpr int TK_TRACE_N = 12; // prologue, issue, remainder, barrier B, emission, vm wait, barrier A, epilogue, iterations, end,
// the workgroup's start and end on the 100 MHz s_memrealtime clock
__device__ uint64_t g_tk_trace[4096 * 2 * TK_TRACE_N];
// decode: prologue, issue, remainder, barrier B, correction (+ barrier C), emission, vm wait, barrier A,
// iterations, end
__device__ uint64_t g_tk_trace_dec[4096 * 2 * TK_TRACE_N];
#define PPFS_TK_MARK(i)                                                                                                \
    do {                                                                                                               \
        const uint64_t now_ = clock64();                                                                               \
        tr_[i] += now_ - tlast_;                                                                                       \
        tlast_ = now_;                                                                                                 \
    } while (0)
#else
#define PPFS_TK_MARK(i) ((void)0)
#endif

// Interior emission pieces: the 16 bytes at LDS byte a + sh / 8 (a dword aligned, sh = 0, 8, 16, 24).
// A window of 5 dwords is read by exactly ds_read2_b32 (0, 1), ds_read2_b32 (2, 3), ds_read_b32 (4)
// (left to itself the compiler reads dwords (0, 1), (1, 2), (3, 4): 6 dword reads), N windows in
// flight at once before one wait; asm reads are not tracked by the compiler, so the wait is explicit
// and names the results.
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
struct Win5 {
    u32x2v d01, d23;
    uint32_t d4;
};
__device__ __forceinline__ uint4 win_piece(const Win5& w, uint32_t sh)
{
    return make_uint4(__builtin_amdgcn_alignbit(w.d01.y, w.d01.x, sh), __builtin_amdgcn_alignbit(w.d23.x, w.d01.y, sh),
        __builtin_amdgcn_alignbit(w.d23.y, w.d23.x, sh), __builtin_amdgcn_alignbit(w.d4, w.d23.y, sh));
}
__device__ __forceinline__ void win5x1(Win5& w0, uint32_t a0)
{
    asm volatile("ds_read2_b32 %0, %3 offset1:1\n\tds_read2_b32 %1, %3 offset0:2 offset1:3\n\tds_read_b32 %2, %3 offset:16\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(w0.d01), "=&v"(w0.d23), "=&v"(w0.d4) // early clobber: no result may overwrite
                 : "v"(a0)                                        // the address before the last read issues
                 : "memory");
}
__device__ __forceinline__ void win5x3(Win5& w0, Win5& w1, Win5& w2, uint32_t a0, uint32_t a1, uint32_t a2)
{
    asm volatile("ds_read2_b32 %0, %9 offset1:1\n\tds_read2_b32 %1, %9 offset0:2 offset1:3\n\tds_read_b32 %2, %9 offset:16\n\t"
                 "ds_read2_b32 %3, %10 offset1:1\n\tds_read2_b32 %4, %10 offset0:2 offset1:3\n\tds_read_b32 %5, %10 offset:16\n\t"
                 "ds_read2_b32 %6, %11 offset1:1\n\tds_read2_b32 %7, %11 offset0:2 offset1:3\n\tds_read_b32 %8, %11 offset:16\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(w0.d01), "=&v"(w0.d23), "=&v"(w0.d4), "=&v"(w1.d01), "=&v"(w1.d23), "=&v"(w1.d4), "=&v"(w2.d01),
                 "=&v"(w2.d23), "=&v"(w2.d4)
                 : "v"(a0), "v"(a1), "v"(a2)
                 : "memory");
}
// rs_sched.hpp enc_src / dec_src on the device: LDS byte of an interior piece's first source byte
template <int T2> __device__ __forceinline__ uint32_t sched_enc_src(uint32_t p)
{
    const uint32_t j0 = 16u * p, b = j0 / 255u, off = j0 - 255u * b;
    return (uint32_t)PAD + (255u - T2) * b + off - (uint32_t)T2;
}

// Every wave at s_setprio 2 from barrier B to its next remainder phase (emission, corrections, DMA
// issue): with 2-3 workgroups per CU in different phases, the output side issues ahead of another
// workgroup's remainder steps.  Round 5: step 4,508-4,509 vs 4,476-4,497 GiB/s (r5t).
template <int T2, int WPC = 2, int NTST = 1>
__global__ __launch_bounds__(256, WPC) void rs_wg_encode_tk_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables, uint32_t* __restrict__ ctr,
    uint32_t* __restrict__ ctr_clear)
{
    constexpr int NBUF = 3;
    using L = RsWgLayout<T2>;
    // phase 1 through the 5-bit field tables (rs_layout.hpp SL5 / SLX5): 13 lookups a step, not 16
    // (round 4: -1.4% encode time, the 3 lower segments' remainder ~100 cycles shorter per tile)
    constexpr bool T5 = true;
    using D = Lds<T2, false, NBUF, false, 2>; // SL5 + SLX5
    constexpr int BUF = D::BUFB;
    constexpr uint32_t OFF_TK = D::BYTES; // 4 ticket slots: slot i & 3 = tile of iteration i
    // the output tile staged in LDS (natural piece order for the stores); the emission schedule
    // (rs_sched.hpp) is read from the same bytes once, before the first tile
    constexpr uint32_t OFF_STG = D::BYTES + 64, OFF_SCHED = OFF_STG;
    constexpr int OUT_PIECES = TB * 255 / 16;
    constexpr int STG_BYTES = OUT_PIECES * 16;
    static_assert(STG_BYTES >= L::SCHED_BYTES + 64, "the schedule and row map fit the staging buffer");
    constexpr int LDS_ALLOC = lds_alloc<D::BYTES + 64 + STG_BYTES, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * K / 16;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    uint32_t* const s_tk = (uint32_t*)(lds + OFF_TK);
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const bool dmaw = wave != 0, tk_lane = wave == 0 && lane == 0;
    const uint32_t kd = dmaw ? dma_count<IN_PIECES>(wave) : 0u; // this wave's DMA instructions per tile
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    const TkGeom g = tk_geom();
    uint32_t* const my_ctr = ctr + 32u * g.xc; // 128-byte lines
#ifdef PPFS_TK_TRACE
    uint64_t tr_[TK_TRACE_N] = {};
    tr_[10] = __builtin_amdgcn_s_memrealtime();
    uint64_t tlast_ = clock64();
    const uint64_t t0_ = tlast_;
#endif
    // the first three tiles are static: local tickets rank, rank + gx, rank + 2 gx
    uint64_t q0 = tk_tile(g.rank, g, nfull), q1 = tk_tile(g.rank + g.gx, g, nfull);
    uint32_t hist = 0;
    if (dmaw) {
        if (q0 < nfull)
            dma_tile192<IN_PIECES>(lds + D::OFF_BUF + PAD, data + q0 * (TB * K), tid, data, nblocks * K);
        const bool go = q1 < nfull;
        if (go)
            dma_tile192<IN_PIECES>(lds + D::OFF_BUF + BUF + PAD, data + q1 * (TB * K), tid, data, nblocks * K);
        hist = go ? 1u : 0u;
    } else {
        dma_tables_w0<L::SL5_BYTES>(lds, tables + L::OFF_SL5, lane);
        dma_tables_w0<L::SLX5_BYTES>(lds + D::OFF_SLX, tables + L::OFF_SLX5, lane);
        dma_tables_w0<L::SCHED_BYTES>(lds + OFF_SCHED, tables + L::OFF_ESCHED, lane);
        dma_tables_w0<64>(lds + OFF_SCHED + L::SCHED_BYTES, tables + L::OFF_ROWMAP, lane);
        *(uint64_t*)(lds + D::OFF_PAR + 8u * lane) = 0; // both parity slot sets (2 x 64 x 8 B)
        *(uint64_t*)(lds + D::OFF_PAR + 512u + 8u * lane) = 0;
        if (tk_lane) {
            if (blockIdx.x == 0)
                tk_clear(ctr_clear);
            s_tk[2] = (uint32_t)tk_tile(g.rank + 2u * g.gx, g, nfull); // the tile of iteration 2 (static)
            const uint32_t t3 = atomicInc(my_ctr, 0xFFFFFFFFu) + 3u * g.gx; // the tile of iteration 3
            s_tk[3] = (uint32_t)tk_tile(t3, g, nfull);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // tables landed, ticket returned
    }
    if (dmaw)
        vm_wait_exact(kd * hist); // tile q0 landed, q1 may fly
    barrier_lds();
    // this thread's emission pieces, one per round (rs_sched.hpp): rounds 0-2 are interior pieces
    // (LDS window at a[k], funnel shift sh[k], output byte o[k]); round 3 interior, boundary or none
    uint32_t ea[4], esh[4], eo[4], kind3;
    const uint32_t row = lds[OFF_SCHED + L::SCHED_BYTES + lane]; // phase 1's payload row (rs_sched.hpp row_map)
    {
        const uint2 sc = *(const uint2*)(lds + OFF_SCHED + 8u * tid);
        const uint32_t e[4] = { sc.x & 0xFFFFu, sc.x >> 16, sc.y & 0xFFFFu, sc.y >> 16 };
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t pk = e[k] & 0x3FFu, S = sched_enc_src<T2>(pk);
            ea[k] = S & ~3u;
            esh[k] = (S & 3u) * 8u;
            eo[k] = 16u * pk;
        }
        kind3 = e[3] == 0xFFFFu ? 2u : (e[3] >> 15);
    }
    PPFS_TK_MARK(0);
    uint32_t cur = 0, pc = 0, iter = 0;
    // Tickets (round 4): wave 0, lane 0 takes one at the END of an iteration, after the tile's stores,
    // and publishes it after barrier B of the next (the tile of iteration + 4 of the taking one): the
    // compiler's wait for the atomic then covers only operations a phase old.  (Taken at the top and
    // published at the end, the wait drained the tile's fresh stores: ~700 cycles per tile of wave 0,
    // and waves 1-3 behind it at barrier A.)  No initial value: writing the register outside wave
    // 0's branch would make every wave wait for the ticket (the compiler tracks it per register).
    uint32_t tk;
    while (q0 < nfull) {
        // A: tile q0 in LDS, the last emission reads done, the next ticket published (the first
        // pass: tables, parity slots and the iteration-2 and -3 tiles in place)
        if (iter) {
            barrier_lds();
            PPFS_TK_MARK(6);
        }
        const uint64_t ahead = __builtin_amdgcn_readfirstlane(s_tk[(iter + 2u) & 3u]);
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        const bool go = ahead < nfull;
        if (dmaw && go)
            dma_tile192<IN_PIECES>(lds + D::OFF_BUF + ring_add(cur, NBUF - 1, NBUF) * BUF + PAD, data + ahead * (TB * K),
                tid, data, nblocks * K);
        hist = (hist << 1) | (go ? 1u : 0u);
        PPFS_TK_MARK(1);
        if (wave == 0)
            *(uint64_t*)(lds + D::OFF_PAR + (pc ^ 1u) * 512u + 8u * lane) = 0;
        __builtin_amdgcn_s_setprio(0);
        phase_remainder<T2, K, D::NMAP, D::OFF_SLX, T5>(lds, buf, par, wave, row);
        PPFS_TK_MARK(2);
        barrier_lds(); // B: parity slots complete
        __builtin_amdgcn_s_setprio(2);
        PPFS_TK_MARK(3);
        if (tk_lane && iter)
            s_tk[(iter + 3u) & 3u] = (uint32_t)tk_tile(tk + 3u * g.gx, g, nfull); // the tile of iteration iter + 3
        uint8_t* dst = raw + q0 * (TB * 255);
        { // rounds 0-2, interior pieces: 4 funnel shifts each, the 3 windows read together
            const uint32_t lb = lds_addr(lds) + buf;
            Win5 w[3];
            win5x3(w[0], w[1], w[2], lb + ea[0], lb + ea[1], lb + ea[2]);
#pragma unroll
            for (int k = 0; k < 3; ++k)
                *(uint4*)(lds + OFF_STG + eo[k]) = win_piece(w[k], esh[k]);
        }
        { // round 3: the last interior pieces, then the boundary pieces (general merge)
            uint4 o;
            if (kind3 == 0u) {
                Win5 w;
                win5x1(w, lds_addr(lds) + buf + ea[3]);
                o = win_piece(w, esh[3]);
            } else {
                o = enc_piece<T2>(lds, buf, par, eo[3] >> 4);
            }
            if (kind3 != 2u)
                *(uint4*)(lds + OFF_STG + eo[3]) = o;
        }
        barrier_lds(); // S: the whole output tile staged
        // stores in the natural order: a wave writes 1 KiB of consecutive output per instruction
        // (round 4: stored straight from the schedule's lanes, 128-byte runs from four blocks, the
        // t = 3 encode ran at half speed -- partial lines everywhere)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = tid + 256u * k;
            if ((k < 3 || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, raw, nblocks * 255u))
                st_nt<NTST>(dst + 16u * p, *(const uint4*)(lds + OFF_STG + 16u * p));
        }
        ++iter;
        PPFS_TK_MARK(4);
        if (dmaw) {
            // the next tile's DMA (issued an iteration ago, or in the prologue) landed; newer: the
            // last two iterations' stores and this iteration's DMA
            const uint32_t st = 4u * (iter < 2u ? iter : 2u);
            vm_wait_exact(st + kd * (hist & 1u));
        }
        if (tk_lane)
            tk = atomicInc(my_ctr, 0xFFFFFFFFu); // the tile of (iteration iter - 1) + 4, published next iteration
        PPFS_TK_MARK(5);
        cur = ring_add(cur, 1, NBUF);
        pc ^= 1u;
        q0 = q1;
        q1 = ahead;
    }
    if (q0 == nfull && nfull < ntiles) { // the partial tile
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        const uint64_t t = nfull;
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        if (PPFS_DBG_OK(data + t * (TB * K), nb * K, data, nblocks * K))
            stage_bytes(lds + buf + PAD, data + t * (TB * K), nb * K, tid);
        barrier_lds();
        phase_remainder<T2, K, D::NMAP, D::OFF_SLX, T5>(lds, buf, par, wave, row);
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
#ifdef PPFS_TK_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PPFS_TK_MARK(7);
    tr_[8] = iter;
    tr_[9] = clock64() - t0_;
    tr_[11] = __builtin_amdgcn_s_memrealtime();
    if (wave < 2 && lane == 0 && blockIdx.x < 4096)
        for (int i = 0; i < TK_TRACE_N; ++i)
            g_tk_trace[(blockIdx.x * 2 + wave) * TK_TRACE_N + i] = tr_[i];
#endif
}

// ------------------------------------------------------------------------------------
// The t <= 4 decode (rs_wg_decode_kernel, double-buffered, 3 workgroups per CU) on the same
// ticket scheme: waves 1-3 issue the DMA, wave 0 (the corrector) brings the tables and takes the
// tickets.  With two buffers the first tile is static and ticket j is the tile of iteration j + 1
// (taken at the top of iteration j - 1, read at the top of iteration j for the DMA one tile ahead).
// Counter sets: the decode halves of the stream's pair (api.cpp ctr_for).
// ------------------------------------------------------------------------------------
template <int T2, int WPC = 3, int NTST = 1>
__global__ __launch_bounds__(256, WPC) void rs_wg_decode_tk_kernel(uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint64_t nblocks, const uint8_t* __restrict__ tables, int write_back,
    uint32_t* __restrict__ ctr, uint32_t* __restrict__ ctr_clear, uint8_t* __restrict__ raw_wb)
{
    constexpr int NBUF = 2;
    using L = RsWgLayout<T2>;
    // nibble tables (the 5-bit field tables of the encode measured no gain here: round 4, r4u)
    using D = Lds<T2, true, NBUF, false, 1>; // decode tables + SLX
    constexpr uint32_t OFF_TK = D::BYTES; // 4 ticket slots: slot i & 3 = tile of iteration i
    constexpr int LDS_ALLOC = lds_alloc<D::BYTES + 64, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * 255 / 16;
    constexpr int OUT_PIECES = TB * K / 16;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    uint32_t* const s_tk = (uint32_t*)(lds + OFF_TK);
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const bool dmaw = wave != 0, tk_lane = wave == 0 && lane == 0;
    const uint32_t row = lane_row(lane);
    const bool wb = write_back != 0, want = data != nullptr;
    // write-back target: the codewords in place, or (raw_wb, the host path's page-locked caller image
    // mapped into the device) the caller's image directly
    uint8_t* const wbp = raw_wb ? raw_wb : raw;
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB;
    const TkGeom g = tk_geom();
    uint32_t* const my_ctr = ctr + 32u * g.xc;
#ifdef PPFS_TK_TRACE
    uint64_t tr_[TK_TRACE_N] = {};
    tr_[10] = __builtin_amdgcn_s_memrealtime();
    uint64_t tlast_ = clock64();
    const uint64_t t0_ = tlast_;
#endif
    uint64_t q0 = tk_tile(g.rank, g, nfull); // static first tile
    if (dmaw) {
        if (q0 < nfull)
            dma_tile192<IN_PIECES>(lds + D::OFF_BUF + PAD, raw + q0 * (TB * 255), tid, raw, nblocks * 255u);
    } else {
        dma_tables_w0<L::TABLE_BYTES>(lds, tables, lane); // the decode tables, then SLX after them
        dma_tables_w0<L::SLX_BYTES>(lds + D::OFF_SLX, tables + L::OFF_SLX, lane);
        *(uint64_t*)(lds + D::OFF_PAR + 8u * lane) = 0;
        *(uint64_t*)(lds + D::OFF_PAR + 512u + 8u * lane) = 0;
        if (tk_lane) {
            if (blockIdx.x == 0)
                tk_clear(ctr_clear);
            s_tk[1] = (uint32_t)tk_tile(atomicInc(my_ctr, 0xFFFFFFFFu) + g.gx, g, nfull); // the tile of iteration 1
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // tile q0 / tables and the ticket landed
    barrier_lds();
    PPFS_TK_MARK(0);
    uint32_t cur = 0, pc = 0, iter = 0;
    while (q0 < nfull) {
        if (iter) {
            barrier_lds(); // A: tile q0 in LDS, the last emission reads done, the next ticket published
            PPFS_TK_MARK(7);
        }
        const uint64_t q1 = __builtin_amdgcn_readfirstlane(s_tk[(iter + 1u) & 3u]);
        // taken at the top, published at the end (round 4: taken at the end and published after the
        // next barrier B, as the encode does, the decode ran ~1 % slower -- its wave 0 then waits for
        // the contended atomic right before the corrections, r4q)
        uint32_t tk; // no initial value (see the encode)
        if (tk_lane)
            tk = atomicInc(my_ctr, 0xFFFFFFFFu); // the tile of iteration iter + 2
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        if (dmaw && q1 < nfull)
            dma_tile192<IN_PIECES>(lds + D::OFF_BUF + (cur ^ 1u) * BUF + PAD, raw + q1 * (TB * 255), tid, raw,
                nblocks * 255u);
        PPFS_TK_MARK(1);
        if (wave == 0)
            *(uint64_t*)(lds + D::OFF_PAR + (pc ^ 1u) * 512u + 8u * lane) = 0;
        __builtin_amdgcn_s_setprio(0);
        phase_remainder<T2, 255, D::NMAP, D::OFF_SLX>(lds, buf, par, wave, row);
        PPFS_TK_MARK(2);
        barrier_lds(); // B: remainders complete
        __builtin_amdgcn_s_setprio(2);
        PPFS_TK_MARK(3);
        if (wave == 0) {
            const uint32_t st_tile = phase_correct<T2>(lds, buf, par, row, true, wbp, q0 * TB + row, wb, nblocks * 255u);
            if (status && PPFS_DBG_OK(status + q0 * TB + row, 1, status, nblocks))
                status[q0 * TB + row] = (uint8_t)st_tile;
        }
        barrier_lds(); // C: corrections patched into the LDS rows
        PPFS_TK_MARK(4);
        if (want) {
            uint8_t* dst = data + q0 * (TB * K);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t p = tid + 256u * k;
                const uint4 o = dec_piece<T2>(lds, buf, p);
                if ((k < 3 || p < (uint32_t)OUT_PIECES) && PPFS_DBG_OK(dst + 16u * p, 16, data, nblocks * K))
                    st_nt<NTST>(dst + 16u * p, o);
            }
        }
        ++iter;
        PPFS_TK_MARK(5);
        if (dmaw) { // the next tile's DMA landed; this tile's stores may fly
            if (want)
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (tk_lane)
            s_tk[(iter + 1u) & 3u] = (uint32_t)tk_tile(tk + g.gx, g, nfull); // the tile of (iteration iter - 1) + 2
        PPFS_TK_MARK(6);
        cur ^= 1u;
        pc ^= 1u;
        q0 = q1;
    }
    if (q0 == nfull && nfull < ntiles) { // the partial tile
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        const uint64_t t = nfull;
        const uint32_t nb = (uint32_t)(nblocks - t * TB);
        const uint32_t buf = D::OFF_BUF + cur * BUF, par = D::OFF_PAR + pc * 512u;
        if (PPFS_DBG_OK(raw + t * (TB * 255), nb * 255u, raw, nblocks * 255u))
            stage_bytes(lds + buf + PAD, raw + t * (TB * 255), nb * 255u, tid);
        barrier_lds();
        phase_remainder<T2, 255, D::NMAP, D::OFF_SLX>(lds, buf, par, wave, row);
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
#ifdef PPFS_TK_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tr_[8] = iter;
    tr_[9] = clock64() - t0_;
    tr_[11] = __builtin_amdgcn_s_memrealtime();
    if (wave < 2 && lane == 0 && blockIdx.x < 4096)
        for (int i = 0; i < TK_TRACE_N; ++i)
            g_tk_trace_dec[(blockIdx.x * 2 + wave) * TK_TRACE_N + i] = tr_[i];
#endif
}

} // namespace wg
} // namespace ppfs
