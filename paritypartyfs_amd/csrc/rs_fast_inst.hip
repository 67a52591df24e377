// rs_fast_inst.hip -- the shipped fast-path dispatch for one 2t = PPFS_T2 (compiled once per 2t).
// Only the kernels the engine launches are instantiated here; the variants measured in rounds 1-2
// (register prefetch, 8-wave and wave-independent encodes, image encodes, deeper rings, the nibble
// pair kernels) live in tools/ablations/ and are built by tools/build_alt.sh.
//   2t <= 8      rs_wg_tk.hpp ticket-counter encode / decode (every context hands a counter set
//                for its first 16 streams, api.cpp ctr_for); rs_wg.hpp static-walk kernels otherwise
//   8 < 2t <= 16 rs_fast.hpp lane-per-block kernels; 2t = 16 encodes with rs_pair.hpp's solo image kernel
//   2t = 32      rs_bs.hpp byte-slice kernels (cfg5, RS(255,223))
#include "rs_fast.hpp"
#include "rs_wg.hpp"
#include "rs_wg_tk.hpp"
#include "rs_pair.hpp"
#include "rs_bs.hpp"
#include "launch.hpp"

#ifndef PPFS_T2
#error "compile with -DPPFS_T2=<2t>"
#endif
static_assert(PPFS_T2 <= 16 || PPFS_T2 == 32, "the 16 < 2t < 32 codes take the generic path (ppfs_rs_fast_supported)");

#define PPFS_CAT2(a, b) a##b
#define PPFS_CAT(a, b) PPFS_CAT2(a, b)

using namespace ppfs;

static int cu_count()
{
    static int cus[64] = { 0 };
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64)
        dev = 0;
    if (!cus[dev]) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            c = 256;
        cus[dev] = c;
    }
    return cus[dev];
}

// persistent tile grid: WPC resident workgroups per CU, capped by the tiles (tb blocks each)
static uint32_t rs_tile_grid(uint64_t nb, int wpc, int tb = 64)
{
    const uint64_t tiles = (nb + (uint64_t)tb - 1) / (uint64_t)tb;
    const uint64_t cap = (uint64_t)wpc * (uint64_t)cu_count();
    return (uint32_t)(tiles < cap ? (tiles ? tiles : 1) : cap);
}

#if PPFS_T2 <= 8
// 2t <= 8 (rs_wg.hpp).  Encode: a ring of 3 LDS tile buffers, 2 workgroups per CU;
// decode: double-buffered, 3 per CU.  Non-temporal output stores in both.
// The static-walk encode fits as many workgroups as its LDS allows (at most 4); the ticket encode
// runs 2 per CU (its LDS carries the ticket slots).
constexpr int fit_wpc(int bytes, int most) { return 163840 / bytes < most ? 163840 / bytes : most; }
constexpr int TK_NTST = 1; // ticket kernels' output stores non-temporal (plain stores: slower)
constexpr int ENC_NBUF = 3, ENC_WPC = 2, DEC_NBUF = 2, DEC_WPC = 3;
constexpr int ENC_WPC_STATIC = fit_wpc(wg::lds_bytes<PPFS_T2, false, ENC_NBUF>(), 4);
#elif PPFS_T2 == 32
// 2t = 32 (rs_bs.hpp): one workgroup per CU, every wave on its own 32-block tiles;
// encode 12 waves (3 per SIMD), decode 8 (LDS- and register-bound).  Decode: GF block, S12 table and
// the XP rows in LDS (TLDS 3; round 3: 139 -> 130 us in the cfg5 step), register prefetch of the next
// tile (NBUF 0); encode: one LDS image, the next tile's DMA after the emission (NBUF 1).  Both take
// their tiles by per-XCD ticket when the launch has a counter set (rs_bs.hpp BsWalk).
constexpr int BS_ENC_NW = 12, BS_ENC_NBUF = 1, BS_DEC_NW = 8, BS_DEC_TLDS = 3, BS_DEC_NBUF = 0;
#else
// 8 < 2t <= 16: rs_fast.hpp lane-per-block kernels; 2t = 16 encodes with the solo image kernel
constexpr bool SOLO_IMG = PPFS_T2 == 16;
constexpr int SOLO_NW = 2, SOLO_WPC = 4;
// grid of the lane-per-block kernels: two 256-thread workgroups per CU, capped by the work
static uint32_t rs_grid(uint64_t nb)
{
    const uint64_t wave_tiles = (nb + RS_WT - 1) / RS_WT;
    const uint64_t want = (wave_tiles + RS_WAVES - 1) / RS_WAVES;
    const uint64_t cap = 2ull * (uint64_t)cu_count();
    return (uint32_t)(want < cap ? (want ? want : 1) : cap);
}
#endif

// ctr / ctr_clear: the stream's ticket-counter set for this launch and the one to zero (the previous
// launch's; api.cpp ctr_for alternates them), or null: the static walk
extern "C" hipError_t PPFS_CAT(ppfs_rs_fast_encode_t, PPFS_T2)(const uint8_t* d, uint8_t* r, uint64_t nb,
    const uint8_t* tab, hipStream_t s, [[maybe_unused]] uint32_t* ctr, [[maybe_unused]] uint32_t* ctr_clear)
{
#if PPFS_T2 <= 8
    if (ctr && ctr_clear)
        PPFS_LAUNCH((wg::rs_wg_encode_tk_kernel<PPFS_T2, ENC_WPC, TK_NTST>), dim3(rs_tile_grid(nb, ENC_WPC)), dim3(256), 0, s,
            d, r, nb, tab, ctr, ctr_clear);
    else
        PPFS_LAUNCH((wg::rs_wg_encode_kernel<PPFS_T2, ENC_NBUF, ENC_WPC_STATIC, 3, 1, false>), dim3(rs_tile_grid(nb, ENC_WPC_STATIC)),
            dim3(256), 0, s, d, r, nb, tab);
#elif PPFS_T2 == 32
    PPFS_LAUNCH((bs::rs_bs_encode_kernel<PPFS_T2, BS_ENC_NW, BS_ENC_NBUF>), dim3(rs_tile_grid(nb, 1, bs::TBW * BS_ENC_NW)),
        dim3(64 * BS_ENC_NW), 0, s, d, r, nb, tab, ctr, ctr_clear);
#else
    if constexpr (SOLO_IMG)
        PPFS_LAUNCH((pair::rs_solo_encode_img_kernel<PPFS_T2, SOLO_WPC, SOLO_NW>),
            dim3(rs_tile_grid(nb, SOLO_WPC, 64 * SOLO_NW)), dim3(64 * SOLO_NW), 0, s, d, r, nb, tab);
    else
        PPFS_LAUNCH(rs255_encode_kernel<PPFS_T2>, dim3(rs_grid(nb)), dim3(256), 0, s, d, r, nb, tab);
#endif
    return hipGetLastError();
}

extern "C" const char* PPFS_CAT(ppfs_rs_fast_path_t, PPFS_T2)()
{
#if PPFS_T2 <= 8
    // the ticket kernels (rs_wg_tk.hpp) when the caller hands a counter set; api.cpp reports the
    // static walk ("rs255-wg-seg4-lds") for a launch without one
    return "rs255-wg-tk-lds";
#elif PPFS_T2 == 32
    return "rs255-bs-byte-lds";
#else
    return "rs255-slice8-lds";
#endif
}

// wb_dst: where the write-backs go (null: the codewords in place; 2t <= 8 only: api.cpp's host path
// passes the page-locked caller image, mapped into the device)
extern "C" hipError_t PPFS_CAT(ppfs_rs_fast_decode_t, PPFS_T2)(uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb,
    const uint8_t* tab, int wb, hipStream_t s, [[maybe_unused]] uint32_t* ctr, [[maybe_unused]] uint32_t* ctr_clear,
    [[maybe_unused]] uint8_t* wb_dst)
{
#if PPFS_T2 <= 8
    if (ctr && ctr_clear)
        PPFS_LAUNCH((wg::rs_wg_decode_tk_kernel<PPFS_T2, DEC_WPC, TK_NTST>), dim3(rs_tile_grid(nb, DEC_WPC)), dim3(256), 0, s,
            r, d, st, nb, tab, wb, ctr, ctr_clear, wb_dst);
    else
        PPFS_LAUNCH((wg::rs_wg_decode_kernel<PPFS_T2, DEC_NBUF, DEC_WPC, 7, 1>), dim3(rs_tile_grid(nb, DEC_WPC)),
            dim3(256), 0, s, r, d, st, nb, tab, wb, wb_dst);
#elif PPFS_T2 == 32
    if (wb_dst)
        return hipErrorInvalidValue;
    PPFS_LAUNCH((bs::rs_bs_decode_kernel<PPFS_T2, BS_DEC_NW, BS_DEC_NBUF, 1, BS_DEC_TLDS>),
        dim3(rs_tile_grid(nb, 1, bs::TBW * BS_DEC_NW)), dim3(64 * BS_DEC_NW), 0, s, r, d, st, nb, tab, wb,
        ctr, ctr_clear);
#else
    if (wb_dst)
        return hipErrorInvalidValue;
    PPFS_LAUNCH(rs255_decode_kernel<PPFS_T2>, dim3(rs_grid(nb)), dim3(256), 0, s, r, d, st, nb, tab, wb);
#endif
    return hipGetLastError();
}
PPFS_DBG_ACCESSOR(PPFS_CAT(ppfs_dbg_faults_rs_t, PPFS_T2))

// resident small-batch servers (api.cpp server_call): 2t <= 8 rs_wg.hpp rs_wg_server_kernel,
// 8 < 2t <= 16 rs_fast.hpp rs255_server_kernel, 2t = 32 rs_pair.hpp rs_pair_server_kernel
extern "C" hipError_t PPFS_CAT(ppfs_rs_server_launch_t, PPFS_T2)(ppfs::SrvBox* box, uint8_t* zc, uint64_t zc_bytes,
    const uint8_t* tab, uint32_t gen, uint32_t idle_us, hipStream_t s)
{
#if PPFS_T2 <= 8
    PPFS_LAUNCH((wg::rs_wg_server_kernel<PPFS_T2>), dim3(1), dim3(256), 0, s, box, zc, zc_bytes, tab, gen, idle_us);
#elif PPFS_T2 == 32
    PPFS_LAUNCH((pair::rs_pair_server_kernel<PPFS_T2, true>), dim3(1), dim3(pair::NTHR), 0, s, box, zc, zc_bytes, tab,
        gen, idle_us);
#else
    PPFS_LAUNCH((rs255_server_kernel<PPFS_T2>), dim3(1), dim3(64), 0, s, box, zc, zc_bytes, tab, gen, idle_us);
#endif
    return hipGetLastError();
}

#if defined(PPFS_TK_TRACE) && PPFS_T2 == 32
// profiling builds: the 2t = 32 decode's per-wave phase sums (rs_bs.hpp g_bs_trace)
extern "C" hipError_t ppfs_bs_trace_read(void* dst, size_t bytes)
{
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(bs::g_bs_trace), bytes < sizeof(bs::g_bs_trace) ? bytes : sizeof(bs::g_bs_trace), 0,
        hipMemcpyDeviceToHost);
}
#endif
#if defined(PPFS_TK_TRACE) && PPFS_T2 <= 8
// profiling builds: the encode's per-phase cycle sums (rs_wg_tk.hpp g_tk_trace) into host memory
extern "C" hipError_t PPFS_CAT(ppfs_tk_trace_read_t, PPFS_T2)(void* dst, size_t bytes)
{
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(wg::g_tk_trace), bytes < sizeof(wg::g_tk_trace) ? bytes : sizeof(wg::g_tk_trace), 0,
        hipMemcpyDeviceToHost);
}
extern "C" hipError_t PPFS_CAT(ppfs_tk_trace_dec_read_t, PPFS_T2)(void* dst, size_t bytes)
{
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(wg::g_tk_trace_dec),
        bytes < sizeof(wg::g_tk_trace_dec) ? bytes : sizeof(wg::g_tk_trace_dec), 0, hipMemcpyDeviceToHost);
}
#endif
