// rs_fast_inst_ablate.hip -- ABLATION builds only (tools/build_alt.sh): the fast-path instantiation
// with every compile-time switch of rounds 1-2 (the product dispatch is csrc/rs_fast_inst.hip).
#include "rs_fast.hpp"
#include "rs_wg.hpp"
#include "rs_wg_img.hpp"
#include "rs_pair.hpp"
#include "rs_pair_ablate.hpp"
#include "rs_bs.hpp"
#include "rs_w1.hpp"

#ifndef PPFS_T2
#error "compile with -DPPFS_T2=<2t>"
#endif

#define PPFS_CAT2(a, b) a##b
#define PPFS_CAT(a, b) PPFS_CAT2(a, b)

using namespace ppfs;

// persistent grid: two 256-thread workgroups per CU (LDS-limited), capped by the work
static uint32_t rs_grid(uint64_t nb)
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
    const uint64_t wave_tiles = (nb + RS_WT - 1) / RS_WT;
    const uint64_t want = (wave_tiles + RS_WAVES - 1) / RS_WAVES;
    const uint64_t cap = 2ull * (uint64_t)cus[dev];
    return (uint32_t)(want < cap ? (want ? want : 1) : cap);
}

// persistent tile grid: WPC resident workgroups per CU, capped by the tiles (tb blocks each)
static uint32_t rs_tile_grid(uint64_t nb, int wpc, int tb = 64)
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
        c = 256;
    const uint64_t tiles = (nb + (uint64_t)tb - 1) / (uint64_t)tb;
    const uint64_t cap = (uint64_t)wpc * (uint64_t)c;
    return (uint32_t)(tiles < cap ? (tiles ? tiles : 1) : cap);
}

#if PPFS_T2 <= 8
// segment workgroup path (2t <= 8): one 256-thread workgroup per 64-block tile, WPC resident per CU
// PPFS_WG_FULL = N (ablation): one single-buffered workgroup per tile over a full grid, N per CU
#ifndef PPFS_WG_FULL
#define PPFS_WG_FULL 0
#endif
constexpr bool WG_FULL = PPFS_WG_FULL != 0;
constexpr int fit_wpc(int bytes, int most) { return 163840 / bytes < most ? 163840 / bytes : most; }
// PPFS_WG_ENC_NBUF / PPFS_WG_DEC_NBUF = LDS tile buffers per workgroup: 2 = double buffer;
// 3, 4 = a ring with the DMA NBUF - 1 tiles ahead and as many workgroups per CU as fit.
// Encode ships with 3 (2 workgroups / CU, 2 tiles in flight each): in the bench step the encode
// runs 110-112 -> 101-102 us (0.59 -> 0.65 of 8 TB/s) and from HBM 107-108 -> 102 us, while with
// the payload cache-resident it is slower (89 -> 99 us: half the waves to hide LDS latency).
// Decode stays at 2: its ring variants are 10 % slower in the step (profiles/r2_ablations/).
#ifndef PPFS_WG_ENC_NBUF
#define PPFS_WG_ENC_NBUF 3
#endif
#ifndef PPFS_WG_DEC_NBUF
#define PPFS_WG_DEC_NBUF 2
#endif
static_assert(PPFS_WG_ENC_NBUF >= 2 && PPFS_WG_ENC_NBUF <= 4 && PPFS_WG_DEC_NBUF >= 2 && PPFS_WG_DEC_NBUF <= 4, "NBUF 2..4");
// PPFS_WG_ENC_COMPACT = 1 (ablation): the compact encode LDS layout (rs_wg.hpp Lds: 2 maps,
// payload-sized tile buffers), so a ring of 3 buffers fits 3 workgroups per CU.  Slower: 2^20
// blocks hot / from HBM 101 / 104 -> 108 / 111 us (3 ring buffers) and 103 / 106 us (4 buffers,
// 2 workgroups) (profiles/r2_ablations/compact_enc_kablate.jsonl)
#ifndef PPFS_WG_ENC_COMPACT
#define PPFS_WG_ENC_COMPACT 0
#endif
constexpr bool ENC_COMPACT = PPFS_WG_ENC_COMPACT != 0 && !WG_FULL;
constexpr int ENC_NBUF = WG_FULL ? 0 : PPFS_WG_ENC_NBUF;
[[maybe_unused]] constexpr int ENC_WPC = WG_FULL ? fit_wpc(wg::lds_bytes<PPFS_T2, false, 0>(), PPFS_WG_FULL)
    : ENC_NBUF >= 3          ? fit_wpc(wg::lds_bytes<PPFS_T2, false, ENC_NBUF, ENC_COMPACT>(), 4)
                             : ((4 * wg::lds_bytes<PPFS_T2, false, 2, ENC_COMPACT>() <= 163840) ? 4 : 3);
// PPFS_WG_DEC_FULL = N (ablation): decode on a full grid, N workgroups per CU, one tile each.
// Standalone from HBM ("cold") it is faster (2^20 blocks: 106-108 -> 91-99 us), but inside the
// bench step slower (99.7 -> 103.7 us) and in the step is where the headline is measured,
// so the persistent double-buffered grid (0) stays the default.
#ifndef PPFS_WG_DEC_FULL
#define PPFS_WG_DEC_FULL 0
#endif
constexpr bool DEC_FULL = PPFS_WG_DEC_FULL != 0;
constexpr int DEC_NBUF = DEC_FULL ? 0 : PPFS_WG_DEC_NBUF;
[[maybe_unused]] constexpr int DEC_WPC = DEC_FULL ? fit_wpc(wg::lds_bytes<PPFS_T2, true, 0>(), PPFS_WG_DEC_FULL)
    : DEC_NBUF >= 3          ? fit_wpc(wg::lds_bytes<PPFS_T2, true, DEC_NBUF>(), 3)
                             : 3;
// PPFS_WG_ENC_IMG = 1 (ablation): encode into a codeword image on a full grid
// (rs_wg_encode_img_kernel).  A third fewer VALU instructions; standalone with the payload
// cache-resident ("hot") 89-92 -> 83-85 us, but from HBM 108 -> 114 us and in the step 111 -> 114 us
// (its DMA sources are byte-misaligned: 9 lines per 1 KiB wave read), so the default stays 0.
#ifndef PPFS_WG_ENC_IMG
#define PPFS_WG_ENC_IMG 0
#endif
#ifndef PPFS_WG_ENC_IMG_WPC
#define PPFS_WG_ENC_IMG_WPC 6
#endif
// PPFS_WG_RP = N: register-prefetch kernels (rs_wg_*_rp_kernel), N workgroups per CU; 0 = off
#ifndef PPFS_WG_RP
#define PPFS_WG_RP 0
#endif
// PPFS_WG_DYN: bit 0 = encode, bit 1 = decode take their tiles from a ticket counter (rs_wg_ablate.hpp
// rs_wg_encode_dyn_kernel) instead of the static t += G walk; bit 2 = the static walk through the
// same kernel (ablation)
#ifndef PPFS_WG_DYN
#define PPFS_WG_DYN 0
#endif
// PPFS_WG_ENC_W8 = NBUF (3 or 4): the 8-wave encode (rs_wg_ablate.hpp rs_wg_encode8_kernel); 0 = off
#ifndef PPFS_WG_ENC_W8
#define PPFS_WG_ENC_W8 0
#endif
#if PPFS_WG_RP
#include "rs_wg_rp.hpp"
#endif
// dynamic tiles (rs_wg_tk.hpp) when the caller passes a counter set: bit 0 = encode, bit 1 = decode
#ifndef PPFS_WG_TK
#define PPFS_WG_TK 3
#endif
#include "rs_wg_tk.hpp"
// PPFS_WG_TKN = NBUF (ablation): the ticket encode over a ring of NBUF buffers (rs_wg_tk_ablate.hpp)
#ifndef PPFS_WG_TKN
#define PPFS_WG_TKN 0
#endif
#if PPFS_WG_TKN
#include "rs_wg_tk_ablate.hpp"
#endif
#if PPFS_WG_ENC_W8 || PPFS_WG_DYN
#include "rs_wg_ablate.hpp"
#endif
// round 3: the barrier-free wave-quarter encode (rs_wq.hpp): PPFS_WG_WQ = 1 static walk of 16-block
// wave tiles (ring PPFS_WQ_NBUF), 2 = per-wave ticket counters (ring of 3)
#ifndef PPFS_WG_WQ
#define PPFS_WG_WQ 0
#endif
#ifndef PPFS_WQ_NBUF
#define PPFS_WQ_NBUF 3
#endif
#if PPFS_T2 <= 8
#include "rs_wq.hpp"
#endif
// wave-independent kernels (rs_w1.hpp): one workgroup of PPFS_W1_NW waves per CU, every wave on
// its own 64-block tiles; PPFS_W1_NBUF 1 = LDS-DMA, 0 = register prefetch
#ifndef PPFS_WG_W1
#define PPFS_WG_W1 0
#endif
#ifndef PPFS_W1_NW
#define PPFS_W1_NW 8
#endif
#ifndef PPFS_W1_DEC_NW
#define PPFS_W1_DEC_NW 8
#endif
#ifndef PPFS_W1_NBUF
#define PPFS_W1_NBUF 1
#endif
#ifndef PPFS_W1_DEC_NBUF
#define PPFS_W1_DEC_NBUF PPFS_W1_NBUF
#endif
#ifndef PPFS_ENC_MODE
#define PPFS_ENC_MODE 3 // ablation builds only: rs_wg.hpp MODE bits (remainder / codeword emission)
#endif
#ifndef PPFS_DEC_MODE
#define PPFS_DEC_MODE 7
#endif
#ifndef PPFS_ENC_NTST
#define PPFS_ENC_NTST 1
#endif
#ifndef PPFS_DEC_NTST
#define PPFS_DEC_NTST 1
#endif
#elif PPFS_T2 > 16
// pair workgroup path (16 < 2t <= 32, rs_pair.hpp): 128-thread workgroups, (WPC, NBUF) per CU.
// Single-buffered tiles let 6 (encode) / 4 (decode) workgroups share a CU: the chains are
// latency-bound, and more resident tiles beat the in-workgroup prefetch (measured at 2t = 32:
// encode 270 -> 197 us, decode 241 -> 206 us vs 3 double-buffered workgroups).  The column
// kernels of tools/ablations/rs_col.hpp are kept for ablation.
#ifndef PPFS_PAIR_ENC
#define PPFS_PAIR_ENC 6, 1
#endif
#ifndef PPFS_PAIR_DEC_RM
#define PPFS_PAIR_DEC_RM 1 // decode from c mod g (payload remainder ^ parity) where 2t = 32
#endif
#ifndef PPFS_PAIR_DEC
#define PPFS_PAIR_DEC 5, 1, 1, (PPFS_T2 == 32 && PPFS_PAIR_DEC_RM)
#endif
// encode into a codeword image (rs_pair_encode_img_kernel) where 16 | 2t; 0 = the window emission
#ifndef PPFS_PAIR_IMG
#define PPFS_PAIR_IMG 1
#endif
#ifndef PPFS_PAIR_IMG_NW
#define PPFS_PAIR_IMG_NW 4 // waves per workgroup (32 blocks each): 4 x 4 = 16 waves per CU, +1-2 % over 2
#endif
#ifndef PPFS_PAIR_IMG_WPC
#define PPFS_PAIR_IMG_WPC (PPFS_PAIR_IMG_NW == 4 ? 4 : 6)
#endif
// byte-slice kernels (rs_bs.hpp) for 2t = 32: one workgroup of PPFS_BS_NW waves per CU, each wave
// on its own 32-block tiles; PPFS_BS_ENC_NBUF image buffers per wave for encode (decode: 1)
#ifndef PPFS_PAIR_BS
#define PPFS_PAIR_BS 1
#endif
#ifndef PPFS_BS_NW
#define PPFS_BS_NW 8
#endif
#ifndef PPFS_BS_ENC_NW
#define PPFS_BS_ENC_NW 12 // 3 waves per SIMD (decode: PPFS_BS_NW = 8, LDS- and register-bound)
#endif
#ifndef PPFS_BS_ENC_NBUF
#define PPFS_BS_ENC_NBUF 1
#endif
#ifndef PPFS_BS_DEC_NBUF
#define PPFS_BS_DEC_NBUF 1 // 0 = register prefetch
#endif
#ifndef PPFS_BS_DEC_NTST
#define PPFS_BS_DEC_NTST 1 // non-temporal payload stores of the decode
#endif
constexpr bool PAIR_BS = PPFS_PAIR_BS && PPFS_T2 == 32;
constexpr bool PAIR_IMG = PPFS_PAIR_IMG && (PPFS_T2 % 16 == 0);
constexpr int PAIR_ENC_WPC = PAIR_IMG ? PPFS_PAIR_IMG_WPC : pair::wpc_of(PPFS_PAIR_ENC), PAIR_DEC_WPC = pair::wpc_of(PPFS_PAIR_DEC);
#endif
// 8 < 2t <= 16: lane-per-block kernels (rs_fast.hpp); the column path leaves half of its lanes on
// all-zero state columns there and measured slower on decode.  2t = 16
// encodes with the solo image kernel (rs_pair.hpp) over the same slicing tables.
#if PPFS_T2 > 8 && PPFS_T2 <= 16
#ifndef PPFS_SOLO_IMG
#define PPFS_SOLO_IMG 1
#endif
#ifndef PPFS_SOLO_NW
#define PPFS_SOLO_NW 2
#endif
#ifndef PPFS_SOLO_WPC
#define PPFS_SOLO_WPC 4
#endif
constexpr bool SOLO_IMG = PPFS_SOLO_IMG && PPFS_T2 == 16;
constexpr int SOLO_NW = PPFS_SOLO_NW, SOLO_WPC = PPFS_SOLO_WPC;
#endif

// pair decode grid: 1 = one workgroup per 64-block tile (workgroups dispatched in address order;
// 1-error decode 0.203 -> 0.190 ms per 2^20 blocks, clean decode unchanged: DESIGN.md 4.1b),
// 0 = persistent, PAIR_DEC_WPC per CU
#ifndef PPFS_PAIR_DEC_FULL
#define PPFS_PAIR_DEC_FULL 1
#endif

extern "C" hipError_t PPFS_CAT(ppfs_rs_fast_encode_t, PPFS_T2)(const uint8_t* d, uint8_t* r, uint64_t nb,
    const uint8_t* tab, hipStream_t s, [[maybe_unused]] uint32_t* ctr, [[maybe_unused]] uint32_t* ctr_clear)
{
#if PPFS_T2 <= 8
#if PPFS_WG_RP
    hipLaunchKernelGGL((wg::rs_wg_encode_rp_kernel<PPFS_T2, PPFS_WG_RP, PPFS_ENC_NTST>),
        dim3(rs_tile_grid(nb, PPFS_WG_RP)), dim3(256), 0, s, d, r, nb, tab);
#elif PPFS_WG_DYN & 1
    hipLaunchKernelGGL((wg::rs_wg_encode_dyn_kernel<PPFS_T2, ENC_NBUF, ENC_WPC, PPFS_ENC_MODE, PPFS_ENC_NTST, (PPFS_WG_DYN & 4) != 0>),
        dim3(rs_tile_grid(nb, ENC_WPC)), dim3(320), 0, s, d, r, nb, tab, ctr); // the caller's counter set
#elif PPFS_WG_ENC_W8
    hipLaunchKernelGGL((wg::rs_wg_encode8_kernel<PPFS_T2, (PPFS_T2 > 6 ? 3 : PPFS_WG_ENC_W8), 2, PPFS_ENC_NTST>),
        dim3(rs_tile_grid(nb, 2)), dim3(512), 0, s, d, r, nb, tab);
#else
#if PPFS_WG_TKN
    if (ctr)
        hipLaunchKernelGGL((wg::rs_wg_encode_tkn_kernel<PPFS_T2, PPFS_WG_TKN, 2, PPFS_ENC_NTST>), dim3(rs_tile_grid(nb, 2)), dim3(256), 0,
            s, d, r, nb, tab, ctr);
    else
#endif
    if (PPFS_WG_WQ == 2 && ctr && ctr_clear)
        hipLaunchKernelGGL((wq::rs_wq_encode_kernel<PPFS_T2, 2, 3, 1, true>), dim3(rs_tile_grid(nb, 2, 4 * wq::QB)), dim3(256), 0,
            s, d, r, nb, tab, ctr, ctr_clear);
    else if (PPFS_WG_WQ)
        hipLaunchKernelGGL((wq::rs_wq_encode_kernel<PPFS_T2, PPFS_WQ_NBUF >= 3 ? 2 : 3, PPFS_WQ_NBUF, 1>),
            dim3(rs_tile_grid(nb, PPFS_WQ_NBUF >= 3 ? 2 : 3, 4 * wq::QB)), dim3(256), 0, s, d, r, nb, tab, nullptr, nullptr);
    else if ((PPFS_WG_TK & 1) && ctr && PPFS_ENC_MODE == 3 && !WG_FULL && !PPFS_WG_ENC_IMG && !(PPFS_WG_W1 & 1))
        hipLaunchKernelGGL((wg::rs_wg_encode_tk_kernel<PPFS_T2, 2, PPFS_ENC_NTST>), dim3(rs_tile_grid(nb, 2)), dim3(256), 0, s, d,
            r, nb, tab, ctr, ctr_clear);
    else if constexpr (PPFS_WG_W1 & 1)
        hipLaunchKernelGGL((w1::rs_w1_encode_kernel<PPFS_T2, PPFS_W1_NW, PPFS_W1_NBUF, PPFS_ENC_MODE, PPFS_ENC_NTST>),
            dim3(rs_tile_grid(nb, 1, w1::TB * PPFS_W1_NW)), dim3(64 * PPFS_W1_NW), 0, s, d, r, nb, tab);
    else if constexpr (PPFS_WG_ENC_IMG)
        hipLaunchKernelGGL((wg::rs_wg_encode_img_kernel<PPFS_T2, PPFS_WG_ENC_IMG_WPC, PPFS_ENC_NTST>),
            dim3(rs_tile_grid(nb, 1 << 24)), dim3(256), 0, s, d, r, nb, tab);
    else
        hipLaunchKernelGGL((wg::rs_wg_encode_kernel<PPFS_T2, ENC_NBUF, ENC_WPC, PPFS_ENC_MODE, PPFS_ENC_NTST, ENC_COMPACT>), dim3(rs_tile_grid(nb, WG_FULL ? (1 << 24) : ENC_WPC)), dim3(256),
            0, s, d, r, nb, tab);
#endif
#elif PPFS_T2 > 16
    if constexpr (PAIR_BS)
        hipLaunchKernelGGL((bs::rs_bs_encode_kernel<PPFS_T2, PPFS_BS_ENC_NW, PPFS_BS_ENC_NBUF>),
            dim3(rs_tile_grid(nb, 1, bs::TBW * PPFS_BS_ENC_NW)), dim3(64 * PPFS_BS_ENC_NW), 0, s, d, r, nb, tab, nullptr, nullptr);
    else if constexpr (PAIR_IMG)
        hipLaunchKernelGGL((pair::rs_pair_encode_img_kernel<PPFS_T2, PPFS_PAIR_IMG_WPC, PPFS_PAIR_IMG_NW>),
            dim3(rs_tile_grid(nb, PAIR_ENC_WPC, 32 * PPFS_PAIR_IMG_NW)), dim3(64 * PPFS_PAIR_IMG_NW), 0, s, d, r, nb, tab);
    else
        hipLaunchKernelGGL((pair::rs_pair_encode_kernel<PPFS_T2, PPFS_PAIR_ENC>), dim3(rs_tile_grid(nb, PAIR_ENC_WPC)),
            dim3(pair::NTHR), 0, s, d, r, nb, tab);
#else
    if constexpr (SOLO_IMG)
        hipLaunchKernelGGL((pair::rs_solo_encode_img_kernel<PPFS_T2, SOLO_WPC, SOLO_NW>),
            dim3(rs_tile_grid(nb, SOLO_WPC, 64 * SOLO_NW)), dim3(64 * SOLO_NW), 0, s, d, r, nb, tab);
    else
        hipLaunchKernelGGL(rs255_encode_kernel<PPFS_T2>, dim3(rs_grid(nb)), dim3(256), 0, s, d, r, nb, tab);
#endif
    return hipGetLastError();
}

extern "C" const char* PPFS_CAT(ppfs_rs_fast_path_t, PPFS_T2)()
{
#if PPFS_T2 <= 8
    // the ticket kernels (rs_wg_tk.hpp) when the caller hands a counter set, which every engine
    // context does for its first 16 streams
    return (PPFS_WG_W1 & 1) ? "rs255-w1-lds"
        : (PPFS_WG_TK & 3) == 3 ? "rs255-wg-tk-lds"
        : (PPFS_WG_TK & 1)      ? "rs255-wg-tkenc-lds"
                                : "rs255-wg-seg4-lds";
#elif PPFS_T2 > 16
    return PAIR_BS ? "rs255-bs-byte-lds" : "rs255-pair-nibble-lds";
#else
    return "rs255-slice8-lds";
#endif
}

extern "C" hipError_t PPFS_CAT(ppfs_rs_fast_decode_t, PPFS_T2)(uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb,
    const uint8_t* tab, int wb, hipStream_t s, [[maybe_unused]] uint32_t* ctr, [[maybe_unused]] uint32_t* ctr_clear,
    [[maybe_unused]] uint8_t* wb_dst)
{
#if PPFS_T2 <= 8
#if PPFS_WG_RP
    if (d)
        hipLaunchKernelGGL((wg::rs_wg_decode_rp_kernel<PPFS_T2, PPFS_WG_RP, PPFS_DEC_NTST, true>),
            dim3(rs_tile_grid(nb, PPFS_WG_RP)), dim3(256), 0, s, r, d, st, nb, tab, wb);
    else
        hipLaunchKernelGGL((wg::rs_wg_decode_rp_kernel<PPFS_T2, PPFS_WG_RP, PPFS_DEC_NTST, false>),
            dim3(rs_tile_grid(nb, PPFS_WG_RP)), dim3(256), 0, s, r, d, st, nb, tab, wb);
#else
    if ((PPFS_WG_TK & 2) && ctr && PPFS_DEC_MODE == 7 && !DEC_FULL && DEC_NBUF == 2 && DEC_WPC == 3 && !(PPFS_WG_W1 & 2))
        hipLaunchKernelGGL((wg::rs_wg_decode_tk_kernel<PPFS_T2, 3, PPFS_DEC_NTST>), dim3(rs_tile_grid(nb, 3)), dim3(256), 0, s,
            r, d, st, nb, tab, wb, ctr, ctr_clear, wb_dst);
    else if constexpr (PPFS_WG_W1 & 2)
        hipLaunchKernelGGL((w1::rs_w1_decode_kernel<PPFS_T2, PPFS_W1_DEC_NW, PPFS_W1_DEC_NBUF, PPFS_DEC_NTST>),
            dim3(rs_tile_grid(nb, 1, w1::TB * PPFS_W1_DEC_NW)), dim3(64 * PPFS_W1_DEC_NW), 0, s, r, d, st, nb, tab, wb);
    else
    hipLaunchKernelGGL((wg::rs_wg_decode_kernel<PPFS_T2, DEC_NBUF, DEC_WPC, PPFS_DEC_MODE, PPFS_DEC_NTST>), dim3(rs_tile_grid(nb, DEC_FULL ? (1 << 24) : DEC_WPC)), dim3(256),
        0, s, r, d, st, nb, tab, wb, wb_dst);
#endif
#elif PPFS_T2 > 16
    if constexpr (PAIR_BS)
        hipLaunchKernelGGL((bs::rs_bs_decode_kernel<PPFS_T2, PPFS_BS_NW, PPFS_BS_DEC_NBUF, PPFS_BS_DEC_NTST>), dim3(rs_tile_grid(nb, 1, bs::TBW * PPFS_BS_NW)),
            dim3(64 * PPFS_BS_NW), 0, s, r, d, st, nb, tab, wb, nullptr, nullptr);
    else
    hipLaunchKernelGGL((pair::rs_pair_decode_kernel<PPFS_T2, PPFS_PAIR_DEC>),
        dim3(rs_tile_grid(nb, PPFS_PAIR_DEC_FULL ? (1 << 24) : PAIR_DEC_WPC)),
        dim3(pair::NTHR), 0, s, r, d, st, nb, tab, wb);
#else
    hipLaunchKernelGGL(rs255_decode_kernel<PPFS_T2>, dim3(rs_grid(nb)), dim3(256), 0, s, r, d, st, nb, tab, wb);
#endif
    return hipGetLastError();
}
PPFS_DBG_ACCESSOR(PPFS_CAT(ppfs_dbg_faults_rs_t, PPFS_T2))

// resident small-batch servers (api.cpp server_call): 2t <= 8 rs_wg.hpp rs_wg_server_kernel,
// 2t > 16 rs_pair.hpp rs_pair_server_kernel
#if PPFS_T2 > 8 && PPFS_T2 <= 16
extern "C" hipError_t PPFS_CAT(ppfs_rs_server_launch_t, PPFS_T2)(ppfs::SrvBox* box, uint8_t* zc, uint64_t zc_bytes,
    const uint8_t* tab, uint32_t gen, uint32_t idle_us, hipStream_t s)
{
    hipLaunchKernelGGL((rs255_server_kernel<PPFS_T2>), dim3(1), dim3(64), 0, s, box, zc, zc_bytes, tab, gen, idle_us);
    return hipGetLastError();
}
#endif
#if PPFS_T2 > 16
extern "C" hipError_t PPFS_CAT(ppfs_rs_server_launch_t, PPFS_T2)(ppfs::SrvBox* box, uint8_t* zc, uint64_t zc_bytes,
    const uint8_t* tab, uint32_t gen, uint32_t idle_us, hipStream_t s)
{
    hipLaunchKernelGGL((pair::rs_pair_server_kernel<PPFS_T2, (PPFS_T2 == 32 && PPFS_PAIR_DEC_RM)>), dim3(1), dim3(pair::NTHR),
        0, s, box, zc, zc_bytes, tab, gen, idle_us);
    return hipGetLastError();
}
#endif
#if PPFS_T2 <= 8
extern "C" hipError_t PPFS_CAT(ppfs_rs_server_launch_t, PPFS_T2)(ppfs::SrvBox* box, uint8_t* zc, uint64_t zc_bytes,
    const uint8_t* tab, uint32_t gen, uint32_t idle_us, hipStream_t s)
{
    hipLaunchKernelGGL((wg::rs_wg_server_kernel<PPFS_T2>), dim3(1), dim3(256), 0, s, box, zc, zc_bytes, tab, gen, idle_us);
    return hipGetLastError();
}
#endif
