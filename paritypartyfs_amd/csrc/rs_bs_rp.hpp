#pragma once
// rs_bs_rp.hpp -- RS(255,223) (2t = 32, cfg5) decode with the codeword rows in registers (round 5).
//
// Reference semantics as rs_bs.hpp rs_bs_decode_kernel (rs_block_device.cpp:119-183, 210-280):
// c mod g per block, a single error confirmed against the x^p mod g row, else the reference's
// BM / root search over all 255 values / Forney; status 0 / 1; write-back of every corrected byte.
//
// rs_bs_decode_kernel keeps a wave's 32-block tile in its LDS image for the whole iteration: the
// remainder chain reads every 8-byte chunk from the image (two 2-way ds_read_b32 per step, a fifth
// of the chain's LDS cycles), the corrections patch the image, the emission reads it back, and the
// next tile arrives through registers (register prefetch + 8 ds_write_b128).  The decode is bound by
// the LDS (~75 % of its cycles).  Here:
//   - a lane copies its bytes out of the image once per tile (lane c of block b's pair: parity
//     bytes [16c, +16) = its column of the stored parity, payload bytes [112c, +112)), 34 dword
//     reads, and the next tile's LDS-DMA is issued right after into the same image;
//   - the chain takes each chunk from the owner lane's registers by a DPP broadcast within the
//     pair (no image reads), the state fold as in rs_bs.hpp;
//   - a single error is patched in the owner lane's registers (and written back to HBM);
//   - the payload leaves straight from the registers: lane c stores its 112 (111) bytes at the
//     223-byte row stride, 16 bytes at a time;
//   - blocks with 2+ errors (or a miscorrection pattern) take the general path after the emission
//     (after a vmcnt(0), so the patch stores land after the row stores): lane 0 of the pair runs
//     the reference BM / roots / Forney and patches the emitted payload byte and, with write-back,
//     the codeword byte in HBM (read back from HBM: no other path has written that block).
#include "rs_bs.hpp"

namespace ppfs {
namespace bs {

// A lane's bytes of its block: parity [16c, 16c+16) in par, payload [112c, 112c+112) in P (c = 1:
// payload bytes 112..222 and one byte past the payload, never used)
struct RpRow {
    uint32_t par[4];
    uint32_t P[28];
};

// the value of lane 0 / lane 1 of the pair, in both lanes (quad_perm [0,0,2,2] / [1,1,3,3])
__device__ __forceinline__ uint32_t bc0(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xA0, 0xF, 0xF, true); }
__device__ __forceinline__ uint32_t bc1(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xF5, 0xF, 0xF, true); }

// copy the lane's bytes out of the image row (row: LDS byte of the block's codeword byte 0; the
// reads may run up to 5 bytes past the row: the next row or the image slack)
__device__ __forceinline__ void rp_load(RpRow& R, const uint8_t* lds, uint32_t row, uint32_t c)
{
    const uint32_t sh = (row & 3u) * 8u;
    const uint32_t* wp = (const uint32_t*)(lds + ((row + 16u * c) & ~3u));
    uint32_t d[5];
#pragma unroll
    for (int m = 0; m < 5; ++m)
        d[m] = wp[m];
#pragma unroll
    for (int m = 0; m < 4; ++m)
        R.par[m] = __builtin_amdgcn_alignbit(d[m + 1], d[m], sh);
    const uint32_t* wq = (const uint32_t*)(lds + ((row + 32u + 112u * c) & ~3u));
    uint32_t e[29];
#pragma unroll
    for (int m = 0; m < 29; ++m)
        e[m] = wq[m];
#pragma unroll
    for (int m = 0; m < 28; ++m)
        R.P[m] = __builtin_amdgcn_alignbit(e[m + 1], e[m], sh);
}

// c mod g of the block from the registers: payload chunk j (bytes [8j, 8j+8)) is in lane j >= 14
// (P[2 (j - 14 c)], P[2 (j - 14 c) + 1]); the top chunk j = 27 holds 7 bytes
__device__ __forceinline__ void rp_cmodg(uint32_t (&s)[4], const RpRow& R, const uint8_t* lds, const BsLane& L)
{
    uint32_t cm = L.c ? ~0u : 0u;
    asm("" : "+v"(cm));
    s[0] = s[1] = s[2] = s[3] = 0;
    bs_lookups(s, lds, L, bc1(R.P[26]), bc1(R.P[27] & 0x00FFFFFFu));
#pragma unroll
    for (int j = 26; j >= 0; --j) {
        uint32_t lo, hi;
        if (j >= 14) { // chunk and the state's top 8 bytes both in lane 1
            lo = bc1(R.P[2 * (j - 14)] ^ s[2]);
            hi = bc1(R.P[2 * (j - 14) + 1] ^ s[3]);
        } else {
            lo = bc0(R.P[2 * j]) ^ bc1(s[2]);
            hi = bc0(R.P[2 * j + 1]) ^ bc1(s[3]);
        }
        uint32_t n[4] = { bc0(s[2]) & cm, bc0(s[3]) & cm, s[0], s[1] }; // state * x^8
        bs_lookups(n, lds, L, lo, hi);
        s[0] = n[0];
        s[1] = n[1];
        s[2] = n[2];
        s[3] = n[3];
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
        s[m] ^= R.par[m]; // + the stored parity (column c)
}

// Codeword byte pos ^= ev in the lane that holds it (both lanes of the pair call with the same
// pos / ev) and, with write-back, in HBM (rs_block_device.cpp:165-180)
__device__ __forceinline__ void rp_fix(RpRow& R, uint32_t c, uint32_t pos, uint32_t ev, uint8_t* __restrict__ raw_g,
    uint64_t gblk, bool wb, [[maybe_unused]] uint64_t raw_bytes)
{
    if (ev == 0)
        return;
    const bool inpar = pos < 32u;
    const uint32_t q = pos - 32u; // payload byte (pos >= 32)
    const bool mine = inpar ? (pos >> 4) == c : (q >= 112u) == (c != 0u);
    const uint32_t idx = inpar ? (pos & 15u) >> 2 : (q - 112u * c) >> 2;
    const uint32_t mask = ev << (8u * (pos & 3u));
    uint32_t fixed = 0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const bool hit = mine && inpar && (uint32_t)m == idx;
        R.par[m] ^= hit ? mask : 0u;
        fixed = hit ? R.par[m] : fixed;
    }
#pragma unroll
    for (int m = 0; m < 28; ++m) {
        const bool hit = mine && !inpar && (uint32_t)m == idx;
        R.P[m] ^= hit ? mask : 0u;
        fixed = hit ? R.P[m] : fixed;
    }
    if (mine && wb && PPFS_DBG_OK(raw_g + gblk * 255u + pos, 1, raw_g, raw_bytes))
        wb_byte(raw_g + gblk * 255u + pos, (uint8_t)(fixed >> (8u * (pos & 3u))));
}

// Single-error correction (bs_correct's S12 / XP-row test) into the registers; general = the
// pair needs the general path (2+ errors or a non-single-error pattern)
template <int T2>
__device__ __forceinline__ uint32_t rp_correct(RpRow& R, const uint8_t* gfp, const uint8_t* s12p, const uint8_t* __restrict__ xp,
    uint32_t c, const uint32_t (&s)[4], bool valid, uint8_t* __restrict__ raw_g, uint64_t gblk, bool wb, uint64_t raw_bytes,
    bool& general)
{
    general = false;
    const bool err = valid && pair::pair_or<1>(s[0] | s[1] | s[2] | s[3]) != 0u;
    if (!__builtin_amdgcn_ballot_w64(err))
        return 0u;
    const Gf gf { gfp };
    const uint16_t* t = (const uint16_t*)(s12p + 8192u * c); // state byte u = 16c + k
    uint32_t s12 = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k)
        s12 ^= t[256 * k + ((s[k >> 2] >> (8 * (k & 3))) & 0xFFu)];
    s12 ^= pair::pair_xchg<1>(s12);
    const uint32_t s1 = s12 & 0xFFu, s2 = s12 >> 8;
    const uint32_t l1 = gf.log(s1), l2 = gf.log(s2);
    uint32_t lx = l2 + 255u - l1;
    lx = lx >= 255u ? lx - 255u : lx;
    uint32_t le = l1 + 255u - lx;
    le = le >= 255u ? le - 255u : le;
    const uint4 xr = *(const uint4*)(xp + 32u * lx + 16u * c);
    const uint32_t xw[4] = { xr.x, xr.y, xr.z, xr.w };
    uint32_t bad = (s1 == 0u || s2 == 0u) ? 1u : 0u;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t x = (xw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const uint32_t rb = (s[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const uint32_t ev = x == 0xFFu ? 0u : gf.exp(le + x);
        bad |= ev != rb ? 1u : 0u;
    }
    const bool geo = err && pair::pair_or<1>(bad) == 0u;
    if (geo)
        rp_fix(R, c, lx, gf.exp(le), raw_g, gblk, wb, raw_bytes);
    general = err && !geo;
    return err ? 1u : 0u;
}

// General correction (2+ errors), out of line, after the row's emission has completed: both lanes
// compute half of S_1..S_32 over the c mod g state (bs_correct_general), lane 0 runs the reference
// BM / roots / Forney and patches codeword byte pos: the emitted payload byte (pos >= 32) and, with
// write-back, the HBM codeword byte (read back: nothing else has written this block)
template <int T2>
__device__ __noinline__ void rp_correct_general(const uint8_t* gfp, uint32_t c, uint32_t s0, uint32_t s1, uint32_t s2,
    uint32_t s3, uint8_t* __restrict__ raw_g, uint8_t* __restrict__ data, uint64_t gblk, bool wb,
    [[maybe_unused]] uint64_t raw_bytes, [[maybe_unused]] uint64_t data_bytes)
{
    static_assert(T2 == 32, "state byte q = coefficient q");
    constexpr uint32_t K = 255u - T2;
    const Gf gf { gfp };
    const uint32_t own[4] = { s0, s1, s2, s3 };
    uint32_t rw[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t p = pair::pair_xchg<1>(own[k]);
        rw[k] = c ? p : own[k];
        rw[4 + k] = c ? own[k] : p;
    }
    uint32_t sw[4] = { 0u, 0u, 0u, 0u };
#pragma unroll
    for (int ii = 0; ii < 16; ++ii) {
        const uint32_t i = 16u * c + 1u + (uint32_t)ii;
        uint32_t e = 0, sacc = 0;
#pragma unroll
        for (int q = 0; q < T2; ++q) {
            const uint32_t rv = (rw[q >> 2] >> (8 * (q & 3))) & 0xFFu;
            const uint32_t v = gf.exp(gf.log(rv) + e);
            sacc ^= rv ? v : 0u;
            e += i;
            e = e >= 255u ? e - 255u : e;
        }
        sw[ii >> 2] |= sacc << (8 * (ii & 3));
    }
    uint32_t hi[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        hi[k] = pair::pair_xchg<1>(sw[k]); // lane 0: S_17..S_32 from lane 1
    if (c == 0) {
        uint32_t S[T2];
#pragma unroll
        for (int i = 0; i < T2; ++i)
            S[i] = ((i < 16 ? sw[i >> 2] : hi[(i - 16) >> 2]) >> (8 * (i & 3))) & 0xFFu;
        rs_correct_general<T2>(S, gf, [&](uint32_t pos, uint32_t ev) {
            if (ev == 0)
                return;
            uint8_t* rp = raw_g + gblk * 255u + pos;
            if (!PPFS_DBG_OK(rp, 1, raw_g, raw_bytes))
                return;
            const uint8_t fixed = (uint8_t)(*rp ^ ev);
            if (wb)
                wb_byte(rp, fixed);
            if (data && pos >= (uint32_t)T2 && PPFS_DBG_OK(data + gblk * K + (pos - T2), 1, data, data_bytes))
                data[gblk * K + (pos - T2)] = fixed;
        });
    }
}

// the lane's 112 (c = 1: 111) payload bytes at dst (any alignment)
template <int NTST>
__device__ __forceinline__ void rp_emit(uint8_t* dst, const RpRow& R, uint32_t c)
{
#pragma unroll
    for (int i = 0; i < 6; ++i)
        st_nt<NTST>(dst + 16 * i, make_uint4(R.P[4 * i], R.P[4 * i + 1], R.P[4 * i + 2], R.P[4 * i + 3]));
    if (c == 0) {
        st_nt<NTST>(dst + 96, make_uint4(R.P[24], R.P[25], R.P[26], R.P[27]));
    } else {
        *(uint2*)(dst + 96) = make_uint2(R.P[24], R.P[25]);
        *(uint32_t*)(dst + 104) = R.P[26];
        *(uint16_t*)(dst + 108) = (uint16_t)R.P[27];
        dst[110] = (uint8_t)(R.P[27] >> 16);
    }
}

// Decode with status and write-back (rs_bs_decode_kernel's interface): workgroup b's wave w takes
// the 32-block wave tiles b NW + w + j S (S = grid NW); LDS as rs_bs_decode_kernel's NBUF = 1 plan
template <int T2, int NW, int NTST = 1, int TLDS = 3>
__global__ __launch_bounds__(64 * NW, 1) void rs_bs_decode_rp_kernel(uint8_t* __restrict__ raw,
    uint8_t* __restrict__ data, uint8_t* __restrict__ status, uint64_t nblocks, const uint8_t* __restrict__ tables,
    int write_back)
{
    static_assert(T2 == 32, "byte-slice path: 2t = 32");
    using L = RsPairLayout<T2>;
    using D = BsLds<NW, 1, true, TLDS>;
    constexpr int K = L::K;
    __shared__ __attribute__((aligned(16))) uint8_t lds[D::BYTES];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    for (uint32_t p = tid; p < (uint32_t)TAB_BYTES / 16; p += 64u * NW)
        *(uint4*)(lds + OFF_TAB + 16 * p) = *(const uint4*)(tables + L::OFF_BS + 16 * p);
    if constexpr (D::GF_IN)
        for (uint32_t p = tid; p < (uint32_t)GF_BYTES / 16; p += 64u * NW)
            *(uint4*)(lds + D::OFF_GF + 16 * p) = *(const uint4*)(tables + L::OFF_GF + 16 * p);
    if constexpr (D::S12_IN)
        for (uint32_t p = tid; p < (uint32_t)L::S12_BYTES / 16; p += 64u * NW)
            *(uint4*)(lds + D::OFF_S12 + 16 * p) = *(const uint4*)(tables + L::OFF_S12 + 16 * p);
    if constexpr (D::XP_IN)
        for (uint32_t p = tid; p < 255u * 2u; p += 64u * NW)
            *(uint4*)(lds + D::OFF_XP + 16 * p) = *(const uint4*)(tables + L::OFF_XPM + 16 * p);
    __syncthreads();
    const uint8_t* const gfp = D::GF_IN ? lds + D::OFF_GF : tables + L::OFF_GF;
    const uint8_t* const s12p = D::S12_IN ? lds + D::OFF_S12 : tables + L::OFF_S12;
    const uint8_t* const xpm = D::XP_IN ? lds + D::OFF_XP : tables + L::OFF_XPM;
    const BsLane Ln = bs_lane(lane);
    const bool wb = write_back != 0, want = data != nullptr;
    const uint32_t img = D::OFF_IMG + wave * (uint32_t)IMGW;
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(lds + img));
    const uint32_t row = img + 255u * Ln.blk;
    const uint64_t nfull = nblocks / TBW, ntiles = (nblocks + TBW - 1) / TBW;
    const uint64_t S = (uint64_t)gridDim.x * NW;
    const uint64_t raw_bytes = nblocks * 255u, data_bytes = nblocks * (uint64_t)K;
    uint64_t t = (uint64_t)blockIdx.x * NW + wave;
    auto src_off = [](uint32_t i) { return (int)(16u * i); };

    // one tile from the image: rows into registers, (next DMA), chain, corrections, status, emission,
    // general path; nb valid blocks
    auto tile = [&](uint64_t tt, uint32_t nb, bool next_dma) {
        RpRow R;
        rp_load(R, lds, row, Ln.c);
        if (next_dma) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the image is read: free for the next tile
            dma_wave(base, raw + (tt + S) * (TBW * 255), lane, src_off, raw, raw_bytes);
        }
        uint32_t s[4];
        rp_cmodg(s, R, lds, Ln);
        const bool valid = Ln.blk < nb;
        const uint64_t gblk = tt * TBW + Ln.blk;
        bool general = false;
        const uint32_t st = rp_correct<T2>(R, gfp, s12p, xpm, Ln.c, s, valid, raw, gblk, wb, raw_bytes, general);
        if (status && valid && Ln.c == 0 && PPFS_DBG_OK(status + gblk, 1, status, nblocks))
            status[gblk] = (uint8_t)st;
        if (want && valid && PPFS_DBG_OK(data + gblk * K + 112u * Ln.c, 112u - Ln.c, data, data_bytes))
            rp_emit<NTST>(data + gblk * K + 112u * Ln.c, R, Ln.c);
        if (__builtin_amdgcn_ballot_w64(general)) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // the row stores land before the patches
            if (general)
                rp_correct_general<T2>(gfp, Ln.c, s[0], s[1], s[2], s[3], raw, data, gblk, wb, raw_bytes, data_bytes);
        }
    };

    if (t < nfull)
        dma_wave(base, raw + t * (TBW * 255), lane, src_off, raw, raw_bytes);
    bool first = true;
    for (; t < nfull; t += S) {
        // this tile's DMA was issued before the previous tile's emission: at least 6 row-store
        // wave-instructions are younger than it (vector-memory operations complete in issue order)
        if (first || !want)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        first = false;
        tile(t, TBW, t + S < nfull);
    }
    if (t == nfull && nfull < ntiles) {
        // the one partial tile (nblocks % 32 blocks), staged byte by byte into the image
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t nb = (uint32_t)(nblocks - t * TBW);
        const uint8_t* src = raw + t * (TBW * 255);
        if (!PPFS_DBG_OK(src, nb * 255u, raw, raw_bytes))
            return;
        for (uint32_t j = lane; j < nb * 255u; j += 64u)
            lds[img + j] = src[j];
        wave_fence();
        tile(t, nb, false);
    }
}

} // namespace bs
} // namespace ppfs
