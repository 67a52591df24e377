// rs_wg_rp.hpp -- ABLATION ONLY (built with -DPPFS_WG_RP=N, tools/build_alt.sh): register-prefetch
// variants of the 2t <= 8 RS kernels of rs_wg.hpp.  Correct (the RS device tests pass with it) but
// 6 % slower in the bench step than the shipped DMA kernels (profiles/r2_ablations/rp4_*.jsonl,
// DESIGN.md 4.1): the compiler's vmcnt waits on the register tiles end up covering both sets.
#pragma once
#include "rs_wg.hpp"

namespace ppfs {
namespace wg {

// ------------------------------------------------------------------------------------
// Register-prefetch variants (persistent grid, ONE LDS tile buffer, two tiles in flight in VGPRs).
// The double-buffered kernels above hold one tile in flight per workgroup, and LDS capacity caps
// that at 4 x 16 KiB per CU -- their memory skeleton alone runs 12 % behind a full-grid copy from
// HBM.  Here the tiles a workgroup will compute two and one iterations later are
// loaded into registers (16 VGPRs each: 4 x 16 B per thread), so every tile has two iterations of
// latency budget, and the single LDS buffer is filled from the registers (4 ds_write_b128 per
// thread) right before its tile is computed.  The loop is unrolled by two so the two register
// sets alternate roles without moves (a move would force the wait a whole iteration early).
// Emission pieces are computed and stored one at a time (few live registers).
// ------------------------------------------------------------------------------------
// One register tile: four 16-byte pieces per thread.  Native vector fields: HIP's uint4 is a
// struct whose copies lower to memcpy, which kept the tiles in scratch.
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
struct RTile {
    v4u32 v0, v1, v2, v3;
};

template <int NPIECE>
__device__ __forceinline__ void rp_load(RTile& R, const uint8_t* __restrict__ src, uint32_t tid)
{
    static_assert(NPIECE > 768 && NPIECE <= 1024, "four pieces per thread");
    const v4u32* s = (const v4u32*)src + tid;
    R.v0 = s[0];
    R.v1 = s[256];
    R.v2 = s[512];
    // Lanes past the tile's last piece re-read that piece: every load is unconditional, so the
    // compiler's wait counts do not fall back to the no-load path (which serialised the prefetch).
    R.v3 = ((const v4u32*)src)[min(tid + 768u, (uint32_t)NPIECE - 1u)];
}

template <int NPIECE> __device__ __forceinline__ void rp_store(uint8_t* dst, const RTile& R, uint32_t tid)
{
    v4u32* d = (v4u32*)dst + tid;
    d[0] = R.v0;
    d[256] = R.v1;
    d[512] = R.v2;
    ((v4u32*)dst)[min(tid + 768u, (uint32_t)NPIECE - 1u)] = R.v3; // duplicates write equal bytes
}

template <int T2, int WPC = 4, int NTST = 1>
__global__ __launch_bounds__(256, WPC) void rs_wg_encode_rp_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, const uint8_t* __restrict__ tables)
{
    using L = RsWgLayout<T2>;
    using D = Lds<T2, false, 1>;
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
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB, G = gridDim.x;
    const uint32_t buf = D::OFF_BUF;
    uint64_t t = blockIdx.x;
    uint32_t pc = 0;
    RTile R0, R1; // register sets: tiles t and t + G (alternating roles)
    // Prefetches past the last full tile re-read that tile (unused): loads stay unconditional.
    const uint64_t tlast = nfull ? nfull - 1 : 0;
    if (t < nfull) {
        rp_load<IN_PIECES>(R0, data + t * (TB * K), tid);
        asm volatile("" ::: "memory"); // all of R0's loads issue before R1's (in-loop wait counts)
        rp_load<IN_PIECES>(R1, data + min(t + G, tlast) * (TB * K), tid);
    }
    auto step = [&](RTile& R) {
        rp_store<IN_PIECES>(lds + buf + PAD, R, tid); // waits for this set's loads only
        barrier_lds(); // A: tile t in LDS
        rp_load<IN_PIECES>(R, data + min(t + 2 * G, tlast) * (TB * K), tid);
        const uint32_t par = D::OFF_PAR + pc * 512u;
        if (wave == 0)
            *(uint64_t*)(lds + D::OFF_PAR + (pc ^ 1u) * 512u + 8u * lane) = 0;
        phase_remainder<T2, K>(lds, buf, par, wave, row);
        barrier_lds(); // B: parity slots complete
        uint8_t* dst = raw + t * (TB * 255);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            // lanes past the last piece redo it (equal bytes): the store stays unconditional
            uint32_t p = k < 3 ? tid + 256u * k : min(tid + 768u, (uint32_t)OUT_PIECES - 1u);
            asm volatile("" : "+v"(p)); // this piece's index maths starts after the last store
            const uint4 o = enc_piece<T2>(lds, buf, par, p);
            st_nt<NTST>(dst + 16u * p, o);
            asm volatile("" ::: "memory");
        }
        barrier_lds(); // C: the buffer is free for the next tile
        pc ^= 1u;
        t += G;
    };
    // The first step is peeled so that the loop is entered in the steady-state order of memory
    // operations (R1 loads, stores, R0 loads, stores): the compiler's wait counts at the loop
    // head are the minimum over its entry paths, and an un-peeled entry (R0 loads, R1 loads)
    // made every iteration wait for both register sets.
    if (t < nfull) {
        step(R0);
        while (t < nfull) {
            step(R1);
            if (t >= nfull)
                break;
            step(R0);
        }
    }
    if (t == nfull && nfull < ntiles) {
        const uint32_t nb = (uint32_t)(nblocks - t * TB), par = D::OFF_PAR + pc * 512u;
        stage_bytes(lds + buf + PAD, data + t * (TB * K), nb * K, tid);
        barrier_lds();
        phase_remainder<T2, K>(lds, buf, par, wave, row);
        barrier_lds();
        uint8_t* dst = raw + t * (TB * 255);
        const uint32_t nout = nb * 255u;
        for (uint32_t p = tid; 16u * p < nout; p += NTHR) {
            const uint4 v = enc_piece<T2>(lds, buf, par, p);
            if (16u * p + 16u <= nout)
                *(uint4*)(dst + 16u * p) = v;
            else
                st_bytes(dst + 16u * p, v, nout - 16u * p);
        }
    }
}

template <int T2, int WPC = 4, int NTST = 1, bool WANT = true>
__global__ __launch_bounds__(256, WPC) void rs_wg_decode_rp_kernel(uint8_t* __restrict__ raw,
    uint8_t* __restrict__ data, uint8_t* __restrict__ status, uint64_t nblocks, const uint8_t* __restrict__ tables,
    int write_back)
{
    using L = RsWgLayout<T2>;
    using D = Lds<T2, true, 1>;
    constexpr int LDS_ALLOC = lds_alloc<D::BYTES, WPC>();
    static_assert(WPC * LDS_ALLOC <= 163840, "LDS for WPC workgroups per CU");
    constexpr int K = L::K;
    constexpr int IN_PIECES = TB * 255 / 16; // 1020
    constexpr int OUT_PIECES = TB * K / 16;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALLOC];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = wave_id();
    const uint32_t row = lane_row(lane);
    const bool wb = write_back != 0; // WANT == (data != nullptr): decided at launch, so the wait counts see one path
    for (uint32_t p = tid; p < (uint32_t)D::TBL / 16; p += NTHR)
        *(uint4*)(lds + 16 * p) = *(const uint4*)(tables + 16 * p);
    if (tid < 128)
        *(uint64_t*)(lds + D::OFF_PAR + 8 * tid) = 0;
    const uint64_t nfull = nblocks / TB, ntiles = (nblocks + TB - 1) / TB, G = gridDim.x;
    const uint32_t buf = D::OFF_BUF;
    uint64_t t = blockIdx.x;
    uint32_t pc = 0;
    RTile R0, R1;
    const uint64_t tlast = nfull ? nfull - 1 : 0;
    if (t < nfull) {
        rp_load<IN_PIECES>(R0, raw + t * (TB * 255), tid);
        asm volatile("" ::: "memory"); // all of R0's loads issue before R1's (in-loop wait counts)
        rp_load<IN_PIECES>(R1, raw + min(t + G, tlast) * (TB * 255), tid);
    }
    auto step = [&](RTile& R) {
        rp_store<IN_PIECES>(lds + buf + PAD, R, tid);
        barrier_lds(); // A: tile t in LDS
        rp_load<IN_PIECES>(R, raw + min(t + 2 * G, tlast) * (TB * 255), tid);
        const uint32_t par = D::OFF_PAR + pc * 512u;
        if (wave == 0)
            *(uint64_t*)(lds + D::OFF_PAR + (pc ^ 1u) * 512u + 8u * lane) = 0;
        phase_remainder<T2, 255>(lds, buf, par, wave, row);
        barrier_lds(); // B: remainders complete
        if (wave == 0) {
            const uint32_t st = phase_correct<T2>(lds, buf, par, row, true, raw, t * TB + row, wb, nblocks * 255u);
            if (status)
                status[t * TB + row] = (uint8_t)st;
        }
        barrier_lds(); // C: corrections patched into the LDS rows
        if (WANT) {
            uint8_t* dst = data + t * (TB * K);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t p = k < 3 ? tid + 256u * k : min(tid + 768u, (uint32_t)OUT_PIECES - 1u);
                asm volatile("" : "+v"(p));
                const uint4 o = dec_piece<T2>(lds, buf, p);
                st_nt<NTST>(dst + 16u * p, o);
                asm volatile("" ::: "memory");
            }
        }
        barrier_lds(); // D: the buffer is free for the next tile
        pc ^= 1u;
        t += G;
    };
    // The first step is peeled so that the loop is entered in the steady-state order of memory
    // operations (R1 loads, stores, R0 loads, stores): the compiler's wait counts at the loop
    // head are the minimum over its entry paths, and an un-peeled entry (R0 loads, R1 loads)
    // made every iteration wait for both register sets.
    if (t < nfull) {
        step(R0);
        while (t < nfull) {
            step(R1);
            if (t >= nfull)
                break;
            step(R0);
        }
    }
    if (t == nfull && nfull < ntiles) {
        const uint32_t nb = (uint32_t)(nblocks - t * TB), par = D::OFF_PAR + pc * 512u;
        stage_bytes(lds + buf + PAD, raw + t * (TB * 255), nb * 255u, tid);
        barrier_lds();
        phase_remainder<T2, 255>(lds, buf, par, wave, row);
        barrier_lds();
        if (wave == 0) {
            const bool valid = row < nb;
            const uint32_t st = phase_correct<T2>(lds, buf, par, row, valid, raw, t * TB + row, wb, nblocks * 255u);
            if (status && valid)
                status[t * TB + row] = (uint8_t)st;
        }
        barrier_lds();
        if (WANT) {
            uint8_t* dst = data + t * (TB * K);
            const uint32_t nout = nb * (uint32_t)K;
            for (uint32_t p = tid; 16u * p < nout; p += NTHR) {
                const uint4 v = dec_piece<T2>(lds, buf, p);
                if (16u * p + 16u <= nout)
                    *(uint4*)(dst + 16u * p) = v;
                else
                    st_bytes(dst + 16u * p, v, nout - 16u * p);
            }
        }
    }
}

} // namespace wg
} // namespace ppfs
