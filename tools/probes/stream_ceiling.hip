// stream_ceiling.hip -- diagnostic build (not shipped): the HBM ceilings the cfg4 streaming kernels
// (bit_fast.hip: one wave per 4 KiB block, lane l loads pieces 64k + l) can reach with no coding
// work, so that the CRC check / Hamming decode (read-mostly) and the CRC / Hamming encode (read +
// write) can be quoted against what the memory system delivers for their shape, not only 8 TB/s.
//   ro_wave<NT,BPW,WGW>  read-only: a wave reads BPW whole 4 KiB blocks (all loads in flight), XORs
//                        them; a store only on an impossible value (nothing is written)
//   ro_wave_st<...>      the same plus one status byte per block (the CRC check's output)
//   ro_flat<NT>          grid-stride 4 x 16 B per thread, 8 workgroups of 256 per CU
//   cp_wave<NTL,NTS>     copy: a wave per block, 4 x 16 B in, 4 x 16 B out (the encode's shape)
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/stream_ceiling.hip -o tools/stream_ceiling.bin
// usage: stream_ceiling [blocks=1048576] [reps=20]   (one JSON line per variant)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));             \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

template <bool NT> __device__ __forceinline__ u32x4 ld(const u32x4* p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

template <bool NT, int BPW, int WGW, bool ST>
__global__ __launch_bounds__(64 * WGW) void ro_wave(const u32x4* __restrict__ in, uint8_t* __restrict__ out, uint32_t nblk)
{
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t b0 = (blockIdx.x * WGW + w) * BPW;
    u32x4 v[BPW][4];
#pragma unroll
    for (int b = 0; b < BPW; ++b)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v[b][k] = (b0 + b < nblk) ? ld<NT>(in + (size_t)(b0 + b) * 256 + 64 * k + lane) : u32x4 { 0, 0, 0, 0 };
#pragma unroll
    for (int b = 0; b < BPW; ++b) {
        uint32_t a = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            a ^= v[b][k].x ^ v[b][k].y ^ v[b][k].z ^ v[b][k].w;
        if (b0 + b < nblk) {
            if constexpr (ST) {
                // one byte per block from lane 0 (its own XOR: no reduction, the status-byte traffic only)
                if (lane == 0)
                    out[b0 + b] = (uint8_t)(a & 1u);
            } else if (a == 0x9E3779B9u && lane == 63u) {
                out[b0 + b] = 1;
            }
        }
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void ro_flat(const u32x4* __restrict__ in, uint8_t* __restrict__ out, size_t n16)
{
    const size_t stride = (size_t)gridDim.x * 256 * 4;
    uint32_t a = 0;
    for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v[k] = i + 256 * k < n16 ? ld<NT>(in + i + 256 * k) : u32x4 { 0, 0, 0, 0 };
#pragma unroll
        for (int k = 0; k < 4; ++k)
            a ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (a == 0x9E3779B9u)
        out[blockIdx.x] = 1;
}

template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void cp_wave(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint32_t nblk)
{
    const uint32_t lane = threadIdx.x & 63u, blk = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (blk >= nblk)
        return;
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        v[k] = ld<NTL>(in + (size_t)blk * 256 + 64 * k + lane);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if constexpr (NTS)
            __builtin_nontemporal_store(v[k], out + (size_t)blk * 256 + 64 * k + lane);
        else
            out[(size_t)blk * 256 + 64 * k + lane] = v[k];
    }
}

// copy, one 16-B piece per thread (the flat full-grid shape), NTL: non-temporal loads
template <bool NTL>
__global__ __launch_bounds__(256) void cp_flat1(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n16)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16)
        __builtin_nontemporal_store(ld<NTL>(in + i), out + i);
}

// copy, a wave per block with WGW waves per workgroup; ILV: store piece k as soon as it lands
template <bool NTL, int WGW, bool ILV>
__global__ __launch_bounds__(64 * WGW) void cp_wave_w(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint32_t nblk)
{
    const uint32_t lane = threadIdx.x & 63u, blk = blockIdx.x * WGW + (threadIdx.x >> 6);
    if (blk >= nblk)
        return;
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        v[k] = ld<NTL>(in + (size_t)blk * 256 + 64 * k + lane);
    if constexpr (ILV) {
        u32x4* o = out + (size_t)blk * 256 + lane; // vmcnt(3 - k): piece k landed (stores count too)
        __builtin_amdgcn_s_waitcnt(0x3F73);
        __builtin_nontemporal_store(v[0], o);
        __builtin_amdgcn_s_waitcnt(0x3F73);
        __builtin_nontemporal_store(v[1], o + 64);
        __builtin_amdgcn_s_waitcnt(0x3F73);
        __builtin_nontemporal_store(v[2], o + 128);
        __builtin_amdgcn_s_waitcnt(0x3F73);
        __builtin_nontemporal_store(v[3], o + 192);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            __builtin_nontemporal_store(v[k], out + (size_t)blk * 256 + 64 * k + lane);
    }
}

// copy, persistent: each wave walks blocks blk, blk + W, ... (W = all waves of the grid)
template <bool NTL>
__global__ __launch_bounds__(256) void cp_persist(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint32_t nblk)
{
    const uint32_t lane = threadIdx.x & 63u, W = gridDim.x * 4;
    for (uint32_t blk = blockIdx.x * 4 + (threadIdx.x >> 6); blk < nblk; blk += W) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v[k] = ld<NTL>(in + (size_t)blk * 256 + 64 * k + lane);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            __builtin_nontemporal_store(v[k], out + (size_t)blk * 256 + 64 * k + lane);
    }
}

// copy, PPT pieces per thread strided by the workgroup (256 threads cover 4 KiB per instruction)
template <int PPT>
__global__ __launch_bounds__(256) void cp_flatn(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n16)
{
    const size_t i0 = (size_t)blockIdx.x * 256 * PPT + threadIdx.x;
    u32x4 v[PPT];
#pragma unroll
    for (int k = 0; k < PPT; ++k)
        v[k] = ld<true>(in + i0 + 256 * k);
#pragma unroll
    for (int k = 0; k < PPT; ++k)
        __builtin_nontemporal_store(v[k], out + i0 + 256 * k);
}

// copy, persistent waves drawing BPT-block tiles from per-XCD ticket counters (the t <= 4 RS
// kernels' walk): XCD xc = blockIdx.x mod 8 walks tiles j * 8 + xc; a wave's first tile is static,
// then one atomic per tile (taken a tile ahead); block 0 zeroes the other counter set for the next launch
template <int BPT>
__global__ __launch_bounds__(1024) void cp_ticket(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint32_t nblk,
    uint32_t* __restrict__ ctr, uint32_t* __restrict__ ctr_clear)
{
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t nx = gridDim.x < 8u ? gridDim.x : 8u, xc = blockIdx.x % nx, rank = blockIdx.x / nx;
    const uint32_t gx = (gridDim.x - xc + nx - 1u) / nx;
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (uint32_t x = 0; x < 8u; ++x)
            __hip_atomic_store(ctr_clear + 32u * x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t* const my = ctr + 32u * xc;
    const uint64_t G = (uint64_t)gx * nw;
    uint64_t j = (uint64_t)rank * nw + wave;
    const uint64_t ntiles = (nblk + BPT - 1) / BPT;
    for (;;) {
        const uint64_t tile = j * nx + xc;
        if (tile >= ntiles)
            break;
        uint32_t tk = 0;
        if (lane == 0)
            tk = atomicAdd(my, 1u);
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const uint64_t blk = tile * BPT + b;
            if (blk < nblk) {
                u32x4 v[4];
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    v[k] = ld<true>(in + blk * 256 + 64 * k + lane);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    __builtin_nontemporal_store(v[k], out + blk * 256 + 64 * k + lane);
            }
        }
        j = G + (uint64_t)__builtin_amdgcn_readfirstlane(tk);
    }
}

template <typename F> static double time_ms(F launch, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> t;
    for (int r = 0; r < reps + 3; ++r) {
        CK(hipEventRecord(a));
        launch();
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 3)
            t.push_back(ms);
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char** argv)
{
    const uint32_t nblk = argc > 1 ? (uint32_t)atoi(argv[1]) : 1u << 20;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const size_t bytes = (size_t)nblk * 4096;
    u32x4 *in = nullptr, *out = nullptr;
    uint8_t* st = nullptr;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&st, nblk + 4096));
    CK(hipMemset(in, 0x5A, bytes));
    CK(hipMemset(out, 0, bytes));
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto report = [&](const char* name, double ms, double moved) {
        const double gbs = moved / (ms * 1e-3) / 1e9;
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f, \"frac_8TBs\": %.4f}\n", name, ms, gbs, gbs / 8000.0);
        fflush(stdout);
    };
    const double rd = (double)bytes, rds = (double)bytes + nblk, cp = 2.0 * (double)bytes;
#define RO(NT, BPW, WGW, ST_)                                                                        \
    report("ro_wave nt=" #NT " bpw=" #BPW " wgw=" #WGW " st=" #ST_,                               \
        time_ms([&] { ro_wave<NT, BPW, WGW, ST_><<<(nblk + BPW * WGW - 1) / (BPW * WGW), 64 * WGW>>>(in, st, nblk); }, reps), \
        ST_ ? rds : rd)
    RO(false, 1, 4, false);
    RO(true, 1, 4, false);
    RO(false, 2, 4, false);
    RO(true, 2, 4, false);
    RO(false, 4, 4, false);
    RO(true, 4, 4, false);
    RO(false, 1, 16, false);
    RO(true, 1, 16, false);
    RO(false, 1, 4, true);
    RO(true, 1, 4, true);
    RO(true, 2, 4, true);
    RO(true, 4, 4, true);
    for (int g : { 8, 16, 32 }) {
        char nm[64];
        snprintf(nm, sizeof nm, "ro_flat nt=0 g=%d/CU", g);
        report(nm, time_ms([&] { ro_flat<false><<<cus * g, 256>>>(in, st, bytes / 16); }, reps), rd);
        snprintf(nm, sizeof nm, "ro_flat nt=1 g=%d/CU", g);
        report(nm, time_ms([&] { ro_flat<true><<<cus * g, 256>>>(in, st, bytes / 16); }, reps), rd);
    }
    report("cp_wave ntl=0 nts=1", time_ms([&] { cp_wave<false, true><<<(nblk + 3) / 4, 256>>>(in, out, nblk); }, reps), cp);
    report("cp_wave ntl=1 nts=1", time_ms([&] { cp_wave<true, true><<<(nblk + 3) / 4, 256>>>(in, out, nblk); }, reps), cp);
    report("cp_wave ntl=0 nts=0", time_ms([&] { cp_wave<false, false><<<(nblk + 3) / 4, 256>>>(in, out, nblk); }, reps), cp);
    report("cp_flat1 ntl=0", time_ms([&] { cp_flat1<false><<<(uint32_t)(bytes / 16 / 256), 256>>>(in, out, bytes / 16); }, reps), cp);
    report("cp_flat1 ntl=1", time_ms([&] { cp_flat1<true><<<(uint32_t)(bytes / 16 / 256), 256>>>(in, out, bytes / 16); }, reps), cp);
#define CW(NTL, WGW, ILV)                                                                             \
    report("cp_wave_w ntl=" #NTL " wgw=" #WGW " ilv=" #ILV,                                         \
        time_ms([&] { cp_wave_w<NTL, WGW, ILV><<<(nblk + WGW - 1) / WGW, 64 * WGW>>>(in, out, nblk); }, reps), cp)
    CW(true, 1, false);
    CW(true, 2, false);
    CW(true, 4, false);
    CW(true, 8, false);
    CW(true, 16, false);
    CW(true, 4, true);
    CW(false, 4, true);
    report("cp_flatn ppt=2", time_ms([&] { cp_flatn<2><<<(uint32_t)(bytes / 16 / 512), 256>>>(in, out, bytes / 16); }, reps), cp);
    report("cp_flatn ppt=4", time_ms([&] { cp_flatn<4><<<(uint32_t)(bytes / 16 / 1024), 256>>>(in, out, bytes / 16); }, reps), cp);
    for (int wpc : { 3, 4, 6 }) { // 256-thread workgroups per CU, capped by dynamic LDS
        char nm[64];
        const uint32_t lds = 160 * 1024 / wpc - 256;
        snprintf(nm, sizeof nm, "cp_wave_w ntl=1 wgw=4 wg/CU=%d", wpc);
        report(nm, time_ms([&] { cp_wave_w<true, 4, false><<<(nblk + 3) / 4, 256, lds>>>(in, out, nblk); }, reps), cp);
        snprintf(nm, sizeof nm, "cp_flat1 ntl=1 wg/CU=%d", wpc);
        report(nm, time_ms([&] { cp_flat1<true><<<(uint32_t)(bytes / 16 / 256), 256, lds>>>(in, out, bytes / 16); }, reps), cp);
    }
    for (int wpc : { 4, 6, 8, 10, 12, 16, 20 }) { // one-wave workgroups, waves per CU capped by LDS
        char nm[64];
        const uint32_t lds = 160 * 1024 / wpc - 256;
        snprintf(nm, sizeof nm, "cp_wave_w ntl=1 wgw=1 waves/CU=%d", wpc);
        report(nm, time_ms([&] { cp_wave_w<true, 1, false><<<nblk, 64, lds>>>(in, out, nblk); }, reps), cp);
        snprintf(nm, sizeof nm, "cp_wave_w ntl=0 wgw=1 waves/CU=%d", wpc);
        report(nm, time_ms([&] { cp_wave_w<false, 1, false><<<nblk, 64, lds>>>(in, out, nblk); }, reps), cp);
    }
    for (int wpc : { 8, 12, 16, 24 }) {
        char nm[64];
        const uint32_t lds = 160 * 1024 / wpc - 256;
        snprintf(nm, sizeof nm, "ro_wave nt=1 bpw=1 wgw=1 waves/CU=%d", wpc);
        report(nm, time_ms([&] { ro_wave<true, 1, 1, true><<<nblk, 64, lds>>>(in, st, nblk); }, reps), rds);
        snprintf(nm, sizeof nm, "ro_wave nt=0 bpw=1 wgw=1 waves/CU=%d", wpc);
        report(nm, time_ms([&] { ro_wave<false, 1, 1, true><<<nblk, 64, lds>>>(in, st, nblk); }, reps), rds);
    }
    {
        uint32_t* ctr = nullptr;
        CK(hipMalloc(&ctr, 2 * 8 * 32 * 4));
        CK(hipMemset(ctr, 0, 2 * 8 * 32 * 4));
        int it = 0;
        struct Shape { int threads, wg_per_cu; };
        for (Shape sh : { Shape { 1024, 1 }, Shape { 512, 2 }, Shape { 256, 4 }, Shape { 64, 16 }, Shape { 768, 1 }, Shape { 512, 1 },
                 Shape { 256, 3 }, Shape { 64, 12 }, Shape { 64, 8 } }) {
            for (int bpt : { 1, 4 }) {
                char nm[96];
                snprintf(nm, sizeof nm, "cp_ticket threads=%d wg/CU=%d bpt=%d", sh.threads, sh.wg_per_cu, bpt);
                const uint32_t grid = (uint32_t)(cus * sh.wg_per_cu);
                report(nm, time_ms([&] {
                    uint32_t* c0 = ctr + 256 * (it & 1);
                    uint32_t* c1 = ctr + 256 * ((it + 1) & 1);
                    ++it;
                    if (bpt == 1)
                        cp_ticket<1><<<grid, sh.threads>>>(in, out, nblk, c0, c1);
                    else
                        cp_ticket<4><<<grid, sh.threads>>>(in, out, nblk, c0, c1);
                }, reps), cp);
            }
        }
        CK(hipFree(ctr));
    }
    for (int g : { 4, 8, 16 }) {
        char nm[64];
        snprintf(nm, sizeof nm, "cp_persist ntl=1 g=%d/CU", g);
        report(nm, time_ms([&] { cp_persist<true><<<cus * g, 256>>>(in, out, nblk); }, reps), cp);
    }
    CK(hipDeviceSynchronize());
    CK(hipFree(in));
    CK(hipFree(out));
    CK(hipFree(st));
    return 0;
}
