// rs_ablate_dec.hip -- diagnostic build (not shipped): RS(255,249) decode staging variants timed
// in one process on real codewords carrying one byte error each (the bench workload); every
// variant's payload output is checked against the original data.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I paritypartyfs_amd/csrc -I include \
//     tools/probes/rs_ablate_dec.hip -o tools/rs_ablate_dec.bin
#include "../paritypartyfs_amd/csrc/api.cpp" // host table builders (same TU: anonymous namespace)
#include "rs_fast.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

// the rs_fast launchers api.cpp declares are not linked here; provide what api.cpp references
extern "C" {
int ppfs_rs_fast_supported(int, int) { return 0; }
int ppfs_rs_fast_tables_bytes(int t2) { return t2 <= 16 ? 4096 : 8192; }
hipError_t ppfs_rs_fast_encode(int, const uint8_t*, uint8_t*, uint64_t, const uint8_t*, hipStream_t) { return hipErrorInvalidValue; }
hipError_t ppfs_rs_fast_decode(int, uint8_t*, uint8_t*, uint8_t*, uint64_t, const uint8_t*, int, hipStream_t) { return hipErrorInvalidValue; }
hipError_t ppfs_rs_generic_encode(const uint8_t*, uint8_t*, uint64_t, int, int, const uint8_t*, hipStream_t) { return hipErrorInvalidValue; }
hipError_t ppfs_rs_generic_decode(uint8_t*, uint8_t*, uint8_t*, uint8_t*, uint64_t, int, int, int, const uint8_t*, hipStream_t) { return hipErrorInvalidValue; }
int ppfs_crc_tables_bytes(void) { return 0; }
hipError_t ppfs_crc_encode(const uint8_t*, uint8_t*, const uint8_t*, uint64_t, uint32_t, uint32_t, uint32_t, uint64_t, const uint8_t*, hipStream_t) { return hipErrorInvalidValue; }
hipError_t ppfs_crc_check(const uint8_t*, uint8_t*, uint8_t*, uint64_t, uint32_t, uint32_t, uint32_t, uint64_t, const uint8_t*, hipStream_t) { return hipErrorInvalidValue; }
hipError_t ppfs_ham_encode(const uint8_t*, uint8_t*, const uint8_t*, uint64_t, uint32_t, uint32_t, uint32_t, hipStream_t) { return hipErrorInvalidValue; }
hipError_t ppfs_ham_decode(uint8_t*, uint8_t*, uint8_t*, uint64_t, int, uint32_t, uint32_t, uint32_t, hipStream_t) { return hipErrorInvalidValue; }
hipError_t ppfs_parity_encode(const uint8_t*, uint8_t*, const uint8_t*, uint64_t, uint32_t, hipStream_t) { return hipErrorInvalidValue; }
hipError_t ppfs_parity_check(const uint8_t*, uint8_t*, uint8_t*, uint64_t, uint32_t, hipStream_t) { return hipErrorInvalidValue; }
}

using namespace ppfs;

struct Bufs {
    uint8_t *d, *cw, *bad, *out, *st, *tab;
    uint64_t nb;
    int grid;
    int grid1; // one wave per tile
};

__global__ void inject(uint8_t* cw, uint64_t nb)
{
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) {
        uint32_t h = (uint32_t)(b * 2654435761u) ^ 0x9E3779B9u;
        h ^= h >> 13;
        h *= 0x85EBCA6Bu;
        h ^= h >> 16;
        cw[b * 255 + (h % 255)] ^= (uint8_t)(1 + (h >> 8) % 255);
    }
}

static bool g_inject = true;
template <int STAGE, int NT = 1, int WB = 1> float t_dec(const Bufs& b, bool check)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float tot = 0;
    for (int i = 0; i < 10; ++i) {
        hipMemcpy(b.bad, b.cw, b.nb * 255, hipMemcpyDeviceToDevice);
        if (g_inject)
            hipLaunchKernelGGL(inject, dim3((b.nb + 255) / 256), dim3(256), 0, 0, b.bad, b.nb);
        hipEventRecord(e0);
        hipLaunchKernelGGL((rs255_decode_kernel<6, 0, STAGE, NT>), dim3(STAGE == 4 ? b.grid1 : b.grid), dim3(256), 0, 0, b.bad, b.out, b.st,
            b.nb, b.tab, WB);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        tot += ms;
    }
    if (check) {
        std::vector<uint8_t> x(b.nb * 249), y(b.nb * 249), c(b.nb * 255), c2(b.nb * 255);
        hipMemcpy(x.data(), b.out, x.size(), hipMemcpyDeviceToHost);
        hipMemcpy(y.data(), b.d, y.size(), hipMemcpyDeviceToHost);
        hipMemcpy(c.data(), b.bad, c.size(), hipMemcpyDeviceToHost);
        hipMemcpy(c2.data(), b.cw, c2.size(), hipMemcpyDeviceToHost);
        if (x != y || (WB && c != c2))
            printf("STAGE %d NT %d: MISMATCH (payload %d, write-back %d)\n", STAGE, NT, x != y, c != c2);
    }
    return tot / 10 * 1e3f;
}

template <int PF, int NT, int MO> float t_enc(const Bufs& b)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((rs255_encode_kernel<6, 0, PF, NT, MO>), dim3(PF == 2 ? b.grid1 : b.grid), dim3(256), 0, 0, b.d, b.cw, b.nb, b.tab);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i)
        hipLaunchKernelGGL((rs255_encode_kernel<6, 0, PF, NT, MO>), dim3(PF == 2 ? b.grid1 : b.grid), dim3(256), 0, 0, b.d,
            b.cw, b.nb, b.tab);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    // MEMONLY leaves cw garbage: restore real codewords
    if (MO)
        hipLaunchKernelGGL((rs255_encode_kernel<6>), dim3(b.grid), dim3(256), 0, 0, b.d, b.cw, b.nb, b.tab);
    return ms / 10 * 1e3f;
}

template <int PF, int NT> float t_enc_grid(const Bufs& b, int grid)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((rs255_encode_kernel<6, 0, PF, NT, 0>), dim3(grid), dim3(256), 0, 0, b.d, b.cw, b.nb, b.tab);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i)
        hipLaunchKernelGGL((rs255_encode_kernel<6, 0, PF, NT, 0>), dim3(grid), dim3(256), 0, 0, b.d, b.cw, b.nb, b.tab);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 10 * 1e3f;
}

template <int STAGE, int NT> float t_dec_grid(const Bufs& b, int grid)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float tot = 0;
    for (int i = 0; i < 10; ++i) {
        hipMemcpy(b.bad, b.cw, b.nb * 255, hipMemcpyDeviceToDevice);
        hipLaunchKernelGGL(inject, dim3((b.nb + 255) / 256), dim3(256), 0, 0, b.bad, b.nb);
        hipEventRecord(e0);
        hipLaunchKernelGGL((rs255_decode_kernel<6, 0, STAGE, NT>), dim3(grid), dim3(256), 0, 0, b.bad, b.out, b.st,
            b.nb, b.tab, 1);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        tot += ms;
    }
    return tot / 10 * 1e3f;
}

int main()
{
    Bufs b;
    b.nb = 1ull << 20;
    hipMalloc(&b.d, b.nb * 249);
    hipMalloc(&b.cw, b.nb * 255);
    hipMalloc(&b.bad, b.nb * 255);
    hipMalloc(&b.out, b.nb * 249);
    hipMalloc(&b.st, b.nb);
    std::vector<uint8_t> tab = build_rs_slice_tables(6);
    const size_t sl = tab.size();
    tab.resize(sl + 1024);
    build_gf_block(tab.data() + sl);
    hipMalloc(&b.tab, tab.size());
    hipMemcpy(b.tab, tab.data(), tab.size(), hipMemcpyHostToDevice);
    std::vector<uint8_t> h(b.nb * 249);
    srand(1);
    for (auto& x : h)
        x = (uint8_t)rand();
    hipMemcpy(b.d, h.data(), h.size(), hipMemcpyHostToDevice);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    b.grid = 2 * cus;
    b.grid1 = (int)((b.nb / 64 + 3) / 4);
    const double bytes = b.nb * 504.0;
    printf("encode (default) %.1f us\n", t_enc<1, 1, 0>(b));
    for (int mult : { 2, 4, 8, 16, 32, 64 }) {
        const int g = std::min(mult * cus, b.grid1);
        std::vector<float> e, d1, d2;
        for (int rep = 0; rep < 5; ++rep) {
            e.push_back(t_enc_grid<1, 1>(b, g));
            d1.push_back(t_dec_grid<1, 2>(b, g));
            d2.push_back(t_dec_grid<2, 2>(b, g));
        }
        std::sort(e.begin(), e.end());
        std::sort(d1.begin(), d1.end());
        std::sort(d2.begin(), d2.end());
        printf("grid %5d (%4.1f tiles/wave): enc PF1 %.1f us | dec S1 NTstore %.1f us | dec S2 NTstore %.1f us\n", g,
            (double)(b.nb / 64) / (4.0 * g), e[2], d1[2], d2[2]);
    }
    // oneshot encode correctness: codewords equal the persistent kernel's
    {
        std::vector<uint8_t> c1(b.nb * 255), c2(b.nb * 255);
        hipLaunchKernelGGL((rs255_encode_kernel<6>), dim3(b.grid), dim3(256), 0, 0, b.d, b.cw, b.nb, b.tab);
        hipMemcpy(c1.data(), b.cw, c1.size(), hipMemcpyDeviceToHost);
        hipLaunchKernelGGL((rs255_encode_kernel<6, 0, 2, 1, 0>), dim3(b.grid1), dim3(256), 0, 0, b.d, b.cw, b.nb, b.tab);
        hipMemcpy(c2.data(), b.cw, c2.size(), hipMemcpyDeviceToHost);
        printf("oneshot encode %s\n", c1 == c2 ? "matches" : "MISMATCH");
    }
    return 0;
}
