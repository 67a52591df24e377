// rs_ablate_dec.hip -- diagnostic build (not shipped): RS(255,249) decode staging variants timed
// in one process on real codewords carrying one byte error each (the bench workload); every
// variant's payload output is checked against the original data.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I paritypartyfs_amd/csrc -I include \
//     tools/rs_ablate_dec.hip -o tools/rs_ablate_dec.bin
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
        hipLaunchKernelGGL((rs255_decode_kernel<6, 0, STAGE, NT>), dim3(b.grid), dim3(256), 0, 0, b.bad, b.out, b.st,
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

float t_enc(const Bufs& b)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i)
        hipLaunchKernelGGL((rs255_encode_kernel<6>), dim3(b.grid), dim3(256), 0, 0, b.d, b.cw, b.nb, b.tab);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 10 * 1e3f;
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
    const double bytes = b.nb * 504.0;
    printf("encode (default) %.1f us\n", t_enc(b));
    t_dec<1, 0>(b, true);
    t_dec<1, 1>(b, true);
    t_dec<1, 2>(b, true);
    t_dec<1, 3>(b, true);
    t_dec<2, 0>(b, true);
    t_dec<2, 2>(b, true);
    t_dec<0, 0>(b, true);
    t_dec<1, 0, 0>(b, true);
    t_dec<1, 2, 0>(b, true);
    const char* names[] = { "S1 NT0", "S1 NTload", "S1 NTstore", "S2 NTstore", "S2 NT0", "S0 NT0",
        "S1 NT0 no-wb", "S1 NTstore no-wb", "encode default", "S1 NT0 clean", "S1 NTstore clean" };
    constexpr int NV = 11;
    std::vector<float> dec[NV];
    for (int rep = 0; rep < 5; ++rep) {
        dec[0].push_back(t_dec<1, 0>(b, false));
        dec[1].push_back(t_dec<1, 1>(b, false));
        dec[2].push_back(t_dec<1, 2>(b, false));
        dec[3].push_back(t_dec<2, 2>(b, false));
        dec[4].push_back(t_dec<2, 0>(b, false));
        dec[5].push_back(t_dec<0, 0>(b, false));
        dec[6].push_back(t_dec<1, 0, 0>(b, false));
        dec[7].push_back(t_dec<1, 2, 0>(b, false));
        dec[8].push_back(t_enc(b));
        g_inject = false;
        dec[9].push_back(t_dec<1, 0>(b, false));
        dec[10].push_back(t_dec<1, 2>(b, false));
        g_inject = true;
    }
    for (int v = 0; v < NV; ++v) {
        std::sort(dec[v].begin(), dec[v].end());
        printf("%-22s %.1f us (%.0f GB/s)  [min %.1f max %.1f]\n", names[v], dec[v][2],
            bytes / (dec[v][2] * 1e-6) / 1e9, dec[v][0], dec[v][4]);
    }
    return 0;
}
