// rs_ablate.hip -- diagnostic build (not shipped): RS(255,249) encode/decode variants timed in
// one process on random data (interleaved rounds, median).  Variant knobs: NSEG (independent
// remainder chains per lane) and PF (prefetch next tile into VGPRs during compute).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I paritypartyfs_amd/csrc tools/probes/rs_ablate.hip -o tools/rs_ablate.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rs_fast.hpp"

using namespace ppfs;

struct Bufs {
    uint8_t *d, *r, *out, *st, *tab, *bad;
    uint64_t nb;
    int grid;
};

template <int NS, int PF, int NT = 0, int MO = 0> float t_enc(const Bufs& b)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((rs255_encode_kernel<6, NS, PF, NT, MO>), dim3(b.grid), dim3(256), 0, 0, b.d, b.r, b.nb, b.tab);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i)
        hipLaunchKernelGGL((rs255_encode_kernel<6, NS, PF, NT, MO>), dim3(b.grid), dim3(256), 0, 0, b.d, b.r, b.nb, b.tab);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 10 * 1e3f;
}

template <int NS, int PF> float t_dec(const Bufs& b)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((rs255_decode_kernel<6, NS, PF>), dim3(b.grid), dim3(256), 0, 0, b.bad, b.out, b.st, b.nb,
        b.tab, 0);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i)
        hipLaunchKernelGGL((rs255_decode_kernel<6, NS, PF>), dim3(b.grid), dim3(256), 0, 0, b.bad, b.out, b.st, b.nb,
            b.tab, 0);
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
    hipMalloc(&b.r, b.nb * 255);
    hipMalloc(&b.bad, b.nb * 255);
    hipMalloc(&b.out, b.nb * 249);
    hipMalloc(&b.st, b.nb);
    hipMalloc(&b.tab, 65536);
    std::vector<uint8_t> h(b.nb * 255);
    srand(1);
    for (auto& x : h)
        x = (uint8_t)rand();
    hipMemcpy(b.d, h.data(), b.nb * 249, hipMemcpyHostToDevice);
    hipMemcpy(b.bad, h.data(), b.nb * 255, hipMemcpyHostToDevice); // random codewords: every block "erroneous"
    std::vector<uint8_t> t(65536);
    for (auto& x : t)
        x = (uint8_t)rand();
    hipMemcpy(b.tab, t.data(), 65536, hipMemcpyHostToDevice);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    b.grid = 2 * cus;
    const double bytes = b.nb * 504.0;
    const char* names[] = { "NS1 PF0 NT0", "NS1 PF1 NT0", "NS1 PF0 NT1", "NS1 PF1 NT1", "MEMONLY PF0 NT0",
        "MEMONLY PF1 NT0", "MEMONLY PF0 NT1", "NS2 PF0 NT0" };
    constexpr int NV = 8;
    std::vector<float> enc[NV], dec[2];
    for (int rep = 0; rep < 5; ++rep) {
        enc[0].push_back(t_enc<1, 0, 0>(b));
        enc[1].push_back(t_enc<1, 1, 0>(b));
        enc[2].push_back(t_enc<1, 0, 1>(b));
        enc[3].push_back(t_enc<1, 1, 1>(b));
        enc[4].push_back(t_enc<1, 0, 0, 1>(b));
        enc[5].push_back(t_enc<1, 1, 0, 1>(b));
        enc[6].push_back(t_enc<1, 0, 1, 1>(b));
        enc[7].push_back(t_enc<2, 0, 0>(b));
    }
    for (int v = 0; v < NV; ++v) {
        std::sort(enc[v].begin(), enc[v].end());
        printf("%-16s encode %.1f us (%.0f GB/s)  [min %.1f max %.1f]\n", names[v], enc[v][2],
            bytes / (enc[v][2] * 1e-6) / 1e9, enc[v][0], enc[v][4]);
    }
    return 0;
}
