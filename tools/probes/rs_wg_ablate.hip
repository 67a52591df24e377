// rs_wg_ablate.hip -- diagnostic build (not shipped): the workgroup RS(255,249) kernels with phases
// switched off (MODE bits) and at several grid sizes, 2^20 blocks, 1 byte error per block for
// decode.  Median of 5 rounds of 10 back-to-back launches.
#include "../paritypartyfs_amd/csrc/api.cpp" // host table builders (same TU)
#include "rs_wg.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

using namespace ppfs;

template <class F> float timeit(F f)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    std::vector<float> v;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(a);
        for (int i = 0; i < 10; ++i)
            f();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        v.push_back(ms / 10 * 1e3f);
    }
    std::sort(v.begin(), v.end());
    return v[2];
}

int main()
{
    const uint64_t nb = 1ull << 20;
    std::vector<uint8_t> tab = build_rs_fast_tables(6);
    uint8_t *d, *r, *bad, *out, *st, *tb;
    hipMalloc(&d, nb * 249);
    hipMalloc(&r, nb * 255);
    hipMalloc(&bad, nb * 255);
    hipMalloc(&out, nb * 249);
    hipMalloc(&st, nb);
    hipMalloc(&tb, tab.size());
    hipMemcpy(tb, tab.data(), tab.size(), hipMemcpyHostToDevice);
    std::vector<uint8_t> h(nb * 249);
    srand(1);
    for (auto& x : h)
        x = (uint8_t)rand();
    hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipLaunchKernelGGL((wg::rs_wg_encode_kernel<6, 2, 3, 3>), dim3(3 * cus), dim3(256), 0, 0, d, r, nb, tb);
    std::vector<uint8_t> cw(nb * 255);
    hipMemcpy(cw.data(), r, cw.size(), hipMemcpyDeviceToHost);
    for (uint64_t b = 0; b < nb; ++b)
        cw[b * 255 + rand() % 255] ^= (uint8_t)(1 + rand() % 255);
    const double bytes = nb * 504.0;
    auto rep = [&](const char* name, float us) { printf("%-44s %7.1f us  %6.0f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9); };
    char nm[96];
    hipMemcpy(bad, cw.data(), cw.size(), hipMemcpyHostToDevice);
#define E(NBUF, WPC, M)                                                                                               \
    snprintf(nm, sizeof nm, "encode nbuf%d wpc%d MODE%d", NBUF, WPC, M);                                           \
    rep(nm, timeit([&] {                                                                                             \
        hipLaunchKernelGGL((wg::rs_wg_encode_kernel<6, NBUF, WPC, M>), dim3(WPC * cus), dim3(256), 0, 0, d, r, nb, tb); \
    }));
#define D(NBUF, WPC, M)                                                                                               \
    snprintf(nm, sizeof nm, "decode nbuf%d wpc%d MODE%d", NBUF, WPC, M);                                           \
    rep(nm, timeit([&] {                                                                                             \
        hipLaunchKernelGGL((wg::rs_wg_decode_kernel<6, NBUF, WPC, M>), dim3(WPC * cus), dim3(256), 0, 0, bad, out, st, \
            nb, tb, 0, nullptr);                                                                                     \
    }));
    for (int rnd = 0; rnd < 3; ++rnd) {
        printf("-- round %d\n", rnd);
        E(2, 3, 3) E(2, 4, 3) E(1, 3, 3) E(1, 4, 3)
        D(2, 3, 7) D(1, 3, 7) D(1, 4, 7)
    }
    E(2, 3, 1) E(2, 3, 2) E(2, 3, 0) E(2, 4, 1) E(2, 4, 2) E(2, 4, 0) E(1, 4, 1) E(1, 4, 2)
    D(2, 3, 3) D(2, 3, 5) D(2, 3, 6) D(2, 3, 0) D(1, 4, 3) D(1, 4, 5) D(1, 4, 6)
    // correctness spot check of the full decode
    hipMemcpy(bad, cw.data(), cw.size(), hipMemcpyHostToDevice);
    hipLaunchKernelGGL((wg::rs_wg_decode_kernel<6, 2, 3, 7>), dim3(3 * cus), dim3(256), 0, 0, bad, out, st, nb, tb, 1, nullptr);
    std::vector<uint8_t> o(nb * 249);
    hipMemcpy(o.data(), out, o.size(), hipMemcpyDeviceToHost);
    printf("decode payload %s\n", o == h ? "matches" : "DIFFERS");
    return 0;
}
