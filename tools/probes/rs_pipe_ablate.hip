// rs_pipe_ablate.hip -- diagnostic build (not shipped): the bench step (encode -> inject one byte error
// per block -> decode with write-back, 2^20 RS(255,249) blocks) with the kernels' phases switched
// off (MODE 0 = same bytes moved, no compute), to see what the memory system allows in THIS
// sequence (each kernel inherits the previous one's dirty lines and cache state).
#include "../paritypartyfs_amd/csrc/api.cpp" // host table builders (same TU)
#include "rs_wg.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>

using namespace ppfs;

__global__ void inject_kernel(uint8_t* cw, const uint8_t* pos, const uint8_t* val, uint64_t nb)
{
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb)
        cw[b * 255 + pos[b]] ^= val[b];
}

__global__ void inject_store_kernel(uint8_t* cw, const uint8_t* pos, const uint8_t* bytes, uint64_t nb)
{
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb)
        cw[b * 255 + pos[b]] = bytes[b];
}

int g_store = 0;
uint8_t* g_bytes = nullptr;

int main()
{
    const uint64_t nb = 1ull << 20;
    std::vector<uint8_t> tab = build_rs_fast_tables(6);
    uint8_t *d, *cw, *out, *st, *tb, *pos, *val;
    hipMalloc(&d, nb * 249);
    hipMalloc(&cw, nb * 255);
    hipMalloc(&out, nb * 249);
    hipMalloc(&st, nb);
    hipMalloc(&pos, nb);
    hipMalloc(&val, nb);
    hipMalloc(&tb, tab.size());
    hipMemcpy(tb, tab.data(), tab.size(), hipMemcpyHostToDevice);
    std::vector<uint8_t> h(nb * 249), hp(nb), hv(nb);
    srand(1);
    for (auto& x : h)
        x = (uint8_t)rand();
    for (uint64_t b = 0; b < nb; ++b) {
        hp[b] = (uint8_t)(rand() % 255);
        hv[b] = (uint8_t)(1 + rand() % 255);
    }
    hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice);
    hipMemcpy(pos, hp.data(), nb, hipMemcpyHostToDevice);
    hipMemcpy(val, hv.data(), nb, hipMemcpyHostToDevice);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t ev[4];
    for (auto& e : ev)
        hipEventCreate(&e);
    auto run = [&](const char* name, auto enc, auto dec, int steps) {
        // 1 s clock ramp, then `steps` timed steps
        auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(700)) {
            for (int i = 0; i < 16; ++i) {
                enc();
                if (g_store)
                    hipLaunchKernelGGL(inject_store_kernel, dim3(nb / 256), dim3(256), 0, 0, cw, pos, g_bytes, nb);
                else
                    hipLaunchKernelGGL(inject_kernel, dim3(nb / 256), dim3(256), 0, 0, cw, pos, val, nb);
                dec();
            }
            hipDeviceSynchronize();
        }
        double se = 0, si = 0, sd = 0;
        for (int i = 0; i < steps; ++i) {
            hipEventRecord(ev[0]);
            enc();
            hipEventRecord(ev[1]);
            if (g_store)
                hipLaunchKernelGGL(inject_store_kernel, dim3(nb / 256), dim3(256), 0, 0, cw, pos, g_bytes, nb);
            else
                hipLaunchKernelGGL(inject_kernel, dim3(nb / 256), dim3(256), 0, 0, cw, pos, val, nb);
            hipEventRecord(ev[2]);
            dec();
            hipEventRecord(ev[3]);
            hipEventSynchronize(ev[3]);
            float a, b, c;
            hipEventElapsedTime(&a, ev[0], ev[1]);
            hipEventElapsedTime(&b, ev[1], ev[2]);
            hipEventElapsedTime(&c, ev[2], ev[3]);
            se += a;
            si += b;
            sd += c;
        }
        se *= 1e3 / steps;
        si *= 1e3 / steps;
        sd *= 1e3 / steps;
        printf("%-34s enc %6.1f  inj %5.1f  dec %6.1f  step %6.1f us  (enc %4.0f dec %4.0f GB/s)\n", name, se, si, sd,
            se + si + sd, nb * 504.0 / se / 1e3, nb * 504.0 / sd / 1e3);
    };
#define ENC(NB, W, M, ...) [&] { hipLaunchKernelGGL((wg::rs_wg_encode_kernel<6, NB, W, M, ##__VA_ARGS__>), dim3(W * cus), dim3(256), 0, 0, d, cw, nb, tb); }
#define DEC(NB, W, M, ...) [&] { hipLaunchKernelGGL((wg::rs_wg_decode_kernel<6, NB, W, M, ##__VA_ARGS__>), dim3(W * cus), dim3(256), 0, 0, cw, out, st, nb, tb, 1, (uint8_t*)nullptr); }
    {
        // precomputed wrong bytes (the bench's store-only injection)
        ENC(2, 4, 3)();
        std::vector<uint8_t> c(nb * 255), wb(nb);
        hipMemcpy(c.data(), cw, c.size(), hipMemcpyDeviceToHost);
        for (uint64_t b = 0; b < nb; ++b)
            wb[b] = c[b * 255 + hp[b]] ^ hv[b];
        hipMalloc(&g_bytes, nb);
        hipMemcpy(g_bytes, wb.data(), nb, hipMemcpyHostToDevice);
    }
    for (int rnd = 0; rnd < 2; ++rnd) {
        g_store = 1;
        run("store-inj: enc nt, dec nt", ENC(2, 4, 3, 1), DEC(2, 3, 7, 1), 200);
        run("store-inj: enc plain, dec nt", ENC(2, 4, 3, 0), DEC(2, 3, 7, 1), 200);
        run("store-inj: enc nt, dec plain", ENC(2, 4, 3, 1), DEC(2, 3, 7, 0), 200);
        run("store-inj: enc plain, dec plain", ENC(2, 4, 3, 0), DEC(2, 3, 7, 0), 200);
        run("store-inj: skel plain/plain", ENC(2, 4, 0, 0), DEC(2, 3, 0, 0), 200);
        g_store = 0;
        run("xor-inj: enc plain, dec plain", ENC(2, 4, 3, 0), DEC(2, 3, 7, 0), 200);
        run("xor-inj: enc plain, dec nt", ENC(2, 4, 3, 0), DEC(2, 3, 7, 1), 200);
    }
    g_store = 0;
    // check
    ENC(2, 4, 3)();
    hipLaunchKernelGGL(inject_kernel, dim3(nb / 256), dim3(256), 0, 0, cw, pos, val, nb);
    DEC(2, 3, 7)();
    std::vector<uint8_t> o(nb * 249);
    hipMemcpy(o.data(), out, o.size(), hipMemcpyDeviceToHost);
    printf("decode payload %s\n", o == h ? "matches" : "DIFFERS");
    return 0;
}
