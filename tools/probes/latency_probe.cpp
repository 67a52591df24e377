// latency_probe.cpp -- where does a per-block readBlock / writeBlock spend its time?
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/probes/latency_probe.cpp -I include
//            -L paritypartyfs_amd/_lib -lppfs_ecc -Wl,-rpath,$PWD/paritypartyfs_amd/_lib -o tools/probes/latency_probe.bin
// Prints one JSON line per probe: median / p10 / p90 microseconds over N calls.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "ppfs_ecc.h"

__global__ void empty_kernel() {}

// one wave writes a flag into host-coherent memory (system-scope release)
__global__ void flag_kernel(unsigned* flag, unsigned v)
{
    if (threadIdx.x == 0)
        __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <class F> static void probe(const char* name, int n, F&& f)
{
    std::vector<double> t;
    for (int i = 0; i < n / 10; ++i)
        f();
    for (int i = 0; i < n; ++i) {
        const auto a = std::chrono::steady_clock::now();
        f();
        const auto b = std::chrono::steady_clock::now();
        t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
    }
    std::sort(t.begin(), t.end());
    printf("{\"probe\": \"%s\", \"n\": %d, \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f}\n", name, n, t[n / 2],
        t[n / 10], t[9 * n / 10]);
    fflush(stdout);
}

int main()
{
    const int N = 2000;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
        return 2;
    probe("launch_empty+streamsync", N, [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        (void)hipStreamSynchronize(s);
    });
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    probe("launch_empty+event_spin", N, [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        (void)hipEventRecord(ev, s);
        while (hipEventQuery(ev) == hipErrorNotReady) {
        }
    });
    unsigned* flag = nullptr;
    (void)hipHostMalloc((void**)&flag, 64, hipHostMallocMapped | hipHostMallocCoherent);
    unsigned* dflag = nullptr;
    (void)hipHostGetDevicePointer((void**)&dflag, flag, 0);
    unsigned seq = 0;
    probe("launch_flag+host_spin", N, [&] {
        ++seq;
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, dflag, seq);
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
        }
    });
    (void)hipStreamSynchronize(s);

    ppfs_ecc_params p {};
    p.ecc_type = 4; // RS
    p.block_size = 512;
    p.rs_correctable_bytes = 3;
    ppfs_ecc_ctx* c = nullptr;
    if (ppfs_ecc_create(&p, 0, &c) != 0)
        return 3;
    const size_t n = ppfs_ecc_raw_block_size(c), k = ppfs_ecc_data_size(c);
    std::vector<uint8_t> data(k * 64), raw(n * 64), out(k * 64), st(64);
    for (size_t i = 0; i < data.size(); ++i)
        data[i] = (uint8_t)(i * 131 + 7);
    (void)ppfs_ecc_encode_host(c, data.data(), raw.data(), 64);
    probe("rs_encode_host_1", N, [&] { (void)ppfs_ecc_encode_host(c, data.data(), raw.data(), 1); });
    probe("rs_decode_host_1_clean", N, [&] { (void)ppfs_ecc_decode_host(c, raw.data(), out.data(), st.data(), 1, 1, nullptr); });
    probe("rs_write_host_1", N, [&] { (void)ppfs_ecc_write_host(c, data.data(), raw.data(), st.data(), 1); });
    probe("rs_decode_host_64_clean", N / 4,
        [&] { (void)ppfs_ecc_decode_host(c, raw.data(), out.data(), st.data(), 64, 1, nullptr); });
    uint8_t *d_raw = nullptr, *d_data = nullptr, *d_st = nullptr;
    (void)hipMalloc(&d_raw, n * 64);
    (void)hipMalloc(&d_data, k * 64);
    (void)hipMalloc(&d_st, 64);
    (void)hipMemcpy(d_raw, raw.data(), n * 64, hipMemcpyHostToDevice);
    probe("rs_decode_device_1+streamsync", N, [&] {
        (void)ppfs_ecc_decode_device(c, d_raw, d_data, d_st, 1, 1, nullptr, s);
        (void)hipStreamSynchronize(s);
    });
    probe("rs_encode_device_1+streamsync", N, [&] {
        (void)ppfs_ecc_encode_device(c, d_data, d_raw, 1, s);
        (void)hipStreamSynchronize(s);
    });
    probe("memcpy_h2d_512+d2h_512", N, [&] {
        (void)hipMemcpyAsync(d_raw, raw.data(), 512, hipMemcpyHostToDevice, s);
        (void)hipMemcpyAsync(out.data(), d_data, 512, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    });
    (void)hipFree(d_raw);
    (void)hipFree(d_data);
    (void)hipFree(d_st);
    ppfs_ecc_destroy(c);
    (void)hipHostFree(flag);
    (void)hipEventDestroy(ev);
    (void)hipStreamDestroy(s);
    return 0;
}
