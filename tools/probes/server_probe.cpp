// server_probe.cpp -- round-trip latency of a resident "mailbox" kernel polling host-coherent
// memory (the design question behind the per-block server path): the host posts a sequence number
// (and, variant 2, 255 payload bytes the kernel reads and 249 it writes back), one lane of the
// resident workgroup polls for it, the workgroup answers with a system-scope release store.
// The kernel exits on a stop flag, after 200 ms without a request, or after 2 s in any case.
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/probes/server_probe.cpp -o tools/server_probe.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

struct Box {
    unsigned req;  // host -> device: request sequence number
    unsigned stop; // host -> device
    unsigned done; // device -> host
    unsigned alive;
    unsigned char pad[48];
    unsigned char in[256];
    unsigned char out[256];
};

__device__ __forceinline__ unsigned ld_sys(const unsigned* p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void mailbox_kernel(Box* b, int payload)
{
    __shared__ unsigned s_req, s_go;
    __shared__ unsigned char buf[256];
    const unsigned tid = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(); // 100 MHz
    unsigned long long last = t0;
    unsigned seen = ld_sys(&b->done);
    if (tid == 0)
        __hip_atomic_store(&b->alive, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    for (;;) {
        if (tid == 0) {
            unsigned go = 0, r = seen;
            for (int spin = 0; spin < 4096; ++spin) {
                r = ld_sys(&b->req);
                if (r != seen || ld_sys(&b->stop)) {
                    go = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            s_req = r;
            s_go = go;
        }
        __syncthreads();
        const unsigned r = s_req;
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        if (!s_go) {
            __syncthreads();
            if (now - last > 20000000ull || now - t0 > 200000000ull) // 200 ms idle / 2 s total
                break;
            continue;
        }
        if (ld_sys(&b->stop))
            break;
        last = now;
        if (payload) {
            if (tid < 255)
                buf[tid] = b->in[tid];
            __syncthreads();
            if (tid < 249)
                b->out[tid] = (unsigned char)(buf[tid + 6] ^ 0x5A);
        }
        __threadfence_system();
        __syncthreads();
        if (tid == 0)
            __hip_atomic_store(&b->done, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        seen = r;
        __syncthreads();
    }
    if (tid == 0)
        __hip_atomic_store(&b->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main()
{
    Box* h = nullptr;
    if (hipHostMalloc((void**)&h, sizeof(Box), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return 2;
    Box* d = nullptr;
    (void)hipHostGetDevicePointer((void**)&d, h, 0);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int payload = 0; payload < 2; ++payload) {
        *h = Box {};
        hipLaunchKernelGGL(mailbox_kernel, dim3(1), dim3(256), 0, s, d, payload);
        const auto w0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(&h->alive, __ATOMIC_ACQUIRE) != 1) {
            if (std::chrono::steady_clock::now() - w0 > std::chrono::seconds(2)) {
                printf("{\"payload\": %d, \"ok\": false, \"error\": \"kernel did not start\"}\n", payload);
                __atomic_store_n(&h->stop, 1u, __ATOMIC_RELEASE);
                (void)hipStreamSynchronize(s);
                return 1;
            }
        }
        std::vector<double> t;
        unsigned seq = 0;
        bool ok = true;
        for (int i = 0; i < 3000; ++i) {
            for (int j = 0; j < 255; ++j)
                h->in[j] = (unsigned char)(i + j);
            const auto a = std::chrono::steady_clock::now();
            ++seq;
            __atomic_store_n(&h->req, seq, __ATOMIC_RELEASE);
            while (__atomic_load_n(&h->done, __ATOMIC_ACQUIRE) != seq) {
                if (std::chrono::steady_clock::now() - a > std::chrono::milliseconds(100)) {
                    ok = false;
                    break;
                }
            }
            const auto b = std::chrono::steady_clock::now();
            if (!ok)
                break;
            if (payload && h->out[10] != (unsigned char)((i + 16) ^ 0x5A))
                ok = false;
            if (i >= 300)
                t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
        }
        __atomic_store_n(&h->stop, 1u, __ATOMIC_RELEASE);
        (void)hipStreamSynchronize(s);
        if (t.empty()) {
            printf("{\"payload\": %d, \"ok\": false}\n", payload);
            continue;
        }
        std::sort(t.begin(), t.end());
        const size_t n = t.size();
        printf("{\"payload\": %d, \"ok\": %s, \"n\": %zu, \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, \"p99_us\": %.2f}\n",
            payload, ok ? "true" : "false", n, t[n / 2], t[n / 10], t[9 * n / 10], t[99 * n / 100]);
        fflush(stdout);
    }
    (void)hipHostFree(h);
    (void)hipStreamDestroy(s);
    return 0;
}
