// dma_align_test.hip -- does global_load_lds_dwordx4 (LDS-DMA) accept a global source address that
// is not 16- / 4-byte aligned on gfx950?  One workgroup: 64 lanes each DMA 16 bytes from
// src + misalign + 16 * lane into LDS, then copy LDS out; the host compares against the source.
// Build: hipcc --offload-arch=gfx950 -O2 tools/probes/dma_align_test.hip -o tools/dma_align_test.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

__global__ void dma_kernel(const uint8_t* src, uint8_t* out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[1024];
    const uint32_t lane = threadIdx.x;
    const uint32_t base = (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)lds;
    const uint8_t* g = src + 16u * lane;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off\n\ts_waitcnt vmcnt(0)" ::"v"(g), "s"(base)
                 : "memory", "m0");
    __syncthreads();
    for (int i = 0; i < 16; ++i)
        out[16 * lane + i] = lds[16 * lane + i];
}

int main()
{
    uint8_t h[2048];
    for (int i = 0; i < 2048; ++i)
        h[i] = (uint8_t)(i * 7 + 3);
    uint8_t *d_src = nullptr, *d_out = nullptr;
    if (hipMalloc(&d_src, 2048) != hipSuccess || hipMalloc(&d_out, 1024) != hipSuccess)
        return 2;
    hipMemcpy(d_src, h, 2048, hipMemcpyHostToDevice);
    int bad_total = 0;
    for (int mis : { 0, 4, 2, 1, 3 }) {
        hipMemset(d_out, 0, 1024);
        hipLaunchKernelGGL(dma_kernel, dim3(1), dim3(64), 0, 0, d_src + mis, d_out);
        hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) {
            printf("misalign %d: error %s\n", mis, hipGetErrorString(e));
            return 1;
        }
        uint8_t o[1024];
        hipMemcpy(o, d_out, 1024, hipMemcpyDeviceToHost);
        int bad = 0, first = -1;
        for (int i = 0; i < 1024; ++i)
            if (o[i] != h[mis + i]) {
                if (first < 0)
                    first = i;
                bad++;
            }
        printf("misalign %d: %d wrong bytes%s", mis, bad, bad ? "" : " (exact)\n");
        if (bad) {
            printf(" (first at %d: got %02x want %02x; aligned-down would be %02x)\n", first, o[first], h[mis + first],
                h[(mis & ~3) + first]);
        }
        bad_total += bad;
    }
    hipFree(d_src);
    hipFree(d_out);
    return 0;
}
