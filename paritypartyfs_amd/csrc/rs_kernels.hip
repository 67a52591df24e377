// rs_kernels.hip -- Reed-Solomon generic path (any n <= 255, any 2t) and fast-path dispatch.
// The fast-path templates live in rs_fast.hpp and are instantiated per 2t by rs_fast_inst.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dbg.hpp"
#include "gf_common.hpp"
#include "rs_layout.hpp"
#include "srv_device.hpp"

namespace ppfs {

// ------------------------------------------------------------------------------------
// Generic path: any n <= 255 and any 2t.  One thread per block; bytewise LFSR for the
// remainder; private arrays for Berlekamp-Massey; exhaustive Chien search.  Used for
// shortened codes (block_size < 255) and parity lengths without a fast instantiation.
// ------------------------------------------------------------------------------------
struct GfG {
    const uint8_t* t; // global memory tables
    __device__ uint32_t log(uint32_t a) const { return t[GF_LOG + a]; }
    __device__ uint32_t exp(uint32_t i) const { return t[GF_EXP2 + i]; }
    __device__ uint32_t mul(uint32_t a, uint32_t b) const
    {
        return (a && b) ? t[GF_EXP2 + t[GF_LOG + a] + t[GF_LOG + b]] : 0u;
    }
    __device__ uint32_t div(uint32_t a, uint32_t b) const
    {
        return (a && b) ? t[GF_EXP2 + 255u + t[GF_LOG + a] - t[GF_LOG + b]] : 0u;
    }
};

// tables layout for the generic path: gf block (1 KiB) then generator g[0..2t] (256 B)
// one block per thread (the kernel below and rs_generic_server_kernel)
__device__ __forceinline__ void rs_generic_encode_one(const uint8_t* __restrict__ data, uint8_t* __restrict__ raw,
    uint64_t blk, uint64_t nblocks, int n, int t2, const uint8_t* __restrict__ tables)
{
    const GfG gf { tables };
    const uint8_t* g = tables + GF_BYTES;
    const int k = n - t2;
    const uint8_t* d = data + blk * (uint64_t)k;
    uint8_t* o = raw + blk * (uint64_t)n;
    if (!PPFS_DBG_OK(d, k, data, nblocks * k) || !PPFS_DBG_OK(o, n, raw, nblocks * n))
        return;
    uint8_t r[256];
    for (int q = 0; q < t2; ++q)
        r[q] = 0;
    for (int j = k - 1; j >= 0; --j) {
        const uint32_t fb = d[j] ^ (t2 ? r[t2 - 1] : 0);
        for (int q = t2 - 1; q >= 1; --q)
            r[q] = (uint8_t)(r[q - 1] ^ gf.mul(fb, g[q]));
        if (t2)
            r[0] = (uint8_t)gf.mul(fb, g[0]);
    }
    for (int q = 0; q < t2; ++q)
        o[q] = r[q];
    for (int j = 0; j < k; ++j)
        o[t2 + j] = d[j];
}

__global__ __launch_bounds__(256) void rs_generic_encode_kernel(const uint8_t* __restrict__ data,
    uint8_t* __restrict__ raw, uint64_t nblocks, int n, int t2, const uint8_t* __restrict__ tables)
{
    const uint64_t blk = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (blk < nblocks)
        rs_generic_encode_one(data, raw, blk, nblocks, n, t2, tables);
}

__device__ __forceinline__ void rs_generic_decode_one(uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint8_t* __restrict__ spill, uint64_t blk, uint64_t nblocks, int n, int t2,
    int write_back, const uint8_t* __restrict__ tables)
{
    const GfG gf { tables };
    const int k = n - t2;
    uint8_t* c = raw + blk * (uint64_t)n;
    if (!PPFS_DBG_OK(c, n, raw, nblocks * n) || (data && !PPFS_DBG_OK(data + blk * (uint64_t)k, k, data, nblocks * k))
        || (status && !PPFS_DBG_OK(status + blk, 1, status, nblocks))
        || (spill && !PPFS_DBG_OK(spill + blk * (uint64_t)(256 - n), 256 - n, spill, nblocks * (256 - n))))
        return;
    uint8_t cw[256];
    for (int i = 0; i < n; ++i)
        cw[i] = c[i];
    for (int i = n; i < 256; ++i)
        cw[i] = 0;
    // syndromes by power-sum evaluation (polynomial_gf256.cpp:129-138)
    uint8_t S[256];
    bool clean = true;
    for (int i = 1; i <= t2; ++i) {
        const uint32_t li = (uint32_t)i;
        uint32_t s = 0;
        uint32_t lp = 0; // log of alpha^(i*m)
        for (int m = 0; m < n; ++m) {
            if (cw[m])
                s ^= gf.exp((gf.log(cw[m]) + lp) % 255u);
            lp = (lp + li) % 255u;
        }
        S[i - 1] = (uint8_t)s;
        clean = clean && s == 0;
    }
    int wb_len = 0;
    if (!clean) {
        uint8_t sig[256], B[256], T[256];
        for (int i = 0; i <= t2; ++i) {
            sig[i] = i == 0;
            B[i] = i == 0;
        }
        uint32_t b = 1;
        int L = 0, m = 1;
        for (int nn = 0; nn < t2; ++nn) {
            uint32_t d = S[nn];
            for (int i = 1; i <= L; ++i)
                d ^= gf.mul(sig[i], S[nn - i]);
            if (d) {
                const uint32_t coef = gf.div(d, b);
                for (int i = 0; i <= t2; ++i)
                    T[i] = sig[i];
                for (int i = m; i <= t2; ++i)
                    sig[i] ^= (uint8_t)gf.mul(coef, B[i - m]);
                if (2 * L <= nn) {
                    L = nn + 1 - L;
                    for (int i = 0; i <= t2; ++i)
                        B[i] = T[i];
                    b = d;
                    m = 1;
                } else {
                    m++;
                }
            } else {
                m++;
            }
        }
        uint8_t om[256];
        for (int j = 0; j < t2; ++j) {
            uint32_t o = 0;
            for (int a = 0; a <= j; ++a)
                o ^= gf.mul(S[a], sig[j - a]);
            om[j] = (uint8_t)o;
        }
        // code_word.size(): trimmed length of the raw block, extended by correction positions
        int size = n;
        while (size > 0 && cw[size - 1] == 0)
            size--;
        for (uint32_t mm = 0; mm < 255; ++mm) {
            uint32_t s = 0, ds = 0;
            for (int i = 0; i <= t2; ++i) {
                if (!sig[i])
                    continue;
                const uint32_t e = (gf.log(sig[i]) + (uint32_t)i * mm) % 255u;
                s ^= gf.exp(e);
                if (i & 1)
                    ds ^= gf.exp((e + 255u - mm) % 255u);
            }
            if (s)
                continue;
            uint32_t acc = 0;
            for (int j = t2 - 1; j >= 0; --j)
                acc = gf.mul(acc, gf.exp(mm)) ^ om[j];
            const uint32_t e = gf.div(acc, ds);
            const int pos = mm == 0 ? 0 : 255 - (int)mm;
            cw[pos] ^= (uint8_t)e;
            if (pos + 1 > size)
                size = pos + 1;
        }
        wb_len = size;
        if (write_back)
            for (int i = 0; i < n; ++i)
                c[i] = cw[i];
    }
    if (status)
        status[blk] = clean ? 0 : 1;
    if (spill) {
        uint8_t* sp = spill + blk * (uint64_t)(256 - n);
        const int extra = wb_len > n ? wb_len - n : 0;
        sp[0] = (uint8_t)extra;
        for (int i = 0; i < 255 - n; ++i)
            sp[1 + i] = i < extra ? cw[n + i] : 0;
    }
    if (data) {
        uint8_t* o = data + blk * (uint64_t)k;
        for (int j = 0; j < k; ++j)
            o[j] = cw[t2 + j];
    }
}

__global__ __launch_bounds__(64) void rs_generic_decode_kernel(uint8_t* __restrict__ raw, uint8_t* __restrict__ data,
    uint8_t* __restrict__ status, uint8_t* __restrict__ spill, uint64_t nblocks, int n, int t2, int write_back,
    const uint8_t* __restrict__ tables)
{
    const uint64_t blk = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (blk < nblocks)
        rs_generic_decode_one(raw, data, status, spill, blk, nblocks, n, t2, write_back, tables);
}

// Resident small-batch server for the generic RS path (shortened codes, parity lengths without a
// fast instantiation; server_box.hpp protocol): one 64-thread workgroup, thread b takes block b of
// a request, requests without spill only (a shortened code's write-back past the block end goes
// through the launch path).  A write is the old block's decode for its status, then the encode.
__global__ __launch_bounds__(64, 1) void rs_generic_server_kernel(SrvBox* box, uint8_t* zc, uint64_t zc_bytes, int n,
    int t2, const uint8_t* __restrict__ tables, uint32_t gen, uint32_t idle_us)
{
    __shared__ uint32_t s_cmd[2];
    const uint32_t k = (uint32_t)(n - t2);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t last = t0;
    uint32_t seen = srv::ld_sys(&box->done), served = 0;
    if (threadIdx.x == 0)
        srv::st_sys(&box->alive, gen);
    for (;;) {
        const uint32_t r = srv::next_request(box, seen, last, t0, idle_us, s_cmd);
        if (r == 0)
            break;
        const SrvCmd cmd = srv_cmd_unpack(r);
        const uint32_t nb = cmd.nb, b = threadIdx.x;
        const SrvLayout lay = srv_layout(nb, k, (uint32_t)n);
        uint8_t* data = zc + lay.data;
        uint8_t* raw = zc + lay.raw;
        uint8_t* status = zc + lay.status;
        const bool ok = nb >= 1 && nb <= SRV_MAX_BLOCKS && PPFS_DBG_OK(data, nb * k, zc, zc_bytes)
            && PPFS_DBG_OK(raw, nb * (uint32_t)n, zc, zc_bytes) && PPFS_DBG_OK(status, nb, zc, zc_bytes);
        if (ok && b < nb) {
            if (cmd.op == SRV_DECODE)
                rs_generic_decode_one(raw, cmd.want_data ? data : nullptr, status, nullptr, b, nb, n, t2,
                    cmd.write_back ? 1 : 0, tables);
            if (cmd.op == SRV_WRITE) // the old block's status only (rs_block_device.cpp:61-93)
                rs_generic_decode_one(raw, nullptr, status, nullptr, b, nb, n, t2, 0, tables);
            if (cmd.op == SRV_ENCODE || cmd.op == SRV_WRITE)
                rs_generic_encode_one(data, raw, b, nb, n, t2, tables);
        }
        seen = r;
        srv::finish_request(box, r, ++served);
    }
    if (threadIdx.x == 0)
        srv::st_sys(&box->alive, gen | SRV_EXITED);
}

} // namespace ppfs

using namespace ppfs;

// Fast-path instantiations (t = 1..5, 8, 16: the reference tests' and BASELINE configs' t).
#define PPFS_RS_CASES(X) X(2) X(4) X(6) X(8) X(10) X(16) X(32)

#define X(T)                                                                                                           \
    extern "C" hipError_t ppfs_rs_fast_encode_t##T(const uint8_t*, uint8_t*, uint64_t, const uint8_t*, hipStream_t,   \
        uint32_t*, uint32_t*);                                                                                         \
    extern "C" hipError_t ppfs_rs_fast_decode_t##T(uint8_t*, uint8_t*, uint8_t*, uint64_t, const uint8_t*, int,       \
        hipStream_t, uint32_t*, uint32_t*, uint8_t*);
PPFS_RS_CASES(X)
#undef X

extern "C" int ppfs_rs_fast_supported(int n, int t2)
{
    if (n != 255)
        return 0;
    switch (t2) {
#define X(T)                                                                                                           \
    case T:                                                                                                            \
        return 1;
        PPFS_RS_CASES(X)
#undef X
    default:
        return 0;
    }
}

// device table blob of the fast path (rs_layout.hpp): segment layout for 2t <= 8, lane-per-block
// nibble slicing tables (4 KiB; the 1 KiB GF block is appended by the builder) for 8 < 2t <= 16,
// pair layout (nibble planes of 16-byte columns, GF block, XP rows) for 16 < 2t <= 32
extern "C" int ppfs_rs_fast_tables_bytes(int t2)
{
    return t2 <= 8 ? rs_wg_table_bytes(t2) : (t2 <= 16 ? 4096 : rs_pair_table_bytes());
}

extern "C" hipError_t ppfs_rs_fast_encode(int t2, const uint8_t* d, uint8_t* r, uint64_t nb, const uint8_t* tab,
    hipStream_t s, uint32_t* ctr, uint32_t* ctr_clear)
{
    switch (t2) {
#define X(T)                                                                                                           \
    case T:                                                                                                            \
        return ppfs_rs_fast_encode_t##T(d, r, nb, tab, s, ctr, ctr_clear);
        PPFS_RS_CASES(X)
#undef X
    default:
        return hipErrorInvalidValue;
    }
}

#define X(T) extern "C" const char* ppfs_rs_fast_path_t##T();
PPFS_RS_CASES(X)
#undef X
// name of the kernel path an instantiation was built with (ppfs_ecc_kernel_name)
extern "C" const char* ppfs_rs_fast_path(int t2)
{
    switch (t2) {
#define X(T)                                                                                                           \
    case T:                                                                                                            \
        return ppfs_rs_fast_path_t##T();
        PPFS_RS_CASES(X)
#undef X
    default:
        return "";
    }
}

extern "C" hipError_t ppfs_rs_fast_decode(int t2, uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb,
    const uint8_t* tab, int wb, hipStream_t s, uint32_t* ctr, uint32_t* ctr_clear, uint8_t* wb_dst)
{
    switch (t2) {
#define X(T)                                                                                                           \
    case T:                                                                                                            \
        return ppfs_rs_fast_decode_t##T(r, d, st, nb, tab, wb, s, ctr, ctr_clear, wb_dst);
        PPFS_RS_CASES(X)
#undef X
    default:
        return hipErrorInvalidValue;
    }
}

// resident small-batch servers (2t <= 8: segment-layout tables; 10, 16: lane-per-block; 32: pair layout)
#define PPFS_RS_SERVER_CASES(X) X(2) X(4) X(6) X(8) X(10) X(16) X(32)
#define X(T)                                                                                                           \
    extern "C" hipError_t ppfs_rs_server_launch_t##T(ppfs::SrvBox*, uint8_t*, uint64_t, const uint8_t*, uint32_t,      \
        uint32_t, hipStream_t);
PPFS_RS_SERVER_CASES(X)
#undef X
extern "C" hipError_t ppfs_rs_server_launch(int t2, ppfs::SrvBox* box, uint8_t* zc, uint64_t zc_bytes, const uint8_t* tab,
    uint32_t gen, uint32_t idle_us, hipStream_t s)
{
    switch (t2) {
#define X(T)                                                                                                           \
    case T:                                                                                                            \
        return ppfs_rs_server_launch_t##T(box, zc, zc_bytes, tab, gen, idle_us, s);
        PPFS_RS_SERVER_CASES(X)
#undef X
    default:
        return hipErrorInvalidValue;
    }
}

extern "C" hipError_t ppfs_rs_generic_server_launch(int n, int t2, SrvBox* box, uint8_t* zc, uint64_t zc_bytes,
    const uint8_t* tab, uint32_t gen, uint32_t idle_us, hipStream_t s)
{
    hipLaunchKernelGGL(rs_generic_server_kernel, dim3(1), dim3(64), 0, s, box, zc, zc_bytes, n, t2, tab, gen, idle_us);
    return hipGetLastError();
}

extern "C" hipError_t ppfs_rs_generic_encode(const uint8_t* d, uint8_t* r, uint64_t nb, int n, int t2,
    const uint8_t* tab, hipStream_t s)
{
    const uint32_t grid = (uint32_t)((nb + 255) / 256);
    hipLaunchKernelGGL(rs_generic_encode_kernel, dim3(grid), dim3(256), 0, s, d, r, nb, n, t2, tab);
    return hipGetLastError();
}

extern "C" hipError_t ppfs_rs_generic_decode(uint8_t* r, uint8_t* d, uint8_t* st, uint8_t* spill, uint64_t nb, int n,
    int t2, int wb, const uint8_t* tab, hipStream_t s)
{
    const uint32_t grid = (uint32_t)((nb + 63) / 64);
    hipLaunchKernelGGL(rs_generic_decode_kernel, dim3(grid), dim3(64), 0, s, r, d, st, spill, nb, n, t2, wb, tab);
    return hipGetLastError();
}

PPFS_DBG_ACCESSOR(ppfs_dbg_faults_rs_generic)
