// api.cpp -- host implementation of the ppfs_ecc C ABI (include/ppfs_ecc.h).
//
// Builds the per-context codec tables (GF(2^8) log/antilog, RS slicing tables, CRC shift
// tables), uploads them once, and dispatches batches to the HIP kernels in rs_kernels.hip and
// bit_kernels.hip.  Parameter handling mirrors the reference constructors:
//   ReedSolomonBlockDevice  rs_block_device.cpp:52-60  (n = min(bs,255), t = min(t, n/2))
//   CrcBlockDevice          crc_block_device.cpp:71-76, dataSize :117-120
//   HammingBlockDevice      hamming_block_device.cpp:11-19 (bs = 2^binLog(block_size))
//   ParityBlockDevice       parity_block_device.cpp:9-15
//   RawBlockDevice          raw_block_device.cpp:5-9
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <cstdio>
#include <map>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <unistd.h>
#if defined(__x86_64__) || defined(__i386__)
#include <immintrin.h>
#define PPFS_HOST_X86 1
#else
#define PPFS_HOST_X86 0
#endif
#include <pthread.h>
#include <vector>

#include "../../include/ppfs_ecc.h"
#include "rs_layout.hpp"
#include "rs_sched.hpp"
#include "launch.hpp"
#include "server_box.hpp"

// kernels (rs_kernels.hip / bit_kernels.hip)
extern "C" {
int ppfs_rs_fast_supported(int n, int t2);
int ppfs_rs_fast_tables_bytes(int t2);
hipError_t ppfs_rs_fast_encode(int t2, const uint8_t* d, uint8_t* r, uint64_t nb, const uint8_t* tab, hipStream_t s,
    uint32_t* ctr, uint32_t* ctr_clear);
const char* ppfs_rs_fast_path(int t2);
hipError_t ppfs_flag_launch(uint32_t* flag, uint32_t v, hipStream_t s);
hipError_t ppfs_rs_generic_server_launch(int n, int t2, ppfs::SrvBox* box, uint8_t* zc, uint64_t zc_bytes,
    const uint8_t* tab, uint32_t gen, uint32_t idle_us, hipStream_t s);
hipError_t ppfs_bit_server_launch(int ecc_type, uint32_t bs, uint32_t ds, uint32_t crc_n, uint64_t crc_mask, uint32_t ham_L,
    ppfs::SrvBox* box, uint8_t* zc, uint64_t zc_bytes, const uint8_t* tab, uint32_t gen, uint32_t idle_us, hipStream_t s);
hipError_t ppfs_rs_server_launch(int t2, ppfs::SrvBox* box, uint8_t* zc, uint64_t zc_bytes, const uint8_t* tab,
    uint32_t gen, uint32_t idle_us, hipStream_t s);
hipError_t ppfs_rs_fast_decode(int t2, uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb, const uint8_t* tab, int wb,
    hipStream_t s, uint32_t* ctr, uint32_t* ctr_clear, uint8_t* wb_dst);
hipError_t ppfs_rs_generic_encode(const uint8_t* d, uint8_t* r, uint64_t nb, int n, int t2, const uint8_t* tab,
    hipStream_t s);
hipError_t ppfs_rs_generic_decode(uint8_t* r, uint8_t* d, uint8_t* st, uint8_t* spill, uint64_t nb, int n, int t2,
    int wb, const uint8_t* tab, hipStream_t s);
int ppfs_crc_tables_bytes(void);
int ppfs_crc_fast_layout(int32_t* v, int n);
int ppfs_crc_fast_supported(uint32_t bs, uint32_t n);
int ppfs_bitfast_supported(uint32_t bs);
hipError_t ppfs_crc_encode(const uint8_t* d, uint8_t* r, const uint8_t* skip, uint64_t nb, uint32_t bs, uint32_t ds,
    uint32_t n, uint64_t mask, const uint8_t* tab, hipStream_t s);
hipError_t ppfs_crc_check(const uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb, uint32_t bs, uint32_t ds, uint32_t n,
    uint64_t mask, const uint8_t* tab, hipStream_t s);
hipError_t ppfs_ham_encode(const uint8_t* d, uint8_t* r, const uint8_t* skip, uint64_t nb, uint32_t bs, uint32_t ds,
    uint32_t L, hipStream_t s);
hipError_t ppfs_ham_decode(uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb, int wb, uint32_t bs, uint32_t ds,
    uint32_t L, hipStream_t s);
hipError_t ppfs_parity_encode(const uint8_t* d, uint8_t* r, const uint8_t* skip, uint64_t nb, uint32_t bs,
    hipStream_t s);
hipError_t ppfs_parity_check(const uint8_t* r, uint8_t* d, uint8_t* st, uint64_t nb, uint32_t bs, hipStream_t s);
hipError_t ppfs_gather_rows_launch(const uint8_t* src, uint64_t src_rows, uint8_t* dst, const uint32_t* idx, uint32_t nrows,
    uint32_t row_bytes, hipStream_t s);
hipError_t ppfs_vote3_launch(const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* out, uint64_t rec_bytes,
    uint64_t nrec, uint32_t* damaged, hipStream_t s);
hipError_t ppfs_copy_launch(uint8_t* dst, const uint8_t* src, uint64_t bytes, hipStream_t s);
hipError_t ppfs_patch_list_launch(const uint8_t* cur, const uint8_t* orig, const uint8_t* status, uint32_t n, uint64_t nb,
    uint32_t S, uint32_t* patch, uint8_t* image, hipStream_t s);
hipError_t ppfs_inject_launch(uint8_t* raw, uint64_t stride, uint64_t nblocks, const uint8_t* pos, const uint8_t* val,
    int mode, hipStream_t s);
}

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* what, hipError_t e = hipSuccess)
{
    g_last_error = what;
    if (e != hipSuccess) {
        g_last_error += ": ";
        g_last_error += hipGetErrorString(e);
    }
    return code;
}

// Runs a scope on a context's device and restores the caller's current device afterwards
// (the HIP runtime may be shared with the caller's framework, e.g. torch's current device).
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
        if (prev != dev)
            err = hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

#define HIP_TRY(expr, what)                                                                                            \
    do {                                                                                                               \
        hipError_t _e = (expr);                                                                                        \
        if (_e != hipSuccess)                                                                                          \
            return fail(PPFS_ECC_EHIP, what, _e);                                                                      \
    } while (0)

// ---------------------------------------------------------------------------------------
// GF(2^8) host tables (gf256.cpp:6-29)
// ---------------------------------------------------------------------------------------
struct GfHost {
    uint8_t exp[256], log[256];
    GfHost()
    {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = (uint8_t)x;
            x <<= 1;
            if (x & 0x100)
                x ^= 0x11D;
        }
        exp[255] = exp[0];
        std::memset(log, 0, sizeof log);
        for (int i = 0; i < 255; ++i)
            log[exp[i]] = (uint8_t)i;
    }
    uint8_t mul(uint8_t a, uint8_t b) const
    {
        if (!a || !b)
            return 0;
        return exp[(log[a] + log[b]) % 255];
    }
};
const GfHost& gf()
{
    static GfHost g;
    return g;
}

// 1 KiB block: EXP2[512] | LOG[256] | QS[256]
void build_gf_block(uint8_t* out)
{
    const GfHost& g = gf();
    for (int i = 0; i < 512; ++i)
        out[i] = g.exp[i % 255];
    std::memcpy(out + 512, g.log, 256);
    uint8_t* qs = out + 768;
    std::memset(qs, 0, 256);
    for (int y = 2; y < 256; ++y) {
        const uint8_t c = (uint8_t)(g.mul((uint8_t)y, (uint8_t)y) ^ y);
        if (!qs[c])
            qs[c] = (uint8_t)y;
    }
}

// generator g(x) = prod_{i=1..2t}(x + alpha^i), low -> high (rs_block_device.cpp:195-208)
std::vector<uint8_t> rs_generator(int t2)
{
    const GfHost& G = gf();
    std::vector<uint8_t> g(1, 1);
    uint8_t power = 2;
    for (int i = 0; i < t2; ++i) {
        std::vector<uint8_t> ng(g.size() + 1, 0);
        for (size_t k = 0; k < g.size(); ++k) {
            ng[k] ^= G.mul(g[k], power);
            ng[k + 1] ^= g[k];
        }
        g.swap(ng);
        power = G.mul(power, 2);
    }
    return g;
}

// x^e mod g (monic, degree t2): returns t2 coefficients
std::vector<uint8_t> rs_xpow_mod(int e, const std::vector<uint8_t>& g, int t2)
{
    const GfHost& G = gf();
    std::vector<uint8_t> r(t2, 0);
    r[0] = 1;
    if (t2 == 0)
        return r;
    for (int k = 0; k < e; ++k) {
        const uint8_t top = r[t2 - 1];
        for (int q = t2 - 1; q >= 1; --q)
            r[q] = (uint8_t)(r[q - 1] ^ G.mul(top, g[q]));
        r[0] = G.mul(top, g[0]);
    }
    return r;
}

// slicing tables for the fast path (see rs_kernels.hip: slice8)
std::vector<uint8_t> build_rs_slice_tables(int t2)
{
    const GfHost& G = gf();
    const int W = t2 <= 8 ? 2 : (t2 <= 16 ? 4 : 8);
    const int bytes = ppfs_rs_fast_tables_bytes(t2);
    std::vector<uint8_t> out((size_t)bytes, 0);
    const std::vector<uint8_t> g = rs_generator(t2);
    for (int i = 0; i < 8; ++i) {
        const std::vector<uint8_t> xi = rs_xpow_mod(t2 + i, g, t2);
        for (int h = 0; h < 2; ++h) {
            for (int v = 0; v < 16; ++v) {
                const uint8_t val = (uint8_t)(v << (4 * h));
                uint8_t entry[32] = { 0 };
                for (int q = 0; q < t2; ++q)
                    entry[4 * W - t2 + q] = G.mul(val, xi[q]);
                const size_t slot = (size_t)((2 * i + h) * 16 + v) * 16;
                if (W <= 4) {
                    std::memcpy(&out[slot], entry, (size_t)(4 * W));
                } else {
                    std::memcpy(&out[slot], entry, 16);
                    std::memcpy(&out[4096 + slot], entry + 16, 16);
                }
            }
        }
    }
    return out;
}

// tables of the workgroup-cooperative RS path, 2t <= 8 (layout: rs_layout.hpp)
template <int T2> std::vector<uint8_t> build_rs_wg_tables_t()
{
    using L = ppfs::RsWgLayout<T2>;
    const GfHost& G = gf();
    std::vector<uint8_t> out((size_t)L::BLOB_BYTES, 0);
    const std::vector<uint8_t> g = rs_generator(T2);
    // top-aligned 8-byte entry of a remainder r (coefficient q at byte 8 - 2t + q)
    auto put = [&](int off, int table, int v, const std::vector<uint8_t>& r, uint8_t scale) {
        for (int q = 0; q < T2; ++q)
            out[(size_t)off + (size_t)table * L::TBL + (size_t)v * L::ES + (8 - T2 + q)] = G.mul(scale, r[q]);
    };
    for (int i = 0; i < 8; ++i) {
        const std::vector<uint8_t> xi = rs_xpow_mod(T2 + i, g, T2);
        for (int h = 0; h < 2; ++h)
            for (int v = 0; v < 16; ++v)
                put(L::OFF_SL, 2 * i + h, v, xi, (uint8_t)(v << (4 * h)));
    }
    for (int m = 0; m < 3; ++m)
        for (int q = 0; q < T2; ++q) {
            const std::vector<uint8_t> xq = rs_xpow_mod(q + 64 * (m + 1), g, T2);
            for (int h = 0; h < 2; ++h)
                for (int v = 0; v < 16; ++v)
                    put(L::OFF_MAP + m * L::MAP_STRIDE, 2 * q + h, v, xq, (uint8_t)(v << (4 * h)));
        }
    for (int m = 0; m < 7; ++m)
        for (int q = 0; q < T2; ++q) {
            const std::vector<uint8_t> xq = rs_xpow_mod(q + 32 * (m + 1), g, T2);
            for (int h = 0; h < 2; ++h)
                for (int v = 0; v < 16; ++v)
                    put(L::OFF_MAP32 + m * L::MAP_STRIDE, 2 * q + h, v, xq, (uint8_t)(v << (4 * h)));
        }
    for (int m = 1; m <= 3; ++m)
        for (int i = 0; i < 8; ++i) {
            const std::vector<uint8_t> xi = rs_xpow_mod(T2 + i + 64 * m, g, T2);
            for (int h = 0; h < 2; ++h)
                for (int v = 0; v < 16; ++v)
                    put(L::OFF_SLX + (m - 1) * 16 * L::TBL, 2 * i + h, v, xi, (uint8_t)(v << (4 * h)));
        }
    for (int q = 0; q < T2; ++q)
        for (int h = 0; h < 2; ++h)
            for (int v = 0; v < 16; ++v)
                for (int i = 1; i <= T2; ++i) {
                    const int e = ((i * (q - T2)) % 255 + 255) % 255;
                    out[(size_t)L::OFF_SYN + (size_t)(2 * q + h) * L::TBL + (size_t)v * L::ES + (i - 1)] =
                        G.mul((uint8_t)(v << (4 * h)), G.exp[e]);
                }
    build_gf_block(out.data() + L::OFF_GF);
    const std::vector<uint16_t> es = ppfs::sched::build_encode(T2);
    std::memcpy(out.data() + L::OFF_ESCHED, es.data(), es.size() * sizeof(uint16_t));
    const std::vector<uint8_t> rm = ppfs::sched::row_map(L::K);
    std::memcpy(out.data() + L::OFF_ROWMAP, rm.data(), rm.size());
    // SL5 / SLX5 from the nibble tables by linearity: bit m of the 64-bit chunk (byte m / 8, nibble
    // half (m % 8) / 4, bit m % 4) contributes nibble table 2 (m / 8) + (m % 8) / 4, entry 1 << (m % 4)
    auto five = [&](int nib_off, int five_off) {
        for (int i = 0; i < 13; ++i)
            for (int v = 0; v < 32; ++v)
                for (int k = 0; k < 5; ++k) {
                    const int m = 5 * i + k;
                    if (!(v >> k & 1) || m >= 64)
                        continue;
                    const size_t src = (size_t)nib_off + (size_t)(2 * (m / 8) + (m % 8) / 4) * L::TBL + (size_t)(1 << (m % 4)) * L::ES;
                    const size_t dst = (size_t)five_off + (size_t)i * 32 * L::ES + (size_t)v * L::ES;
                    for (int b = 0; b < L::ES; ++b)
                        out[dst + (size_t)b] ^= out[src + (size_t)b];
                }
    };
    five(L::OFF_SL, L::OFF_SL5);
    for (int m = 0; m < 3; ++m)
        five(L::OFF_SLX + m * 16 * L::TBL, L::OFF_SLX5 + m * L::SL5_BYTES);
    return out;
}

// tables of the pair RS path, 16 < 2t <= 32 (layout: rs_layout.hpp RsPairLayout)
std::vector<uint8_t> build_rs_pair_tables(int t2)
{
    const GfHost& G = gf();
    std::vector<uint8_t> out((size_t)ppfs::rs_pair_table_bytes(), 0);
    const std::vector<uint8_t> g = rs_generator(t2);
    for (int i = 0; i < 8; ++i) {
        const std::vector<uint8_t> xi = rs_xpow_mod(t2 + i, g, t2);
        for (int h = 0; h < 2; ++h)
            for (int v = 0; v < 16; ++v) {
                uint8_t entry[32] = { 0 };
                for (int q = 0; q < t2; ++q)
                    entry[32 - t2 + q] = G.mul((uint8_t)(v << (4 * h)), xi[q]);
                for (int c = 0; c < 2; ++c)
                    std::memcpy(&out[(size_t)(2 * i + h) * 512 + (size_t)c * 256 + (size_t)v * 16], entry + 16 * c, 16);
            }
    }
    build_gf_block(out.data() + 16 * 512);
    uint8_t* xp = out.data() + 16 * 512 + 1024;
    std::memset(xp, 0xFF, 255 * 32);
    for (int p = 0; p < 255; ++p) {
        const std::vector<uint8_t> xr = rs_xpow_mod(p + t2, g, t2);
        for (int q = 0; q < t2; ++q)
            if (xr[q])
                xp[p * 32 + (32 - t2 + q)] = G.log[xr[q]];
    }
    // the same rows for x^p mod g: the single-error check on c mod g (rs_pair.hpp, RM decode)
    uint8_t* xpm = xp + 255 * 32;
    std::memset(xpm, 0xFF, 255 * 32);
    for (int p = 0; p < 255; ++p) {
        const std::vector<uint8_t> xr = rs_xpow_mod(p, g, t2);
        for (int q = 0; q < t2; ++q)
            if (xr[q])
                xpm[p * 32 + (32 - t2 + q)] = G.log[xr[q]];
    }
    // byte-slice tables (rs_bs.hpp): by linearity, byte v at chunk position q maps to the XOR of
    // its two nibble entries; row v, slot 2q + c
    uint8_t* bs = xpm + 255 * 32;
    for (int v = 0; v < 256; ++v)
        for (int q = 0; q < 8; ++q)
            for (int c = 0; c < 2; ++c)
                for (int k = 0; k < 16; ++k)
                    bs[v * 256 + (2 * q + c) * 16 + k] = out[(size_t)(2 * q) * 512 + (size_t)c * 256 + (size_t)(v & 15) * 16 + k]
                        ^ out[(size_t)(2 * q + 1) * 512 + (size_t)c * 256 + (size_t)(v >> 4) * 16 + k];
    // S_1, S_2 contributions of the c mod g state bytes (rs_bs.hpp bs_correct; coefficient q of
    // the state is byte 32 - 2t + q, exponent i q)
    uint8_t* s12 = bs + 256 * 256;
    for (int u = 0; u < 32; ++u) {
        const int q = u - (32 - t2);
        for (int v = 0; v < 256; ++v) {
            if (q < 0)
                continue;
            s12[u * 512 + 2 * v] = G.mul((uint8_t)v, G.exp[q % 255]);
            s12[u * 512 + 2 * v + 1] = G.mul((uint8_t)v, G.exp[(2 * q) % 255]);
        }
    }
    return out;
}

std::vector<uint8_t> build_rs_fast_tables_uncached(int t2)
{
    if (t2 > 16)
        return build_rs_pair_tables(t2);
    switch (t2) {
    case 2:
        return build_rs_wg_tables_t<2>();
    case 4:
        return build_rs_wg_tables_t<4>();
    case 6:
        return build_rs_wg_tables_t<6>();
    case 8:
        return build_rs_wg_tables_t<8>();
    default: {
        std::vector<uint8_t> s = build_rs_slice_tables(t2);
        s.resize(s.size() + 1024);
        build_gf_block(s.data() + s.size() - 1024);
        return s;
    }
    }
}

// the blob depends on 2t only; built once per process (the emission schedule search of the t <= 4
// layouts takes tens of ms)
std::vector<uint8_t> build_rs_fast_tables(int t2)
{
    static std::mutex mu;
    static std::map<int, std::vector<uint8_t>> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(t2);
    if (it == cache.end())
        it = cache.emplace(t2, build_rs_fast_tables_uncached(t2)).first;
    return it->second;
}

// ---------------------------------------------------------------------------------------
// CRC host maths over GF(2)[x] / P  (P explicit, degree n <= 63)
// ---------------------------------------------------------------------------------------
struct CrcHost {
    uint64_t P;
    int n;
    uint64_t mask;
    uint64_t mod(uint64_t a) const // reduce a polynomial of degree <= 63
    {
        for (int k = 63; k >= n; --k)
            if ((a >> k) & 1u)
                a ^= P << (k - n);
        return a;
    }
    uint64_t mulx(uint64_t a) const
    {
        const bool top = (a >> (n - 1)) & 1u;
        a = (a << 1) & mask;
        return top ? a ^ (P & mask) : a;
    }
    uint64_t mul(uint64_t a, uint64_t b) const // a*b mod P (a, b reduced)
    {
        uint64_t r = 0;
        for (int k = n - 1; k >= 0; --k) {
            r = mulx(r);
            if ((b >> k) & 1u)
                r ^= a;
        }
        return r;
    }
    uint64_t xpow(long e) const // x^e mod P, e may be negative (x is invertible: P(0) = 1)
    {
        uint64_t base = e >= 0 ? mod(2u) : (P >> 1); // x or x^-1 = (P - 1)/x
        if (e < 0)
            e = -e;
        uint64_t r = mod(1u);
        while (e) {
            if (e & 1)
                r = mul(r, base);
            base = mul(base, base);
            e >>= 1;
        }
        return r;
    }
};

std::vector<uint8_t> build_crc_tables(uint64_t P, int n, uint32_t ds)
{
    CrcHost c { P, n, n == 64 ? ~0ull : ((1ull << n) - 1) };
    const uint32_t G = (ds + 63) / 64;
    const long z = 64L * G - ds;
    std::vector<uint8_t> out((size_t)ppfs_crc_tables_bytes(), 0);
    uint64_t* pt = (uint64_t*)out.data();
    for (int pos = 0; pos < 64; ++pos) {
        const uint64_t f = c.xpow(8L * (63 - pos) + n - 8 * z - 1);
        for (int h = 0; h < 2; ++h)
            for (int v = 0; v < 16; ++v)
                pt[(pos * 2 + h) * 16 + v] = c.mul(c.mod((uint64_t)v << (4 * h)), f);
    }
    uint64_t* lv = (uint64_t*)(out.data() + 64 * 2 * 16 * 8);
    for (int j = 0; j < 6; ++j) {
        const uint64_t f = c.xpow(512L << j);
        for (int k = 0; k < 16; ++k)
            for (int v = 0; v < 16; ++v)
                lv[(j * 16 + k) * 16 + v] = (4 * k < 64) ? c.mul(c.mod((uint64_t)v << (4 * k)), f) : 0;
    }
    return out;
}

// Maps of the CRC fast path (bit_fast.hip, n <= 32), at the offsets bit_fast.hip reports
// (ppfs_crc_fast_layout): nibble maps (8 nibble tables x 16 u32 entries, T[i][v] = (v << 4i) * C mod
// P for a constant C = x^e mod P): x^0, x^32, x^64, x^96 (piece dwords), x^8192 (one lane's pieces,
// 1 KiB apart), x^(128 2^j) j < 6 (lane tree; the kernels use j = 4, 5 after the lane maps), the
// encode's placement factors x^(8 (ds + m - 1024 (NP + 1)) + n - 1) for each payload misalignment
// m < 16 and the check's x^(8 (ds - bs) + n - 1); the 16 transposed lane maps; the 6-bit tree maps;
// the 8-bit piece / Horner maps.
std::vector<uint8_t> build_crc_fast_tables(uint64_t P, int n, uint32_t ds, uint32_t bs)
{
    struct Lay {
        int32_t map, nmaps, lane_off, lanes, six_off, nsix, map6, eight_off, neight, eight, bytes;
    } ly;
    if (ppfs_crc_fast_layout((int32_t*)&ly, (int)(sizeof(ly) / 4)) != (int)(sizeof(ly) / 4) || ly.map != 8 * 16 * 4
        || ly.lane_off < ly.nmaps * ly.map || ly.six_off < ly.lane_off + ly.lanes * ly.map
        || ly.eight_off < ly.six_off + ly.nsix * ly.map6 || ly.bytes < ly.eight_off + ly.neight * ly.eight || ly.neight != 5
        || ly.nsix != 2 || ly.map6 < 5 * 256 + 16 || ly.eight != 4096)
        return {}; // the device layout changed under this builder: refuse (create fails) rather than misplace
    CrcHost c { P, n, n == 64 ? ~0ull : ((1ull << n) - 1) };
    const long NP = bs / 1024;
    std::vector<long> ex = { 0, 32, 64, 96, 8192 };
    for (int j = 0; j < 6; ++j)
        ex.push_back(128L << j);
    for (long m = 0; m < 16; ++m)
        ex.push_back(8L * ((long)ds + m - 1024L * (NP + 1)) + n - 1);
    ex.push_back(8L * ((long)ds - (long)bs) + n - 1);
    if ((int)ex.size() != ly.nmaps)
        return {};

    std::vector<uint8_t> out((size_t)ly.bytes, 0);
    auto nibble_map = [&](uint8_t* dst, long e) {
        const uint64_t C = c.xpow(e);
        uint32_t* t = (uint32_t*)dst;
        for (int i = 0; i < 8; ++i)
            for (int v = 0; v < 16; ++v)
                t[i * 16 + v] = (uint32_t)c.mul(c.mod((uint64_t)v << (4 * i)), C);
    };
    for (size_t mi = 0; mi < ex.size(); ++mi)
        nibble_map(out.data() + mi * ly.map, ex[mi]);
    // lane maps: lane b of NL = 16 multiplies by x^(128 (NL - 1 - b)), transposed: dword (16 i + v) NL + b
    const int NL = ly.lanes;
    uint32_t* lt = (uint32_t*)(out.data() + ly.lane_off);
    for (int b = 0; b < NL; ++b) {
        const uint64_t C = c.xpow(128L * (NL - 1 - b));
        for (int i = 0; i < 8; ++i)
            for (int v = 0; v < 16; ++v)
                lt[(16 * i + v) * NL + b] = (uint32_t)c.mul(c.mod((uint64_t)v << (4 * i)), C);
    }
    // 6-bit tables of the lane-tree maps x^2048, x^4096 (bit_fast.hip CF_MAP6): sub-table j < 5 = 64
    // entries (v << 6j) C, then 4 entries (v << 30) C
    for (int q = 0; q < 2; ++q) {
        const uint64_t C = c.xpow(ex[9 + q]);
        uint32_t* e = (uint32_t*)(out.data() + ly.six_off + q * ly.map6);
        for (int j = 0; j < 5; ++j)
            for (int v = 0; v < 64; ++v)
                e[64 * j + v] = (uint32_t)c.mul(c.mod((uint64_t)v << (6 * j)), C);
        for (int v = 0; v < 4; ++v)
            e[320 + v] = (uint32_t)c.mul(c.mod((uint64_t)v << 30), C);
    }
    // 8-bit tables (bit_fast.hip CF_EIGHT): x^0, x^32, x^64, x^96 indexed by the bytes of the payload
    // dword in memory order (table k = byte 3 - k of the value), x^8192 by the bytes of a value
    uint32_t* e8 = (uint32_t*)(out.data() + ly.eight_off);
    for (int q = 0; q < 5; ++q) {
        const uint64_t C = c.xpow(ex[q]);
        for (int k = 0; k < 4; ++k) {
            const int vb = q < 4 ? 3 - k : k; // the value byte that input byte k holds
            for (int v = 0; v < 256; ++v)
                e8[q * 1024 + k * 256 + v] = (uint32_t)c.mul(c.mod((uint64_t)v << (8 * vb)), C);
        }
    }
    return out;
}

int bitlen64(uint64_t v)
{
    int c = 0;
    while (v) {
        v >>= 1;
        c++;
    }
    return c;
}

} // namespace

// ---------------------------------------------------------------------------------------
// Context
// ---------------------------------------------------------------------------------------
struct ppfs_ecc_ctx {
    ppfs_ecc_params p {};
    int device = 0;
    // derived
    uint32_t raw = 0, data = 0;
    int rs_n = 0, rs_t2 = 0;
    bool rs_fast = false;
    int crc_n = 0;
    uint64_t crc_mask = 0;
    uint32_t ham_L = 0;
    const char* kname = "";
    // device tables
    uint8_t* d_tables = nullptr;
    // ticket counters of the dynamic-tile t <= 4 encode and decode (rs_wg_tk.hpp): per stream that
    // runs them through this context a slot of two 2,560-byte sets (launch parity), each an encode
    // half then a decode half.  A launch counts on one set and zeroes the other, which the previous
    // launch of the same kind on the stream used (launches on one stream are ordered; no two streams
    // share a slot); tk_par = the set the next launch of each kind uses.  Further streams use the
    // static walk.
    // Ordering (round 4): a slot remembers the caller-stream event slot (ev[] below) of the stream
    // that last launched on it; a slot passes to another stream only once that event has completed,
    // and every device call first waits for the previous call's event on its stream handle, so a
    // stream created at a destroyed stream's address never runs beside a kernel still counting on
    // the old stream's set.
    static constexpr int kTkSlots = 16, kTkSetWords = 1024; // encode 512 words (rs_wq: 32 counters 64 B apart), decode 512
    uint32_t* d_ctr = nullptr;
    hipStream_t tk_stream[kTkSlots] = {};
    uint8_t tk_par[kTkSlots][2] = {};
    int tk_ev[kTkSlots] = {}; // ev[] slot of the slot's last user
    int tk_n = 0;
    // scratch for write_device status when the caller passes none
    uint8_t* d_scratch = nullptr;
    size_t scratch_bytes = 0;
    // host staging (round 5): a stream per link direction, so that chunk i + 1's H2D runs beside
    // chunk i's D2H (with a stream per slot the slots fell into lockstep: both H2Ds, then both
    // D2Hs, one link direction idle at a time); an event per slot orders its kernel after its H2D.
    // hs[0]: H2D copies (SDMA), the small-batch path and decode write-back fix-ups; hs[1]: kernels
    // and D2H copies (the runtime's D2H into page-locked memory is a blit kernel anyway).  Two, not
    // one per stage: a process gets few hardware queues (GPU_MAX_HW_QUEUES, 4 by default) and
    // streams beyond them share queues with torch's -- measured: 4 streams ran slower in bench.py's
    // process than in a torch-free one
    static constexpr int kSlots = 3, kHostStreams = 2;
    hipStream_t hs[kHostStreams] = {};
    hipEvent_t hev[kSlots][2] = {}; // per slot: inputs landed, outputs landed
    uint8_t* h_pin[kSlots] = {};
    uint8_t* d_stage[kSlots] = {};
    size_t stage_bytes = 0;
    bool host_eager = false; // the last chunked decode's write-back predictor, where the next one starts
    // zero-copy staging for small host batches (the per-block IBlockDevice calls): coherent
    // host memory the kernels read and write in place, no H2D / D2H
    uint8_t* h_zc = nullptr;
    uint8_t* d_zc = nullptr;
    size_t zc_bytes = 0;
    // resident small-batch server (RS 2t <= 8, server_box.hpp): mailbox, its stream, the current
    // launch generation, the last request number; srv_ok = -1 undecided, 0 off, 1 on
    ppfs::SrvBox* h_box = nullptr;
    ppfs::SrvBox* d_box = nullptr;
    hipStream_t srv_stream = nullptr;
    uint32_t srv_gen = 0, srv_seq = 0, flag_seq = 0;
    bool srv_launched = false;
    int srv_ok = -1;
    // a resident launch that did not leave when asked (server_stop): the context is unusable and
    // destroy leaks what the launch may still read instead of freeing it under it
    bool srv_stuck = false;
    // Completion of the work this context queued on CALLER streams (the device entry points):
    // one fence-free event per stream, re-recorded after every call, so that destroy waits for
    // exactly that work (it reads the tables, counters and scratch destroy frees) and not for the
    // whole device -- other contexts' resident servers, unrelated torch streams.  A stream beyond
    // kEvSlots sets ev_overflow and destroy falls back to a device-wide synchronize.
    static constexpr int kEvSlots = 32;
    hipStream_t ev_stream[kEvSlots] = {};
    hipEvent_t ev[kEvSlots] = {};
    bool ev_rec[kEvSlots] = {}; // recorded at least once
    int ev_n = 0;
    bool ev_overflow = false;
    // the context's own stream for its stream-ordered device allocations (mem_alloc / mem_free)
    hipStream_t ms = nullptr;
    size_t pin_bytes = 0; // bytes of each h_pin[] buffer (pin cache key)
};

// PPFS_ECC_TRACE=1 (diagnostics): timestamped steps of context creation on stderr
static void trace_step(const char* what)
{
    static const bool on = [] {
        const char* v = std::getenv("PPFS_ECC_TRACE");
        return v && *v && *v != '0';
    }();
    if (!on)
        return;
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    std::fprintf(stderr, "[ppfs_ecc %.6f] %s\n", t, what);
}

namespace {
// ---------------------------------------------------------------------------------------
// Memory that never synchronizes the device when it is freed.  hipFree and hipHostFree wait for
// every stream of the device, so a context destroyed (or resizing its staging) beside another
// context's resident server, or beside a long kernel of the caller's, waited for them -- 1 to 51 s
// in r3d's destroy test.  Device buffers come from the stream-ordered pool on the context's own
// stream (hipFreeAsync after the work that reads them is known complete); page-locked host
// buffers go back to a process-wide cache (exact size and flags) instead of hipHostFree.
// ---------------------------------------------------------------------------------------
#ifdef PPFS_ECC_DEBUG
// PPFS_ECC_DEBUG: the engine's stream-ordered device allocations, for dma_async's range check
// (the runtime keeps no address-range record for pool memory)
std::mutex g_pool_mu;
std::map<uintptr_t, size_t> g_pool;
void pool_note(void* p, size_t n)
{
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (n)
        g_pool[(uintptr_t)p] = n;
    else
        g_pool.erase((uintptr_t)p);
}
bool pool_covers(const void* p, size_t n)
{
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto it = g_pool.upper_bound((uintptr_t)p);
    if (it == g_pool.begin())
        return false;
    --it;
    return (uintptr_t)p >= it->first && (uintptr_t)p + n <= it->first + it->second;
}
#else
inline void pool_note(void*, size_t) {}
#endif
// hipMallocAsync on stream s (recorded for the debug build's copy checks)
hipError_t pool_alloc(void** p, size_t n, hipStream_t s)
{
    const hipError_t e = hipMallocAsync(p, n, s);
    if (e == hipSuccess)
        pool_note(*p, n);
    return e;
}
void pool_free(void* p, hipStream_t s)
{
    if (!p)
        return;
    pool_note(p, 0);
    (void)hipFreeAsync(p, s);
}

hipError_t mem_alloc(ppfs_ecc_ctx* c, void** p, size_t n)
{
    *p = nullptr;
    if (!c->ms) {
        const hipError_t e = hipStreamCreateWithFlags(&c->ms, hipStreamNonBlocking);
        trace_step("mem_alloc: stream created");
        if (e != hipSuccess)
            return e;
    }
    hipError_t e = pool_alloc(p, n, c->ms);
    trace_step("mem_alloc: pool allocation queued");
    if (e == hipSuccess)
        e = hipStreamSynchronize(c->ms); // usable from any stream from here on
    trace_step("mem_alloc: stream synchronized");
    return e;
}
// caller: nothing still queued reads p
void mem_free(ppfs_ecc_ctx* c, void* p)
{
    pool_free(p, c->ms);
}

struct PinCache {
    std::mutex mu;
    std::multimap<std::pair<size_t, unsigned>, void*> idle;
    size_t idle_bytes = 0;
    static constexpr size_t kMaxIdle = 512ull << 20;
};
PinCache& pin_cache()
{
    static PinCache* pc = new PinCache(); // never destroyed: buffers may be returned at process exit
    return *pc;
}
hipError_t pin_alloc(void** p, size_t n, unsigned flags)
{
    PinCache& pc = pin_cache();
    {
        std::lock_guard<std::mutex> lk(pc.mu);
        auto it = pc.idle.find({ n, flags });
        if (it != pc.idle.end()) {
            *p = it->second;
            pc.idle.erase(it);
            pc.idle_bytes -= n;
            return hipSuccess;
        }
    }
    return hipHostMalloc(p, n, flags);
}
// caller: nothing still queued reads or writes p
void pin_free(void* p, size_t n, unsigned flags)
{
    if (!p)
        return;
    PinCache& pc = pin_cache();
    {
        std::lock_guard<std::mutex> lk(pc.mu);
        if (pc.idle_bytes + n <= PinCache::kMaxIdle) {
            pc.idle.insert({ { n, flags }, p });
            pc.idle_bytes += n;
            return;
        }
    }
    (void)hipHostFree(p); // beyond the cache: the synchronizing free
}
constexpr unsigned kPinStage = hipHostMallocDefault, kPinMapped = hipHostMallocMapped | hipHostMallocCoherent;

// Is s capturing a hipGraph?  Work queued then runs later, once per replay, possibly on another
// stream or concurrently with itself.
bool capturing(hipStream_t s)
{
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return st != hipStreamCaptureStatusNone;
}

// The caller-stream event slot of handle s (-1: none, and with `create` none could be made).
int ev_slot(ppfs_ecc_ctx* c, hipStream_t s, bool create)
{
    int i = 0;
    while (i < c->ev_n && c->ev_stream[i] != s)
        ++i;
    if (i < c->ev_n)
        return i;
    if (!create)
        return -1;
    if (c->ev_n == ppfs_ecc_ctx::kEvSlots
        || hipEventCreateWithFlags(&c->ev[i], hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) {
        (void)hipGetLastError();
        c->ev_overflow = true;
        return -1;
    }
    c->ev_stream[i] = s;
    c->ev_rec[i] = false;
    c->ev_n++;
    return i;
}

// The context's own host-path streams -- compared only once they exist: before the host path first
// runs they are null, which is also the default stream's handle.
static bool own_stream(const ppfs_ecc_ctx* c, hipStream_t s)
{
    for (hipStream_t h : c->hs)
        if (h && s == h)
            return true;
    return false;
}

// Before a device entry point queues work on caller stream s: order it after the last call queued
// on the same handle.  For the same stream the runtime returns at once (an event recorded on the
// waiting stream itself); it matters when s is a new stream created at the address of a destroyed
// one whose work may still run: the new stream's kernels then never share that work's ticket set
// (ctr_for) or outlive-check (destroy waits on the event re-recorded after this call).
void order_caller_stream(ppfs_ecc_ctx* c, hipStream_t s)
{
    static const bool off = [] { // diagnostics: PPFS_ECC_NO_ORDER=1 skips the wait
        const char* v = std::getenv("PPFS_ECC_NO_ORDER");
        return v && *v && *v != '0';
    }();
    if (off || own_stream(c, s) || capturing(s))
        return;
    const int i = ev_slot(c, s, false);
    if (i >= 0 && c->ev_rec[i] && hipStreamWaitEvent(s, c->ev[i], 0) != hipSuccess)
        (void)hipGetLastError();
}

// The ticket-counter set of stream s (nullptr: the static-walk kernel runs).  A set is shared by
// every launch on its stream, which is safe only because launches on one stream are ordered.  A
// launch captured into a graph gets no set: its replays may run on other streams or overlap each
// other (two kernels on one set would skip or repeat tiles).  A stream without a slot takes a free
// one, or one whose last user's work has completed (its event); with none, or without a caller
// event slot to order it by, it falls back to the static walk.  ppfs_ecc_stream_kernel_name reports
// which path a stream gets.
struct TkSets {
    uint32_t* mine = nullptr;  // the set this launch counts on
    uint32_t* clear = nullptr; // the set it zeroes (the previous launch's)
    int slot = -1, op = 0;
};
// the slot stream s would use (-1: none); with `take`, assign it
int tk_slot(ppfs_ecc_ctx* c, hipStream_t s, bool take)
{
    if (!c->d_ctr || capturing(s))
        return -1;
    const int e = ev_slot(c, s, take);
    if (take && e < 0)
        return -1;
    int i = 0;
    while (i < c->tk_n && c->tk_stream[i] != s)
        ++i;
    if (i == c->tk_n) {
        if (c->tk_n < ppfs_ecc_ctx::kTkSlots) {
            if (take)
                c->tk_n++;
        } else {
            // recycle a slot whose last user's work is complete (the event query is not a wait);
            // the set its next launch counts on was zeroed by that completed work
            i = -1;
            for (int j = 0; j < c->tk_n && i < 0; ++j) {
                if (!c->ev_rec[c->tk_ev[j]]) // its last record failed: nothing tells when it is done
                    continue;
                const hipError_t q = hipEventQuery(c->ev[c->tk_ev[j]]);
                if (q == hipSuccess)
                    i = j;
                else if (q != hipErrorNotReady)
                    (void)hipGetLastError();
            }
            if (i < 0)
                return -1;
        }
        if (take)
            c->tk_stream[i] = s;
    }
    if (take)
        c->tk_ev[i] = e;
    return i;
}
TkSets ctr_for(ppfs_ecc_ctx* c, hipStream_t s, int op /* 0 encode, 1 decode */)
{
    TkSets t;
    const int i = tk_slot(c, s, true);
    if (i < 0)
        return t;
    const int par = c->tk_par[i][op];
    uint32_t* base = c->d_ctr + (size_t)i * 2 * ppfs_ecc_ctx::kTkSetWords + (size_t)op * (ppfs_ecc_ctx::kTkSetWords / 2);
    t.mine = base + (size_t)par * ppfs_ecc_ctx::kTkSetWords;
    t.clear = base + (size_t)(par ^ 1) * ppfs_ecc_ctx::kTkSetWords;
    t.slot = i;
    t.op = op;
    return t;
}
// after a launch with sets t went into the stream: the next launch of its kind uses the other set
// (a launch that failed to enqueue zeroed nothing and counted on nothing: the parity stays)
hipError_t tk_commit(ppfs_ecc_ctx* c, const TkSets& t, hipError_t e)
{
    if (e == hipSuccess && t.slot >= 0)
        c->tk_par[t.slot][t.op] ^= 1;
    return e;
}

// After a device entry point queued work on caller stream s: (re-)record s's completion event.
// Captured work is the graph's: the caller keeps the context alive while graphs that use it exist.
void note_caller_stream(ppfs_ecc_ctx* c, hipStream_t s)
{
    // the context's own streams (destroy drains them) -- compared only once they exist: before the
    // host path first runs they are null, which is also the default stream's handle, and work on
    // the default stream must be tracked like any other caller stream's
    if (own_stream(c, s) || capturing(s))
        return;
    const int i = ev_slot(c, s, true);
    if (i < 0)
        return; // ev_overflow: destroy synchronizes the device
    if (hipEventRecord(c->ev[i], s) != hipSuccess) {
        (void)hipGetLastError();
        c->ev_overflow = true;
        c->ev_rec[i] = false;
        return;
    }
    c->ev_rec[i] = true;
}
} // namespace

// every copy the engine queues (checked in PPFS_ECC_DEBUG builds; defined with host_pinned below)
static hipError_t dma_async(void* dst, const void* src, size_t n, hipMemcpyKind kind, hipStream_t s);

extern "C" uint64_t ppfs_ecc_crc_implicit_to_explicit(uint64_t implicit_poly) { return (implicit_poly << 1) + 1; }

extern "C" const char* ppfs_ecc_last_error(void) { return g_last_error.c_str(); }

extern "C" int ppfs_ecc_create(const ppfs_ecc_params* params, int device, ppfs_ecc_ctx** out)
{
    if (!params || !out)
        return fail(PPFS_ECC_EINVAL, "null argument");
    *out = nullptr;
    const ppfs_ecc_params p = *params;
    if (p.block_size == 0 || p.block_size > 4096)
        return fail(PPFS_ECC_EINVAL, "block_size must be in [1, 4096] (MAX_BLOCK_SIZE)");
    ppfs_ecc_ctx* c = new (std::nothrow) ppfs_ecc_ctx();
    if (!c)
        return fail(PPFS_ECC_ENOMEM, "ctx alloc");
    c->p = p;
    c->device = device;
    std::vector<uint8_t> tables;
    switch (p.ecc_type) {
    case PPFS_ECC_NONE:
        c->raw = c->data = p.block_size;
        c->kname = "raw-copy";
        break;
    case PPFS_ECC_REED_SOLOMON: {
        c->rs_n = (int)std::min<uint32_t>(p.block_size, 255);
        const int t = (int)std::min<uint32_t>(p.rs_correctable_bytes, (uint32_t)c->rs_n / 2);
        c->rs_t2 = 2 * t;
        c->raw = (uint32_t)c->rs_n;
        c->data = (uint32_t)(c->rs_n - c->rs_t2);
        c->rs_fast = ppfs_rs_fast_supported(c->rs_n, c->rs_t2) != 0;
        tables.resize(4096 + 8192 + 1024, 0);
        if (c->rs_fast) {
            tables = build_rs_fast_tables(c->rs_t2);
            c->kname = ppfs_rs_fast_path(c->rs_t2);
        } else {
            tables.assign(1024 + 256, 0);
            build_gf_block(tables.data());
            std::vector<uint8_t> g = rs_generator(c->rs_t2);
            std::memcpy(tables.data() + 1024, g.data(), g.size());
            c->kname = "rs-generic-lfsr";
        }
        break;
    }
    case PPFS_ECC_CRC: {
        const int n = bitlen64(p.crc_polynomial) - 1;
        if (n < 1 || n > 63) {
            delete c;
            return fail(PPFS_ECC_EINVAL, "CRC polynomial degree must be in [1, 63]");
        }
        const uint32_t nbc = (uint32_t)((n + 7) / 8);
        if (p.block_size <= nbc) {
            delete c;
            return fail(PPFS_ECC_EINVAL, "block too small for the CRC");
        }
        c->crc_n = n;
        c->crc_mask = (1ull << n) - 1;
        c->raw = p.block_size;
        c->data = p.block_size - nbc;
        tables = build_crc_tables(p.crc_polynomial, n, c->data);
        if (ppfs_crc_fast_supported(p.block_size, (uint32_t)n)) {
            const std::vector<uint8_t> f = build_crc_fast_tables(p.crc_polynomial, n, c->data, p.block_size);
            if (f.empty()) {
                delete c;
                return fail(PPFS_ECC_EINVAL, "CRC fast tables: device layout mismatch");
            }
            tables.insert(tables.end(), f.begin(), f.end());
        }
        c->kname = ppfs_crc_fast_supported(p.block_size, (uint32_t)n) ? "crc-piecemap-wave" : "crc-nibble-shift";
        break;
    }
    case PPFS_ECC_HAMMING: {
        int pw = 0;
        while ((1u << (pw + 1)) <= p.block_size)
            pw++;
        c->raw = 1u << pw;
        c->data = c->raw - (uint32_t)((3 * pw + 1 + 7) / 8);
        // raw index of the last payload bit (HammingDataBitsIterator, hamming_block_device.cpp:180-198)
        uint32_t idx = 0;
        for (uint32_t i = 0; i < 8 * c->data; ++i) {
            while ((idx & (idx - 1)) == 0)
                idx++;
            c->ham_L = idx++;
        }
        c->kname = ppfs_bitfast_supported(c->raw) ? "hamming-stream-wave"
                                                  : (c->raw < 8 ? "hamming-tiny" : "hamming-funnel");
        break;
    }
    case PPFS_ECC_PARITY: // block_size 1: no payload, the block's own parity (parity_block_device.cpp:9-15)
        c->raw = p.block_size;
        c->data = p.block_size - 1;
        c->kname = ppfs_bitfast_supported(c->raw) ? "parity-stream-wave" : "parity-popcount";
        break;
    default:
        delete c;
        return fail(PPFS_ECC_EINVAL, "unknown ecc_type");
    }
    DeviceGuard guard(device);
    hipError_t e = guard.err;
    if (e != hipSuccess) {
        delete c;
        return fail(PPFS_ECC_EHIP, "hipSetDevice", e);
    }
    trace_step("create: device set");
    if (c->rs_fast && (c->rs_t2 <= 8 || c->rs_t2 == 32)) { // the ticket kernels (rs_wg_tk.hpp, rs_bs.hpp)
        const size_t cb = sizeof(uint32_t) * ppfs_ecc_ctx::kTkSlots * 2 * ppfs_ecc_ctx::kTkSetWords;
        e = mem_alloc(c, (void**)&c->d_ctr, cb);
        trace_step("create: counters allocated");
        if (e == hipSuccess)
            e = hipMemsetAsync(c->d_ctr, 0, cb, c->ms);
        if (e == hipSuccess)
            e = hipStreamSynchronize(c->ms);
        trace_step("create: counters zeroed");
        if (e != hipSuccess) {
            ppfs_ecc_destroy(c);
            return fail(PPFS_ECC_EHIP, "ticket counters", e);
        }
    }
    if (!tables.empty()) {
        // through a page-locked bounce buffer: the engine never hands pageable memory to a copy
        uint8_t* bounce = nullptr;
        e = mem_alloc(c, (void**)&c->d_tables, tables.size());
        trace_step("create: tables allocated");
        if (e == hipSuccess)
            e = pin_alloc((void**)&bounce, tables.size(), kPinStage);
        trace_step("create: bounce buffer");
        if (e == hipSuccess) {
            std::memcpy(bounce, tables.data(), tables.size());
            e = dma_async(c->d_tables, bounce, tables.size(), hipMemcpyHostToDevice, c->ms);
            if (e == hipSuccess)
                e = hipStreamSynchronize(c->ms);
        }
        trace_step("create: tables uploaded");
        if (bounce) {
            // whatever e is: no copy from the bounce may still be queued when it returns to the cache
            if (e != hipSuccess)
                (void)hipStreamSynchronize(c->ms);
            pin_free(bounce, tables.size(), kPinStage);
        }
        if (e != hipSuccess) {
            ppfs_ecc_destroy(c);
            return fail(PPFS_ECC_EHIP, "table upload", e);
        }
    }
    *out = c;
    return 0;
}

// Ask the resident server launch to leave and wait for it, bounded: it polls `stop` every few
// microseconds, so a launch still running after kSrvStopMs has stopped polling (a hung or
// faulted kernel).  Never blocks past the deadline; false = the launch did not leave.
constexpr int kSrvStopMs = 2000;
static bool server_halt(ppfs_ecc_ctx* c)
{
    if (!c->srv_launched)
        return true;
    __atomic_store_n(&c->h_box->stop, 1u, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(c->srv_stream);
        if (e != hipErrorNotReady) {
            (void)hipGetLastError();
            c->srv_launched = false;
            return true;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(kSrvStopMs)) {
            c->srv_stuck = true;
            c->srv_ok = 0;
            return false;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

extern "C" void ppfs_ecc_destroy(ppfs_ecc_ctx* c)
{
    if (!c)
        return;
    DeviceGuard guard(c->device);
    // the resident server leaves at `stop` before anything it reads is freed
    const bool srv_gone = !c->srv_stuck && server_halt(c);
    if (c->srv_stream && srv_gone)
        (void)hipStreamDestroy(c->srv_stream);
    // Nothing the context queued may outlive it, and destroy waits for nothing else:
    //  - its own streams (host paths) drain before they are destroyed and before the staging
    //    buffers their copies and kernels use are freed;
    //  - work it queued on caller streams (device entry points: it reads the tables, ticket
    //    counters and scratch freed below) is waited for through the per-stream completion events
    //    note_caller_stream recorded after every call;
    //  - only when more caller streams were used than there are event slots does destroy fall back
    //    to a device-wide synchronize.
    // Other contexts' resident servers and unrelated streams are not waited for.
    for (hipStream_t h : c->hs)
        if (h)
            (void)hipStreamSynchronize(h);
    for (int i = 0; i < c->ev_n; ++i) {
        (void)hipEventSynchronize(c->ev[i]);
        (void)hipEventDestroy(c->ev[i]);
    }
    if (c->ev_overflow && (c->d_tables || c->d_scratch || c->d_ctr))
        (void)hipDeviceSynchronize();
    (void)hipGetLastError();
    if (!srv_gone) {
        // a launch that ignored `stop` may still read the tables and the mailbox / zero-copy
        // buffers: leak those rather than free memory under a running kernel
        std::fprintf(stderr, "ppfs_ecc_destroy: resident server did not stop within %d ms; its buffers are leaked\n",
            kSrvStopMs);
        c->d_tables = nullptr;
        c->h_zc = nullptr;
        c->h_box = nullptr;
    }
    // frees that never synchronize the device (mem_free, pin_free)
    for (hipStream_t h : c->hs)
        if (h)
            (void)hipStreamDestroy(h);
    for (int i = 0; i < ppfs_ecc_ctx::kSlots; ++i) {
        for (hipEvent_t e : c->hev[i])
            if (e)
                (void)hipEventDestroy(e);
        pin_free(c->h_pin[i], c->pin_bytes, kPinStage);
        mem_free(c, c->d_stage[i]);
    }
    mem_free(c, c->d_tables);
    mem_free(c, c->d_ctr);
    mem_free(c, c->d_scratch);
    pin_free(c->h_zc, c->zc_bytes, kPinMapped);
    pin_free(c->h_box, sizeof(ppfs::SrvBox), kPinMapped); // after the streams drained: flag kernels write it
    if (c->ms)
        (void)hipStreamDestroy(c->ms); // its frees complete first
    delete c;
}

extern "C" size_t ppfs_ecc_raw_block_size(const ppfs_ecc_ctx* c) { return c ? c->raw : 0; }
extern "C" size_t ppfs_ecc_data_size(const ppfs_ecc_ctx* c) { return c ? c->data : 0; }
extern "C" const char* ppfs_ecc_kernel_name(const ppfs_ecc_ctx* c) { return c ? c->kname : ""; }

// PPFS_ECC_DEBUG builds: out-of-bounds global accesses the kernels detected and skipped (dbg.hpp),
// summed over the kernel translation units; -1 in normal builds
#ifdef PPFS_ECC_DEBUG
#define PPFS_DBG_UNITS(X) X(ppfs_dbg_faults_rs_t2) X(ppfs_dbg_faults_rs_t4) X(ppfs_dbg_faults_rs_t6) \
    X(ppfs_dbg_faults_rs_t8) X(ppfs_dbg_faults_rs_t10) X(ppfs_dbg_faults_rs_t16) X(ppfs_dbg_faults_rs_t32)   \
    X(ppfs_dbg_faults_rs_generic) X(ppfs_dbg_faults_bit) X(ppfs_dbg_faults_bitfast) X(ppfs_dbg_faults_vote)
#define PPFS_DBG_DECL(f) extern "C" long long f(void);
PPFS_DBG_UNITS(PPFS_DBG_DECL)
extern "C" long long ppfs_ecc_debug_faults(void)
{
    long long sum = 0;
#define PPFS_DBG_ADD(f)                                                                                                \
    {                                                                                                                  \
        const long long v = f();                                                                                       \
        if (v < 0)                                                                                                     \
            return v;                                                                                                  \
        sum += v;                                                                                                      \
    }
    PPFS_DBG_UNITS(PPFS_DBG_ADD)
    return sum;
}
#else
extern "C" long long ppfs_ecc_debug_faults(void) { return -1; }
#endif

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

static int check_hip(hipError_t e, const char* what)
{
    if (e != hipSuccess)
        return fail(PPFS_ECC_EHIP, what, e);
    return 0;
}

// PPFS_ECC_SYNC_CHECK=1 (debug runs): every device-resident entry point drains its stream and
// reports an asynchronous fault of the work it queued under its own name, instead of at some later
// unrelated call.  Off by default: the entry points are asynchronous.
static bool sync_check_enabled()
{
    static const bool on = [] {
        const char* v = std::getenv("PPFS_ECC_SYNC_CHECK");
        return v && *v && *v != '0';
    }();
    return on;
}

static int sync_check(int r, void* stream, const char* what)
{
    if (r || !sync_check_enabled() || capturing((hipStream_t)stream)) // a capture runs nothing yet
        return r;
    hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    if (e == hipSuccess)
        e = hipGetLastError();
    return e != hipSuccess ? fail(PPFS_ECC_EHIP, what, e) : 0;
}

static int ppfs_ecc_encode_device_impl(ppfs_ecc_ctx* c, const uint8_t* d_data, uint8_t* d_raw, size_t nblocks,
    void* stream)
{
    if (!c || (nblocks && ((!d_data && c->data) || !d_raw)))
        return fail(PPFS_ECC_EINVAL, "encode: null argument");
    if (nblocks == 0)
        return 0;
    hipStream_t s = (hipStream_t)stream;
    switch (c->p.ecc_type) {
    case PPFS_ECC_NONE:
        return check_hip(dma_async(d_raw, d_data, nblocks * c->raw, hipMemcpyDeviceToDevice, s), "copy");
    case PPFS_ECC_REED_SOLOMON:
        if (c->rs_fast && aligned16(d_data) && aligned16(d_raw)) {
            const TkSets t = ctr_for(c, s, 0);
            return check_hip(
                tk_commit(c, t, ppfs_rs_fast_encode(c->rs_t2, d_data, d_raw, nblocks, c->d_tables, s, t.mine, t.clear)),
                "rs encode");
        }
        if (c->rs_fast) {
            // fast tables but unaligned pointers: the generic kernel needs gf block + generator
            return fail(PPFS_ECC_EINVAL, "rs encode: device pointers must be 16-byte aligned");
        }
        return check_hip(ppfs_rs_generic_encode(d_data, d_raw, nblocks, c->rs_n, c->rs_t2, c->d_tables, s),
            "rs generic encode");
    case PPFS_ECC_CRC:
        return check_hip(ppfs_crc_encode(d_data, d_raw, nullptr, nblocks, c->raw, c->data, (uint32_t)c->crc_n,
                             c->crc_mask, c->d_tables, s),
            "crc encode");
    case PPFS_ECC_HAMMING:
        if (c->raw >= 8 && !aligned16(d_raw))
            return fail(PPFS_ECC_EINVAL, "hamming: raw pointer must be 16-byte aligned");
        return check_hip(ppfs_ham_encode(d_data, d_raw, nullptr, nblocks, c->raw, c->data, c->ham_L, s),
            "hamming encode");
    case PPFS_ECC_PARITY:
        return check_hip(ppfs_parity_encode(d_data, d_raw, nullptr, nblocks, c->raw, s), "parity encode");
    }
    return fail(PPFS_ECC_EINVAL, "bad ctx");
}

// The RS(255, 255 - 2t), 2t <= 8 decodes (rs_wg_tk.hpp / rs_wg.hpp) can put their write-backs
// somewhere other than the codewords they read: the host path points them at a page-locked caller
// image mapped into the device, so a chunk's corrections land there with no codeword copy and no
// patch pass (round 6)
static bool rs_wb_direct(const ppfs_ecc_ctx* c)
{
    return c->p.ecc_type == PPFS_ECC_REED_SOLOMON && c->rs_fast && c->rs_n == 255 && c->rs_t2 <= 8;
}

// wb_dst (the host path only, rs_wb_direct): the write-backs go there instead of into d_raw
static int ppfs_ecc_decode_device_impl(ppfs_ecc_ctx* c, uint8_t* d_raw, uint8_t* d_data, uint8_t* d_status,
    size_t nblocks, int write_back, uint8_t* d_spill, void* stream, uint8_t* wb_dst = nullptr)
{
    if (!c || (nblocks && !d_raw))
        return fail(PPFS_ECC_EINVAL, "decode: null argument");
    if (nblocks == 0)
        return 0;
    if (wb_dst && !rs_wb_direct(c))
        return fail(PPFS_ECC_EINVAL, "decode: no direct write-back for this codec");
    hipStream_t s = (hipStream_t)stream;
    switch (c->p.ecc_type) {
    case PPFS_ECC_NONE:
        if (d_status) {
            int r = check_hip(hipMemsetAsync(d_status, 0, nblocks, s), "status");
            if (r)
                return r;
        }
        if (d_data)
            return check_hip(dma_async(d_data, d_raw, nblocks * c->raw, hipMemcpyDeviceToDevice, s), "copy");
        return 0;
    case PPFS_ECC_REED_SOLOMON:
        if (c->rs_fast) {
            if (!aligned16(d_raw) || (d_data && !aligned16(d_data)) || (d_status && !aligned16(d_status)))
                return fail(PPFS_ECC_EINVAL, "rs decode: device pointers must be 16-byte aligned");
            if (d_spill) {
                int r = check_hip(hipMemsetAsync(d_spill, 0, nblocks * (256 - (size_t)c->rs_n), s), "spill");
                if (r)
                    return r;
            }
            const TkSets t = ctr_for(c, s, 1);
            return check_hip(tk_commit(c, t,
                                 ppfs_rs_fast_decode(c->rs_t2, d_raw, d_data, d_status, nblocks, c->d_tables, write_back, s,
                                     t.mine, t.clear, wb_dst)),
                "rs decode");
        }
        return check_hip(ppfs_rs_generic_decode(d_raw, d_data, d_status, d_spill, nblocks, c->rs_n, c->rs_t2,
                             write_back, c->d_tables, s),
            "rs generic decode");
    case PPFS_ECC_CRC:
        return check_hip(ppfs_crc_check(d_raw, d_data, d_status, nblocks, c->raw, c->data, (uint32_t)c->crc_n,
                             c->crc_mask, c->d_tables, s),
            "crc check");
    case PPFS_ECC_HAMMING:
        if (c->raw >= 8 && !aligned16(d_raw))
            return fail(PPFS_ECC_EINVAL, "hamming: raw pointer must be 16-byte aligned");
        return check_hip(ppfs_ham_decode(d_raw, d_data, d_status, nblocks, write_back, c->raw, c->data, c->ham_L, s),
            "hamming decode");
    case PPFS_ECC_PARITY:
        return check_hip(ppfs_parity_check(d_raw, d_data, d_status, nblocks, c->raw, s), "parity check");
    }
    return fail(PPFS_ECC_EINVAL, "bad ctx");
}

static int ensure_scratch(ppfs_ecc_ctx* c, size_t bytes, hipStream_t s)
{
    if (c->scratch_bytes >= bytes)
        return 0;
    if (c->d_scratch) {
        // an earlier write on this stream may still read the old scratch status
        HIP_TRY(hipStreamSynchronize(s), "scratch sync");
        mem_free(c, c->d_scratch);
    }
    c->d_scratch = nullptr;
    c->scratch_bytes = 0;
    HIP_TRY(mem_alloc(c, (void**)&c->d_scratch, bytes), "scratch alloc");
    c->scratch_bytes = bytes;
    return 0;
}

static int ppfs_ecc_write_device_impl(ppfs_ecc_ctx* c, const uint8_t* d_data, uint8_t* d_raw, uint8_t* d_status,
    size_t nblocks, void* stream)
{
    if (!c || (nblocks && ((!d_data && c->data) || !d_raw)))
        return fail(PPFS_ECC_EINVAL, "write: null argument");
    if (nblocks == 0)
        return 0;
    hipStream_t s = (hipStream_t)stream;
    uint8_t* st = d_status;
    if (!st) {
        int r = ensure_scratch(c, (nblocks + 15) & ~(size_t)15, s);
        if (r)
            return r;
        st = c->d_scratch;
    }
    int r = 0;
    switch (c->p.ecc_type) {
    case PPFS_ECC_NONE:
        if (d_status && (r = check_hip(hipMemsetAsync(d_status, 0, nblocks, s), "status")))
            return r;
        return check_hip(dma_async(d_raw, d_data, nblocks * c->raw, hipMemcpyDeviceToDevice, s), "copy");
    case PPFS_ECC_REED_SOLOMON:
        // old block decoded for its status (correction event) only; the new codeword does
        // not depend on it (rs_block_device.cpp:61-93)
        if ((r = ppfs_ecc_decode_device(c, d_raw, nullptr, st, nblocks, 0, nullptr, stream)))
            return r;
        return ppfs_ecc_encode_device(c, d_data, d_raw, nblocks, stream);
    case PPFS_ECC_CRC:
        if ((r = check_hip(ppfs_crc_check(d_raw, nullptr, st, nblocks, c->raw, c->data, (uint32_t)c->crc_n,
                               c->crc_mask, c->d_tables, s),
                 "crc check")))
            return r;
        return check_hip(ppfs_crc_encode(d_data, d_raw, st, nblocks, c->raw, c->data, (uint32_t)c->crc_n,
                             c->crc_mask, c->d_tables, s),
            "crc encode");
    case PPFS_ECC_HAMMING:
        if ((r = ppfs_ecc_decode_device(c, d_raw, nullptr, st, nblocks, 1, nullptr, stream)))
            return r;
        return check_hip(ppfs_ham_encode(d_data, d_raw, st, nblocks, c->raw, c->data, c->ham_L, s), "hamming encode");
    case PPFS_ECC_PARITY:
        if ((r = check_hip(ppfs_parity_check(d_raw, nullptr, st, nblocks, c->raw, s), "parity check")))
            return r;
        return check_hip(ppfs_parity_encode(d_data, d_raw, st, nblocks, c->raw, s), "parity encode");
    }
    return fail(PPFS_ECC_EINVAL, "bad ctx");
}

// device entry points: queue, then record the caller stream's completion event (destroy waits
// on it), then (PPFS_ECC_SYNC_CHECK) report an asynchronous fault under the entry's own name
static int queued(ppfs_ecc_ctx* c, int r, size_t nblocks, void* stream, const char* what)
{
    if (!r && nblocks)
        note_caller_stream(c, (hipStream_t)stream);
    return sync_check(r, stream, what);
}
// ... and before it queues anything: after the last call on the same stream handle
static void* ordered(ppfs_ecc_ctx* c, size_t nblocks, void* stream)
{
    if (c && nblocks)
        order_caller_stream(c, (hipStream_t)stream);
    return stream;
}

extern "C" int ppfs_ecc_encode_device(ppfs_ecc_ctx* c, const uint8_t* d_data, uint8_t* d_raw, size_t nblocks,
    void* stream)
{
    return queued(c, ppfs_ecc_encode_device_impl(c, d_data, d_raw, nblocks, ordered(c, nblocks, stream)), nblocks,
        stream, "encode (async)");
}

extern "C" int ppfs_ecc_decode_device(ppfs_ecc_ctx* c, uint8_t* d_raw, uint8_t* d_data, uint8_t* d_status,
    size_t nblocks, int write_back, uint8_t* d_spill, void* stream)
{
    return queued(c,
        ppfs_ecc_decode_device_impl(c, d_raw, d_data, d_status, nblocks, write_back, d_spill, ordered(c, nblocks, stream)),
        nblocks, stream, "decode (async)");
}

extern "C" int ppfs_ecc_write_device(ppfs_ecc_ctx* c, const uint8_t* d_data, uint8_t* d_raw, uint8_t* d_status,
    size_t nblocks, void* stream)
{
    return queued(c, ppfs_ecc_write_device_impl(c, d_data, d_raw, d_status, nblocks, ordered(c, nblocks, stream)),
        nblocks, stream, "write (async)");
}

namespace ppfs {
thread_local TimeHook g_time_hook;
}

extern "C" int ppfs_ecc_time_next_launch(void* start_event, void* stop_event)
{
    if ((start_event == nullptr) != (stop_event == nullptr))
        return -EINVAL;
    ppfs::g_time_hook = ppfs::TimeHook { (hipEvent_t)start_event, (hipEvent_t)stop_event };
    return 0;
}

extern "C" const char* ppfs_ecc_stream_kernel_name(ppfs_ecc_ctx* c, void* stream)
{
    if (!c)
        return "";
    if (c->d_ctr && (c->rs_t2 <= 8 || c->rs_t2 == 32)) {
        // 2t <= 8 and 2t = 32: ticket walks while the stream has (or can get) a counter set
        const hipStream_t s = (hipStream_t)stream;
        const bool evok = ev_slot(c, s, false) >= 0 || c->ev_n < ppfs_ecc_ctx::kEvSlots;
        if (!evok || tk_slot(c, s, false) < 0)
            return c->rs_t2 <= 8 ? "rs255-wg-seg4-lds" // rs_wg.hpp static walk
                                 : "rs255-bs-byte-lds-static"; // rs_bs.hpp, BsWalk without counters
    }
    return c->kname;
}

// ---------------------------------------------------------------------------------------
// Host-memory paths: chunked, triple-buffered pinned staging, H2D / kernel / D2H overlapped.
// ---------------------------------------------------------------------------------------
static int ensure_staging(ppfs_ecc_ctx* c, size_t bytes)
{
    if (c->stage_bytes >= bytes)
        return 0;
    for (hipStream_t h : c->hs)
        if (h)
            HIP_TRY(hipStreamSynchronize(h), "staging sync");
    for (int i = 0; i < ppfs_ecc_ctx::kSlots; ++i) {
        pin_free(c->h_pin[i], c->pin_bytes, kPinStage);
        mem_free(c, c->d_stage[i]);
        c->h_pin[i] = nullptr;
        c->d_stage[i] = nullptr;
    }
    c->stage_bytes = c->pin_bytes = 0;
    for (hipStream_t& h : c->hs)
        if (!h)
            HIP_TRY(hipStreamCreateWithFlags(&h, hipStreamNonBlocking), "stream");
    for (int i = 0; i < ppfs_ecc_ctx::kSlots; ++i) {
        for (hipEvent_t& e : c->hev[i])
            if (!e)
                HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
        HIP_TRY(pin_alloc((void**)&c->h_pin[i], bytes, kPinStage), "pinned alloc");
        c->pin_bytes = bytes;
        HIP_TRY(mem_alloc(c, (void**)&c->d_stage[i], bytes), "stage alloc");
    }
    c->stage_bytes = bytes;
    return 0;
}

namespace {
// 16 MiB of codewords per chunk: 64 Ki RS(255, k) blocks (round 6, r6e: page-locked encode / 1-error
// decode 75.9-76.1 / 42.9-43.1 GiB/s vs 71.9-72.1 / 40.9-41.0 at 32 Ki, 98-262 Ki no better), 4 Ki
// blocks of 4 KiB
constexpr size_t kChunkBytes = 16u << 20;
// Chunk sizes of a pipelined host call of at least 8 chunks: the first chunks ramp up (chunk / 8,
// / 4, / 2) and the last ones ramp down (halving the remainder), so the pipeline's fill (the first
// H2D before any kernel or D2H) and drain (the last D2H with no H2D beside it) move small chunks,
// not whole ones.  r6g (page-locked, 2 rounds x 7 reps): clean decode 70.3-72.3 vs 64.0-65.3 GiB/s,
// 1-error decode 41.6-42.6 vs 41.3-42.7, encode 71.5-75.4 vs 71.6-76.1.  (Four staging slots
// instead of three: encode 51-52, decode 31-37 GiB/s; a decode's codewords returned on the H2D
// stream: 26 GiB/s -- both dropped.)
size_t ramp_chunk(size_t index, size_t remaining, size_t chunk)
{
    const size_t least = std::max<size_t>(chunk / 8, 1024);
    size_t nb = chunk;
    if (index < 3)
        nb = std::max(least, chunk >> (3 - index));
    if (remaining < 2 * nb) // ramp down: half of what is left (at least `least`)
        nb = std::max(least, (remaining / 2 + 1023) & ~(size_t)1023);
    return remaining < nb + least ? remaining : nb; // no piece smaller than `least` after it
}
// Blocks per chunk of a context's host calls (a multiple of 1 Ki, at least 1 Ki);
// PPFS_ECC_CHUNK_BLOCKS (1 Ki .. 4 Mi): another chunk size (the r6e sweep)
size_t chunk_blocks(const ppfs_ecc_ctx* c)
{
    static const size_t env = [] {
        const char* e = std::getenv("PPFS_ECC_CHUNK_BLOCKS");
        const long v = e ? std::atol(e) : 0;
        return v >= 1024 && v <= (1l << 22) ? (size_t)v : 0;
    }();
    return env ? env : std::max<size_t>(1024, (kChunkBytes / std::max<size_t>(c->raw, 1)) & ~(size_t)1023);
}


// Host staging copies of the pageable host path (caller buffer <-> page-locked staging): one CPU
// thread moves ~10 GB/s, well under the link rate the page-locked path reaches, so copies of
// >= 2 MiB are split in 512 KiB pieces over PPFS_ECC_COPY_THREADS threads (default 8 -- the
// calling thread and 7 pool workers; 1 = single-threaded).  The workers persist (a spawn per copy
// cost ~10-20 us a thread), and one job carries every region of a chunk (payload and codewords).
int copy_threads()
{
    static const int n = [] {
        const char* e = std::getenv("PPFS_ECC_COPY_THREADS");
        const int v = e ? std::atoi(e) : 8;
        return v < 1 ? 1 : (v > 16 ? 16 : v);
    }();
    return n;
}

// Streaming copy of one staging piece (round 5, PPFS_ECC_COPY_NT=0: plain memcpy): 64-byte
// non-temporal stores skip the read-for-ownership of every destination line, so the copy moves
// its bytes once instead of twice -- the destinations (the page-locked staging the DMA reads, or
// a multi-MB caller buffer) do not fit in the caches anyway.  AVX-512 or AVX2 by the CPU, memcpy
// for the unaligned head and the tail; an sfence makes the stores visible before the job's
// completion is published.  x86 hosts only; elsewhere piece_copy is a memcpy.
#if PPFS_HOST_X86
__attribute__((target("avx512f"))) void nt_copy512(uint8_t* d, const uint8_t* s, size_t n)
{
    size_t i = 0;
    for (; i + 256 <= n; i += 256) {
        const __m512i a = _mm512_loadu_si512((const void*)(s + i)), b = _mm512_loadu_si512((const void*)(s + i + 64));
        const __m512i c = _mm512_loadu_si512((const void*)(s + i + 128)), e = _mm512_loadu_si512((const void*)(s + i + 192));
        _mm512_stream_si512((__m512i*)(d + i), a);
        _mm512_stream_si512((__m512i*)(d + i + 64), b);
        _mm512_stream_si512((__m512i*)(d + i + 128), c);
        _mm512_stream_si512((__m512i*)(d + i + 192), e);
    }
    for (; i + 64 <= n; i += 64)
        _mm512_stream_si512((__m512i*)(d + i), _mm512_loadu_si512((const void*)(s + i)));
    if (i < n)
        std::memcpy(d + i, s + i, n - i);
}
__attribute__((target("avx2"))) void nt_copy256(uint8_t* d, const uint8_t* s, size_t n)
{
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256((const __m256i*)(s + i)), b = _mm256_loadu_si256((const __m256i*)(s + i + 32));
        const __m256i c = _mm256_loadu_si256((const __m256i*)(s + i + 64)), e = _mm256_loadu_si256((const __m256i*)(s + i + 96));
        _mm256_stream_si256((__m256i*)(d + i), a);
        _mm256_stream_si256((__m256i*)(d + i + 32), b);
        _mm256_stream_si256((__m256i*)(d + i + 64), c);
        _mm256_stream_si256((__m256i*)(d + i + 96), e);
    }
    if (i < n)
        std::memcpy(d + i, s + i, n - i);
}
#endif
void piece_copy(void* dst, const void* src, size_t n)
{
#if !PPFS_HOST_X86
    std::memcpy(dst, src, n);
#else
    static const int mode = [] { // 2 AVX-512, 1 AVX2, 0 memcpy
        const char* e = std::getenv("PPFS_ECC_COPY_NT");
        if (e && *e == '0')
            return 0;
        // the CPU's flags from /proc/cpuinfo (this TU is also parsed for the GPU, where the
        // compiler's CPU-feature builtins do not exist)
        bool a512 = false, a2 = false;
        if (FILE* f = std::fopen("/proc/cpuinfo", "r")) {
            char line[8192];
            while (std::fgets(line, sizeof(line), f))
                if (std::strncmp(line, "flags", 5) == 0) {
                    a512 = std::strstr(line, " avx512f") != nullptr;
                    a2 = std::strstr(line, " avx2") != nullptr;
                    break;
                }
            std::fclose(f);
        }
        return a512 ? 2 : (a2 ? 1 : 0);
    }();
    uint8_t* d = (uint8_t*)dst;
    const uint8_t* s = (const uint8_t*)src;
    if (mode == 0 || n < 4096) {
        std::memcpy(d, s, n);
        return;
    }
    const size_t head = (64 - ((uintptr_t)d & 63)) & 63; // stores 64-byte aligned
    std::memcpy(d, s, head);
    if (mode == 2)
        nt_copy512(d + head, s + head, n - head);
    else
        nt_copy256(d + head, s + head, n - head);
    _mm_sfence();
#endif
}

struct CopySeg {
    void* dst;
    const void* src;
    size_t n;
};

class CopyPool {
    struct Job;

public:
    static constexpr size_t kPiece = 512u << 10;
    static constexpr int kMaxSegs = 4;

    // one pool per process, its workers blocked on cv_ between jobs; leaked at exit (the workers
    // never touch freed state).  Never used in a forked child (par_memcpy_n): the parent's workers
    // do not exist there, and a mutex another parent thread held at the fork stays locked.
    static CopyPool& get()
    {
        static CopyPool* pool = new CopyPool(copy_threads() - 1);
        return *pool;
    }

    void run(const CopySeg* segs, int nseg)
    {
        Job j;
        for (int i = 0; i < nseg; ++i) {
            j.seg[i] = segs[i];
            j.first[i + 1] = j.first[i] + (segs[i].n + kPiece - 1) / kPiece;
        }
        j.nseg = nseg;
        j.total = j.first[nseg];
        submit(j);
    }

    // fn(i) for i in [0, n), spread over the workers and the caller
    void run_for(size_t n, const std::function<void(size_t)>& fn)
    {
        Job j;
        j.fn = &fn;
        j.total = n;
        submit(j);
    }

private:
    void submit(Job& j)
    {
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &j;
            ++gen_;
        }
        cv_.notify_all();
        work(j);
        std::unique_lock<std::mutex> lk(m_);
        if (job_ == &j) // late wakers find no job (concurrent callers: each one finishes its own job)
            job_ = nullptr;
        done_.wait(lk, [&] { return j.finished.load() == j.total && j.users == 0; });
    }

    struct Job {
        CopySeg seg[kMaxSegs] {};
        size_t first[kMaxSegs + 1] {}; // first piece of each segment
        int nseg = 0;
        size_t total = 0;
        std::atomic<size_t> next { 0 }, finished { 0 };
        int users = 0; // workers holding the job (guarded by m_)
        const std::function<void(size_t)>* fn = nullptr; // run_for: item p is fn(p), not a copy piece
    };

    explicit CopyPool(int workers)
    {
        for (int i = 0; i < workers; ++i)
            std::thread([this] { loop(); }).detach();
    }

    void work(Job& j)
    {
        size_t done = 0;
        for (size_t p; (p = j.next.fetch_add(1)) < j.total; ++done) {
            if (j.fn) {
                (*j.fn)(p);
                continue;
            }
            int s = 0;
            while (p >= j.first[s + 1])
                ++s;
            const size_t off = (p - j.first[s]) * kPiece;
            const size_t len = std::min(kPiece, j.seg[s].n - off);
            piece_copy((uint8_t*)j.seg[s].dst + off, (const uint8_t*)j.seg[s].src + off, len);
        }
        if (done && j.finished.fetch_add(done) + done == j.total) {
            std::lock_guard<std::mutex> g(m_);
            done_.notify_all();
        }
    }

    void loop()
    {
        uint64_t seen = 0;
        for (;;) {
            Job* j;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (!(j = job_))
                    continue;
                ++j->users;
            }
            work(*j);
            std::lock_guard<std::mutex> g(m_);
            if (--j->users == 0)
                done_.notify_all();
        }
    }

    std::mutex m_;
    std::condition_variable cv_, done_;
    uint64_t gen_ = 0;
    Job* job_ = nullptr;
};

// Set in a forked child (pthread_atfork, registered at load): its copies run single-threaded.
std::atomic<bool> g_fork_child { false };
[[maybe_unused]] const int g_atfork_registered = pthread_atfork(nullptr, nullptr, [] { g_fork_child.store(true); });

void par_memcpy_n(const CopySeg* segs, int nseg)
{
    size_t total = 0;
    for (int i = 0; i < nseg; ++i)
        total += segs[i].n;
    if (g_fork_child.load(std::memory_order_relaxed) || copy_threads() == 1 || total < (2u << 20)) {
        for (int i = 0; i < nseg; ++i)
            std::memcpy(segs[i].dst, segs[i].src, segs[i].n);
        return;
    }
    CopyPool::get().run(segs, nseg);
}

void par_memcpy(void* dst, const void* src, size_t n)
{
    const CopySeg s { dst, src, n };
    par_memcpy_n(&s, 1);
}

struct Layout { // offsets inside one staging buffer
    size_t data, raw, status, spill, idx, gat, orig, patch, total;
};

// Slots per block of a decode's patch list (vote.hip patch_list_kernel) -- RS(255, k): 2 (a block
// with more changed bytes -- up to 2t, one per root of sigma -- comes back whole); Hamming: 1, the
// one corrected byte -- or 0: the codec returns whole codewords (shortened RS, whose write-back
// also spills past the block, and the codecs without a write-back).  PPFS_ECC_PATCH=0: always whole
// codewords (A/B).
uint32_t patch_slots(const ppfs_ecc_ctx* c)
{
    static const bool off = [] {
        const char* e = std::getenv("PPFS_ECC_PATCH");
        return e && *e == '0';
    }();
    if (off)
        return 0;
    if (c->p.ecc_type == PPFS_ECC_REED_SOLOMON && c->rs_n == 255)
        return 2; // one or two changed bytes (at most 2t; more come back whole)
    if (c->p.ecc_type == PPFS_ECC_HAMMING)
        return 1;
    return 0;
}

// a decode with write-back returns only the codewords it changed (status 1): as a packed gather
// when at most nb / kGatherDiv blocks changed, else the chunk's whole codeword range
constexpr size_t kGatherDiv = 8;

Layout layout_for(const ppfs_ecc_ctx* c, size_t nb)
{
    Layout L {};
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    L.data = 0;
    L.raw = al(L.data + nb * c->data);
    L.status = al(L.raw + nb * c->raw);
    L.spill = al(L.status + nb);
    L.idx = al(L.spill + nb * (256 - std::min<size_t>(c->raw, 255)));
    L.gat = al(L.idx + (nb / kGatherDiv + 1) * sizeof(uint32_t));
    const uint32_t S = patch_slots(c);
    L.orig = al(L.gat + (nb / kGatherDiv + 1) * c->raw);
    L.patch = al(L.orig + (S ? nb * c->raw : 0));
    L.total = al(L.patch + nb * S * sizeof(uint32_t));
    return L;
}
} // namespace

enum HostOp { OP_ENCODE, OP_DECODE, OP_WRITE };

// Does encode read the old raw block?  (CRC tail bits, Hamming unused bits, parity fix byte)
static bool raw_is_rmw(const ppfs_ecc_ctx* c)
{
    return c->p.ecc_type == PPFS_ECC_HAMMING || c->p.ecc_type == PPFS_ECC_PARITY
        || (c->p.ecc_type == PPFS_ECC_CRC && (c->crc_n % 8) != 0);
}

// page-locked host memory (hipHostMalloc / hipHostRegister, e.g. ppfs_ecc_host_register): the
// DMA engines can reach it directly, so the host paths skip the CPU copy through staging
static bool host_pinned_byte(const void* p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// The whole range [p, p + bytes) must be page-locked before the DMA engines may touch it: a buffer
// that starts inside a registered region and runs past its end would otherwise be DMA'd from / to
// unlocked pages.  The runtime's allocation record of the first byte (hipMemGetAddressRange: the
// hipHostMalloc / hipHostRegister extent) has to cover the last byte; where the runtime keeps no
// such record the range is probed at both ends and every 64 KiB in between.
static bool host_pinned(const void* p, size_t bytes)
{
    if (!p || !bytes)
        return true;
    const uintptr_t a = (uintptr_t)p, last = a + bytes - 1;
    if (!host_pinned_byte(p) || !host_pinned_byte((const void*)last))
        return false;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) == hipSuccess && base && size) {
        const uintptr_t b = (uintptr_t)base;
        if (b <= a && last < b + size)
            return true;
    }
    (void)hipGetLastError();
    constexpr uintptr_t kStride = 64 << 10;
    for (uintptr_t q = (a & ~(kStride - 1)) + kStride; q < last; q += kStride)
        if (!host_pinned_byte((const void*)q))
            return false;
    return true;
}

// Device memory over the whole range [p, p + n): both ends device memory and, where the runtime
// keeps an allocation record (hipMalloc; not stream-ordered pool memory), inside one allocation.
[[maybe_unused]] static bool device_range(const void* p, size_t n)
{
    if (!p || !n)
        return true;
#ifdef PPFS_ECC_DEBUG
    if (pool_covers(p, n)) // the engine's own stream-ordered allocations
        return true;
#endif
    auto dev_byte = [](const void* q) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        return a.type == hipMemoryTypeDevice;
    };
    const uintptr_t a = (uintptr_t)p, last = a + n - 1;
    if (!dev_byte(p) || !dev_byte((const void*)last))
        return false;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) == hipSuccess && base && size)
        return (uintptr_t)base <= a && last < (uintptr_t)base + size;
    (void)hipGetLastError();
    return true;
}

[[maybe_unused]] static std::atomic<long long> g_dma_rejects { 0 };

// Every hipMemcpyAsync of this file.  PPFS_ECC_DEBUG builds check both ends first: a host end
// must be page-locked over its whole range (host_pinned: the engine's own staging, a hipHostMalloc'd
// or ppfs_ecc_host_register'd caller buffer), a device end device memory over its whole range
// (device_range).  A copy that fails the check is refused -- counted (ppfs_ecc_debug_dma_rejects),
// printed, returned as an error -- never handed to the runtime's pageable-copy path or to the DMA
// engines.  Normal builds: the copy as is.
static hipError_t dma_async(void* dst, const void* src, size_t n, hipMemcpyKind kind, hipStream_t s)
{
#ifdef PPFS_ECC_DEBUG
    if (n) {
        const bool src_dev = kind == hipMemcpyDeviceToHost || kind == hipMemcpyDeviceToDevice;
        const bool dst_dev = kind == hipMemcpyHostToDevice || kind == hipMemcpyDeviceToDevice;
        const bool src_ok = src_dev ? device_range(src, n) : host_pinned(src, n);
        const bool dst_ok = dst_dev ? device_range(dst, n) : host_pinned(dst, n);
        if (!src_ok || !dst_ok) {
            const long long k = ++g_dma_rejects;
            if (k <= 16)
                std::fprintf(stderr, "PPFS_ECC_DEBUG: refused copy of %zu B %p -> %p (kind %d): %s end not %s over its range\n",
                    n, src, dst, (int)kind, src_ok ? "destination" : "source",
                    (src_ok ? dst_dev : src_dev) ? "device memory" : "page-locked");
            return hipErrorInvalidValue;
        }
    }
#endif
    return hipMemcpyAsync(dst, src, n, kind, s);
}

extern "C" long long ppfs_ecc_debug_dma_rejects(void)
{
#ifdef PPFS_ECC_DEBUG
    return g_dma_rejects.load();
#else
    return -1;
#endif
}

// Positive control of the copy checks: a copy from malloc'd (pageable) memory and one into a range
// that runs past its device allocation must both be refused.  1 = both refused (the reject counter
// is restored, so the control does not count as a finding), 0 = a check let one through, -1 in
// normal builds.
extern "C" long long ppfs_ecc_debug_dma_selftest(void)
{
#ifdef PPFS_ECC_DEBUG
    const long long before = g_dma_rejects.load();
    uint8_t* pageable = (uint8_t*)std::malloc(4096);
    uint8_t* d = nullptr;
    if (!pageable || hipMalloc(&d, 4096) != hipSuccess) {
        std::free(pageable);
        return 0;
    }
    const bool r1 = dma_async(d, pageable, 4096, hipMemcpyHostToDevice, nullptr) != hipSuccess;
    const bool r2 = dma_async(d + 4096 - 16, d, 32, hipMemcpyDeviceToDevice, nullptr) != hipSuccess;
    (void)hipGetLastError();
    (void)hipStreamSynchronize(nullptr);
    (void)hipFree(d);
    std::free(pageable);
    g_dma_rejects.store(before);
    return (r1 && r2) ? 1 : 0;
#else
    return -1;
#endif
}

static int device_op(ppfs_ecc_ctx* c, HostOp op, uint8_t* d, const Layout& L, size_t nb, int write_back, bool want_data,
    bool want_spill, hipStream_t s)
{
    switch (op) {
    case OP_ENCODE:
        return ppfs_ecc_encode_device(c, d + L.data, d + L.raw, nb, s);
    case OP_WRITE:
        return ppfs_ecc_write_device(c, d + L.data, d + L.raw, d + L.status, nb, s);
    case OP_DECODE:
        return ppfs_ecc_decode_device(c, d + L.raw, want_data ? d + L.data : nullptr, d + L.status, nb, write_back,
            want_spill ? d + L.spill : nullptr, s);
    }
    return fail(PPFS_ECC_EINVAL, "bad op");
}

constexpr size_t kSmallBlocks = 64; // one tile: the per-block IBlockDevice calls

// ---- resident small-batch server (server_box.hpp, rs_wg.hpp rs_wg_server_kernel) ----
// every codec (RS: rs_wg / rs255 / rs_pair / generic servers by table layout; CRC, Hamming, parity:
// bit_server_kernel):
// a per-block call posts its request to the resident
// workgroup instead of launching kernels and synchronizing a stream (measured on the box, RS(255,249),
// one block: launch + stream synchronize alone 10.3 us, a whole decode_host call 16.2 us).
// PPFS_ECC_SERVER=0 turns it off (the launch path below).
constexpr uint32_t kSrvIdleUs = 20000; // a launch leaves after 20 ms without a request

static bool server_eligible(ppfs_ecc_ctx* c)
{
    if (c->srv_ok < 0) {
        const char* e = std::getenv("PPFS_ECC_SERVER");
        const bool off = e && e[0] == '0';
        const bool rs = c->p.ecc_type == PPFS_ECC_REED_SOLOMON
            && (!c->rs_fast || c->rs_t2 <= 8 || c->rs_t2 == 10 || c->rs_t2 == 16 || c->rs_t2 == 32);
        // Hamming blocks < 8 bytes run thread-per-block kernels the bit server does not carry
        const bool bit = c->p.ecc_type == PPFS_ECC_CRC || (c->p.ecc_type == PPFS_ECC_HAMMING && c->raw >= 8)
            || c->p.ecc_type == PPFS_ECC_PARITY;
        c->srv_ok = (!off && (rs || bit)) ? 1 : 0;
    }
    return c->srv_ok == 1;
}

// stop the resident launch (if any) and wait until it has returned (bounded, server_halt); an
// error when it did not: the context is then unusable (srv_stuck)
static int server_stop(ppfs_ecc_ctx* c)
{
    if (server_halt(c))
        return 0;
    return fail(PPFS_ECC_EHIP, "small-batch server did not stop: context unusable");
}

static int server_launch(ppfs_ecc_ctx* c)
{
    const uint32_t gen = (++c->srv_gen) & ~ppfs::SRV_EXITED;
    c->srv_gen = gen;
    trace_step("server: launch");
    __atomic_store_n(&c->h_box->stop, 0u, __ATOMIC_RELEASE);
    if (c->p.ecc_type == PPFS_ECC_REED_SOLOMON && c->rs_fast)
        HIP_TRY(ppfs_rs_server_launch(c->rs_t2, c->d_box, c->d_zc, c->zc_bytes, c->d_tables, gen, kSrvIdleUs, c->srv_stream),
            "server launch");
    else if (c->p.ecc_type == PPFS_ECC_REED_SOLOMON)
        HIP_TRY(ppfs_rs_generic_server_launch(c->rs_n, c->rs_t2, c->d_box, c->d_zc, c->zc_bytes, c->d_tables, gen, kSrvIdleUs,
                    c->srv_stream),
            "server launch");
    else
        HIP_TRY(ppfs_bit_server_launch((int)c->p.ecc_type, c->raw, c->data, (uint32_t)c->crc_n, c->crc_mask, c->ham_L, c->d_box,
                    c->d_zc, c->zc_bytes, c->d_tables, gen, kSrvIdleUs, c->srv_stream),
            "server launch");
    c->srv_launched = true;
    return 0;
}

// the context's mailbox (server requests, completion flag of the launch path)
static int ensure_box(ppfs_ecc_ctx* c)
{
    if (c->h_box)
        return 0;
    HIP_TRY(pin_alloc((void**)&c->h_box, sizeof(ppfs::SrvBox), kPinMapped), "mailbox");
    std::memset((void*)c->h_box, 0, sizeof(ppfs::SrvBox));
    HIP_TRY(hipHostGetDevicePointer((void**)&c->d_box, c->h_box, 0), "mailbox map");
    return 0;
}

// Wait for the small-batch launch path's work on stream s: a flag kernel after it stores a fresh
// number into the mailbox and the host spins on it (hipStreamSynchronize's completion signal
// costs ~4 us more per call).  A faulting kernel never lets the flag arrive: the stream is queried
// every few thousand spins and its error returned.
static int wait_flag(ppfs_ecc_ctx* c, hipStream_t s)
{
    int r = ensure_box(c);
    if (r)
        return r;
    const uint32_t v = ++c->flag_seq;
    HIP_TRY(ppfs_flag_launch(&c->d_box->flag, v, s), "flag launch");
    for (uint32_t spin = 1;; ++spin) {
        if (__atomic_load_n(&c->h_box->flag, __ATOMIC_ACQUIRE) == v)
            return 0;
        if ((spin & 4095u) == 0) {
            const hipError_t e = hipStreamQuery(s);
            if (e != hipErrorNotReady && e != hipSuccess)
                return check_hip(e, "small-batch kernels");
            if (e == hipSuccess && __atomic_load_n(&c->h_box->flag, __ATOMIC_ACQUIRE) != v)
                return fail(PPFS_ECC_EHIP, "small-batch completion flag missing");
        }
    }
}

static int server_call(ppfs_ecc_ctx* c, HostOp op, const Layout& L, size_t nb, int write_back, bool want_data)
{
    using namespace ppfs;
    if (!c->srv_stream) {
        const int r = ensure_box(c);
        if (r)
            return r;
        // The resident launch gets a stream of its own priority level: HIP maps streams of one
        // priority onto GPU_MAX_HW_QUEUES hardware queues, and a stream sharing the server's queue
        // waits behind the resident launch (round 4: another context's creation in a fresh process
        // waited for good; with more hardware queues, or the server at high priority, it did not)
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess || least == greatest
            || hipStreamCreateWithPriority(&c->srv_stream, hipStreamNonBlocking, greatest) != hipSuccess) {
            (void)hipGetLastError();
            HIP_TRY(hipStreamCreateWithFlags(&c->srv_stream, hipStreamNonBlocking), "server stream");
        }
    }
    SrvBox* b = c->h_box;
    const SrvLayout sl = srv_layout((uint32_t)nb, c->data, c->raw);
    if (nb < 1 || nb > SRV_MAX_BLOCKS || sl.data != L.data || sl.raw != L.raw || sl.status != L.status)
        return fail(PPFS_ECC_EINVAL, "small-batch server: layout mismatch");
    const SrvCmd sc { (uint32_t)nb, op == OP_ENCODE ? SRV_ENCODE : (op == OP_DECODE ? SRV_DECODE : SRV_WRITE),
        write_back != 0, want_data };
    c->srv_seq = (c->srv_seq + 1) & 0xFFFFu;
    const uint32_t seq = srv_cmd_pack(c->srv_seq, sc);
    __atomic_store_n(&b->cmd, seq, __ATOMIC_RELEASE); // publishes the request and its input bytes
    auto exited = [&]() { return __atomic_load_n(&b->alive, __ATOMIC_ACQUIRE) == (c->srv_gen | SRV_EXITED); };
    if (!c->srv_launched || exited()) {
        const int r = server_launch(c);
        if (r)
            return r;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 1;; ++spin) {
        if (__atomic_load_n(&b->done, __ATOMIC_ACQUIRE) == seq)
            return 0;
        if ((spin & 255u) == 0) {
            if (exited()) { // the launch left (idle / lifetime) without seeing this request
                const int r = server_launch(c);
                if (r)
                    return r;
            } else if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                const bool stopped = server_stop(c) == 0; // bounded: never hangs on a launch that stopped polling
                c->srv_ok = 0; // this context uses the launch path from now on
                if (stopped && __atomic_load_n(&b->done, __ATOMIC_ACQUIRE) == seq)
                    return 0;
                return fail(PPFS_ECC_EHIP, stopped ? "small-batch server: no answer within 10 s"
                                                   : "small-batch server: no answer within 10 s and did not stop: context unusable");
            }
        }
    }
}

// Small batches run the kernels on coherent host memory in place: no H2D / D2H copies on the
// critical path of a per-block readBlock / writeBlock (each async copy costs microseconds).
static int host_run_small(ppfs_ecc_ctx* c, HostOp op, const uint8_t* data_in, uint8_t* data_out, uint8_t* raw,
    uint8_t* status, uint8_t* spill, size_t nb, int write_back)
{
    const Layout L = layout_for(c, nb);
    if (c->zc_bytes < L.total) {
        if (server_stop(c)) // it holds the buffer's address
            return PPFS_ECC_EHIP;
        if (c->h_zc && c->hs[0])
            HIP_TRY(hipStreamSynchronize(c->hs[0]), "zero-copy sync");
        pin_free(c->h_zc, c->zc_bytes, kPinMapped);
        c->h_zc = c->d_zc = nullptr;
        c->zc_bytes = 0;
        const size_t bytes = std::max(L.total, layout_for(c, kSmallBlocks).total);
        HIP_TRY(pin_alloc((void**)&c->h_zc, bytes, kPinMapped), "zero-copy alloc");
        HIP_TRY(hipHostGetDevicePointer((void**)&c->d_zc, c->h_zc, 0), "zero-copy map");
        c->zc_bytes = bytes;
    }
    if (!c->hs[0])
        HIP_TRY(hipStreamCreateWithFlags(&c->hs[0], hipStreamNonBlocking), "stream");
    uint8_t* h = c->h_zc;
    const size_t spill_b = 256 - std::min<size_t>(c->raw, 255);
    if (op == OP_ENCODE || op == OP_WRITE)
        std::memcpy(h + L.data, data_in, nb * c->data);
    if (op != OP_ENCODE || raw_is_rmw(c))
        std::memcpy(h + L.raw, raw, nb * c->raw);
    if (server_eligible(c) && !spill) {
        const int r = server_call(c, op, L, nb, write_back, data_out != nullptr);
        if (r)
            return r;
    } else {
        int r = device_op(c, op, c->d_zc, L, nb, write_back, data_out != nullptr, spill != nullptr, c->hs[0]);
        if (!r)
            r = wait_flag(c, c->hs[0]);
        if (r)
            return r;
    }
    if (op == OP_ENCODE || op == OP_WRITE)
        std::memcpy(raw, h + L.raw, nb * c->raw);
    else if (write_back) // only the codewords the decode changed (status 1)
        for (size_t b = 0; b < nb; ++b)
            if (h[L.status + b] == 1)
                std::memcpy(raw + b * c->raw, h + L.raw + b * c->raw, c->raw);
    if (op == OP_DECODE && data_out)
        std::memcpy(data_out, h + L.data, nb * c->data);
    if (status && op != OP_ENCODE)
        std::memcpy(status, h + L.status, nb);
    if (spill)
        std::memcpy(spill, h + L.spill, nb * spill_b);
    return 0;
}

static int host_run_chunks(ppfs_ecc_ctx* c, HostOp op, const uint8_t* data_in, uint8_t* data_out, uint8_t* raw,
    uint8_t* status, uint8_t* spill, size_t nblocks, int write_back);

// A host call returns only once nothing it queued is still in flight: on an error part-way through
// (a failed copy or launch in one slot) the other slots' H2D / kernel / D2H may still be running,
// and their DMA targets the caller's buffers (direct mode) and the staging the next call reuses.
// Every stream is drained before the error goes back; the first error's message is kept.
static int host_run(ppfs_ecc_ctx* c, HostOp op, const uint8_t* data_in, uint8_t* data_out, uint8_t* raw,
    uint8_t* status, uint8_t* spill, size_t nblocks, int write_back)
{
    if (!c)
        return fail(PPFS_ECC_EINVAL, "null ctx");
    if (c->srv_stuck)
        return fail(PPFS_ECC_EHIP, "context unusable: its resident server launch did not stop");
    if (nblocks == 0)
        return 0;
    DeviceGuard guard(c->device);
    HIP_TRY(guard.err, "set device");
    const int r = nblocks <= kSmallBlocks
        ? host_run_small(c, op, data_in, data_out, raw, status, spill, nblocks, write_back)
        : host_run_chunks(c, op, data_in, data_out, raw, status, spill, nblocks, write_back);
    if (r) {
        const std::string msg = g_last_error;
        for (hipStream_t h : c->hs)
            if (h)
                (void)hipStreamSynchronize(h);
        g_last_error = msg;
    }
    return r;
}

static int host_run_chunks(ppfs_ecc_ctx* c, HostOp op, const uint8_t* data_in, uint8_t* data_out, uint8_t* raw,
    uint8_t* status, uint8_t* spill, size_t nblocks, int write_back)
{
    const size_t chunk = std::min(nblocks, chunk_blocks(c));
    const Layout L = layout_for(c, chunk);
    int r = ensure_staging(c, L.total);
    if (r)
        return r;
    const size_t spill_b = 256 - std::min<size_t>(c->raw, 255);
    constexpr int NS = ppfs_ecc_ctx::kSlots;
    hipStream_t s_in = c->hs[0], s_out = c->hs[1];
    size_t pending_first[NS] = {}, pending_n[NS] = {};
    // fetched: the chunk's codewords already came back (staging, or the caller's page-locked image)
    bool busy[NS] = {}, fetched[NS] = {}, patched[NS] = {}, landed[NS] = {};
    // every caller buffer page-locked: DMA straight between it and the device staging buffers
    const bool direct = host_pinned(data_in, nblocks * c->data) && host_pinned(data_out, nblocks * c->data)
        && host_pinned(raw, nblocks * c->raw) && host_pinned(status, nblocks) && host_pinned(spill, nblocks * spill_b);

    // decode with write-back: the codewords come back only where the decode changed them
    // (status 1), read from the chunk's status once it has landed
    const bool lazy_raw = op == OP_DECODE && write_back;
    // ... and as a patch list (the changed bytes) where the codec bounds them (patch_slots): the
    // host writes those bytes into its image instead of taking back whole codewords
    const uint32_t S = lazy_raw ? patch_slots(c) : 0u;
    // a page-locked caller image the device can address: the patch kernel stores the changed bytes
    // straight into it (no list, no host work); else the list comes back and the host applies it
    uint8_t* img_dev = nullptr;
    if (S && direct && hipHostGetDevicePointer((void**)&img_dev, raw, 0) != hipSuccess) {
        (void)hipGetLastError();
        img_dev = nullptr;
    }
    // RS with 2t <= 8 into such an image: the decode kernel itself stores its corrections there
    // (rs_wb_direct), so no codeword copy before it and no patch kernel after it
    const bool wb_direct = img_dev && rs_wb_direct(c);
    // predictor: the last drained chunk changed many codewords -> fetch the next ones eagerly
    // (queued behind the kernel, as encode does) instead of after the status has landed.  It starts
    // where the context's previous call left it: the first kSlots chunks are queued before any has
    // landed
    bool eager = c->host_eager;
    auto fetch_changed = [&](int i, size_t b0, size_t nb) -> int {
        uint8_t* h = c->h_pin[i];
        uint8_t* d = c->d_stage[i];
        // the chunk has landed (drain): its staging is idle until reused.  On the H2D stream, whose
        // queue holds at most the next kSlots - 1 chunks' input copies; the other holds their kernels
        hipStream_t s = s_in;
        const uint8_t* sts = (direct && status) ? status + b0 : h + L.status;
        uint32_t* ix = (uint32_t*)(h + L.idx);
        size_t nchg = 0;
        for (size_t b = 0; b < nb; ++b)
            if (sts[b] == 1) {
                if (nchg <= nb / kGatherDiv)
                    ix[nchg] = (uint32_t)b;
                ++nchg;
            }
        eager = nchg > nb / kGatherDiv;
        if (nchg == 0)
            return 0;
        if (fetched[i]) {
            if (direct)
                return 0; // the whole range landed in the caller's image (unchanged blocks: same bytes)
            if (eager)
                par_memcpy(raw + b0 * c->raw, h + L.raw, nb * c->raw);
            else
                for (size_t b = 0; b < nb; ++b)
                    if (sts[b] == 1)
                        std::memcpy(raw + (b0 + b) * c->raw, h + L.raw + b * c->raw, c->raw);
            return 0;
        }
        if (nchg > nb / kGatherDiv) { // many: the whole range
            uint8_t* o = direct ? raw + b0 * c->raw : h + L.raw;
            HIP_TRY(dma_async(o, d + L.raw, nb * c->raw, hipMemcpyDeviceToHost, s), "D2H raw");
            HIP_TRY(hipStreamSynchronize(s), "sync");
            if (!direct)
                par_memcpy(raw + b0 * c->raw, h + L.raw, nb * c->raw);
            return 0;
        }
        HIP_TRY(dma_async(d + L.idx, ix, nchg * sizeof(uint32_t), hipMemcpyHostToDevice, s), "H2D idx");
        HIP_TRY(ppfs_gather_rows_launch(d + L.raw, nb, d + L.gat, (const uint32_t*)(d + L.idx), (uint32_t)nchg,
                    (uint32_t)c->raw, s), "gather");
        HIP_TRY(dma_async(h + L.gat, d + L.gat, nchg * c->raw, hipMemcpyDeviceToHost, s), "D2H gather");
        HIP_TRY(hipStreamSynchronize(s), "sync");
        for (size_t j = 0; j < nchg; ++j)
            std::memcpy(raw + (b0 + ix[j]) * c->raw, h + L.gat + j * c->raw, c->raw);
        return 0;
    };

    // The chunk's patch list into the caller's image: taken back now unless it came behind the
    // kernel (the predictor expected many changed blocks), nothing for a clean chunk; blocks with
    // more changed bytes than their S slots come back whole, by one gather like fetch_changed's.
    auto apply_patches = [&](int i, size_t b0, size_t nb) -> int {
        uint8_t* h = c->h_pin[i];
        uint8_t* d = c->d_stage[i];
        const uint8_t* sts = (direct && status) ? status + b0 : h + L.status;
        size_t nchg = 0;
        for (size_t b = 0; b < nb; ++b)
            nchg += sts[b] == 1;
        eager = nchg > nb / kGatherDiv;
        if (nchg == 0)
            return 0;
        if (!fetched[i]) {
            HIP_TRY(dma_async(h + L.patch, d + L.patch, nb * S * sizeof(uint32_t), hipMemcpyDeviceToHost, s_in), "D2H patch");
            HIP_TRY(hipStreamSynchronize(s_in), "sync");
        }
        const uint32_t* P = (const uint32_t*)(h + L.patch);
        uint8_t* img = raw + b0 * c->raw;
        const size_t n = c->raw;
        constexpr size_t kPart = 4096; // blocks per pool item
        std::atomic<bool> overflow { false };
        const std::function<void(size_t)> part = [&](size_t p) {
            const size_t e = std::min(nb, (p + 1) * kPart);
            for (size_t b = p * kPart; b < e; ++b) {
                if (sts[b] != 1)
                    continue;
                const uint32_t* q = P + b * S;
                if (q[0] == 0xFFFFFFFEu) {
                    overflow.store(true, std::memory_order_relaxed);
                    continue;
                }
                for (uint32_t j = 0; j < S && q[j] != 0xFFFFFFFFu; ++j)
                    img[b * n + (q[j] >> 8)] = (uint8_t)q[j];
            }
        };
        const size_t parts = (nb + kPart - 1) / kPart;
        if (parts > 1 && nchg > 4 * kPart && !g_fork_child.load(std::memory_order_relaxed) && copy_threads() > 1)
            CopyPool::get().run_for(parts, part);
        else
            for (size_t p = 0; p < parts; ++p)
                part(p);
        if (!overflow.load())
            return 0;
        uint32_t* ix = (uint32_t*)(h + L.idx);
        const size_t cap = nb / kGatherDiv + 1; // the gather region's rows
        size_t nov = 0;
        for (size_t b = 0; b < nb; ++b) {
            if (sts[b] != 1 || P[b * S] != 0xFFFFFFFEu)
                continue;
            ix[nov++] = (uint32_t)b;
            if (nov == cap || b + 1 == nb) {
                HIP_TRY(dma_async(d + L.idx, ix, nov * sizeof(uint32_t), hipMemcpyHostToDevice, s_in), "H2D idx");
                HIP_TRY(ppfs_gather_rows_launch(d + L.raw, nb, d + L.gat, (const uint32_t*)(d + L.idx), (uint32_t)nov,
                            (uint32_t)n, s_in), "gather");
                HIP_TRY(dma_async(h + L.gat, d + L.gat, nov * n, hipMemcpyDeviceToHost, s_in), "D2H gather");
                HIP_TRY(hipStreamSynchronize(s_in), "sync");
                for (size_t j = 0; j < nov; ++j)
                    std::memcpy(img + (size_t)ix[j] * n, h + L.gat + j * n, n);
                nov = 0;
            }
        }
        if (nov) {
            HIP_TRY(dma_async(d + L.idx, ix, nov * sizeof(uint32_t), hipMemcpyHostToDevice, s_in), "H2D idx");
            HIP_TRY(ppfs_gather_rows_launch(d + L.raw, nb, d + L.gat, (const uint32_t*)(d + L.idx), (uint32_t)nov,
                        (uint32_t)n, s_in), "gather");
            HIP_TRY(dma_async(h + L.gat, d + L.gat, nov * n, hipMemcpyDeviceToHost, s_in), "D2H gather");
            HIP_TRY(hipStreamSynchronize(s_in), "sync");
            for (size_t j = 0; j < nov; ++j)
                std::memcpy(img + (size_t)ix[j] * n, h + L.gat + j * n, n);
        }
        return 0;
    };

    auto drain = [&](int i) -> int {
        if (!busy[i])
            return 0;
        HIP_TRY(hipEventSynchronize(c->hev[i][1]), "sync");
        const size_t b0 = pending_first[i], nb = pending_n[i];
        if (lazy_raw) {
            const int e = landed[i] ? 0 : patched[i] ? apply_patches(i, b0, nb) : fetch_changed(i, b0, nb);
            if (e)
                return e;
        }
        if (direct) {
            busy[i] = false;
            return 0;
        }
        uint8_t* h = c->h_pin[i];
        CopySeg seg[2];
        int ns = 0;
        if (op == OP_ENCODE || op == OP_WRITE)
            seg[ns++] = { raw + b0 * c->raw, h + L.raw, nb * c->raw };
        if (op == OP_DECODE && data_out)
            seg[ns++] = { data_out + b0 * c->data, h + L.data, nb * c->data };
        par_memcpy_n(seg, ns);
        if (status)
            std::memcpy(status + b0, h + L.status, nb);
        if (spill)
            std::memcpy(spill + b0 * spill_b, h + L.spill, nb * spill_b);
        busy[i] = false;
        return 0;
    };

    // a slot is reused only after drain() saw its outputs land: its H2D then never overwrites
    // staging an earlier chunk's kernel or D2H still reads
    int slot = 0;
    size_t nb = 0;
    for (size_t b0 = 0, ci = 0; b0 < nblocks; b0 += nb, slot = (slot + 1) % NS, ++ci) {
        nb = nblocks >= 8 * chunk ? ramp_chunk(ci, nblocks - b0, chunk) : std::min(chunk, nblocks - b0);
        if ((r = drain(slot)))
            return r;
        uint8_t* h = c->h_pin[slot];
        uint8_t* d = c->d_stage[slot];
        hipEvent_t* ev = c->hev[slot];
        hipStream_t s = s_in;
        // inputs host -> pinned -> device (data and raw regions are adjacent in the layout)
        const bool need_data = op == OP_ENCODE || op == OP_WRITE;
        const bool need_raw = op != OP_ENCODE || raw_is_rmw(c);
        if (direct) {
            if (need_data)
                HIP_TRY(dma_async(d + L.data, data_in + b0 * c->data, nb * c->data, hipMemcpyHostToDevice, s),
                    "H2D data");
            if (need_raw)
                HIP_TRY(dma_async(d + L.raw, raw + b0 * c->raw, nb * c->raw, hipMemcpyHostToDevice, s), "H2D raw");
        } else {
            CopySeg seg[2];
            int ns = 0;
            if (need_data)
                seg[ns++] = { h + L.data, data_in + b0 * c->data, nb * c->data };
            if (need_raw)
                seg[ns++] = { h + L.raw, raw + b0 * c->raw, nb * c->raw };
            par_memcpy_n(seg, ns);
            const size_t in_lo = need_data ? L.data : L.raw;
            const size_t in_hi = need_raw ? L.raw + nb * c->raw : L.data + nb * c->data;
            HIP_TRY(dma_async(d + in_lo, h + in_lo, in_hi - in_lo, hipMemcpyHostToDevice, s), "H2D");
        }
        // patch lists for the big chunks (the small-batch path takes its whole staging span back)
        const bool patch_now = S && !wb_direct && (direct || nb * (c->raw + c->data) > (64u << 10));
        if (patch_now) // the codewords as they came, for the patch list after the decode (on the input
            // stream, which a decode leaves half idle, not ahead of the kernel on the output stream)
            HIP_TRY(ppfs_copy_launch(d + L.orig, d + L.raw, nb * c->raw, s_in), "orig copy");
        HIP_TRY(hipEventRecord(ev[0], s_in), "event");
        HIP_TRY(hipStreamWaitEvent(s_out, ev[0], 0), "wait");
        s = s_out;
        switch (op) {
        case OP_ENCODE:
            r = ppfs_ecc_encode_device(c, d + L.data, d + L.raw, nb, s);
            break;
        case OP_WRITE:
            r = ppfs_ecc_write_device(c, d + L.data, d + L.raw, d + L.status, nb, s);
            break;
        case OP_DECODE:
            if (wb_direct)
                r = queued(c,
                    ppfs_ecc_decode_device_impl(c, d + L.raw, data_out ? d + L.data : nullptr, d + L.status, nb, write_back,
                        nullptr, ordered(c, nb, s), img_dev + b0 * c->raw),
                    nb, s, "decode (async)");
            else
                r = ppfs_ecc_decode_device(c, d + L.raw, data_out ? d + L.data : nullptr, d + L.status, nb, write_back,
                    spill ? d + L.spill : nullptr, s);
            break;
        }
        if (r)
            return r;
        // outputs device -> pinned staging (or straight to page-locked caller buffers)
        const bool want_raw = op == OP_ENCODE || op == OP_WRITE || (lazy_raw && eager && !patch_now && !wb_direct);
        patched[slot] = patch_now && !img_dev;
        // the write-back goes straight into the caller's image (the patch kernel's, or the decode's own)
        landed[slot] = (patch_now && img_dev) || wb_direct;
        const bool want_data = op == OP_DECODE && data_out;
        const bool want_st = (status || lazy_raw) && op != OP_ENCODE;
        if (!direct && nb * (c->raw + c->data) <= (64u << 10)) {
            // small batches (the per-block IBlockDevice calls): one D2H of the staging span
            // instead of up to four -- each copy is a few us of latency on the critical path
            const size_t lo = want_data ? L.data : L.raw;
            const size_t hi = spill ? L.spill + nb * spill_b : (want_st ? L.status + nb : L.raw + nb * c->raw);
            HIP_TRY(dma_async(h + lo, d + lo, hi - lo, hipMemcpyDeviceToHost, s), "D2H");
            fetched[slot] = true;
        } else {
            fetched[slot] = want_raw;
            uint8_t* o_raw = direct ? raw + b0 * c->raw : h + L.raw;
            uint8_t* o_data = direct ? (data_out ? data_out + b0 * c->data : nullptr) : h + L.data;
            uint8_t* o_st = (direct && status) ? status + b0 : h + L.status;
            uint8_t* o_sp = direct ? (spill ? spill + b0 * spill_b : nullptr) : h + L.spill;
            if (want_raw)
                HIP_TRY(dma_async(o_raw, d + L.raw, nb * c->raw, hipMemcpyDeviceToHost, s), "D2H raw");
            if (want_data)
                HIP_TRY(dma_async(o_data, d + L.data, nb * c->data, hipMemcpyDeviceToHost, s), "D2H data");
            if (want_st)
                HIP_TRY(dma_async(o_st, d + L.status, nb, hipMemcpyDeviceToHost, s), "D2H status");
            if (spill)
                HIP_TRY(dma_async(o_sp, d + L.spill, nb * spill_b, hipMemcpyDeviceToHost, s), "D2H spill");
            if (patch_now) {
                HIP_TRY(ppfs_patch_list_launch(d + L.raw, d + L.orig, d + L.status, c->raw, nb, S, (uint32_t*)(d + L.patch),
                            img_dev ? img_dev + b0 * c->raw : nullptr, s), "patch list");
                if (eager && !img_dev) // the list comes back behind the kernel (fetched: apply_patches takes it as landed)
                    HIP_TRY(dma_async(h + L.patch, d + L.patch, nb * S * sizeof(uint32_t), hipMemcpyDeviceToHost, s), "D2H patch");
                fetched[slot] = eager && !img_dev;
            }
        }
        HIP_TRY(hipEventRecord(ev[1], s_out), "event");
        pending_first[slot] = b0;
        pending_n[slot] = nb;
        busy[slot] = true;
    }
    for (int j = 0; j < NS; ++j) // oldest first
        if ((r = drain((slot + j) % NS)))
            return r;
    if (lazy_raw)
        c->host_eager = eager;
    return 0;
}

extern "C" size_t ppfs_ecc_host_chunk_blocks(ppfs_ecc_ctx* c) { return c ? chunk_blocks(c) : 0; }

extern "C" int ppfs_ecc_encode_host(ppfs_ecc_ctx* c, const uint8_t* data, uint8_t* raw, size_t nblocks)
{
    return host_run(c, OP_ENCODE, data, nullptr, raw, nullptr, nullptr, nblocks, 0);
}

extern "C" int ppfs_ecc_decode_host(ppfs_ecc_ctx* c, uint8_t* raw, uint8_t* data, uint8_t* status, size_t nblocks,
    int write_back, uint8_t* spill)
{
    return host_run(c, OP_DECODE, nullptr, data, raw, status, spill, nblocks, write_back);
}

extern "C" int ppfs_ecc_write_host(ppfs_ecc_ctx* c, const uint8_t* data, uint8_t* raw, uint8_t* status, size_t nblocks)
{
    return host_run(c, OP_WRITE, data, nullptr, raw, status, nullptr, nblocks, 0);
}

// ---------------------------------------------------------------------------------------
// Whole-image scrub: the effect of readBlock(i) for i = 0..nblocks-1 in order on
// a disk image of image_bytes bytes, without the payloads: RS writes back the corrected
// codeword (rs_block_device.cpp:175-180), Hamming the flipped byte (hamming_block_device.cpp:
// 41-51), CRC and parity only check.  Blocks are independent except in one case: a shortened RS
// code (n < 255) whose miscorrection lands at a position >= n writes those bytes past the block
// end -- into the next block(s), which the sequential reference then reads modified, or off
// the image, in which case HeapDisk::write (heap_disk.cpp:21-27) rejects the whole write-back.
// Scrub reproduces that: one batch pass without write-back finds the spilling blocks (their
// spill record), and the image is then processed in runs between them.
// ---------------------------------------------------------------------------------------
namespace {
struct ScrubOps { // decode a block range of the image; copy spill bytes into the image
    std::function<int(size_t b0, size_t nb, int wb, uint8_t* st, uint8_t* spill)> decode;
    std::function<int(size_t addr, const uint8_t* src, size_t n)> put;
};

int scrub_run(const ppfs_ecc_ctx* c, size_t image_bytes, size_t nblocks, uint8_t* st, const ScrubOps& ops)
{
    const bool wb = c->p.ecc_type == PPFS_ECC_REED_SOLOMON || c->p.ecc_type == PPFS_ECC_HAMMING;
    if (!(c->p.ecc_type == PPFS_ECC_REED_SOLOMON && c->rs_n < 255))
        return ops.decode(0, nblocks, wb ? 1 : 0, st, nullptr);
    const size_t n = c->raw, sb = 256 - n;
    std::vector<uint8_t> spill(nblocks * sb);
    int r = ops.decode(0, nblocks, 0, st, spill.data()); // status + spill records, image untouched
    if (r)
        return r;
    size_t start = 0;
    for (size_t i = 0; i < nblocks; ++i) {
        const size_t extra = spill[i * sb];
        if (!extra)
            continue;
        if (i > start && (r = ops.decode(start, i - start, 1, st + start, nullptr)))
            return r;
        const size_t end = (i + 1) * n + extra; // the write-back covers [i n, end)
        if (end <= image_bytes) {
            if ((r = ops.decode(i, 1, 1, st + i, nullptr)) || (r = ops.put((i + 1) * n, &spill[i * sb + 1], extra)))
                return r;
            const size_t j = std::min(nblocks - 1, (end - 1) / n); // last block the spill touched
            if (j > i && (r = ops.decode(i + 1, j - i, 0, st + i + 1, &spill[(i + 1) * sb])))
                return r;
        } // else the reference's disk write fails and nothing of block i is written back
        start = i + 1;
    }
    return start < nblocks ? ops.decode(start, nblocks - start, 1, st + start, nullptr) : 0;
}

void scrub_counts(const uint8_t* st, size_t nblocks, size_t* counts)
{
    if (!counts)
        return;
    counts[0] = counts[1] = counts[2] = 0;
    for (size_t i = 0; i < nblocks; ++i)
        counts[st[i] == PPFS_ECC_OK ? 0 : (st[i] == PPFS_ECC_CORRECTED ? 1 : 2)]++;
}
} // namespace

extern "C" int ppfs_ecc_scrub_host(ppfs_ecc_ctx* c, uint8_t* image, size_t image_bytes, size_t nblocks,
    uint8_t* status, size_t* counts)
{
    if (!c || (nblocks && !image) || image_bytes < nblocks * (size_t)c->raw)
        return fail(PPFS_ECC_EINVAL, "scrub: bad argument");
    std::vector<uint8_t> st_local;
    if (!status) {
        st_local.resize(nblocks);
        status = st_local.data();
    }
    const size_t n = c->raw;
    ScrubOps ops;
    ops.decode = [&](size_t b0, size_t nb, int wb, uint8_t* st, uint8_t* spill) {
        return ppfs_ecc_decode_host(c, image + b0 * n, nullptr, st, nb, wb, spill);
    };
    ops.put = [&](size_t addr, const uint8_t* src, size_t len) {
        std::memcpy(image + addr, src, len);
        return 0;
    };
    const int r = scrub_run(c, image_bytes, nblocks, status, ops);
    if (r)
        return r;
    scrub_counts(status, nblocks, counts);
    return 0;
}

extern "C" int ppfs_ecc_scrub_device(ppfs_ecc_ctx* c, uint8_t* d_image, size_t image_bytes, size_t nblocks,
    uint8_t* d_status, void* stream)
{
    if (!c || (nblocks && !d_image) || image_bytes < nblocks * (size_t)c->raw)
        return fail(PPFS_ECC_EINVAL, "scrub: bad argument");
    hipStream_t s = (hipStream_t)stream;
    const size_t n = c->raw, sb = 256 - std::min<size_t>(n, 255);
    const bool chain = c->p.ecc_type == PPFS_ECC_REED_SOLOMON && c->rs_n < 255;
    uint8_t* d_spill = nullptr;
    uint8_t* bounce = nullptr; // page-locked: the spill records and patches never DMA pageable memory
    if (chain) {
        HIP_TRY(pool_alloc((void**)&d_spill, nblocks * sb, s), "scrub spill alloc");
        if (pin_alloc((void**)&bounce, std::max<size_t>(nblocks * sb, 256), kPinStage) != hipSuccess) {
            pool_free(d_spill, s);
            return fail(PPFS_ECC_ENOMEM, "scrub spill bounce");
        }
    }
    ScrubOps ops;
    ops.decode = [&](size_t b0, size_t nb, int wb, uint8_t* st_host, uint8_t* spill_host) {
        uint8_t* st = d_status ? d_status + b0 : nullptr;
        (void)st_host;
        int r = ppfs_ecc_decode_device(c, d_image + b0 * n, nullptr, st, nb, wb, spill_host ? d_spill + b0 * sb : nullptr,
            stream);
        if (r || !spill_host)
            return r;
        HIP_TRY(dma_async(bounce, d_spill + b0 * sb, nb * sb, hipMemcpyDeviceToHost, s), "scrub spill D2H");
        HIP_TRY(hipStreamSynchronize(s), "scrub sync");
        std::memcpy(spill_host, bounce, nb * sb);
        return 0;
    };
    ops.put = [&](size_t addr, const uint8_t* src, size_t len) { // len <= 255 - n < 256
        std::memcpy(bounce, src, len);
        HIP_TRY(dma_async(d_image + addr, bounce, len, hipMemcpyHostToDevice, s), "scrub spill H2D");
        HIP_TRY(hipStreamSynchronize(s), "scrub sync"); // the bounce is reused by the next call
        return 0;
    };
    // status bytes live on the device; scrub_run only indexes st (never reads it)
    std::vector<uint8_t> dummy(chain ? nblocks : 0);
    const int r = scrub_run(c, image_bytes, nblocks, dummy.data(), ops);
    if (d_spill) {
        pool_free(d_spill, s);
        (void)hipStreamSynchronize(s); // the bounce's last copy is done before it is freed
    }
    if (bounce)
        pin_free(bounce, std::max<size_t>(nblocks * sb, 256), kPinStage);
    return r;
}

// ---------------------------------------------------------------------------------------
// 2-of-3 bitwise voting of replicated records (vote.hip)
// ---------------------------------------------------------------------------------------
extern "C" int ppfs_vote3_device(const uint8_t* d_a, const uint8_t* d_b, const uint8_t* d_c, uint8_t* d_out,
    size_t rec_bytes, size_t nrec, uint32_t* d_damaged, void* stream)
{
    if ((nrec && rec_bytes && (!d_a || !d_b || !d_c || !d_out)))
        return fail(PPFS_ECC_EINVAL, "vote3: null argument");
    if (nrec && !rec_bytes)
        return fail(PPFS_ECC_EINVAL, "vote3: zero record size");
    return sync_check(
        check_hip(ppfs_vote3_launch(d_a, d_b, d_c, d_out, rec_bytes, nrec, d_damaged, (hipStream_t)stream), "vote3"),
        stream, "vote3 (async)");
}

extern "C" int ppfs_copy_device(void* d_dst, const void* d_src, size_t bytes, void* stream)
{
    if (bytes && (!d_dst || !d_src))
        return fail(PPFS_ECC_EINVAL, "copy: null argument");
    return sync_check(
        check_hip(ppfs_copy_launch((uint8_t*)d_dst, (const uint8_t*)d_src, bytes, (hipStream_t)stream), "copy"), stream,
        "copy (async)");
}

extern "C" int ppfs_inject_device(uint8_t* d_raw, size_t stride, size_t nblocks, const uint8_t* d_pos,
    const uint8_t* d_val, int mode, void* stream)
{
    if (nblocks && (!d_raw || !d_pos || !d_val))
        return fail(PPFS_ECC_EINVAL, "inject: null argument");
    if (nblocks && !stride)
        return fail(PPFS_ECC_EINVAL, "inject: zero stride");
    if (mode != 0 && mode != 1)
        return fail(PPFS_ECC_EINVAL, "inject: mode must be 0 (set) or 1 (xor)");
    return sync_check(check_hip(ppfs_inject_launch(d_raw, stride, nblocks, d_pos, d_val, mode, (hipStream_t)stream),
                          "inject"),
        stream, "inject (async)");
}

extern "C" int ppfs_vote3_host(int device, const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* out,
    size_t rec_bytes, size_t nrec, uint32_t* damaged)
{
    if (nrec && (!rec_bytes || !a || !b || !c || !out))
        return fail(PPFS_ECC_EINVAL, "vote3: bad argument");
    const size_t nbytes = rec_bytes * nrec;
    if (nbytes == 0) {
        if (damaged)
            std::memset(damaged, 0, nrec * sizeof(uint32_t));
        return 0;
    }
    DeviceGuard guard(device);
    HIP_TRY(guard.err, "set device");
    // its own non-blocking stream, drained before anything is freed (not the legacy null stream,
    // which does not order against other non-blocking streams).  The caller's (pageable) buffers
    // are copied by the CPU through page-locked staging, as the engine's host calls do: the DMA
    // engines only ever touch memory this call allocated and still holds.
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "vote3 stream");
    uint8_t *d = nullptr, *h = nullptr;
    const size_t dmg_off = (4 * nbytes + 255) & ~(size_t)255, total = dmg_off + nrec * sizeof(uint32_t);
    // stream-ordered device memory and the page-locked cache: nothing here synchronizes the device
    hipError_t e = pool_alloc((void**)&d, total, s);
    if (e == hipSuccess)
        e = pin_alloc((void**)&h, total, kPinStage);
    if (e == hipSuccess) {
        std::memcpy(h, a, nbytes);
        std::memcpy(h + nbytes, b, nbytes);
        std::memcpy(h + 2 * nbytes, c, nbytes);
        e = dma_async(d, h, 3 * nbytes, hipMemcpyHostToDevice, s);
    }
    if (e == hipSuccess)
        e = ppfs_vote3_launch(d, d + nbytes, d + 2 * nbytes, d + 3 * nbytes, rec_bytes, nrec,
            damaged ? (uint32_t*)(d + dmg_off) : nullptr, s);
    if (e == hipSuccess)
        e = dma_async(h + 3 * nbytes, d + 3 * nbytes, total - 3 * nbytes, hipMemcpyDeviceToHost, s);
    const hipError_t es = hipStreamSynchronize(s);
    if (e == hipSuccess)
        e = es;
    if (e == hipSuccess) {
        std::memcpy(out, h + 3 * nbytes, nbytes);
        if (damaged)
            std::memcpy(damaged, h + dmg_off, nrec * sizeof(uint32_t));
    }
    const int r = e != hipSuccess ? fail(PPFS_ECC_EHIP, "vote3", e) : 0;
    if (h)
        pin_free(h, total, kPinStage);
    if (d) {
        pool_free(d, s);
        (void)hipStreamSynchronize(s);
    }
    (void)hipStreamDestroy(s);
    return r;
}

// ---------------------------------------------------------------------------------------
// Page-locking of caller memory (a pinned host mirror of the disk image)
// ---------------------------------------------------------------------------------------
// Registry of the ranges registered through this ABI (start -> bytes): ppfs_ecc_host_registered
// lets a caller (tests/conftest.py) check that no engine-registered range outlives its owner --
// a range still registered after its memory went back to the allocator would let a later,
// unrelated buffer at the same address be treated as page-locked.
namespace {
std::mutex g_reg_mu;
std::map<uintptr_t, size_t> g_reg;
} // namespace

extern "C" int ppfs_ecc_host_register(void* ptr, size_t bytes)
{
    if (!ptr || !bytes)
        return fail(PPFS_ECC_EINVAL, "host_register: bad argument");
    std::lock_guard<std::mutex> lk(g_reg_mu);
    HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterDefault), "hipHostRegister");
    g_reg[(uintptr_t)ptr] = bytes;
    return 0;
}

extern "C" int ppfs_ecc_host_unregister(void* ptr)
{
    if (!ptr)
        return fail(PPFS_ECC_EINVAL, "host_unregister: null pointer");
    std::lock_guard<std::mutex> lk(g_reg_mu);
    HIP_TRY(hipHostUnregister(ptr), "hipHostUnregister");
    g_reg.erase((uintptr_t)ptr);
    return 0;
}

extern "C" long long ppfs_ecc_host_registered(size_t* bytes)
{
    std::lock_guard<std::mutex> lk(g_reg_mu);
    if (bytes) {
        size_t b = 0;
        for (const auto& kv : g_reg)
            b += kv.second;
        *bytes = b;
    }
    return (long long)g_reg.size();
}

// ------------------------------------------------------------------------------------------
// Multi-GPU host path: contiguous shards, one host thread per context
// ------------------------------------------------------------------------------------------
struct ppfs_ecc_group {
    std::vector<ppfs_ecc_ctx*> ctx;
};

extern "C" int ppfs_ecc_group_create(const ppfs_ecc_params* params, const int* devices, int ndevices,
    ppfs_ecc_group** out)
{
    if (!out || !devices || ndevices <= 0)
        return fail(PPFS_ECC_EINVAL, "group: devices");
    *out = nullptr;
    ppfs_ecc_group* g = new (std::nothrow) ppfs_ecc_group();
    if (!g)
        return fail(PPFS_ECC_ENOMEM, "group alloc");
    for (int i = 0; i < ndevices; ++i) {
        ppfs_ecc_ctx* c = nullptr;
        const int r = ppfs_ecc_create(params, devices[i], &c);
        if (r) {
            ppfs_ecc_group_destroy(g);
            return r;
        }
        g->ctx.push_back(c);
    }
    *out = g;
    return 0;
}

extern "C" void ppfs_ecc_group_destroy(ppfs_ecc_group* g)
{
    if (!g)
        return;
    for (ppfs_ecc_ctx* c : g->ctx)
        ppfs_ecc_destroy(c);
    delete g;
}

extern "C" int ppfs_ecc_group_size(const ppfs_ecc_group* g) { return g ? (int)g->ctx.size() : 0; }

extern "C" ppfs_ecc_ctx* ppfs_ecc_group_ctx(ppfs_ecc_group* g, int i)
{
    return (g && i >= 0 && i < (int)g->ctx.size()) ? g->ctx[(size_t)i] : nullptr;
}

namespace {
// run(ctx, first block, count) for every shard on its own thread; the first failing shard's
// code and message come back to the calling thread
int group_run(ppfs_ecc_group* g, size_t nblocks, const std::function<int(ppfs_ecc_ctx*, size_t, size_t)>& run)
{
    if (!g || g->ctx.empty())
        return fail(PPFS_ECC_EINVAL, "null group");
    const size_t G = g->ctx.size();
    if (G == 1 || nblocks < G)
        return run(g->ctx[0], 0, nblocks);
    std::vector<int> rc(G, 0);
    std::vector<std::string> msg(G);
    std::vector<std::thread> th;
    th.reserve(G);
    for (size_t i = 0; i < G; ++i) {
        const size_t b0 = nblocks * i / G, b1 = nblocks * (i + 1) / G;
        th.emplace_back([&, i, b0, b1] {
            rc[i] = run(g->ctx[i], b0, b1 - b0);
            if (rc[i])
                msg[i] = g_last_error;
        });
    }
    for (auto& t : th)
        t.join();
    for (size_t i = 0; i < G; ++i)
        if (rc[i]) {
            g_last_error = msg[i];
            return rc[i];
        }
    return 0;
}
} // namespace

extern "C" int ppfs_ecc_group_encode_host(ppfs_ecc_group* g, const uint8_t* data, uint8_t* raw, size_t nblocks)
{
    return group_run(g, nblocks, [&](ppfs_ecc_ctx* c, size_t b0, size_t nb) {
        return ppfs_ecc_encode_host(c, data + b0 * c->data, raw + b0 * c->raw, nb);
    });
}

extern "C" int ppfs_ecc_group_decode_host(ppfs_ecc_group* g, uint8_t* raw, uint8_t* data, uint8_t* status,
    size_t nblocks, int write_back, uint8_t* spill)
{
    return group_run(g, nblocks, [&](ppfs_ecc_ctx* c, size_t b0, size_t nb) {
        const size_t sp = 256 - std::min<size_t>(c->raw, 255);
        return ppfs_ecc_decode_host(c, raw + b0 * c->raw, data ? data + b0 * c->data : nullptr,
            status ? status + b0 : nullptr, nb, write_back, spill ? spill + b0 * sp : nullptr);
    });
}

extern "C" int ppfs_ecc_group_write_host(ppfs_ecc_group* g, const uint8_t* data, uint8_t* raw, uint8_t* status,
    size_t nblocks)
{
    return group_run(g, nblocks, [&](ppfs_ecc_ctx* c, size_t b0, size_t nb) {
        return ppfs_ecc_write_host(c, data + b0 * c->data, raw + b0 * c->raw, status ? status + b0 : nullptr, nb);
    });
}
