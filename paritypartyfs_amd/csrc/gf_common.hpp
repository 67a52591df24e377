// gf_common.hpp -- shared device helpers for the PPFS ECC kernels (gfx950 / CDNA4).
//
// GF(2^8) with primitive polynomial 0x11D and alpha = 2, as in the reference
// lib/ecc_helpers/src/gf256.cpp:6-83 (a/0 == 0, inv(0) == 0).  Device code keeps the
// tables in LDS: EXP2[512] (EXP2[i] = alpha^(i mod 255), so a log sum never needs a mod),
// LOG[256] (LOG[0] = 0 like the reference) and QS[256] (a solution y of y^2 + y = c, 0 if none).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ppfs {

// Byte offsets of the GF tables inside the 1 KiB "gf block" uploaded per context.
constexpr int GF_EXP2 = 0;
constexpr int GF_LOG = 512;
constexpr int GF_QS = 768;
constexpr int GF_BYTES = 1024;

typedef __attribute__((address_space(3))) uint8_t lds_u8;

struct Gf {
    const uint8_t* t; // LDS (generic pointer into __shared__ memory)

    __device__ __forceinline__ uint32_t log(uint32_t a) const { return t[GF_LOG + a]; }
    __device__ __forceinline__ uint32_t exp(uint32_t i) const { return t[GF_EXP2 + i]; }
    __device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b) const
    {
        uint32_t r = t[GF_EXP2 + t[GF_LOG + a] + t[GF_LOG + b]];
        return (a && b) ? r : 0u;
    }
    __device__ __forceinline__ uint32_t div(uint32_t a, uint32_t b) const
    {
        uint32_t r = t[GF_EXP2 + 255u + t[GF_LOG + a] - t[GF_LOG + b]];
        return (a && b) ? r : 0u;
    }
    __device__ __forceinline__ uint32_t inv(uint32_t a) const
    {
        uint32_t r = t[GF_EXP2 + 255u - t[GF_LOG + a]];
        return a ? r : 0u;
    }
    // multiply by a value given in log form (la = LOG[a], a != 0)
    __device__ __forceinline__ uint32_t mul_log(uint32_t la, uint32_t b) const
    {
        uint32_t r = t[GF_EXP2 + la + t[GF_LOG + b]];
        return b ? r : 0u;
    }
    __device__ __forceinline__ uint32_t qs(uint32_t c) const { return t[GF_QS + c]; }
};

// Write-back of one corrected codeword byte to HBM (decode with write_back).  A plain byte store: the
// non-temporal form measured no faster.
__device__ __forceinline__ void wb_byte(uint8_t* p, uint8_t v) { *p = v; }

// Wave-uniform values: keep the compiler honest about what is uniform.
__device__ __forceinline__ uint32_t wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

} // namespace ppfs
