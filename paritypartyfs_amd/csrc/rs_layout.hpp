#pragma once
// rs_layout.hpp -- table layout of the workgroup-cooperative RS(255, 255-2t) kernels (rs_wg.hpp),
// shared by the host table builder (api.cpp) and the device code.  2t <= 8 (t <= 4), so a
// remainder fits one 8-byte entry, stored top-aligned: coefficient q of x^q at byte 8 - 2t + q.
//
// Every table is a set of nibble tables: 16 entries of 8 bytes (one 128-byte table), indexed by
// one nibble of one input byte.  A wave's 64 lanes always read the same table in one
// instruction, so the 16 possible entries sit in 32 distinct LDS banks: conflict-free.
//   SL   slicing-by-8: table 2i+h, value v -> (v << 4h) * x^(2t+i) mod g      (16 tables)
//   MAP  m = 0,1,2: table 2q+h, value v -> (v << 4h) * x^(q + 64(m+1)) mod g (2t tables each):
//        moves a segment remainder from segment m+1 to its place in the codeword
//   MAP32 the same for 32-byte segments, m = 0..6 (the 8-wave encode; appended after GF)
//   SYN  table 2q+h, value v -> bytes i-1 = (v << 4h) * alpha^(i (q - 2t)), i = 1..2t: the
//        syndromes S_i = c(alpha^i) from r' = x^2t c(x) mod g (rs_block_device.cpp:131-141)
//   GF   the 1 KiB EXP2 / LOG / QS block of gf_common.hpp
#include "gf_common.hpp"

namespace ppfs {

template <int T2> struct RsWgLayout {
    static_assert(T2 >= 2 && T2 <= 8 && (T2 % 2) == 0, "workgroup RS path: 2t in {2,4,6,8}");
    static constexpr int N = 255, K = N - T2;
    static constexpr int ES = 8;         // entry bytes
    static constexpr int TBL = 16 * ES;  // one nibble table
    static constexpr int OFF_SL = 0;
    static constexpr int OFF_MAP = OFF_SL + 16 * TBL;
    static constexpr int MAP_STRIDE = 2 * T2 * TBL;
    static constexpr int OFF_SYN = OFF_MAP + 3 * MAP_STRIDE;
    static constexpr int OFF_GF = OFF_SYN + 2 * T2 * TBL;
    static constexpr int TABLE_BYTES = OFF_GF + GF_BYTES;
    // MAP32 (after the decode layout, read by the 8-wave encode only): m = 0..6, the x^(q + 32(m+1))
    // maps of 32-byte segments
    static constexpr int OFF_MAP32 = TABLE_BYTES;
    // SLX (round 3): the slicing tables of segment m = 1..3 with x^(64 m) folded in, 16 nibble
    // tables each: table 2i+h, value v -> (v << 4h) * x^(2t+i+64m) mod g, read by the LAST slicing
    // step of segment m, which then needs no x^(64 m) map (rs_wg.hpp seg_remainder)
    static constexpr int OFF_SLX = OFF_MAP32 + 7 * MAP_STRIDE;
    static constexpr int SLX_BYTES = 3 * 16 * TBL;
    // ESCHED (round 4): the encode's emission schedule (rs_sched.hpp), 256 threads x 4 rounds of u16;
    // the encode DMAs it into the staging buffer once per workgroup (the decode emits in natural
    // order: its schedule is built only by tests/cpp/test_sched.cpp)
    static constexpr int OFF_ESCHED = OFF_SLX + SLX_BYTES;
    static constexpr int SCHED_BYTES = 2048;
    // ROWMAP (round 4): the encode's lane -> payload row of phase 1 (rs_sched.hpp row_map), 64 bytes
    static constexpr int OFF_ROWMAP = OFF_ESCHED + SCHED_BYTES;
    // SL5 / SLX5 (round 4): SL and SLX as 5-bit field tables for the encode's phase 1: table i (of
    // 13), value v -> the contribution of v at bits [5i, 5i+5) of the 64-bit chunk; 32 entries x 8 B
    // = 256 B, the 64 banks of a ds_read_b64 lane group (conflict-free), 13 lookups per step not 16
    static constexpr int SL5_BYTES = 13 * 32 * ES;
    static constexpr int OFF_SL5 = OFF_ROWMAP + 64;
    static constexpr int OFF_SLX5 = OFF_SL5 + SL5_BYTES;
    static constexpr int SLX5_BYTES = 3 * SL5_BYTES;
    static constexpr int BLOB_BYTES = OFF_SLX5 + SLX5_BYTES;
    static_assert(TABLE_BYTES % 16 == 0 && BLOB_BYTES % 16 == 0, "tables are copied in 16-byte pieces");
};

constexpr int rs_wg_table_bytes(int t2)
{
    return t2 == 2 ? RsWgLayout<2>::BLOB_BYTES : t2 == 4 ? RsWgLayout<4>::BLOB_BYTES
         : t2 == 6 ? RsWgLayout<6>::BLOB_BYTES : RsWgLayout<8>::BLOB_BYTES;
}

// Pair RS path (rs_pair.hpp), 16 < 2t <= 32: the same 32-byte top-aligned state, two lanes per
// block each holding a 16-byte column.
//   SL   slicing-by-8, nibble-indexed: table t = 2i + h (byte i of the chunk, nibble h), column
//        plane c: 16 entries x 16 B = bytes [16c, 16c+16) of (v << 4h) * x^(2t+i) mod g, at
//        512 t + 256 c + 16 v (each plane is exactly the 64 LDS banks)
//   GF   the 1 KiB EXP2 / LOG / QS block
//   XP   decode only: row p (32 B, state layout) = LOG of each coefficient of x^(p+2t) mod g, 0xFF
//        for a zero coefficient -- the remainder of a single error e at byte p is e * row p,
//        which is how the decoder confirms the single-error case
//   XPM  the same rows for x^p mod g (decode from c mod g)
//   BS   byte-slice tables of the rs_bs.hpp kernels (2t = 32), 64 KiB: row v (256 B) holds, in
//        slot 2q + c (16 B), bytes [16c, 16c+16) of v * x^(2t+q) mod g = SL[2q][v & 15] ^
//        SL[2q+1][v >> 4] -- the eight byte positions of a chunk side by side, so that lanes
//        reading distinct slots hit distinct banks whatever byte values they look up
//   S12  the rs_bs.hpp decode's first two syndromes from c mod g, 16 KiB: entry (u, v) (2 B at
//        512 u + 2 v) = v alpha^u | (v alpha^(2u)) << 8, the contribution of state byte u = v
template <int T2> struct RsPairLayout {
    static_assert(T2 > 16 && T2 <= 32 && (T2 % 2) == 0, "pair RS path: 2t in (16, 32]");
    static constexpr int N = 255, K = N - T2;
    static constexpr int OFF_SL = 0;
    static constexpr int OFF_GF = OFF_SL + 16 * 512;
    static constexpr int OFF_XP = OFF_GF + GF_BYTES;
    static constexpr int ENC_BYTES = OFF_GF;
    static constexpr int OFF_XPM = OFF_XP + 255 * 32; // rows x^p mod g (decode from c mod g)
    static constexpr int OFF_BS = OFF_XPM + 255 * 32;
    static constexpr int BS_BYTES = 256 * 256;
    static constexpr int OFF_S12 = OFF_BS + BS_BYTES;
    static constexpr int S12_BYTES = 32 * 256 * 2;
    static constexpr int TABLE_BYTES = OFF_S12 + S12_BYTES;
    static_assert(OFF_BS % 16 == 0, "aligned byte-slice tables");
};

constexpr int rs_pair_table_bytes() { return 16 * 512 + GF_BYTES + 2 * 255 * 32 + 256 * 256 + 32 * 256 * 2; }

} // namespace ppfs
