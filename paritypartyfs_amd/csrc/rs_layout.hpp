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
    static_assert(TABLE_BYTES % 16 == 0, "tables are copied in 16-byte pieces");
};

constexpr int rs_wg_table_bytes(int t2)
{
    return 16 * 128 + 3 * 2 * t2 * 128 + 2 * t2 * 128 + GF_BYTES;
}

} // namespace ppfs
