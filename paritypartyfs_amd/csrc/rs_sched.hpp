#pragma once
// rs_sched.hpp -- emission schedules of the t <= 4 RS tile kernels (rs_wg_tk.hpp), built on the host
// once per context and stored in the table blob (rs_layout.hpp OFF_ESCHED / OFF_DSCHED).
//
// A 64-block tile's output is 1020 (encode: 64 x 255 B) or 64 K / 16 (decode: 64 x K B) 16-byte
// pieces; the 256 threads emit them in 4 rounds.  Most pieces are "interior": all 16 bytes come from
// one LDS row at one offset (encode: payload bytes of one block after its 2t parity bytes; decode:
// payload bytes of one codeword), so the piece is 4 funnel shifts of a 5-dword LDS window and
// nothing else.  The rest ("boundary" pieces: an encode piece holding parity bytes or a block
// start, a decode piece crossing a block end) need the general byte-mask merge (rs_wg.hpp enc_piece
// / dec_piece).  The schedule puts every interior piece in rounds 0-2 and the first lanes of round
// 3, and the boundary pieces in the last lanes of round 3, so only one or two waves run the merge,
// once per tile, instead of every piece paying for it.
//
// Within that, interior pieces are grouped per 32-lane half wave (the lane group of ds_read_b32,
// MI355X_MICROARCH.md LDS table) so that the window dword addresses of a half are distinct mod 32
// (banks): taken in piece order, greedily, a piece joins the current half when its window start
// hits a bank no piece of the half hits yet.  For 2t = 6 every full half is conflict-free (the
// natural order p = tid + 256 k is 2-way).  Consecutive pieces of a block have window starts 4
// dwords apart, so a half is mostly runs of 8 consecutive pieces (128 B of output each).
//
// Entry (u16, thread-major: entry 4 tid + k is thread tid's piece of round k):
//   bits 0-9   piece index; bit 15 set = boundary piece; 0xFFFF = no piece in that round.
#include <stdint.h>

#include <vector>

namespace ppfs {
namespace sched {

constexpr int kTile = 64, kThreads = 256, kRounds = 4, kPad = 16;
constexpr uint16_t kBoundary = 0x8000, kNone = 0xFFFF;

// LDS byte (relative to the tile buffer) of an interior piece's first source byte
inline uint32_t enc_src(int t2, uint32_t p)
{
    const uint32_t k = 255u - (uint32_t)t2, j0 = 16u * p, b = j0 / 255u, off = j0 - 255u * b;
    return (uint32_t)kPad + k * b + off - (uint32_t)t2;
}
inline uint32_t dec_src(int t2, uint32_t p)
{
    const uint32_t k = 255u - (uint32_t)t2, j0 = 16u * p, b = j0 / k, off = j0 - k * b;
    return (uint32_t)kPad + 255u * b + (uint32_t)t2 + off;
}
inline bool enc_interior(int t2, uint32_t p)
{
    for (uint32_t j = 16u * p; j < 16u * p + 16u; ++j)
        if (j % 255u < (uint32_t)t2)
            return false;
    return true;
}
inline bool dec_interior(int t2, uint32_t p)
{
    const uint32_t k = 255u - (uint32_t)t2;
    return (16u * p) / k == (16u * p + 15u) / k;
}

// the schedule of `npieces` pieces given the interior test and window start; returns 4 x 256 u16
template <class Interior, class Src>
inline std::vector<uint16_t> build(uint32_t npieces, Interior interior, Src src)
{
    std::vector<uint32_t> inter, bnd;
    for (uint32_t p = 0; p < npieces; ++p)
        (interior(p) ? inter : bnd).push_back(p);
    // greedy halves: distinct window-start banks (dword mod 32) per 32 lanes
    std::vector<uint32_t> seq;
    std::vector<uint32_t> left = inter;
    while (!left.empty()) {
        uint32_t used = 0, n = 0;
        std::vector<uint32_t> rest;
        for (uint32_t p : left) {
            const uint32_t bank = (src(p) >> 2) & 31u;
            if (n < 32 && !(used >> bank & 1u)) {
                used |= 1u << bank;
                seq.push_back(p);
                ++n;
            } else {
                rest.push_back(p);
            }
        }
        left.swap(rest);
    }
    std::vector<uint16_t> out((size_t)kThreads * kRounds, kNone);
    size_t j = 0; // slot j = round k = j / 256, thread j % 256
    for (uint32_t p : seq) {
        out[(j % kThreads) * kRounds + j / kThreads] = (uint16_t)p;
        ++j;
    }
    for (uint32_t p : bnd) {
        out[(j % kThreads) * kRounds + j / kThreads] = (uint16_t)(p | kBoundary);
        ++j;
    }
    return out;
}

inline std::vector<uint16_t> build_encode(int t2)
{
    return build(kTile * 255 / 16, [t2](uint32_t p) { return enc_interior(t2, p); },
        [t2](uint32_t p) { return enc_src(t2, p); });
}
inline std::vector<uint16_t> build_decode(int t2)
{
    return build((uint32_t)(kTile * (255 - t2) / 16), [t2](uint32_t p) { return dec_interior(t2, p); },
        [t2](uint32_t p) { return dec_src(t2, p); });
}

} // namespace sched
} // namespace ppfs
