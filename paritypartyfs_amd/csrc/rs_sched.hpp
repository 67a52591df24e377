#pragma once
// rs_sched.hpp -- emission schedules of the t <= 4 RS tile kernels (rs_wg_tk.hpp), built on the host
// once per context and stored in the table blob (rs_layout.hpp OFF_ESCHED; the decode schedule only in
// tests/cpp/test_sched.cpp).
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

#include <algorithm>
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

// Orders one 32-lane half so that each 8-lane group -- the ds_write_b128 lane group of the encode's
// staging stores, banks (a / 4) mod 32, so piece p takes bank quad p mod 8 -- holds distinct p mod 8
// wherever the half allows.  Lane order within a half leaves the window reads' banking alone (their
// lane groups are the halves).
inline void spread_groups(uint16_t* half)
{
    std::vector<uint16_t> bucket[8], none;
    for (int i = 0; i < 32; ++i)
        (half[i] == kNone ? none : bucket[half[i] & 7u]).push_back(half[i]);
    auto fullest = [&](uint32_t skip) {
        int best = -1;
        for (int r = 0; r < 8; ++r)
            if (!(skip >> r & 1u) && !bucket[r].empty() && (best < 0 || bucket[r].size() > bucket[best].size()))
                best = r;
        return best;
    };
    for (int g = 0; g < 4; ++g) {
        uint32_t used = 0;
        int n = 0;
        for (int r; n < 8 && (r = fullest(used)) >= 0; ++n) { // one piece per residue, fullest first
            half[8 * g + n] = bucket[r].back();
            bucket[r].pop_back();
            used |= 1u << r;
        }
        for (; n < 8 && !none.empty(); ++n) { // then the lanes without a piece
            half[8 * g + n] = none.back();
            none.pop_back();
        }
        for (int r; n < 8 && (r = fullest(0)) >= 0; ++n) { // then (a conflict) what is left
            half[8 * g + n] = bucket[r].back();
            bucket[r].pop_back();
        }
    }
}

// Kuhn's augmenting path for the octet matching below: residue r -> a piece whose shifted bank
// quad u is free (owner[u] = index of the piece holding u, or -1)
inline bool octet_augment(int r, const std::vector<std::vector<int>>& by_r, const std::vector<uint32_t>& u_of,
    int (&owner)[8], int (&pick)[8], uint32_t& seen)
{
    for (int i : by_r[r]) {
        const uint32_t u = u_of[i];
        if (seen >> u & 1u)
            continue;
        seen |= 1u << u;
        if (owner[u] < 0 || octet_augment(owner[u] >> 8, by_r, u_of, owner, pick, seen)) {
            owner[u] = (r << 8) | i; // residue and piece
            pick[r] = i;
            return true;
        }
    }
    return false;
}

// LDS cycles of a 32-lane half's 5 window reads (per dword: the most distinct dwords on one bank)
// plus its four 8-lane staging-store groups (the most pieces on one bank quad p mod 8)
template <class Src> inline int half_cycles(const uint16_t* half, Src src)
{
    int cyc = 0, na = 0;
    uint32_t a[32];
    for (int l = 0; l < 32; ++l)
        if (half[l] != kNone)
            a[na++] = src(half[l] & 0x3FFu) >> 2;
    std::sort(a, a + na);
    na = (int)(std::unique(a, a + na) - a); // equal dwords broadcast
    for (uint32_t i = 0; i < 5; ++i) {
        int bank[32] = {}, m = 0;
        for (int l = 0; l < na; ++l) {
            const int c = ++bank[(a[l] + i) & 31u];
            m = c > m ? c : m;
        }
        cyc += m;
    }
    for (int g = 0; g < 4; ++g) {
        int quad[8] = {}, m = 0;
        for (int l = 8 * g; l < 8 * g + 8; ++l)
            if (half[l] != kNone) {
                const int c = ++quad[half[l] & 7u];
                m = c > m ? c : m;
            }
        cyc += m;
    }
    return cyc;
}

// The last round holds the leftovers (pieces outside full halves, the boundary pieces): a
// deterministic hill climb over swaps of two of its slots of one kind (interior with interior,
// boundary or none with boundary or none), kept when the two halves' LDS cycles do not rise
template <class Src> inline void polish_last_round(std::vector<uint16_t>& slots, Src src)
{
    const size_t base = (size_t)kThreads * (kRounds - 1);
    auto kind = [](uint16_t e) { return e != kNone && !(e & kBoundary) ? 0 : 1; };
    uint32_t rng = 12345u;
    for (int it = 0; it < 20000; ++it) {
        rng = rng * 1664525u + 1013904223u;
        const size_t x = base + (rng >> 8) % (size_t)kThreads;
        rng = rng * 1664525u + 1013904223u;
        const size_t y = base + (rng >> 8) % (size_t)kThreads;
        if (x / 32 == y / 32 && x / 8 == y / 8)
            continue;
        if (kind(slots[x]) != kind(slots[y]))
            continue;
        uint16_t* hx = &slots[x / 32 * 32];
        uint16_t* hy = &slots[y / 32 * 32];
        const int before = half_cycles(hx, src) + (hx != hy ? half_cycles(hy, src) : 0);
        std::swap(slots[x], slots[y]);
        const int after = half_cycles(hx, src) + (hx != hy ? half_cycles(hy, src) : 0);
        if (after > before)
            std::swap(slots[x], slots[y]);
    }
}

// The schedule of `npieces` pieces given the interior test and window start; returns 4 x 256 u16.
//
// An interior piece p whose window starts at LDS dword a = src(p) / 4 has a = 4 p + c (mod 32), c
// constant over a block (the row start's offset).  So its window bank is w = 4 ((r + s) mod 8) + k
// with r = p mod 8 (also its staging-store bank quad: encode, ds_write_b128 of piece p at 16 p),
// k = c mod 4 and s = c / 4.  An "octet" -- 8 pieces of one k with distinct r and distinct
// (r + s) mod 8 -- fills one 8-lane store group without a conflict and 8 distinct banks; four octets
// of distinct k make a 32-lane half whose window reads (ds_read_b32 groups are the halves) are
// conflict-free too.  Octets come first from blocks of one (k, s) (one piece per residue), then from
// what is left of one k (a perfect residue -> shifted-quad matching).  Pieces outside full halves go
// in greedy halves of distinct window banks; boundary pieces last (round 3), and every half is then
// ordered so each 8-lane group holds distinct residues where it can (spread_groups).
template <class Interior, class Src>
inline std::vector<uint16_t> build(uint32_t npieces, Interior interior, Src src)
{
    std::vector<uint32_t> bnd, pool[4][8]; // interior pieces by (k, s)
    for (uint32_t p = 0; p < npieces; ++p) {
        if (!interior(p)) {
            bnd.push_back(p);
            continue;
        }
        const uint32_t c = ((src(p) >> 2) - 4u * p) & 31u;
        pool[c & 3u][c >> 2].push_back(p);
    }
    std::vector<std::vector<uint32_t>> octets[4];
    for (int k = 0; k < 4; ++k) {
        std::vector<uint32_t> rest_p, rest_s;
        for (uint32_t sv = 0; sv < 8; ++sv) {
            std::vector<uint32_t> by[8];
            for (uint32_t p : pool[k][sv])
                by[p & 7u].push_back(p);
            for (;;) {
                bool full = true;
                for (auto& b : by)
                    full = full && !b.empty();
                if (!full)
                    break;
                std::vector<uint32_t> o;
                for (auto& b : by) {
                    o.push_back(b.back());
                    b.pop_back();
                }
                octets[k].push_back(o);
            }
            for (auto& b : by)
                for (uint32_t p : b) {
                    rest_p.push_back(p);
                    rest_s.push_back(sv);
                }
        }
        // octets across s: residue r -> quad u = (r + s) mod 8, a perfect matching of the leftovers
        for (;;) {
            std::vector<std::vector<int>> by_r(8);
            std::vector<uint32_t> u_of(rest_p.size());
            for (size_t i = 0; i < rest_p.size(); ++i) {
                by_r[rest_p[i] & 7u].push_back((int)i);
                u_of[i] = (rest_p[i] + rest_s[i]) & 7u;
            }
            int owner[8], pick[8];
            for (int u = 0; u < 8; ++u)
                owner[u] = -1;
            bool ok = true;
            for (int r = 0; r < 8 && ok; ++r) {
                uint32_t seen = 0;
                ok = octet_augment(r, by_r, u_of, owner, pick, seen);
            }
            if (!ok)
                break;
            std::vector<uint32_t> o;
            std::vector<bool> take(rest_p.size(), false);
            for (int u = 0; u < 8; ++u) {
                const int i = owner[u] & 0xFF;
                take[(size_t)i] = true;
                o.push_back(rest_p[(size_t)i]);
            }
            octets[k].push_back(o);
            std::vector<uint32_t> np, ns;
            for (size_t i = 0; i < rest_p.size(); ++i)
                if (!take[i]) {
                    np.push_back(rest_p[i]);
                    ns.push_back(rest_s[i]);
                }
            rest_p.swap(np);
            rest_s.swap(ns);
        }
        pool[k][0] = rest_p; // the leftovers of class k
    }
    std::vector<uint32_t> seq, left;
    for (;;) { // full halves: one octet of each k
        bool all = true;
        for (auto& o : octets)
            all = all && !o.empty();
        if (!all)
            break;
        for (auto& o : octets) {
            seq.insert(seq.end(), o.back().begin(), o.back().end());
            o.pop_back();
        }
    }
    for (int k = 0; k < 4; ++k) {
        for (auto& o : octets[k])
            left.insert(left.end(), o.begin(), o.end());
        left.insert(left.end(), pool[k][0].begin(), pool[k][0].end());
    }
    std::sort(left.begin(), left.end());
    // greedy halves: distinct window-start banks (dword mod 32) per 32 lanes
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
    std::vector<uint16_t> slots((size_t)kThreads * kRounds, kNone); // slot j = round j / 256, thread j % 256
    size_t j = 0;
    for (uint32_t p : seq)
        slots[j++] = (uint16_t)p;
    for (uint32_t p : bnd)
        slots[j++] = (uint16_t)(p | kBoundary);
    for (size_t h = 0; h < slots.size(); h += 32)
        spread_groups(&slots[h]);
    polish_last_round(slots, src);
    std::vector<uint16_t> out(slots.size());
    for (j = 0; j < slots.size(); ++j)
        out[(j % kThreads) * kRounds + j / kThreads] = slots[j];
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

// The encode's phase 1 (rs_wg.hpp seg_remainder): lane -> payload row.  A lane reads its row's
// segment as dwords from the row start, and the tile buffers and segments start at multiples of 4,
// so row r sits on bank (len r / 4) mod 32 plus a constant.  Rows are ranked per bank (the i-th row
// of a bank has level i); lanes 0-31 take the even levels, lanes 32-63 the odd ones, so for the
// payload rows of t <= 4 (len 247..253: each bank holds 1 to 3 rows) lanes 0-31 read conflict-free
// and lanes 32-63 at most 2-way (the fixed lane_row split is 2-way in both halves).
inline std::vector<uint8_t> row_map(uint32_t len)
{
    std::vector<uint8_t> half[2];
    uint32_t level_of_bank[32] = {};
    for (uint32_t r = 0; r < (uint32_t)kTile; ++r) {
        const uint32_t b = (len * r / 4u) & 31u;
        half[level_of_bank[b]++ & 1u].push_back((uint8_t)r);
    }
    while (half[0].size() > 32) {
        half[1].push_back(half[0].back());
        half[0].pop_back();
    }
    while (half[1].size() > 32) {
        half[0].push_back(half[1].back());
        half[1].pop_back();
    }
    std::vector<uint8_t> out(half[0]);
    out.insert(out.end(), half[1].begin(), half[1].end());
    return out;
}

} // namespace sched
} // namespace ppfs
