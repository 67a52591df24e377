// Host check of the t <= 4 RS emission schedules (paritypartyfs_amd/csrc/rs_sched.hpp) that the tile
// kernels read from the table blob (rs_wg_tk.hpp).  For 2t = 2, 4, 6, 8, encode and decode:
//   - every output piece of a 64-block tile is emitted exactly once;
//   - rounds 0-2 hold interior pieces only (the kernels run the 4-shift path there unconditionally);
//   - every wave has a piece in round 3 (each wave issues exactly 4 stores per tile, which the
//     encode's counted vmcnt waits rely on);
//   - an interior piece emulated as the kernel computes it -- 5 dwords from the LDS tile buffer at
//     (src & ~3), 4 funnel shifts by (src & 3) * 8 -- equals the codeword / payload bytes of that
//     piece, on random rows;
//   - the window reads of a 32-lane half (ds_read_b32 lane group) conflict no more than the natural
//     order p = tid + 256 k does (printed: LDS cycles of the window reads per tile);
//   - the encode's staging stores (ds_write_b128, 8-lane groups, banks (a / 4) mod 32) of rounds
//     0-2 are conflict-free for 2t = 4 and 6 (printed: LDS cycles per tile, all rounds);
//   - row_map(K) is a permutation of the 64 rows whose lanes 0-31 read their row starts on distinct
//     banks and lanes 32-63 at most 2 to a bank (phase 1's dword reads).
// Prints "ALL PASSED".
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <vector>

#include "../../paritypartyfs_amd/csrc/rs_sched.hpp"

using namespace ppfs::sched;

static int fails = 0;
#define CHECK(c, ...)                                                                                                  \
    do {                                                                                                               \
        if (!(c)) {                                                                                                    \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__);                                                          \
            std::printf(__VA_ARGS__);                                                                                  \
            std::printf("\n");                                                                                         \
            ++fails;                                                                                                   \
        }                                                                                                              \
    } while (0)

static uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t sh) { return (uint32_t)((((uint64_t)hi << 32) | lo) >> (sh & 31u)); }

// LDS cycles of the 5 window reads of a wave-round: per 32-lane half, per dword i, max distinct
// dwords on one bank (mod 32)
static int window_cycles(const std::vector<uint32_t>& src_of_lane)
{
    int cyc = 0;
    for (int h = 0; h < 2; ++h)
        for (int i = 0; i < 5; ++i) {
            std::vector<std::set<uint32_t>> bank(32);
            for (int l = 32 * h; l < 32 * h + 32; ++l)
                if (src_of_lane[l] != ~0u) {
                    const uint32_t d = (src_of_lane[l] >> 2) + (uint32_t)i;
                    bank[d & 31u].insert(d);
                }
            size_t m = 0;
            for (auto& b : bank)
                m = b.size() > m ? b.size() : m;
            cyc += (int)m;
        }
    return cyc;
}

static void check(int t2, bool dec)
{
    const uint32_t K = 255u - (uint32_t)t2;
    const uint32_t npieces = dec ? 64u * K / 16u : 64u * 255u / 16u;
    const std::vector<uint16_t> sc = dec ? build_decode(t2) : build_encode(t2);
    CHECK(sc.size() == 1024, "size");
    std::mt19937 rng(1234 + t2 + 100 * dec);
    // the tile as it sits in LDS (kPad front pad, rows packed) and the output it must produce
    const uint32_t row = dec ? 255u : K;
    std::vector<uint8_t> buf(kPad + 64 * 255 + 64, 0), out(npieces * 16);
    for (uint32_t i = 0; i < 64 * row; ++i)
        buf[kPad + i] = (uint8_t)rng();
    std::vector<uint8_t> par(64 * 8);
    for (auto& v : par)
        v = (uint8_t)rng();
    for (uint32_t j = 0; j < npieces * 16; ++j) {
        if (dec) {
            const uint32_t b = j / K, off = j % K;
            out[j] = buf[kPad + 255u * b + (uint32_t)t2 + off];
        } else {
            const uint32_t b = j / 255u, off = j % 255u;
            out[j] = off < (uint32_t)t2 ? par[8 * b + off] : buf[kPad + K * b + off - (uint32_t)t2];
        }
    }
    std::vector<int> seen(npieces, 0);
    int interior = 0, boundary = 0, cyc_sched = 0, cyc_nat = 0, cyc_stage = 0, bnd_waves = 0;
    for (uint32_t k = 0; k < 4; ++k) {
        for (uint32_t w = 0; w < 4; ++w) {
            std::vector<uint32_t> s_lane(64, ~0u), n_lane(64, ~0u);
            int have = 0;
            for (uint32_t l = 0; l < 64; ++l) {
                const uint32_t tid = 64 * w + l;
                const uint16_t e = sc[4 * tid + k];
                const uint32_t pn = tid + 256u * k; // the natural order's piece
                if (pn < npieces) {
                    const bool in = dec ? dec_interior(t2, pn) : enc_interior(t2, pn);
                    n_lane[l] = dec ? dec_src(t2, pn) : (in ? enc_src(t2, pn) : (uint32_t)kPad + K * (16u * pn / 255u));
                }
                if (e == kNone)
                    continue;
                ++have;
                const uint32_t p = e & 0x3FFu;
                CHECK(p < npieces, "t2 %d dec %d: piece %u out of range", t2, dec, p);
                if (p >= npieces)
                    continue;
                seen[p]++;
                const bool bnd = (e & kBoundary) != 0;
                const bool in = dec ? dec_interior(t2, p) : enc_interior(t2, p);
                CHECK(bnd == !in, "t2 %d dec %d: piece %u boundary flag %d, interior %d", t2, dec, p, bnd, in);
                CHECK(k == 3 || !bnd, "t2 %d dec %d: boundary piece %u in round %u", t2, dec, p, k);
                if (bnd) {
                    ++boundary;
                    continue;
                }
                ++interior;
                const uint32_t S = dec ? dec_src(t2, p) : enc_src(t2, p);
                s_lane[l] = S;
                uint32_t d[5];
                std::memcpy(d, &buf[S & ~3u], 20);
                uint32_t o[4];
                for (int m = 0; m < 4; ++m)
                    o[m] = alignbit(d[m + 1], d[m], (S & 3u) * 8u);
                CHECK(std::memcmp(o, &out[16u * p], 16) == 0, "t2 %d dec %d: interior piece %u bytes differ", t2, dec, p);
            }
            CHECK(k < 3 || have > 0, "t2 %d dec %d: wave %u has no round-3 piece", t2, dec, w);
            if (k == 3)
                for (uint32_t l = 0; l < 64; ++l)
                    if (sc[4 * (64 * w + l) + k] != kNone && (sc[4 * (64 * w + l) + k] & kBoundary)) {
                        ++bnd_waves;
                        break;
                    }
            CHECK(k == 3 || have == 64, "t2 %d dec %d: wave %u round %u has %d pieces", t2, dec, w, k, have);
            cyc_sched += window_cycles(s_lane);
            cyc_nat += window_cycles(n_lane);
            // staging stores: per 8-lane group, the most pieces on one bank quad (p mod 8)
            for (uint32_t g = 0; g < 8; ++g) {
                int quad[8] = {}, m = 0, n = 0;
                for (uint32_t l = 8 * g; l < 8 * g + 8; ++l) {
                    const uint16_t e = sc[4 * (64 * w + l) + k];
                    if (e != kNone) {
                        m = std::max(m, ++quad[e & 7u]);
                        ++n;
                    }
                }
                cyc_stage += m;
                CHECK(dec || (t2 != 4 && t2 != 6) || k == 3 || m == 1, "t2 %d: round %u wave %u group %u stores %d-way", t2, k, w, g, m);
            }
        }
    }
    for (uint32_t p = 0; p < npieces; ++p)
        CHECK(seen[p] == 1, "t2 %d dec %d: piece %u emitted %d times", t2, dec, p, seen[p]);
    std::printf("2t=%d %s: %d interior + %d boundary pieces; window-read LDS cycles per tile %d (natural order %d); "
                "staging-store group cycles %d (ideal 128)\n",
        t2, dec ? "decode" : "encode", interior, boundary, cyc_sched, cyc_nat, cyc_stage);
    CHECK(cyc_sched <= cyc_nat, "t2 %d dec %d: schedule conflicts more than the natural order", t2, dec);
    // the boundary pieces (the general byte-mask merge) stay packed at the end of round 3: at most one
    // wave more than they fill runs the merge path (the polish swaps boundary slots with boundary /
    // empty slots only); spread over every wave, each wave would run both emission paths
    const int need = (boundary + 63) / 64;
    CHECK(bnd_waves <= need + 1, "t2 %d dec %d: boundary pieces spread over %d waves (%d needed)", t2, dec, bnd_waves, need);
}

static void check_rows(uint32_t len)
{
    const std::vector<uint8_t> rm = row_map(len);
    CHECK(rm.size() == 64, "row map size");
    std::vector<int> seen(64, 0);
    int worst[2] = { 0, 0 };
    for (int h = 0; h < 2; ++h) {
        int bank[32] = {};
        for (int l = 32 * h; l < 32 * h + 32; ++l) {
            CHECK(rm[l] < 64, "row %u", rm[l]);
            seen[rm[l] & 63]++;
            worst[h] = std::max(worst[h], ++bank[(len * rm[l] / 4u) & 31u]);
        }
    }
    for (int r = 0; r < 64; ++r)
        CHECK(seen[r] == 1, "len %u: row %d mapped %d times", len, r, seen[r]);
    CHECK(worst[0] == 1 && worst[1] <= 2, "len %u: row reads %d-way / %d-way", len, worst[0], worst[1]);
    std::printf("row_map(%u): lanes 0-31 %d-way, lanes 32-63 %d-way\n", len, worst[0], worst[1]);
}

int main()
{
    for (int t2 = 2; t2 <= 8; t2 += 2) {
        check(t2, false);
        check(t2, true);
        check_rows(255u - (uint32_t)t2);
    }
    if (fails) {
        std::printf("%d FAILED\n", fails);
        return 1;
    }
    std::printf("ALL PASSED\n");
    return 0;
}
