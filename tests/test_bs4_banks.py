"""Host model of the cfg5 four-lanes-per-block lookups (paritypartyfs_amd/csrc/rs_bs4.hpp q_lane /
q_lookups), CPU only: for every lookup m of a chunk and any byte values, the 32 lanes of each
ds_read_b64 group (MI355X_MICROARCH.md LDS table: lanes 0-31 and 32-63, bank = (address / 4) mod 64)
read 32 distinct 8-byte slots covering all 64 banks, and every lane reads its own quarter of the
entry for its own rotated chunk byte."""
import random


def q_lane(lane):
    c, blk = lane & 3, lane >> 2
    k = blk & 7
    return c, blk, k


def lookup_address(lane, m, chunk):
    """LDS byte offset (from the table base) lookup m of `lane` reads, and the chunk byte it uses"""
    c, _, k = q_lane(lane)
    q = (m + k) & 7                # rotated position
    byte = chunk[q]                # rotated chunk byte m = chunk byte (m + k) mod 8
    return byte * 256 + 32 * q + 8 * c, q


def test_quad_lookups_conflict_free():
    rng = random.Random(7)
    for _ in range(200):
        chunks = [[rng.randrange(256) for _ in range(8)] for _ in range(16)]  # one chunk per block
        for m in range(8):
            for group in (range(0, 32), range(32, 64)):
                banks = set()
                for lane in group:
                    _, blk, _ = q_lane(lane)
                    a, _ = lookup_address(lane, m, chunks[blk])
                    assert a % 8 == 0
                    banks.add((a // 4) % 64)
                    banks.add((a // 4 + 1) % 64)
                assert len(banks) == 64


def test_quad_lookups_cover_every_position_once():
    chunk = list(range(8))
    for lane in range(64):
        c, _, _ = q_lane(lane)
        seen = set()
        for m in range(8):
            a, q = lookup_address(lane, m, chunk)
            assert (a % 256) == 32 * q + 8 * c and a // 256 == chunk[q]
            seen.add(q)
        assert seen == set(range(8))
