"""GPU tests of the engine's boundary hygiene (round-2 fixes of the asynchronous-fault suspects):

- the Python mirror rejects buffers shorter than a call touches, and buffers of the wrong kind,
  before anything reaches the C ABI (an undersized host array would overflow the heap, an
  undersized tensor would be written out of bounds in HBM);
- a host buffer that is only partly page-locked is not DMA'd directly (api.cpp host_pinned checks
  the whole range) and still gives the oracle's results;
- destroying a context right after queueing device work on the caller's stream is safe: the
  context's tables stay alive until that work is done (ppfs_ecc_destroy drains first);
- the C++ adapter propagates engine errors as Disk_IOError (tests/cpp, EngineErrors).
"""
import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch

from paritypartyfs_amd import ECC_CRC, ECC_HAMMING, ECC_REED_SOLOMON, EccEngine, EccGroup, pinned, vote3, vote3_host


def test_short_and_wrong_kind_buffers_rejected():
    eng = EccEngine(ECC_REED_SOLOMON, 512, 3)
    n, k = eng.raw_block_size, eng.data_size
    nb = 100
    d = torch.zeros(nb * k, dtype=torch.uint8, device="cuda")
    r = torch.zeros(nb * n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        eng.encode(d, r[: nb * n - 1], nblocks=nb)
    with pytest.raises(ValueError):
        eng.encode(d[:-1], r, nblocks=nb)
    with pytest.raises(ValueError):
        eng.decode(r, d, st[:-1], nblocks=nb)
    with pytest.raises(ValueError):
        eng.decode(r, d[: nb * k - 5], st, nblocks=nb)
    with pytest.raises(ValueError):
        eng.write(d, r[:10], st, nblocks=nb)
    with pytest.raises(ValueError):  # host array into a device entry point
        eng.encode(np.zeros(nb * k, np.uint8), r, nblocks=nb)
    hd, hr, hs = np.zeros(nb * k, np.uint8), np.zeros(nb * n, np.uint8), np.zeros(nb, np.uint8)
    with pytest.raises(ValueError):
        eng.encode_host(hd, hr[:-1])
    with pytest.raises(ValueError):
        eng.decode_host(hr, hd[:-1], hs)
    with pytest.raises(ValueError):
        eng.decode_host(hr, hd, hs[:-1])
    with pytest.raises(ValueError):
        eng.write_host(hd, hr, hs[:3])
    with pytest.raises(ValueError):  # tensor into a host entry point
        eng.encode_host(d, hr)
    with pytest.raises(ValueError):
        eng.scrub_host(hr, nblocks=nb + 1)
    # right-sized calls still work
    eng.encode(d, r, nblocks=nb)
    eng.decode(r, d, st, nblocks=nb)
    torch.cuda.synchronize()
    assert int(st.max()) == 0
    grp = EccGroup(ECC_REED_SOLOMON, 512, 3, devices=(0, 0))
    with pytest.raises(ValueError):
        grp.decode_host(hr, hd, hs[:-1])
    grp.close()
    eng.close()


def test_vote3_rejects_bad_sizes():
    a = np.zeros(49 * 3 + 5, np.uint8)
    with pytest.raises(ValueError):  # ragged tail
        vote3_host(a, a, a, 49)
    ta = torch.zeros(49 * 4, dtype=torch.uint8, device="cuda")
    out = torch.empty_like(ta)
    with pytest.raises(ValueError):
        vote3(ta, ta[:-1], ta, out, 49)
    with pytest.raises(ValueError):
        vote3(ta, ta, ta, out[:10], 49)
    with pytest.raises(ValueError):
        vote3(ta, ta, ta, out, 49, torch.zeros(3, dtype=torch.int32, device="cuda"))
    dmg = torch.zeros(4, dtype=torch.int32, device="cuda")
    vote3(ta, ta, ta, out, 49, dmg)
    torch.cuda.synchronize()
    assert int(dmg.abs().sum()) == 0


@pytest.mark.parametrize("codec", ["rs512", "ham1024"])
def test_partly_registered_buffer_is_staged(oracle, codec):
    """Only the first half of the codeword image is page-locked: the call must not take the direct
    DMA path over the unlocked half, and its results equal the fully pageable and fully pinned
    ones (and the oracle's for RS)."""
    if codec == "rs512":
        eng = EccEngine(ECC_REED_SOLOMON, 512, 3)
    else:
        eng = EccEngine(ECC_HAMMING, 1024)
    n, k = eng.raw_block_size, eng.data_size
    nb = 70001
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    results = []
    for mode in ("pageable", "half", "full"):
        raw = np.zeros(nb * n, np.uint8)
        if mode == "half":
            half = raw[: (nb // 2) * n]
            with pinned(half, data):
                eng.encode_host(data, raw)
        elif mode == "full":
            with pinned(raw, data):
                eng.encode_host(data, raw)
        else:
            eng.encode_host(data, raw)
        results.append(raw)
    assert np.array_equal(results[0], results[1]) and np.array_equal(results[0], results[2])
    if codec == "rs512":
        assert np.array_equal(results[0], oracle.rs_encode(512, 3, data))
    eng.close()


def test_destroy_right_after_queued_work(oracle):
    """close() immediately after queueing a large encode on the caller's stream: the kernels still
    read the context's tables, so destroy must wait for them (results stay bit-exact)."""
    rng = np.random.default_rng(8)
    for typ, bs, t, poly in ((ECC_REED_SOLOMON, 512, 3, 0), (ECC_REED_SOLOMON, 4096, 16, 0),
                             (ECC_CRC, 4096, 0, (0x9960034C << 1) + 1)):
        eng = EccEngine(typ, bs, t, crc_polynomial_explicit=poly)
        n, k = eng.raw_block_size, eng.data_size
        nb = 1 << 16
        data = rng.integers(0, 256, nb * k, dtype=np.uint8)
        d = torch.from_numpy(data).cuda()
        r = torch.zeros(nb * n, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        for _ in range(4):
            eng.encode(d, r)
        eng.close()  # work still in flight on the current stream
        torch.cuda.synchronize()
        got = r.cpu().numpy()
        if typ == ECC_REED_SOLOMON:
            want = oracle.rs_encode(bs, t, data[: 2048 * k])
        else:
            want = oracle.crc_encode(bs, poly, data[: 2048 * k], raw_old=np.zeros(2048 * n, np.uint8))
        assert np.array_equal(got[: 2048 * n], want)


def test_many_contexts_created_and_destroyed_across_threads(oracle):
    """Contexts whose streams were first used on worker threads (group shards) and destroyed on
    the main thread, interleaved with device work on torch's stream: no fault, same results."""
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, 20000 * 249, dtype=np.uint8)
    want = oracle.rs_encode(512, 3, data)
    for rep in range(6):
        grp = EccGroup(ECC_REED_SOLOMON, 512, 3, devices=(0,) * (2 + rep % 3))
        raw = np.zeros(20000 * 255, np.uint8)
        grp.encode_host(data, raw)
        d = torch.from_numpy(data).cuda()
        r = torch.zeros(20000 * 255, dtype=torch.uint8, device="cuda")
        eng = EccEngine(ECC_REED_SOLOMON, 512, 3)
        eng.encode(d, r)
        grp.close()
        eng.close()
        assert np.array_equal(raw, want)
        assert np.array_equal(r.cpu().numpy(), want)


def test_debug_bounds_checks_positive_control():
    """PPFS_ECC_DEBUG builds (tools/gpu_debug_suite.sh): a deliberately out-of-range row gather is
    reported and skipped by the kernel, so a green debug suite means the checks ran and found
    nothing.  Normal builds have no checks (-1)."""
    from paritypartyfs_amd import _native

    L = _native.lib()
    n = L.ppfs_ecc_debug_selftest()
    if _native.debug_faults() is None:
        assert n == -1
    else:
        assert n >= 1, n


@pytest.mark.parametrize("nb,stride,xor", [(1, 255, False), (5, 255, True), (1 << 16, 255, False),
                                           (4099, 249, True), (1003, 4096, False)])
def test_inject_bytes_matches_index_put(nb, stride, xor):
    """bench.py's fault injection (ppfs_inject_device): one byte per block, set or XOR, equal to
    torch's indexing of the same bytes; positions >= stride leave their block untouched; ragged
    block counts (not a multiple of the kernel's 4 blocks per thread) and an offset (unaligned)
    position array."""
    from paritypartyfs_amd import inject_bytes

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(nb)
    raw = torch.randint(0, 256, (nb * stride,), dtype=torch.uint8, device=dev, generator=g)
    pos_all = torch.randint(0, 256, (nb + 1,), dtype=torch.uint8, device=dev, generator=g)
    pos = pos_all[1:]  # 1-byte offset: the kernel's unaligned path
    val = torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
    want = raw.clone().view(nb, stride)
    p = pos.long()
    keep = p < stride
    rows = torch.arange(nb, device=dev)[keep]
    cols = p[keep]
    want[rows, cols] = (want[rows, cols] ^ val[keep]) if xor else val[keep]
    inject_bytes(raw, stride, pos, val, xor=xor)
    torch.cuda.synchronize()
    assert torch.equal(raw.view(nb, stride), want)
    with pytest.raises(ValueError):
        inject_bytes(raw, stride, pos, val, nblocks=nb + 1)


@pytest.mark.parametrize("xor", [False, True])
def test_inject_bytes_neighbours_share_sectors(xor):
    """Positions at the start or end of every block put the injected bytes of consecutive blocks
    in one 32-byte sector, within a thread's 4 blocks and across threads (the case a whole-sector
    rewrite would have to merge); the image starts 7 bytes past a 32-byte
    boundary.  Only the chosen bytes change, nothing outside the image."""
    from paritypartyfs_amd import inject_bytes

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(77)
    nb, stride = 40001, 255
    base = torch.randint(0, 256, (nb * stride + 64,), dtype=torch.uint8, device=dev, generator=g)
    raw = base[7: 7 + nb * stride]
    edge = torch.tensor([0, 1, 2, 3, 251, 252, 253, 254], dtype=torch.uint8, device=dev)
    pos = edge[torch.randint(0, 8, (nb,), device=dev, generator=g)]
    val = torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
    before = base.clone()
    want = raw.clone().view(nb, stride)
    rows, cols = torch.arange(nb, device=dev), pos.long()
    want[rows, cols] = (want[rows, cols] ^ val) if xor else val
    inject_bytes(raw, stride, pos, val, xor=xor)
    torch.cuda.synchronize()
    assert torch.equal(raw.view(nb, stride), want)
    assert torch.equal(base[:7], before[:7]) and torch.equal(base[7 + nb * stride:], before[7 + nb * stride:])


def test_rs_encode_on_many_concurrent_streams(oracle):
    """The t <= 4 encode hands tiles out from per-stream ticket counters (rs_wg_tk.hpp, api.cpp
    ctr_for): one context encoding on 20 streams at once -- 16 get their own counter sets, the
    rest the static walk -- gives the oracle's codewords on every stream, twice over (the kernels
    leave their sets at zero for the next launch)."""
    bs, t, nb = 512, 3, 64 * 1536 + 7  # several tiles per workgroup, a ragged tail
    n, k, _ = oracle.rs_sizes(bs, t)
    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    rng = np.random.default_rng(20)
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    want = oracle.rs_encode(bs, t, data)
    d = torch.from_numpy(data).cuda()
    streams = [torch.cuda.Stream() for _ in range(20)]
    outs = [torch.zeros(nb * n, dtype=torch.uint8, device="cuda") for _ in streams]
    torch.cuda.synchronize()
    for _ in range(2):
        for s, o in zip(streams, outs):
            o.zero_()
        torch.cuda.synchronize()
        for s, o in zip(streams, outs):
            eng.encode(d, o, nblocks=nb, stream=s)
        torch.cuda.synchronize()
        for o in outs:
            assert np.array_equal(o.cpu().numpy(), want)
    eng.close()


@pytest.mark.gpu
def test_rs_decode_on_many_concurrent_streams(oracle):
    """The t <= 4 decode takes its tiles from the second half of the stream's ticket set
    (rs_wg_tk.hpp rs_wg_decode_tk_kernel): 20 streams decoding one context's batches at once, one
    byte error in every codeword, give the payloads, status 1 and the repaired codewords on every
    stream, twice over."""
    bs, t, nb = 512, 3, 64 * 1536 + 7
    n, k, _ = oracle.rs_sizes(bs, t)
    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    rng = np.random.default_rng(21)
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    clean = oracle.rs_encode(bs, t, data)
    cw = clean.reshape(nb, n).copy()
    cw[np.arange(nb), rng.integers(0, n, nb)] ^= rng.integers(1, 256, nb).astype(np.uint8)
    bad = torch.from_numpy(cw.reshape(-1)).cuda()
    streams = [torch.cuda.Stream() for _ in range(20)]
    raws = [torch.empty_like(bad) for _ in streams]
    outs = [torch.empty(nb * k, dtype=torch.uint8, device="cuda") for _ in streams]
    sts = [torch.empty(nb, dtype=torch.uint8, device="cuda") for _ in streams]
    for _ in range(2):
        for r, o, st in zip(raws, outs, sts):
            r.copy_(bad)
            o.zero_()
            st.zero_()
        torch.cuda.synchronize()
        for s, r, o, st in zip(streams, raws, outs, sts):
            eng.decode(r, o, st, write_back=True, nblocks=nb, stream=s)
        torch.cuda.synchronize()
        for r, o, st in zip(raws, outs, sts):
            assert np.array_equal(o.cpu().numpy(), data)
            assert int(st.min()) == 1 and int(st.max()) == 1
            assert np.array_equal(r.cpu().numpy(), clean)
    eng.close()
