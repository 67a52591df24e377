"""GPU tests of context lifetime and launch-path bookkeeping (round 3):

- ppfs_ecc_destroy waits for the work its context queued and for nothing else: destroying context A
  while context B's resident server is busy serving per-block calls takes milliseconds, not B's
  server lifetime, and B keeps answering correctly (api.cpp note_caller_stream / ppfs_ecc_destroy);
- a hipGraph captured from encode + decode uses the static-walk kernels, never a stream's
  ticket-counter set, so replays of two such graphs on two streams at once, and a replay beside
  eager work on the capture's stream, stay bit-exact (api.cpp ctr_for);
- ticket-counter slots pass to a 17th stream once an earlier slot's work is complete, and a stream
  created at a destroyed stream's address is ordered after its work (round 4);
- work on the default stream is waited for by destroy;
- every range registered through ppfs_ecc_host_register is released by `pinned` (the registry the
  conftest guard checks after every GPU test);
- the PPFS_ECC_DEBUG build's copy checks refuse a pageable source (positive control).
"""
import threading
import time

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch

from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine, _native, pinned

STATIC = "rs255-wg-seg4-lds"


def _rs_batch(oracle, nb, seed, bs=512, t=3):
    n, k, _ = oracle.rs_sizes(bs, t)
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    return n, k, data, oracle.rs_encode(bs, t, data)


@pytest.mark.timeout(90)
def test_destroy_does_not_wait_for_another_contexts_server(oracle):
    """B serves one-block decodes from its resident launch in a loop (relaunched every <= 20 ms); A is
    created, queues a batch on a caller stream and is destroyed: A's destroy waits for A's batch
    only, and A's creation and copies are not held behind B's launch for long (the server lifetime
    bounds how long a stream sharing its hardware queue waits)."""
    n, k, data, cw = _rs_batch(oracle, 64, 31)
    B = EccEngine(ECC_REED_SOLOMON, 512, 3)
    stop = threading.Event()
    errors, calls = [], [0]

    def serve():
        raw = cw[:n].copy()
        out = np.empty(k, np.uint8)
        st = np.empty(1, np.uint8)
        try:
            while not stop.is_set():
                bad = raw.copy()
                bad[calls[0] % n] ^= 0x41
                B.decode_host(bad, out, st, write_back=True)
                if not (np.array_equal(out, data[:k]) and st[0] == 1 and np.array_equal(bad, raw)):
                    errors.append(calls[0])
                calls[0] += 1
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(repr(e))

    # The main thread never synchronizes the device while B serves: a device-wide wait can starve as
    # long as B keeps relaunching its server (hipDeviceSynchronize waits for the device to go idle).
    nb = 1 << 16
    _, _, adata, acw = _rs_batch(oracle, nb, 32)
    ms = torch.cuda.Stream()
    with torch.cuda.stream(ms):
        d = torch.from_numpy(adata).cuda()
        r = torch.zeros(nb * n, dtype=torch.uint8, device="cuda")
    ms.synchronize()
    hdata = adata[: 200 * k].copy()
    hraw = np.zeros(200 * n, np.uint8)
    times = []
    th = threading.Thread(target=serve)
    th.start()
    try:
        time.sleep(0.2)  # B's server is resident and busy
        t_end = time.perf_counter() + 20.0
        for _ in range(5):
            if time.perf_counter() > t_end:  # a hang here would be the bug under test: fail, do not wait
                break
            A = EccEngine(ECC_REED_SOLOMON, 512, 3)
            A.encode_host(hdata, hraw)  # A's own streams and staging (chunked host path)
            assert np.array_equal(hraw, acw[: 200 * n])
            A.encode(d, r, stream=ms)  # queued on a caller stream
            t0 = time.perf_counter()
            A.close()
            times.append(time.perf_counter() - t0)
            ms.synchronize()
            with torch.cuda.stream(ms):
                got = r.cpu().numpy()
                r.zero_()
            assert np.array_equal(got, acw)  # A's work finished before its tables went away
        time.sleep(0.1)
    finally:
        stop.set()
        th.join(60)
    assert len(times) == 5, times
    assert not errors, errors[:5]
    assert calls[0] > 100, calls[0]  # B kept serving throughout
    # a device-wide synchronize -- hipDeviceSynchronize, or a hipFree / hipHostFree, which wait for
    # every stream of the device -- would wait for B's resident launches, which B relaunches back to
    # back while it serves (each up to SRV_LIFETIME_US = 20 ms): the device is never idle
    assert max(times) < 0.25, times
    B.close()


def test_destroy_waits_for_work_on_every_caller_stream(oracle):
    """Work queued on several caller streams, then destroy at once: every batch is complete and
    bit-exact afterwards (each stream's completion event was waited for)."""
    nb = 1 << 15
    n, k, data, cw = _rs_batch(oracle, nb, 33)
    d = torch.from_numpy(data).cuda()
    streams = [torch.cuda.Stream() for _ in range(5)]
    outs = [torch.zeros(nb * n, dtype=torch.uint8, device="cuda") for _ in streams]
    torch.cuda.synchronize()
    eng = EccEngine(ECC_REED_SOLOMON, 512, 3)
    for s, o in zip(streams, outs):
        for _ in range(3):
            eng.encode(d, o, stream=s)
    eng.close()
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(o.cpu().numpy(), cw)


def _capture(eng, data, cw, out, st, nb, static=STATIC):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        assert eng.stream_kernel_name() == static  # no ticket set inside a capture
        eng.encode(data, cw, nblocks=nb)
        eng.decode(cw, out, st, write_back=True, nblocks=nb)
    return g


@pytest.mark.parametrize("bs,t,kname,static", [(512, 3, "rs255-wg-tk-lds", STATIC),
                                               (4096, 16, "rs255-bs-byte-lds", "rs255-bs-byte-lds-static")], ids=["t3", "t16"])
def test_graph_replays_on_two_streams_at_once(oracle, bs, t, kname, static):
    """Two graphs of encode + decode (each its own buffers) replayed concurrently on two streams,
    and one replayed beside eager launches on its capture's stream: bit-exact every time.  With the
    capture stream's ticket set baked into the graphs, the concurrent replays would share counters
    and skip or repeat tiles.  t = 16: the byte-slice kernels' per-wave tickets (round 5) take the
    static walk inside a capture the same way, reported as "rs255-bs-byte-lds-static"."""
    nb = (1 << 18) + 5
    n, k, data, cw = _rs_batch(oracle, nb, 34, bs, t)
    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    assert eng.kernel_name == kname
    d = torch.from_numpy(data).cuda()
    bufs = [(torch.zeros(nb * n, dtype=torch.uint8, device="cuda"), torch.zeros(nb * k, dtype=torch.uint8, device="cuda"),
             torch.zeros(nb, dtype=torch.uint8, device="cuda")) for _ in range(3)]
    eng.encode(d, bufs[0][0], nblocks=nb)  # eager first: loads the kernels
    torch.cuda.synchronize()
    graphs = [_capture(eng, d, c, o, s, nb, static) for c, o, s in bufs[:2]]
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    want_cw = torch.from_numpy(cw).cuda()
    for _ in range(3):
        for c, o, s in bufs:
            c.zero_(), o.zero_(), s.fill_(9)
        torch.cuda.synchronize()
        with torch.cuda.stream(sa):
            graphs[0].replay()
        with torch.cuda.stream(sb):
            graphs[1].replay()
            eng.encode(d, bufs[2][0], nblocks=nb)  # eager beside the replays (ticket kernels)
            eng.decode(bufs[2][0], bufs[2][1], bufs[2][2], write_back=True, nblocks=nb)
        torch.cuda.synchronize()
        for c, o, s in bufs:
            assert torch.equal(c, want_cw)
            assert torch.equal(o, d)
            assert int(s.max()) == 0
    assert eng.stream_kernel_name() == kname  # outside a capture: ticket kernels again
    del graphs
    eng.close()


def test_stream_slots_are_recycled_past_16_streams(oracle):
    """16 ticket-counter slots: a 17th..20th stream takes a slot whose last user's work has completed
    (round 4; it used to fall back to the static walk for good), and every stream's codewords stay
    bit-exact; during capture the static walk runs."""
    nb = 3 * 64 * 7 + 13
    n, k, data, cw = _rs_batch(oracle, nb, 35)
    eng = EccEngine(ECC_REED_SOLOMON, 512, 3)
    d = torch.from_numpy(data).cuda()
    streams = [torch.cuda.Stream() for _ in range(20)]
    outs = [torch.zeros(nb * n, dtype=torch.uint8, device="cuda") for _ in streams]
    for s, o in zip(streams[:16], outs[:16]):
        assert eng.stream_kernel_name(s) == "rs255-wg-tk-lds"
        eng.encode(d, o, stream=s)
    torch.cuda.synchronize()
    for s, o in zip(streams[16:], outs[16:]):  # every earlier slot's work is complete: recycled
        assert eng.stream_kernel_name(s) == "rs255-wg-tk-lds"
        eng.encode(d, o, stream=s)
        eng.decode(o, None, None, write_back=False, stream=s)
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(o.cpu().numpy(), cw)
    for o in outs[:4]:
        o.zero_()
    torch.cuda.synchronize()  # the zeroing (current stream) before the encodes on the other streams
    for s, o in zip(streams[:4], outs[:4]):  # back on the first streams, after their slots moved on
        eng.encode(d, o, stream=s)
    torch.cuda.synchronize()
    for o in outs[:4]:
        assert np.array_equal(o.cpu().numpy(), cw)
    eng.close()
    hm = EccEngine(ECC_REED_SOLOMON, 4096, 16)  # a fresh context: the stream gets a free counter set
    assert hm.stream_kernel_name(streams[16]) == hm.kernel_name == "rs255-bs-byte-lds"
    hm.close()


def _hip():
    import ctypes
    L = ctypes.CDLL("libamdhip64.so")  # the runtime torch loaded (the engine's too)
    return ctypes, L


def test_recycled_stream_handle_never_shares_a_live_ticket_set(oracle):
    """A stream destroyed with a large encode still in flight, then streams created until one comes
    back at the destroyed stream's address (the runtime reuses the object's memory): the launch on
    the new stream is ordered after the old stream's work (api.cpp order_caller_stream) instead of
    counting on the same ticket set beside it.  Both outputs are bit-exact."""
    ct, L = _hip()
    big = 1 << 20
    n, k, data, cw = _rs_batch(oracle, big, 36)
    d = torch.from_numpy(data).cuda()
    eng = EccEngine(ECC_REED_SOLOMON, 512, 3)
    small_nb = 64 * 40 + 7
    torch.cuda.synchronize()
    hit = 0
    for trial in range(4):
        out_a = torch.zeros(big * n, dtype=torch.uint8, device="cuda")
        out_b = torch.zeros(small_nb * n, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        sa = ct.c_void_p()
        assert L.hipStreamCreateWithFlags(ct.byref(sa), ct.c_uint(1)) == 0  # non-blocking
        for _ in range(3):
            eng.encode(d, out_a, nblocks=big, stream=sa.value)
        assert L.hipStreamDestroy(sa) == 0  # returns with the encodes in flight
        made, sb = [], None
        for _ in range(64):
            s = ct.c_void_p()
            assert L.hipStreamCreateWithFlags(ct.byref(s), ct.c_uint(1)) == 0
            if s.value == sa.value:
                sb = s
                break
            made.append(s)
        if sb is not None:
            hit += 1
            eng.encode(d, out_b, nblocks=small_nb, stream=sb.value)
            assert L.hipStreamSynchronize(sb) == 0
            assert L.hipStreamDestroy(sb) == 0
        for s in made:
            assert L.hipStreamDestroy(s) == 0
        torch.cuda.synchronize()
        assert np.array_equal(out_a.cpu().numpy(), cw)
        if sb is not None:
            assert np.array_equal(out_b.cpu().numpy(), cw[: small_nb * n])
    eng.close()
    if not hit:
        pytest.skip("the runtime never reused a destroyed stream's handle")


def test_default_stream_work_outlives_nothing_at_close(oracle):
    """Encode and decode queued on the default (null) stream, then close at once: destroy waits for
    that work (its completion event is recorded although the context's own host streams do not exist
    yet), so the outputs are complete and the freed tables were not read afterwards."""
    nb = (1 << 19) + 3
    n, k, data, cw = _rs_batch(oracle, nb, 37)
    d = torch.from_numpy(data).cuda()
    for _ in range(3):
        eng = EccEngine(ECC_REED_SOLOMON, 512, 3)
        r = torch.zeros(nb * n, dtype=torch.uint8, device="cuda")
        o = torch.zeros(nb * k, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        eng.encode(d, r, nblocks=nb, stream=0)
        eng.decode(r, o, None, write_back=False, nblocks=nb, stream=0)
        eng.close()
        torch.cuda.synchronize()
        assert np.array_equal(r.cpu().numpy(), cw)
        assert torch.equal(o, d)


def test_pinned_releases_every_registered_range():
    base = _native.host_registered()
    base = base[0] if base else 0
    a = np.zeros(1 << 20, np.uint8)
    b = np.zeros(3 << 20, np.uint8)
    with pinned(a, b):
        cnt, nbytes = _native.host_registered()
        assert cnt == base + 2 and nbytes >= a.nbytes + b.nbytes
    assert _native.host_registered()[0] == base


def test_debug_copy_checks_positive_control():
    """PPFS_ECC_DEBUG builds refuse a copy from pageable memory and one past a device allocation;
    normal builds have no checks (-1)."""
    L = _native.lib()
    v = L.ppfs_ecc_debug_dma_selftest()
    if _native.debug_faults() is None:
        assert v == -1 and _native.debug_dma_rejects() is None
    else:
        assert v == 1, v


@pytest.mark.parametrize("bs,t", [(512, 3), (4096, 16), (4096, 0)], ids=["rs_t3", "rs_t16", "hamming4096"])
def test_time_next_launch_records_the_kernel(bs, t):
    """ppfs_ecc_time_next_launch: the next engine kernel records both events from its dispatch
    packet (a positive duration no longer than the stream-event bracket around the call), the hook
    disarms after one launch, and the launch it timed computes the same codewords as an untimed one."""
    from bench import HipEvents
    from paritypartyfs_amd import ECC_HAMMING

    typ = ECC_REED_SOLOMON if t else ECC_HAMMING
    eng = EccEngine(typ, bs, t)
    n, k, nb = eng.raw_block_size, eng.data_size, 1 << 15
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev)
    ref = torch.zeros(nb * n, dtype=torch.uint8, device=dev)
    cw = torch.zeros_like(ref)
    eng.encode(data, ref, nblocks=nb)
    L = _native.lib()
    ev = HipEvents(4)
    ev.record(0, stream)
    assert L.ppfs_ecc_time_next_launch(ev.ev[2], ev.ev[3]) == 0
    eng.encode(data, cw, nblocks=nb)
    ev.record(1, stream)
    torch.cuda.synchronize()
    kernel_ms, bracket_ms = ev.ms(2, 3), ev.ms(0, 1)
    assert 0.0 < kernel_ms <= bracket_ms + 1e-3
    assert torch.equal(cw, ref)
    # disarmed: a second launch records nothing new (the stop event keeps its timestamp; reading the
    # same pair again may differ in the last nanosecond of the tick -> ms conversion, a new launch's
    # duration by far more)
    eng.encode(data, cw, nblocks=nb)
    torch.cuda.synchronize()
    assert abs(ev.ms(2, 3) - kernel_ms) < 1e-5
    ev.close()
    eng.close()
