"""Batched UDP I/O (rfec_udp_*, razor_amd/csrc/rfec_net.c) and the host
receive path (rfec_host_recv_datagrams).

CPU (loopback sockets, no GPU): datagram slots sent with sendmmsg arrive byte
for byte in order through recvmmsg; the reference's rules hold -- zero-length
slots are not sent (sim_session.c:287-288), datagrams shorter than
SIM_HEADER_SIZE are ignored (:339), at most 1500 bytes are read per datagram
(:333, the excess truncated), and the counters match (:291-292, :343-344).

GPU: a lossy, reordered datagram stream of the product sender goes over
loopback UDP into a pinned slot block and through rfec_host_recv_datagrams;
the parse records and the recovered segments equal the oracle's on exactly the
datagrams that arrived.
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np
import pytest

from razor_amd.fec import RFEC_UDP_SERVER, UDP_ADDR_DTYPE, RfecError, rfec_udp_stats


@pytest.fixture()
def pair(product):
    lib = product
    rx, rx_addr = lib.udp_open("127.0.0.1", 0, RFEC_UDP_SERVER, 4 << 20)
    tx, tx_addr = lib.udp_open("127.0.0.1", 0, RFEC_UDP_SERVER, 4 << 20)
    yield lib, rx, rx_addr, tx, tx_addr
    lib.udp_close(rx)
    lib.udp_close(tx)


def _slots(lens, dstride, rng):
    dg = np.zeros((len(lens), dstride), np.uint8)
    for i, n in enumerate(lens):
        dg[i, :n] = rng.integers(0, 256, n, dtype=np.uint8)
    return dg, np.asarray(lens, np.uint16)


def _recv_all(lib, fd, want, dstride, stats, src=None, max_idle=20):
    out = np.zeros((max(want, 1), dstride), np.uint8)
    ln = np.zeros(max(want, 1), np.uint16)
    got, idle = 0, 0
    while got < want and idle < max_idle:
        part_src = None if src is None else src[got:]
        n = lib.udp_recv(fd, want - got, dstride, out[got:].ctypes.data, ln[got:].ctypes.data, 50, stats, part_src)
        got += n
        idle = idle + 1 if n == 0 else 0
    return out[:got], ln[:got]


def test_udp_open_and_addr(product):
    fd, a = product.udp_open("127.0.0.1", 0)
    try:
        assert fd >= 0 and a.port != 0 and a.ip == 0x7F000001
    finally:
        product.udp_close(fd)
    b = product.udp_addr("10.1.2.3", 16001)
    assert b.ip == 0x0A010203 and b.port == 16001
    with pytest.raises(RfecError):
        product.udp_addr("not-an-ip", 1)
    with pytest.raises(RfecError):
        product.udp_open("300.1.1.1", 0)


def test_udp_round_trip_rules(pair):
    lib, rx, rx_addr, tx, tx_addr = pair
    rng = np.random.default_rng(3)
    dstride = 1504
    # ordinary datagrams, zero-length slots (not sent), too-short ones (sent, ignored by the receiver)
    lens = list(rng.integers(6, 1500, 300))
    for i in (0, 17, 150, 299):
        lens[i] = 0
    for i in (5, 42, 200):
        lens[i] = int(rng.integers(1, 6))
    lens[7], lens[8] = 6, 1500
    dg, dl = _slots(lens, dstride, rng)
    st_tx, st_rx = rfec_udp_stats(), rfec_udp_stats()
    rc, done = lib.udp_send(tx, rx_addr, len(dl), dstride, dg.ctypes.data, dl.ctypes.data, 100, st_tx)
    assert rc == 0 and done == len(dl)
    sent = dl > 0
    assert st_tx.datagrams == sent.sum() and st_tx.skipped == (~sent).sum()
    assert st_tx.bytes == int(dl.astype(np.int64).sum())
    kept = dl >= 6
    src = np.zeros(kept.sum(), UDP_ADDR_DTYPE)
    got, gl = _recv_all(lib, rx, int(kept.sum()), dstride, st_rx, src)
    assert len(gl) == kept.sum()
    assert np.array_equal(gl, dl[kept])
    for i, j in enumerate(np.nonzero(kept)[0]):
        assert np.array_equal(got[i, :gl[i]], dg[j, :dl[j]])
    assert st_rx.datagrams == kept.sum() and st_rx.dropped == (sent & ~kept).sum()
    assert st_rx.bytes == int(dl[kept].astype(np.int64).sum()) and st_rx.truncated == 0
    assert (src["ip"] == 0x7F000001).all() and (src["port"] == tx_addr.port).all()


def test_udp_truncation_and_quiet_wait(pair):
    lib, rx, rx_addr, tx, _ = pair
    rng = np.random.default_rng(4)
    st = rfec_udp_stats()
    # nothing queued: a quiet wait returns 0 datagrams
    buf = np.zeros((4, 512), np.uint8)
    ln = np.zeros(4, np.uint16)
    assert lib.udp_recv(rx, 4, 512, buf.ctypes.data, ln.ctypes.data, 5, st) == 0
    # a 600-byte datagram into 512-byte slots, and a 1600-byte one into 2048-byte slots:
    # at most min(dstride, 1500) bytes are read (the session's 1500-byte buffer)
    for dstride, n in ((512, 600), (2048, 1600)):
        dg, dl = _slots([n], 2048, rng)
        assert lib.udp_send(tx, rx_addr, 1, 2048, dg.ctypes.data, dl.ctypes.data)[0] == 0
        got, gl = _recv_all(lib, rx, 1, dstride, st)
        cap = min(dstride, 1500)
        assert gl[0] == cap and np.array_equal(got[0, :cap], dg[0, :cap])
    assert st.truncated == 2


def test_udp_bad_arguments(pair):
    lib, rx, rx_addr, tx, _ = pair
    dg = np.zeros((2, 64), np.uint8)
    dl = np.array([10, 65], np.uint16)  # longer than the slot
    with pytest.raises(RfecError):
        lib.udp_send(tx, rx_addr, 2, 64, dg.ctypes.data, dl.ctypes.data)
    with pytest.raises(RfecError):
        lib.udp_send(tx, rx_addr, 2, 0, dg.ctypes.data, dl.ctypes.data)


def test_udp_many_chunks(pair):
    """More than one sendmmsg / recvmmsg batch (1024 messages each), receiver draining concurrently."""
    lib, rx, rx_addr, tx, _ = pair
    rng = np.random.default_rng(5)
    dstride, n = 256, 5000
    lens = rng.integers(6, 256, n)
    dg, dl = _slots(lens, dstride, rng)
    st_tx, st_rx = rfec_udp_stats(), rfec_udp_stats()
    res = {}

    def send():
        off = 0
        while off < n:  # paced in chunks so the loopback receive queue does not overflow
            m = min(512, n - off)
            rc, done = lib.udp_send(tx, rx_addr, m, dstride, dg[off:].ctypes.data, dl[off:].ctypes.data, 100, st_tx)
            off += done
        res["sent"] = off

    t = threading.Thread(target=send)
    t.start()
    got, gl = _recv_all(lib, rx, n, dstride, st_rx)
    t.join()
    assert res["sent"] == n and st_tx.datagrams == n and st_tx.syscalls >= n // 1024
    # loopback may drop under pressure; what arrives is an in-order subsequence, byte-exact
    assert len(gl) >= n // 2
    j = 0
    for i in range(len(gl)):
        while j < n and not (dl[j] == gl[i] and np.array_equal(dg[j, :dl[j]], got[i, :gl[i]])):
            j += 1
        assert j < n, "received datagram not found in send order"
        j += 1


# ---------------------------------------------------------------------------
# GPU: UDP -> pinned slots -> parse -> receiver ingestion
# ---------------------------------------------------------------------------
@pytest.mark.gpu
def test_udp_stream_into_receiver(oracle1000):
    import torch

    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")
    from razor_amd.fec import WIRE_REC_DTYPE, native
    from test_receiver import DSTRIDE, STRIDE, _network, _sender_stream

    lib = native(1000)
    order, (sdg, sdl, fdg, fdl), _ = _sender_stream(lib, 800, 21)
    arrivals = _network(order, np.random.default_rng(8), loss=0.1, window=30, dup=0.03)
    n = len(arrivals)
    dg = np.zeros((n, DSTRIDE), np.uint8)
    dl = np.zeros(n, np.uint16)
    for a, (kind, i) in enumerate(arrivals):
        src, ln = (sdg, sdl) if kind == 0 else (fdg, fdl)
        dg[a], dl[a] = src[i], ln[i]
    rx, rx_addr = lib.udp_open("127.0.0.1", 0, RFEC_UDP_SERVER, 8 << 20)
    tx, _ = lib.udp_open("127.0.0.1", 0, RFEC_UDP_SERVER, 8 << 20)
    pin = lib.lib.rfec_pinned_alloc(n * DSTRIDE + n * 2 + 64)
    assert pin
    try:
        slots = np.ctypeslib.as_array((C.c_uint8 * (n * DSTRIDE)).from_address(pin)).reshape(n, DSTRIDE)
        lens = np.ctypeslib.as_array((C.c_uint16 * n).from_address(pin + n * DSTRIDE))

        def send():
            off = 0
            while off < n:
                m = min(256, n - off)
                off += lib.udp_send(tx, rx_addr, m, DSTRIDE, dg[off:].ctypes.data, dl[off:].ctypes.data, 100)[1]

        t = threading.Thread(target=send)
        t.start()
        got, idle = 0, 0
        while got < n and idle < 20:
            k = lib.udp_recv(rx, n - got, DSTRIDE, slots[got:].ctypes.data, lens[got:].ctypes.data, 50)
            got += k
            idle = idle + 1 if k == 0 else 0
        t.join()
        assert got >= n // 2
        out, outp, mts, rep, recs = lib.host_recv_datagrams(got, DSTRIDE, slots.ctypes.data, lens.ctypes.data,
                                                            STRIDE, 1000, 0, 1 << 15, want_recs=True)
        h_dg, h_dl = slots[:got].copy(), lens[:got].copy()
    finally:
        lib.lib.rfec_pinned_free(pin)
        lib.udp_close(rx)
        lib.udp_close(tx)
    erecs, epay = oracle1000.parse_batch(h_dg, h_dl, STRIDE, 1000)
    assert np.array_equal(recs.view(np.uint8), np.asarray(erecs).view(np.uint8).reshape(recs.view(np.uint8).shape))
    assert (recs["status"] == 0).all()
    eo, eop, emts, edrop = oracle1000.rx_recover(recs.view(WIRE_REC_DTYPE), epay, 1000, max_out=1 << 15)
    idx = np.argsort(eo["hdr"]["seq"], kind="stable")
    assert len(out) == len(eo) and len(out) > 0
    assert np.array_equal(out["hdr"], eo["hdr"][idx]) and np.array_equal(outp, eop[idx])
    assert mts == emts and rep.n_fec_dropped == edrop and rep.n_unmodelled == 0
