"""Receiver ingestion on the GPU (rfec_rx_recover): parsed datagrams in
arrival order -> the segments the reference receiver recovers.

  * the reference's own receiver on scripted lossy / reordered / duplicated
    streams (tests/golden/rx.json, oracle/gen_rx.c over sim_fec.c);
  * the event-by-event oracle (oracle_rx_recover, pinned by the same
    fixtures) on larger streams the product sender emits, parsed by the
    device wire codec, with loss, reordering, duplicates and parities late
    enough for the 3000 ms rule;
  * edge cases: empty batch, undecodable records only, output too small.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import pyoracle as po
import rx_cases as rc

pytestmark = pytest.mark.gpu

UID = 0x0BADF00D
DSTRIDE = 1056
STRIDE = 1008


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")
    from razor_amd.fec import native
    return native(1000)


def _dev(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).cuda()


def _rx(lib, recs, pay, max_ts=0, max_out=1 << 16):
    dr, dp = _dev(recs), _dev(pay)
    torch.cuda.synchronize()
    return lib.rx_recover(len(recs), dr.data_ptr(), dp.data_ptr(), pay.shape[1], 1000, max_ts, max_out)


def _sorted(rows):
    return sorted(rows, key=lambda r: r[0])


@pytest.mark.parametrize("name", ["k10_loss10", "k10_loss25_dup", "mixed_loss15", "late_parities",
                                  "peer_large_groups", "peer_huge_groups"])  # (flexes of 130-200 and 300-1,000 segments: line jobs)
def test_rx_reference_fixture(lib, oracle1000, name):
    scn = {s["name"]: s for s in po.rx_fixture()["scenarios"]}[name]
    recs, pay, _, _ = po.rx_stream(oracle1000, scn)
    out, outp, max_ts, rep = _rx(lib, recs, pay)
    assert _sorted(rc.got_rows(out, outp)) == _sorted(rc.expected(scn))
    assert [int(s) for s in out["hdr"]["seq"]] == sorted(int(s) for s in out["hdr"]["seq"])
    assert max_ts == scn["max_ts"]
    _, _, _, dropped = oracle1000.rx_recover(recs, pay, 1000)
    assert rep.n_fec_dropped == dropped and rep.n_unmodelled == 0
    assert rep.n_recovered == len(scn["recovered"])


def _sender_stream(lib, frames_n, seed, k_choices=(10,), pf=(80,)):
    """Datagrams of the product sender in send order: each segment, and a
    group's parities right after the segment that closes it."""
    rng = np.random.default_rng(seed)
    sizes = rng.choice(k_choices, frames_n) * 1000 - rng.integers(0, 900, frames_n)
    blob = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8)
    frames = np.zeros(frames_n, po.FRAME)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    frames["data"] = blob.ctypes.data + offs.astype(np.uint64)
    frames["size"] = sizes
    frames["payload_type"] = 96
    frames["ftype"] = np.arange(frames_n) % 50 == 0
    frames["protect_fraction"] = rng.choice(pf, frames_n)
    frames["now_ms"] = 1_700_000_000_000 + np.arange(frames_n) * 33
    st = lib.sender_init()
    segs, groups, sdg, sdl, fdg, fdl, rep = lib.send_frames(st, frames, UID, DSTRIDE, max_segs=frames_n * 12 + 64,
                                                            max_groups=frames_n + 64, max_parities=frames_n * 16 + 64)
    closes = {}
    p = 0
    for g in groups:
        nl = int(g["n_lines"])
        if int(g["first_seg"]) >= 0:
            closes[int(g["first_seg"]) + int(g["count"]) - 1] = (p, nl)
        p += nl
    order = []
    for i in range(len(segs)):
        order.append((0, i))
        if i in closes:
            p0, nl = closes[i]
            order.extend((1, p0 + l) for l in range(nl))
    return order, (sdg, sdl, fdg, fdl), blob


def _network(order, rng, loss=0.12, window=40, dup=0.04, late=0.0, late_by=4000):
    keys = []
    for pos, item in enumerate(order):
        if rng.random() < loss:
            continue
        key = pos + rng.integers(0, window)
        if item[0] == 1 and rng.random() < late:
            key += late_by
        keys.append((key, pos, item))
        if rng.random() < dup:
            keys.append((key + rng.integers(1, 3 * window), pos, item))
    keys.sort(key=lambda t: (t[0], t[1]))
    return [t[2] for t in keys]


def _arrivals(lib, arrivals, dg):
    sdg, sdl, fdg, fdl = dg
    n = len(arrivals)
    dgram = np.zeros((n, DSTRIDE), np.uint8)
    dlen = np.zeros(n, np.uint16)
    for a, (kind, i) in enumerate(arrivals):
        src, ln = (sdg, sdl) if kind == 0 else (fdg, fdl)
        dgram[a], dlen[a] = src[i], ln[i]
    from razor_amd.fec import WIRE_REC_DTYPE
    d_dg, d_dl = _dev(dgram), _dev(dlen)
    recs = torch.zeros(n * WIRE_REC_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    pay = torch.zeros(n * STRIDE, dtype=torch.uint8, device="cuda")
    lib.wire_parse(n, DSTRIDE, d_dg.data_ptr(), d_dl.data_ptr(), STRIDE, 1000, recs.data_ptr(), pay.data_ptr())
    torch.cuda.synchronize()
    return recs, pay


@pytest.mark.parametrize("case", ["k10", "mixed", "late", "heavy"])
def test_rx_sender_stream_vs_oracle(lib, oracle1000, case):
    cfg = {"k10": dict(frames=3000, k=(10,), pf=(80,), net=dict()),
           "mixed": dict(frames=2000, k=(1, 3, 10, 24), pf=(20, 50, 80, 100), net=dict(loss=0.15, window=80)),
           "late": dict(frames=1500, k=(10,), pf=(80,), net=dict(loss=0.1, late=0.25, late_by=1600)),
           "heavy": dict(frames=800, k=(6, 10), pf=(100,), net=dict(loss=0.35, window=200, dup=0.2))}[case]
    rng = np.random.default_rng({"k10": 1, "mixed": 2, "late": 3, "heavy": 4}[case])
    order, dg, _ = _sender_stream(lib, cfg["frames"], 7, cfg["k"], cfg["pf"])
    arrivals = _network(order, rng, **cfg["net"])
    recs, pay = _arrivals(lib, arrivals, dg)
    from razor_amd.fec import WIRE_REC_DTYPE
    h_recs = recs.cpu().numpy().view(WIRE_REC_DTYPE)
    h_pay = pay.cpu().numpy().reshape(-1, STRIDE)
    assert (h_recs["status"] == 0).all()
    eo, eop, emts, edrop = oracle1000.rx_recover(h_recs, h_pay, 1000, max_out=1 << 17)
    out, outp, mts, rep = lib.rx_recover(len(h_recs), recs.data_ptr(), pay.data_ptr(), STRIDE, 1000, 0, 1 << 17)
    idx = np.argsort(eo["hdr"]["seq"], kind="stable")
    assert len(out) == len(eo) and len(out) > 0
    assert np.array_equal(out["hdr"], eo["hdr"][idx]) and np.array_equal(out["fec_id"], eo["fec_id"][idx])
    assert np.array_equal(outp, eop[idx])
    assert mts == emts and rep.n_fec_dropped == edrop and rep.n_unmodelled == 0
    if case == "late":
        assert edrop > 0


def test_rx_continues_across_calls(lib, oracle1000):
    """max_ts carries across batches (sim_receiver_fec_t.max_ts)."""
    order, dg, _ = _sender_stream(lib, 400, 3)
    arrivals = _network(order, np.random.default_rng(5), loss=0.1, window=10, dup=0.0)
    recs, pay = _arrivals(lib, arrivals, dg)
    _, _, m1, _ = lib.rx_recover(len(arrivals), recs.data_ptr(), pay.data_ptr(), STRIDE, 1000, 0, 1 << 15)
    assert m1 > 0
    _, _, m2, rep = lib.rx_recover(len(arrivals), recs.data_ptr(), pay.data_ptr(), STRIDE, 1000, m1 + 10_000,
                                   1 << 15)
    assert m2 == m1 + 10_000 and rep.n_fec_dropped > 0  # every parity is now > 3 s old


def test_rx_edges(lib):
    from razor_amd.fec import RfecError, WIRE_REC_DTYPE
    out, outp, mts, rep = lib.rx_recover(0, 0, 0, STRIDE, 1000, 77, 4)
    assert len(out) == 0 and mts == 77
    bad = np.zeros(8, WIRE_REC_DTYPE)
    bad["status"] = -1
    out, _, mts, rep = _rx(lib, bad, np.zeros((8, STRIDE), np.uint8), 5)
    assert len(out) == 0 and mts == 5 and rep.n_groups == 0
    order, dg, _ = _sender_stream(lib, 200, 11)
    arrivals = _network(order, np.random.default_rng(2), loss=0.2, window=4, dup=0.0)
    recs, pay = _arrivals(lib, arrivals, dg)
    out, _, _, _ = lib.rx_recover(len(arrivals), recs.data_ptr(), pay.data_ptr(), STRIDE, 1000, 0, 1 << 14)
    assert len(out) > 1
    with pytest.raises(RfecError):
        lib.rx_recover(len(arrivals), recs.data_ptr(), pay.data_ptr(), STRIDE, 1000, 0, len(out) - 1)
    with pytest.raises(RfecError):
        lib.rx_recover(len(arrivals), recs.data_ptr(), pay.data_ptr(), 1000, 1000, 0, 16)  # stride % 16


# ---------------------------------------------------------------------------
# receiver sessions (rfec_rx_session_*): state kept across batches
# ---------------------------------------------------------------------------
def _rows(out, outp):
    return sorted(rc.got_rows(out, outp), key=lambda r: r[0])


@pytest.mark.parametrize("name", ["k10_loss10", "mixed_loss15", "late_parities", "evict_late_segments",
                                  "evict_lost_parities", "no_evict_late_segments", "peer_large_groups", "peer_huge_groups"])
def test_rx_session_reference_fixture(lib, name):
    """The reference receiver's streams pushed in batches, with sim_fec_evict
    between batches where the scenario's heartbeat ran it: the same recovered
    segments (bytes by FNV-1a), max_ts, and the same open flexes / cached
    segments left as the reference's skiplists."""
    scn = {s["name"]: s for s in po.rx_fixture()["scenarios"]}[name]
    recs, pay, _, _ = po.rx_stream(po.Oracle(1000), scn)
    E = scn["evict_every"]
    sess = lib.rx_session(pay.shape[1], 1000)
    rng = np.random.default_rng(7)
    a, rows = 0, []
    while a < len(recs):
        b = min(len(recs), a + (E if E else int(rng.integers(1, 500))))
        dr, dp = _dev(recs[a:b]), _dev(pay[a:b])
        out, outp, rep = sess.push(b - a, dr.data_ptr(), dp.data_ptr())
        assert rep.n_unmodelled == 0
        rows += rc.got_rows(out, outp)
        if E and b - a == E:
            sess.evict()
        a = b
    assert sorted(rows, key=lambda r: r[0]) == sorted(rc.expected(scn), key=lambda r: r[0])
    info = sess.info()
    assert info["max_ts"] == scn["max_ts"]
    if E:
        assert (info["open_flexes"], info["cached_segments"]) == (scn["flexes_left"], scn["cache_left"])
    sess.close()


@pytest.mark.parametrize("evict_every", [0, 300])
def test_rx_session_split_invariance(lib, oracle1000, evict_every, monkeypatch):
    """A product-sender stream pushed in random batches (evict_every == 0) or
    in batches of evict_every with evictions between: the union of what the
    batches deliver == the oracle on the whole stream with the same evictions
    -- including groups whose datagrams straddle batches.  The arena is the
    smallest (RFEC_RX_ARENA_ROWS=4096), so compactions run (an eviction
    compacts once the session holds half its arena, a push when it needs the
    room) and the session keeps only what the open state refers to."""
    monkeypatch.setenv("RFEC_RX_ARENA_ROWS", "4096")
    order, dg, _ = _sender_stream(lib, 2500, 5, (3, 6, 10), (20, 80, 100))
    arrivals = _network(order, np.random.default_rng(13), loss=0.15, window=60, dup=0.03, late=0.05,
                        late_by=2500)
    recs, pay = _arrivals(lib, arrivals, dg)
    from razor_amd.fec import WIRE_REC_DTYPE
    h_recs = recs.cpu().numpy().view(WIRE_REC_DTYPE)
    h_pay = pay.cpu().numpy().reshape(-1, STRIDE)
    n = len(h_recs)
    eo, eop, emts, edrop = oracle1000.rx_recover(h_recs, h_pay, 1000, max_out=1 << 17, evict_every=evict_every)
    sess = lib.rx_session(STRIDE, 1000)
    rng = np.random.default_rng(evict_every + 1)
    a, got, gotp, dropped = 0, [], [], 0
    recs_u8 = recs.view(-1, WIRE_REC_DTYPE.itemsize)
    pay_u8 = pay.view(-1, STRIDE)
    while a < n:
        b = min(n, a + (evict_every if evict_every else int(rng.integers(1, 3000))))
        out, outp, rep = sess.push(b - a, recs_u8[a:b].data_ptr(), pay_u8[a:b].data_ptr(), max_out=1 << 16)
        got.append(out)
        gotp.append(outp)
        dropped += rep.n_fec_dropped
        assert rep.n_unmodelled == 0
        if evict_every and b - a == evict_every:
            sess.evict()
        a = b
    out, outp = np.concatenate(got), np.concatenate(gotp)
    i, j = np.argsort(out["hdr"]["seq"], kind="stable"), np.argsort(eo["hdr"]["seq"], kind="stable")
    assert len(out) == len(eo) > 0
    assert np.array_equal(out["hdr"][i], eo["hdr"][j]) and np.array_equal(out["fec_id"][i], eo["fec_id"][j])
    assert np.array_equal(outp[i], eop[j])
    assert sess.info()["max_ts"] == emts and dropped == edrop
    if evict_every:
        info = sess.info()
        assert info["records_held"] < n // 2  # compaction keeps only what the open state refers to
    sess.close()


@pytest.mark.parametrize("pinned", [False, True])
def test_rx_session_datagrams(lib, oracle1000, pinned):
    """Datagram slots in host memory -> session (parse, ingestion), in batches.
    Pageable slots are copied to the device first; pinned ones (the UDP batch
    slots) are read by the parse kernel itself, and a pinned payload output is
    gathered into directly."""
    order, (sdg, sdl, fdg, fdl), _ = _sender_stream(lib, 600, 9)
    arrivals = _network(order, np.random.default_rng(4), loss=0.1, window=20, dup=0.02)
    n = len(arrivals)
    keep = []
    if pinned:
        dgram, k1 = lib.pinned_array((n, DSTRIDE), np.uint8)
        dlen, k2 = lib.pinned_array((n,), np.uint16)
        keep += [k1, k2]
        dgram[:] = 0
        dlen[:] = 0
    else:
        dgram = np.zeros((n, DSTRIDE), np.uint8)
        dlen = np.zeros(n, np.uint16)
    for a, (kind, i) in enumerate(arrivals):
        src, ln = (sdg, sdl) if kind == 0 else (fdg, fdl)
        dgram[a], dlen[a] = src[i], ln[i]
    sess = lib.rx_session(STRIDE, 1000)
    got, gotp, recs = [], [], []
    for a in range(0, n, 777):
        b = min(n, a + 777)
        out, outp, rep, r = sess.push_datagrams(b - a, DSTRIDE, dgram[a:].ctypes.data, dlen[a:].ctypes.data,
                                                want_recs=True, max_out=4096, pinned_out=pinned)
        got.append(out)
        gotp.append(outp)
        recs.append(r)
    recs = np.concatenate(recs)
    erecs, epay = oracle1000.parse_batch(dgram, dlen, STRIDE, 1000)
    assert np.array_equal(recs.view(np.uint8), np.asarray(erecs).view(np.uint8).reshape(recs.view(np.uint8).shape))
    eo, eop, emts, _ = oracle1000.rx_recover(erecs, epay, 1000, max_out=1 << 16)
    out, outp = np.concatenate(got), np.concatenate(gotp)
    i, j = np.argsort(out["hdr"]["seq"], kind="stable"), np.argsort(eo["hdr"]["seq"], kind="stable")
    assert len(out) == len(eo) > 0 and np.array_equal(out["hdr"][i], eo["hdr"][j])
    assert np.array_equal(outp[i], eop[j]) and sess.info()["max_ts"] == emts
    sess.close()


@pytest.mark.parametrize("pinned", [False, True])
def test_rx_session_datagrams_async(lib, oracle1000, pinned):
    """The pipelined push (rfec_rx_session_push_datagrams_async): random batch
    sizes, evictions between calls (compaction with a parsed, not ingested
    batch behind the kept rows), then the flush.  Deliveries, records and
    payloads equal the synchronous push over the same batches with each
    eviction at the same point of ingestion; a synchronous push is refused
    while a batch is pending."""
    order, (sdg, sdl, fdg, fdl), _ = _sender_stream(lib, 600, 9)
    arrivals = _network(order, np.random.default_rng(5), loss=0.1, window=20, dup=0.02)
    n = len(arrivals)
    keep = []
    if pinned:
        dgram, k1 = lib.pinned_array((n, DSTRIDE), np.uint8)
        dlen, k2 = lib.pinned_array((n,), np.uint16)
        keep += [k1, k2]
    else:
        dgram = np.zeros((n, DSTRIDE), np.uint8)
        dlen = np.zeros(n, np.uint16)
    for a, (kind, i) in enumerate(arrivals):
        src, ln = (sdg, sdl) if kind == 0 else (fdg, fdl)
        dgram[a], dlen[a] = src[i], ln[i]
    rng = np.random.default_rng(6)
    cuts, a = [], 0
    while a < n:
        b = min(n, a + int(rng.integers(1, 1500)))
        cuts.append((a, b))
        a = b
    evict_after = {j for j in range(len(cuts)) if rng.random() < 0.3}  # evict once batch j is ingested

    def collect(parts):
        out = np.concatenate([p[0] for p in parts])
        outp = np.concatenate([p[1] for p in parts])
        recs = np.concatenate([p[2] for p in parts if p[2] is not None and len(p[2])])
        return out, outp, recs

    # synchronous reference
    sess = lib.rx_session(STRIDE, 1000)
    ref = []
    for j, (a, b) in enumerate(cuts):
        out, outp, rep, r = sess.push_datagrams(b - a, DSTRIDE, dgram[a:].ctypes.data, dlen[a:].ctypes.data,
                                                want_recs=True, max_out=4096)
        ref.append((out, outp, r))
        if j in evict_after:
            sess.evict()
    ref_info = sess.info()
    sess.close()
    # pipelined: call j starts batch j and ingests batch j - 1
    sess = lib.rx_session(STRIDE, 1000)
    got = []
    for j, (a, b) in enumerate(cuts):
        out, outp, rep, r = sess.push_datagrams_async(b - a, DSTRIDE, dgram[a:].ctypes.data, dlen[a:].ctypes.data,
                                                      want_recs=True, max_out=4096, pinned_out=pinned)
        got.append((out, outp, r))
        assert sess.info()["pending"] == b - a and (j == 0 or len(r) == cuts[j - 1][1] - cuts[j - 1][0])
        if j == 0:
            with pytest.raises(Exception):
                sess.push_datagrams(1, DSTRIDE, dgram.ctypes.data, dlen.ctypes.data)
        if j - 1 in evict_after:
            sess.evict()
    out, outp, rep, r = sess.push_datagrams_async(0, DSTRIDE, 0, 0, want_recs=True, max_out=4096,
                                                  pinned_out=pinned)
    got.append((out, outp, r))
    assert sess.info()["pending"] == 0
    if len(cuts) - 1 in evict_after:
        sess.evict()
    eo, eop, erecs = collect(ref)
    go, gop, grecs = collect(got)
    assert len(go) == len(eo) > 0
    assert np.array_equal(go.view(np.uint8), eo.view(np.uint8)) and np.array_equal(gop, eop)
    assert np.array_equal(grecs.view(np.uint8), erecs.view(np.uint8))
    assert sess.info()["max_ts"] == ref_info["max_ts"]
    sess.close()


@pytest.mark.gpu
@pytest.mark.parametrize("long_junk", [False, True])
def test_recv_datagrams_wide_slots(oracle1000, long_junk):
    """rfec_host_recv_datagrams over 1,504-B receive slots: with every datagram
    <= 1,280 B the 20-byte-lane parse runs (the host knows the lengths), with a
    few 1,300-1,500-B junk datagrams the 32-byte-lane one; records, recovered
    segments and payloads equal the oracle either way."""
    import torch

    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")
    from razor_amd.fec import WIRE_REC_DTYPE, native

    W = 1504
    lib = native(1000)
    order, (sdg, sdl, fdg, fdl), _ = _sender_stream(lib, 300, 5)
    arrivals = _network(order, np.random.default_rng(9), loss=0.1, window=20, dup=0.02)
    rng = np.random.default_rng(10)
    rows = []
    for kind, i in arrivals:
        src, ln = (sdg, sdl) if kind == 0 else (fdg, fdl)
        rows.append((src[i][:ln[i]].tobytes()))
    if long_junk:
        for p in rng.choice(len(rows), 5, replace=False):
            rows[p] = rng.integers(0, 256, int(rng.integers(1300, 1501)), dtype=np.uint8).tobytes()
    n = len(rows)
    dg = np.zeros((n, W), np.uint8)
    dl = np.zeros(n, np.uint16)
    for a, b in enumerate(rows):
        dg[a, :len(b)] = np.frombuffer(b, np.uint8)
        dl[a] = len(b)
    out, outp, mts, rep, recs = lib.host_recv_datagrams(n, W, dg.ctypes.data, dl.ctypes.data, STRIDE, 1000, 0,
                                                        1 << 15, want_recs=True)
    erecs, epay = oracle1000.parse_batch(dg, dl, STRIDE, 1000)
    assert np.array_equal(recs.view(np.uint8), np.asarray(erecs).view(np.uint8).reshape(recs.view(np.uint8).shape))
    assert (recs["status"] != 0).sum() == (5 if long_junk else 0)
    eo, eop, emts, edrop = oracle1000.rx_recover(recs.view(WIRE_REC_DTYPE), epay, 1000, max_out=1 << 15)
    idx = np.argsort(eo["hdr"]["seq"], kind="stable")
    assert len(out) == len(eo) and len(out) > 0
    assert np.array_equal(out["hdr"], eo["hdr"][idx]) and np.array_equal(outp, eop[idx])
    assert mts == emts


@pytest.mark.parametrize("seed", [0, 1])
def test_rx_peer_geometry(lib, oracle1000, seed):
    """Groups a peer may send that razor's own sender never does (parities of
    columns c >= col; row * col < count, members past the matrix): the batched
    receiver models them as the reference flex receiver does (it takes row,
    col, count and index straight from the parity, flex_fec_receiver.c:69-88,
    105-206) and delivers exactly the oracle's segments, bytes included;
    nothing is left unmodelled.  Then the same stream pushed into a session in
    random batches."""
    recs, pay = rc.peer_stream(oracle1000, np.random.default_rng(70 + seed))
    out, outp, max_ts, rep = _rx(lib, recs, pay)
    eo, ep, emts, edrop = oracle1000.rx_recover(recs, pay, 1000)
    assert rep.n_unmodelled == 0 and len(eo) > 100
    assert _sorted(rc.got_rows(out, outp)) == _sorted(rc.got_rows(eo, ep))
    assert max_ts == emts
    sess = lib.rx_session(pay.shape[1], 1000)
    rng = np.random.default_rng(seed)
    a, rows = 0, []
    while a < len(recs):
        b = min(len(recs), a + int(rng.integers(1, 400)))
        dr, dp = _dev(recs[a:b]), _dev(pay[a:b])
        torch.cuda.synchronize()
        o, op, r = sess.push(b - a, dr.data_ptr(), dp.data_ptr())
        rows += rc.got_rows(o, op)
        assert r.n_unmodelled == 0
        a = b
    sess.close()
    assert _sorted(rows) == _sorted(rc.got_rows(eo, ep))


@pytest.mark.parametrize("k,row,col", [(128, 64, 2), (128, 2, 64), (100, 50, 2), (96, 3, 32)])
def test_rx_huge_shape_small_count(lib, oracle1000, k, row, col):
    """A peer's flex of at most RFEC_MAX_K segments with more than 64 lines
    (128 = 64 x 2 or 2 x 64: 66 lines) is a huge shape: its recovery runs as
    line jobs, not through the batched peel (whose plans hold 64 lines).
    50 x 2 and 3 x 32 (52 / 35 lines) keep a device plan.  Losses: row 0
    whole, member 3 (its row), member 1 two levels deep where the shape
    allows, scattered singles.  Delivered rows equal the event-by-event
    oracle's, nothing unmodelled."""
    erase = {0, 1, 3, 2 * col + 1, 7 * col, k - 2}
    recs, pay = rc.single_group_stream(oracle1000, k, 80, erase, seed=k + row, shape=(row, col))
    out, outp, _, rep = _rx(lib, recs, pay)
    o_out, o_pay, _, _ = oracle1000.rx_recover(recs, pay, 1000)
    assert rep.n_unmodelled == 0
    assert len(o_out) >= 4
    assert _sorted(rc.got_rows(out, outp)) == _sorted(rc.got_rows(o_out, o_pay))


@pytest.mark.parametrize("k,pf", [(200, 80), (600, 80), (1000, 80)])
def test_rx_large_group_cascades_and_rejection(lib, oracle1000, k, pf):
    """Flexes above RFEC_MAX_K (line jobs; above 255 segments and 64 lines:
    huge shapes, lines by FEC index): a recovery two levels deep (members 0
    and 1 of row 0 lost with member `col` of row 1: row 1 recovers `col`, then
    column 0 recovers 0 -- column 1 recovers 1 directly), a row parity whose
    fec_data_size is cut below a member's size (flex_fec_xor.c:88-89: its
    line is rejected, its lost member comes back through its column), and
    scattered single losses.  Delivered rows equal the event-by-event
    oracle's, nothing unmodelled."""
    _, row, col = oracle1000.num_packets(k, pf)
    erase = {0, 1, col, 2 * col + 3, 5 * col + 7, 9 * col + 1}
    recs, pay = rc.single_group_stream(oracle1000, k, pf, erase, tamper=(2, 1), seed=k)
    out, outp, _, rep = _rx(lib, recs, pay)
    o_out, o_pay, _, _ = oracle1000.rx_recover(recs, pay, 1000)
    assert rep.n_unmodelled == 0
    assert _sorted(rc.got_rows(out, outp)) == _sorted(rc.got_rows(o_out, o_pay))
    got = {int(s) for s in out["hdr"]["seq"]}
    assert {1, 2, col + 1, 2 * col + 4} <= got  # the two-level chain and the rejected row's member
