"""Wire-codec checks shared by the oracle tests (CPU) and the HIP tests (GPU).

An *engine* exposes (numpy in, numpy out, layouts of include/razor_fec.h):
    frame_fec(parity[N][stride], meta[N], fsize[N], status|None, stamps[N], capacity, dstride) -> (dgram, dlen)
    frame_seg(shards[N][stride], hdr[N], stamps[N], capacity, dstride) -> (dgram, dlen)
    parse(dgram[N][dstride], dlen[N], stride, capacity) -> (recs[N], payload[N][stride])

Expected values: tests/golden/wire_*.bin, written by oracle/gen_wire.c from the
reference's sim_encode_msg / sim_decode_header / sim_decode_msg.
"""
from __future__ import annotations

import numpy as np

import pyoracle as po

CAP = 1000  # SIM_VIDEO_SIZE of the reference build that wrote the fixtures
STRIDE = 1008


def _r16(n):
    return (n + 15) // 16 * 16


def fec_fixture():
    cases = po.load_wire_fec()
    N = len(cases)
    parity = np.zeros((N, STRIDE), np.uint8)
    meta = np.zeros(N, po.HDR_DTYPE)
    fsize = np.zeros(N, np.uint16)
    stamps = np.zeros(N, po.FEC_STAMP)
    exp = []
    for i, (r, f) in enumerate(cases):
        L = int(r["fec_data_size"])
        parity[i, :L] = f["payload"]
        meta[i] = r["meta"]
        fsize[i] = L
        for k in ("uid", "base_id", "send_ts", "fec_id", "count", "transport_seq", "row", "col", "index"):
            stamps[i][k] = r[k]
        exp.append(f["dgram"])
    return parity, meta, fsize, stamps, exp


def seg_fixture():
    cases = po.load_wire_seg()
    N = len(cases)
    shards = np.zeros((N, STRIDE), np.uint8)
    hdr = np.zeros(N, po.HDR_DTYPE)
    stamps = np.zeros(N, po.SEG_STAMP)
    exp = []
    for i, (r, f) in enumerate(cases):
        L = int(r["data_size"])
        shards[i, :L] = f["payload"]
        for a, b in (("seq", "packet_id"), ("fid", "fid"), ("ts", "timestamp"), ("index", "index"),
                     ("total", "total"), ("ftype", "ftype"), ("payload_type", "payload_type"), ("size", "data_size")):
            hdr[i][a] = r[b]
        for k in ("uid", "fec_id", "send_ts", "transport_seq", "remb"):
            stamps[i][k] = r[k]
        exp.append(f["dgram"])
    return shards, hdr, stamps, exp


def check_frames(dgram, dlen, exp):
    assert dgram.shape[0] == len(exp)
    for i, e in enumerate(exp):
        n = len(e)
        assert int(dlen[i]) == n, f"datagram {i}: length {int(dlen[i])} != reference {n}"
        assert np.array_equal(dgram[i, :n], e), f"datagram {i}: bytes differ from the reference"
        assert not dgram[i, n:].any(), f"datagram {i}: slot not zero past the datagram"


def check_frame_fec(engine):
    parity, meta, fsize, stamps, exp = fec_fixture()
    dstride = _r16(CAP + 49)
    dgram, dlen = engine.frame_fec(parity, meta, fsize, None, stamps, CAP, dstride)
    check_frames(dgram, dlen, exp)
    # status -1 / oversize lines are not emitted
    status = np.zeros(len(exp), np.int8)
    status[::7] = -1
    dgram, dlen = engine.frame_fec(parity, meta, fsize, status, stamps, CAP, dstride)
    for i, e in enumerate(exp):
        if status[i] < 0:
            assert dlen[i] == 0 and not dgram[i].any()
        else:
            assert int(dlen[i]) == len(e) and np.array_equal(dgram[i, :len(e)], e)


def check_frame_seg(engine):
    shards, hdr, stamps, exp = seg_fixture()
    dgram, dlen = engine.frame_seg(shards, hdr, stamps, CAP, _r16(CAP + 36))
    check_frames(dgram, dlen, exp)


def parse_fixture():
    cases = po.load_wire_parse()
    N = len(cases)
    dstride = _r16(max(int(r["len"]) for r, _ in cases))
    dgram = np.zeros((N, dstride), np.uint8)
    dlen = np.zeros(N, np.uint16)
    recs = np.zeros(N, po.WIRE_REC)
    pays = []
    kinds = np.zeros(N, np.uint8)
    for i, (r, f) in enumerate(cases):
        n = int(r["len"])
        dgram[i, :n] = f["dgram"]
        # garbage past the datagram end must not matter
        dgram[i, n:] = (np.arange(dstride - n) * 37 + i) & 0xFF
        dlen[i] = n
        recs[i] = r["rec"]
        kinds[i] = r["kind"]
        pays.append(f["payload"])
    return dgram, dlen, recs, pays, kinds


REC_FIELDS = ("status", "ver", "mid", "remb", "uid", "base_id", "send_ts", "fec_id", "count", "transport_seq",
              "data_size", "row", "col", "index")


def check_recs(got, exp_recs, i, kind=None):
    for k in REC_FIELDS:
        assert got[k] == exp_recs[i][k], f"datagram {i} (kind {kind}): {k} {got[k]} != reference {exp_recs[i][k]}"
    assert got["hdr"].tobytes() == exp_recs[i]["hdr"].tobytes(), f"datagram {i} (kind {kind}): header fields differ"


def check_parse(engine):
    dgram, dlen, exp, pays, kinds = parse_fixture()
    recs, payload = engine.parse(dgram, dlen, STRIDE, CAP)
    seen = set()
    for i in range(len(exp)):
        check_recs(recs[i], exp, i, int(kinds[i]))
        n = int(exp[i]["data_size"])
        assert np.array_equal(payload[i, :n], pays[i]), f"datagram {i}: payload differs"
        assert not payload[i, n:].any(), f"datagram {i}: payload slot not zero past data_size"
        seen.add((int(exp[i]["status"]), int(exp[i]["mid"]) if exp[i]["status"] >= 0 else -1))
    # every outcome the reference produced on the fixtures is exercised
    assert {s for s, _ in seen} >= {0, 1, -1, -2, -3}


def random_batch(rng, N, stride, capacity, seg=False):
    """Random framing inputs, sizes biased to the edges."""
    sizes = rng.integers(0, capacity + 1, N)
    sizes[: min(N, 64)] = np.arange(min(N, 64)) % (capacity + 1)
    sizes[rng.random(N) < 0.1] = capacity
    data = rng.integers(0, 256, (N, stride), dtype=np.uint8)
    data[np.arange(stride)[None, :] >= sizes[:, None]] = 0
    hdr = np.zeros(N, po.HDR_DTYPE)
    for k in ("seq", "fid", "ts"):
        hdr[k] = rng.integers(0, 2**32, N, dtype=np.uint64).astype(np.uint32)
    small = rng.random(N) < 0.5
    hdr["seq"][small] %= 65536
    hdr["fid"][rng.random(N) < 0.5] %= 65536
    hdr["index"] = rng.integers(0, 2**16, N)
    hdr["total"] = rng.integers(0, 2**16, N)
    hdr["total"][rng.random(N) < 0.5] %= 256
    hdr["ftype"] = rng.integers(0, 256, N)
    hdr["payload_type"] = rng.integers(0, 256, N)
    hdr["size"] = sizes
    if seg:
        stamps = np.zeros(N, po.SEG_STAMP)
        stamps["remb"] = rng.integers(0, 3, N)
    else:
        stamps = np.zeros(N, po.FEC_STAMP)
        for k in ("base_id", "send_ts"):
            stamps[k] = rng.integers(0, 2**32, N, dtype=np.uint64).astype(np.uint32)
        for k in ("row", "col", "index"):
            stamps[k] = rng.integers(0, 256, N)
        stamps["count"] = rng.integers(0, 2**16, N)
    stamps["uid"] = rng.integers(0, 2**32, N, dtype=np.uint64).astype(np.uint32)
    stamps["fec_id"] = rng.integers(0, 2**16, N)
    stamps["send_ts"] = rng.integers(0, 2**16, N) if seg else stamps["send_ts"]
    stamps["transport_seq"] = rng.integers(0, 2**16, N)
    return data, hdr, sizes.astype(np.uint16), stamps
