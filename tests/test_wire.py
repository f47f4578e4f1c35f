"""Wire codec (SIM_FEC / SIM_SEG datagrams + CRC32, sim_proto.c / sim_proto.inl):
the oracle against the reference's own encoder/decoder outputs
(tests/golden/wire_*.bin from oracle/gen_wire.c), then the HIP kernels against
the same fixtures and against the oracle on large random batches."""
from __future__ import annotations

import zlib

import numpy as np
import pytest
import torch

import pyoracle as po
import wire_cases as wc


class OracleWire:
    def __init__(self, o):
        self.o = o

    def frame_fec(self, parity, meta, fsize, status, stamps, capacity, dstride):
        return self.o.frame_fec_batch(parity, meta, fsize, status, stamps, capacity, dstride)

    def frame_seg(self, shards, hdr, stamps, capacity, dstride):
        return self.o.frame_seg_batch(shards, hdr, stamps, capacity, dstride)

    def parse(self, dgram, dlen, stride, capacity):
        return self.o.parse_batch(dgram, dlen, stride, capacity)


# -- CPU: oracle pinned to the reference ---------------------------------------
def test_wire_crc_is_zlib_crc32_with_seed(oracle1000):
    """cf_crc32.c:56-68 == zlib crc32 continued from 0x0e3dfc0a; every fixture
    datagram ends in it, big-endian (sim_proto.c:92-94)."""
    for r, f in po.load_wire_fec() + po.load_wire_seg():
        d = f["dgram"].tobytes()
        c = zlib.crc32(d[:-4], po.CRC_SEED)
        assert int.from_bytes(d[-4:], "big") == c == oracle1000.crc32(d[:-4])
    for n in range(0, 9):
        d = bytes(range(n))
        assert oracle1000.crc32(d) == zlib.crc32(d, po.CRC_SEED)


def test_wire_frame_fec_oracle(oracle1000):
    wc.check_frame_fec(OracleWire(oracle1000))


def test_wire_frame_seg_oracle(oracle1000):
    wc.check_frame_seg(OracleWire(oracle1000))


def test_wire_parse_oracle(oracle1000):
    wc.check_parse(OracleWire(oracle1000))


def test_wire_fixture_coverage():
    m = po.wire_manifest()
    assert m["sim_video_size"] == wc.CAP and m["crc_seed"] == po.CRC_SEED
    kinds = np.array([int(r["kind"]) for r, _ in po.load_wire_parse()])
    assert set(kinds.tolist()) == set(range(7))
    segs = po.load_wire_seg()
    masks = {(r["packet_id"] > 65535, r["fid"] > 65535, r["total"] > 255, r["remb"] == 0) for r, _ in segs}
    assert len(masks) == 16  # every header-width / remb combination (sim_proto.inl:85-98)


def test_wire_short_datagram_oracle(oracle1000):
    """Shorter than the CRC trailer: rejected (the reference would read before its buffer)."""
    dgram = np.zeros((4, 64), np.uint8)
    recs, _ = oracle1000.parse_batch(dgram, np.array([0, 1, 2, 3], np.uint16), wc.STRIDE, wc.CAP)
    assert (recs["status"] == -1).all()


# -- GPU -----------------------------------------------------------------------
@pytest.fixture(scope="module")
def gwire():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")
    from gpu_engine import GpuWire
    return GpuWire()


RFEC_TUNE_WAVE_PARSE = 1 << 3


@pytest.fixture(params=["quarter", "wave"])
def pwire(request):
    """The parse both ways: the quarter-wave kernel (default) and the
    wave-per-datagram one (RFEC_TUNE_WAVE_PARSE), the cross-check."""
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")
    from gpu_engine import GpuWire
    return GpuWire(tuning=0 if request.param == "quarter" else RFEC_TUNE_WAVE_PARSE)


@pytest.mark.gpu
def test_wire_frame_fec_gpu(gwire):
    wc.check_frame_fec(gwire)


@pytest.mark.gpu
def test_wire_frame_seg_gpu(gwire):
    wc.check_frame_seg(gwire)


@pytest.mark.gpu
def test_wire_parse_gpu(pwire):
    wc.check_parse(pwire)


@pytest.mark.gpu
def test_wire_short_datagram_gpu(pwire):
    gwire = pwire
    dgram = np.full((5, 64), 0xAB, np.uint8)
    recs, pay = gwire.parse(dgram, np.array([0, 1, 2, 3, 4], np.uint16), wc.STRIDE, wc.CAP)
    assert (recs["status"][:4] == -1).all() and not pay.any()
    # 4 bytes: an empty message whose trailer must equal crc32(seed, "") = seed
    d = np.zeros((1, 64), np.uint8)
    d[0, :4] = np.frombuffer(po.CRC_SEED.to_bytes(4, "big"), np.uint8)
    recs, _ = gwire.parse(d, np.array([4], np.uint16), wc.STRIDE, wc.CAP)
    # CRC accepted; ver/mid then read the trailer bytes themselves (0x0e, 0x3d): mid out of range
    assert recs["status"][0] == -2 and recs["ver"][0] == 0x0E and recs["mid"][0] == 0x3D


@pytest.mark.gpu
@pytest.mark.parametrize("capacity,stride,dstride,N", [(1200, 1200, 1248, 4097), (1200, 1216, 1264, 4099),
                                                       (1000, 1008, 1056, 3001), (230, 240, 288, 2051),
                                                       (1200, 1280, 1280, 2050), (1200, 1200, 1504, 2049),
                                                       (1300, 1312, 1360, 1025)])
def test_wire_parse_mixed_gpu(pwire, oracle1000, capacity, stride, dstride, N):
    """The parse against the oracle on batches that mix SIM_SEG (every header
    width: data at bytes 26-32) and SIM_FEC (data at 45) datagrams in random
    order -- a quarter-wave quad holds datagrams with different data offsets
    -- with flipped bytes (CRC mismatches: record EBADCRC, slot zero), lengths
    cut short or past the slot, data sizes that overrun the datagram, control
    messages and bad message ids; slots of 1,248-1,504 bytes (wider than 1,280:
    the datagrams still fit, the quarter-wave parse reads the first 1,280),
    payload slots up to 1,280 bytes, N not a multiple of 4."""
    rng = np.random.default_rng(capacity + stride * 3 + dstride * 7 + N)
    frames, lens = [], []
    for seg in (True, False):
        data, hdr, sizes, stamps = wc.random_batch(rng, N, stride, capacity, seg=seg)
        over = 36 if seg else 49
        ds = max(dstride, (capacity + over + 15) // 16 * 16)
        if seg:
            g, gl = oracle1000.frame_seg_batch(data, hdr, stamps, capacity, ds)
        else:
            g, gl = oracle1000.frame_fec_batch(data, hdr, sizes, None, stamps, capacity, ds)
        frames.append(g[:, :dstride] if ds > dstride else np.pad(g, ((0, 0), (0, dstride - ds))))
        lens.append(np.minimum(gl, dstride).astype(np.uint16))
    dgram = np.concatenate(frames)
    dlen = np.concatenate(lens)
    pick = rng.permutation(len(dgram))[:N]
    dgram, dlen = dgram[pick].copy(), dlen[pick].copy()
    n = len(dgram)
    flip = rng.random(n) < 0.08  # a flipped byte inside the message
    for i in np.nonzero(flip & (dlen > 8))[0]:
        dgram[i, rng.integers(0, int(dlen[i]))] ^= 1 << int(rng.integers(8))
    cut = rng.random(n) < 0.04  # cut short (the trailer then sits elsewhere: a CRC mismatch)
    dlen[cut] = rng.integers(0, 60, int(cut.sum()))
    over = rng.random(n) < 0.02  # longer than the slot
    dlen[over] = dstride + 1 + rng.integers(0, 100, int(over.sum()))
    mid = rng.random(n) < 0.03  # another message id, CRC recomputed (a control message or a bad id)
    for i in np.nonzero(mid & (dlen >= 10) & (dlen <= dstride))[0]:
        L = int(dlen[i])
        dgram[i, 1] = rng.choice([0x10, 0x12, 0x1D, 0x05, 0x40])
        crc = oracle1000.crc32(dgram[i, :L - 4].tobytes())
        dgram[i, L - 4:L] = np.frombuffer(crc.to_bytes(4, "big"), np.uint8)
    recs, pay = pwire.parse(dgram, dlen, stride, capacity)
    orecs, opay = oracle1000.parse_batch(dgram, dlen, stride, capacity)
    bad = np.nonzero((recs.view(np.uint8).reshape(n, 64) != orecs.view(np.uint8).reshape(n, 64)).any(1))[0]
    assert len(bad) == 0, (bad[:8], recs[bad[:2]], orecs[bad[:2]])
    bad = np.nonzero((pay != opay).any(1))[0]
    assert len(bad) == 0, (bad[:8], recs[bad[:4]]["status"], recs[bad[:4]]["data_size"])
    st = set(int(x) for x in recs["status"])
    assert {0, -1} <= st and (recs["status"] == 0).sum() > n // 2


@pytest.mark.gpu
@pytest.mark.parametrize("capacity,stride", [(1000, 1008), (1200, 1200), (256, 256), (1984, 1984), (1999, 2000)])
def test_wire_random_roundtrip_gpu(gwire, oracle1000, capacity, stride):
    """Large random batches: HIP framing == oracle framing byte for byte, and
    HIP parse(HIP frame(x)) returns x (fields, payload, zero tails)."""
    rng = np.random.default_rng(capacity)
    N = 20000
    for seg in (False, True):
        data, hdr, sizes, stamps = wc.random_batch(rng, N, stride, capacity, seg=seg)
        over = 36 if seg else 49
        dstride = min(2048, (capacity + over + 15) // 16 * 16)
        if seg:
            g, gl = gwire.frame_seg(data, hdr, stamps, capacity, dstride)
            o, ol = oracle1000.frame_seg_batch(data, hdr, stamps, capacity, dstride)
        else:
            g, gl = gwire.frame_fec(data, hdr, sizes, None, stamps, capacity, dstride)
            o, ol = oracle1000.frame_fec_batch(data, hdr, sizes, None, stamps, capacity, dstride)
        assert np.array_equal(gl, ol)
        assert np.array_equal(g, o)
        recs, pay = gwire.parse(g, gl, stride, capacity)
        orecs, opay = oracle1000.parse_batch(g, gl, stride, capacity)
        assert np.array_equal(recs.view(np.uint8), orecs.view(np.uint8))
        assert np.array_equal(pay, opay)
        assert (recs["status"] == 0).all()
        assert np.array_equal(recs["data_size"], sizes)
        assert np.array_equal(pay, data)
        assert np.array_equal(recs["uid"], stamps["uid"])
        assert np.array_equal(recs["transport_seq"], stamps["transport_seq"])
        if seg:
            assert np.array_equal(recs["hdr"]["seq"], hdr["seq"]) and np.array_equal(recs["hdr"]["fid"], hdr["fid"])
            assert np.array_equal(recs["hdr"]["ftype"], hdr["ftype"] & 1)
            assert np.array_equal(recs["remb"], np.where(stamps["remb"] == 0, 0, 0xFF))
        else:
            assert recs["hdr"].tobytes() == hdr.tobytes()
            assert np.array_equal(recs["base_id"], stamps["base_id"])


@pytest.mark.gpu
@pytest.mark.parametrize("capacity,stride,dstride", [(1200, 1200, 1248), (1200, 1216, 1264), (1000, 1008, 1280),
                                                     (1201, 1216, 1248), (1240, 1248, 1280), (230, 240, 272),
                                                     (1300, 1312, 1344)])
def test_wire_frame_seg_edges_gpu(gwire, oracle1000, capacity, stride, dstride):
    """SIM_SEG framing against the oracle where the quarter-wave kernel must
    mask and place bytes itself: garbage past each segment's data (other
    bytes of its slot), sizes above capacity (zero datagram, length 0),
    every header width, an output permutation (`order`), and slot widths
    on both sides of the quarter-wave path's condition (datagram slots up
    to 1,280 B; wider ones take the 32-byte lanes)."""
    rng = np.random.default_rng(capacity * 7 + stride + dstride)
    N = 4099  # not a multiple of 4: the last quad is partial
    data, hdr, sizes, stamps = wc.random_batch(rng, N, stride, capacity, seg=True)
    garbage = rng.integers(0, 256, data.shape, dtype=np.uint8)
    tail = np.arange(stride)[None, :] >= sizes[:, None]
    data = np.where(tail, garbage, data)
    big = rng.random(N) < 0.02
    hdr["size"][big] = capacity + 1 + rng.integers(0, 50, int(big.sum()))
    o, ol = oracle1000.frame_seg_batch(data, hdr, stamps, capacity, dstride)
    assert (ol[big] == 0).all() and not o[big].any()
    g, gl = gwire.frame_seg(data, hdr, stamps, capacity, dstride)
    assert np.array_equal(gl, ol)
    assert np.array_equal(g, o)
    perm = rng.permutation(N).astype(np.uint32)
    g2, gl2 = gwire.frame_seg(data, hdr, stamps, capacity, dstride, order=perm)
    assert np.array_equal(gl2[perm], ol)
    assert np.array_equal(g2[perm], o)


@pytest.mark.gpu
@pytest.mark.parametrize("capacity,stride,dstride", [(1200, 1200, 1264), (1200, 1216, 1280), (1000, 1008, 1056),
                                                     (230, 240, 288), (1300, 1312, 1360)])
def test_wire_frame_fec_edges_gpu(gwire, oracle1000, capacity, stride, dstride):
    """SIM_FEC framing against the oracle with garbage past each line's
    fec_data_size, status -1 and oversize lines (zero datagram, length 0),
    random stamps and meta, a partial last quad and an output permutation,
    on both sides of the quarter-wave path's slot limit (1,280 B)."""
    rng = np.random.default_rng(capacity * 5 + stride + dstride)
    N = 4097
    data, meta, sizes, stamps = wc.random_batch(rng, N, stride, capacity, seg=False)
    garbage = rng.integers(0, 256, data.shape, dtype=np.uint8)
    data = np.where(np.arange(stride)[None, :] >= sizes[:, None], garbage, data)
    sizes = sizes.astype(np.uint16)
    big = rng.random(N) < 0.02
    sizes[big] = capacity + 1 + rng.integers(0, 40, int(big.sum()))
    status = np.where(rng.random(N) < 0.05, -1, 0).astype(np.int8)
    o, ol = oracle1000.frame_fec_batch(data, meta, sizes, status, stamps, capacity, dstride)
    assert (ol[big | (status < 0)] == 0).all()
    g, gl = gwire.frame_fec(data, meta, sizes, status, stamps, capacity, dstride)
    assert np.array_equal(gl, ol)
    assert np.array_equal(g, o)
