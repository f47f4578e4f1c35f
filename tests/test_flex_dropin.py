"""GPU: the group-level drop-in (include/razor_flex.h: flex_fec_sender_* /
flex_fec_receiver_*, razor_amd/csrc/rfec_flex.c) against the reference's
own sender and receiver, through ctypes exactly as razor's C callers use it.

  * sender: every group of every sender fixture (tests/golden/enc_*.bin, the
    reference flex_fec_sender_update's emissions, oracle/gen_golden.c:186-241)
    is fed segment by segment to flex_fec_sender_add_segment and emitted by ONE
    flex_fec_sender_update: parities in the same order with the same stamps,
    meta, fec_data_size and payload bytes;
  * receiver: every erasure pattern of the era_*.bin fixtures is replayed the
    way gen_golden.c:404-451 drove the reference receiver (members, then
    parities, then the recovered segments cascaded back in packet-id order):
    the same recovered set and the same segment hashes.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest
import torch

import parity_cases as pc
import pyoracle as po
from razor_amd.fec import RFEC_TUNE_NO_SERVICE

pytestmark = pytest.mark.gpu

MANIFEST = po.manifest()
CASES = {c["name"]: c for c in MANIFEST["cases"]}

libc = C.CDLL(None)
libc.malloc.restype = C.c_void_p
libc.malloc.argtypes = [C.c_size_t]
libc.free.argtypes = [C.c_void_p]


class base_list_unit_t(C.Structure):
    pass


base_list_unit_t._fields_ = [("next", C.POINTER(base_list_unit_t)), ("pdata", C.c_void_p)]


class base_list_t(C.Structure):  # common/cf_list.h:17-27
    _fields_ = [("head", C.POINTER(base_list_unit_t)), ("tailer", C.POINTER(base_list_unit_t)), ("size", C.c_size_t)]


class flex_fec_sender_t(C.Structure):  # flex_fec_sender.h:7-24
    _fields_ = [("fec_id", C.c_uint16), ("row", C.c_uint8), ("col", C.c_uint8), ("base_id", C.c_uint32),
                ("first", C.c_int), ("fec_ts", C.c_int64), ("seg_size", C.c_uint16), ("segs_count", C.c_uint16),
                ("segs", C.c_void_p), ("cache_size", C.c_uint16), ("cache", C.c_void_p)]


def list_pop(lst: base_list_t):
    """list_pop (common/cf_list.c): the head unit's data; the unit is freed.
    (A POINTER field read from a ctypes Structure aliases the field, so the
    unit's address is taken as an integer before the head moves.)"""
    addr = C.cast(lst.head, C.c_void_p).value
    if not addr:
        return None
    u = base_list_unit_t.from_address(addr)
    d, nxt = u.pdata, C.cast(u.next, C.c_void_p).value
    lst.head = C.cast(nxt, C.POINTER(base_list_unit_t)) if nxt else None
    if not nxt:
        lst.tailer = None
    lst.size -= 1
    libc.free(addr)
    return d


def bind_flex(product):
    """Declares the razor_flex.h symbols on the product's ctypes handle."""
    L = product.lib
    P = C.c_void_p
    for fn, res, args in (("flex_fec_sender_create", C.POINTER(flex_fec_sender_t), []),
                          ("flex_fec_sender_destroy", None, [P]),
                          ("flex_fec_sender_add_segment", None, [P, P]),
                          ("flex_fec_sender_update", None, [P, C.c_uint8, P]),
                          ("flex_fec_sender_release", None, [P, P]),
                          ("flex_fec_receiver_create", P, [P, P, P]),
                          ("flex_fec_receiver_desotry", None, [P]),
                          ("flex_fec_receiver_active", None, [P, C.c_uint16, C.c_uint8, C.c_uint8, C.c_uint32,
                                                              C.c_uint16]),
                          ("flex_fec_receiver_on_fec", P, [P, P]),
                          ("flex_fec_receiver_on_segment", C.c_int, [P, P, P])):
        f = getattr(L, fn)
        f.restype, f.argtypes = res, args
    return product


@pytest.fixture(scope="module", params=["service", "launch"])
def flex(product, request):
    """The drop-in both ways: posted to the resident service (the default) and
    with a kernel launch per call (RFEC_TUNE_NO_SERVICE)."""
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")
    L = product.lib
    before = _svc_stats(L)
    L.rfec_set_tuning(0 if request.param == "service" else RFEC_TUNE_NO_SERVICE)
    yield bind_flex(product)
    L.rfec_set_tuning(0)
    jobs = _svc_stats(L)[0] - before[0]
    assert L.rfec_service_stop() == 0
    if request.param == "service":
        assert jobs > 0, "no drop-in call reached the resident service"
        # the module's sender and (ragged) receiver fixtures ran through the
        # request side in device memory wherever the host maps it
        assert request_in_device(L) == int(bar_host_mapped())
    else:
        assert jobs == 0, "a drop-in call reached the service under RFEC_TUNE_NO_SERVICE"


def bar_host_mapped() -> bool:
    """Independent of the library: is fine-grained device memory mapped
    read-write into this process at its device address (/proc/self/maps)?
    That is the condition under which the service puts its request side
    (doorbell, job, staged segments) in device memory (svc_map_request_side)."""
    hip = C.CDLL("libamdhip64.so")
    p = C.c_void_p()
    n = 1 << 20
    if hip.hipExtMallocWithFlags(C.byref(p), C.c_size_t(n), C.c_uint(1)) != 0 or not p.value:  # Finegrained
        return False
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                lo, hi = (int(x, 16) for x in line.split()[0].split("-"))
                if lo <= p.value and p.value + n <= hi:
                    return line.split()[1].startswith("rw")
        return False
    finally:
        hip.hipFree(p)


def request_in_device(L) -> int:
    from razor_amd.fec import rfec_service_info
    i = rfec_service_info()
    assert L.rfec_service_get_info(C.byref(i)) == 0
    return int(i.request_in_device)


def _svc_stats(L):
    from razor_amd.fec import rfec_service_info
    i = rfec_service_info()
    assert L.rfec_service_get_info(C.byref(i)) == 0
    return i.jobs, i.launches


def make_segments(lib, shards, hdr):
    """sim_segment_t per member (gen_golden.c:150-180, whole payloads)."""
    segs = []
    for i in range(hdr.shape[0]):
        s = lib.sim_segment_t()
        h = hdr[i]
        s.packet_id, s.fid, s.timestamp = int(h["seq"]), int(h["fid"]), int(h["ts"])
        s.index, s.total, s.ftype, s.payload_type = int(h["index"]), int(h["total"]), int(h["ftype"]), int(
            h["payload_type"])
        s.data_size = int(h["size"])
        n = min(int(h["size"]), lib.video_size)
        C.memmove(C.addressof(s) + 34, shards[i, :n].tobytes(), n)
        segs.append(s)
    return segs


def sender_group(lib, snd, segs, pf):
    """gen_golden.c:186-194: add the group's segments, force the update."""
    for s in segs:
        lib.lib.flex_fec_sender_add_segment(snd, C.byref(s))
    snd.contents.fec_ts = 1  # flex_fec_sender_over fires for groups of < 6 too
    lst = base_list_t()
    lib.lib.flex_fec_sender_update(snd, pf, C.byref(lst))
    fecs = []
    while True:
        d = list_pop(lst)
        if d is None:
            break
        f = lib.sim_fec_t()
        C.memmove(C.addressof(f), d, C.sizeof(f))
        libc.free(d)
        fecs.append(f)
    return fecs


@pytest.mark.parametrize("name", [c["name"] for c in MANIFEST["cases"] if c["kind"] in ("sender", "sender_large")])
def test_flex_sender_fixture(flex, oracle1000, name):
    c = CASES[name]
    lib = flex
    shards, hdr = oracle1000.fill_groups(c["config_id"], c["groups"], c["k"], c["S"], ragged=c["ragged"])
    recs, pays = po.load_parities(c)
    snd = lib.lib.flex_fec_sender_create()
    try:
        for g in range(c["groups"]):
            segs = make_segments(lib, shards[g], hdr[g])
            fecs = sender_group(lib, snd, segs, c["protect_fraction"])
            sel = np.nonzero(recs["group"] == g)[0]
            assert len(fecs) == len(sel), f"group {g}: {len(fecs)} parities, reference {len(sel)}"
            for f, ri in zip(fecs, sel):
                r = recs[ri]
                assert (f.fec_id, f.row, f.col, f.index, f.count, f.base_id) == (
                    int(r["fec_id"]), int(r["row"]), int(r["col"]), int(r["index"]), int(r["count"]),
                    int(r["base_id"])), f"group {g}: stamps"
                L = int(r["fec_data_size"])
                assert f.fec_data_size == L
                meta = np.frombuffer(bytes(f.fec_meta), po.HDR_DTYPE)[0]
                assert meta.tobytes() == r["meta"].tobytes(), f"group {g}: meta"
                assert bytes(f.fec_data)[:L] == pays[ri][:L].tobytes(), f"group {g}: payload"
    finally:
        lib.lib.flex_fec_sender_destroy(snd)


def seg_hash(s) -> int:
    h = np.zeros((), po.HDR_DTYPE)
    h["seq"], h["fid"], h["ts"], h["index"], h["total"] = s.packet_id, s.fid, s.timestamp, s.index, s.total
    h["ftype"], h["payload_type"], h["size"] = s.ftype, s.payload_type, s.data_size
    return po.seg_hash(h, np.frombuffer(bytes(s.data), np.uint8))


def run_receiver(lib, segs, fecs, present, pp, base_id):
    """gen_golden.c:404-451 through the drop-in receiver."""
    L = lib.lib
    k = len(segs)
    r = L.flex_fec_receiver_create(None, None, None)
    f0 = fecs[0]
    L.flex_fec_receiver_active(r, f0.fec_id, f0.col, f0.row, f0.base_id, f0.count)
    lst = base_list_t()
    bag = {}

    def add(p):
        if not p:
            return
        s = lib.sim_segment_t()
        C.memmove(C.addressof(s), p, C.sizeof(s))
        libc.free(p)
        bag.setdefault(s.packet_id, s)  # the first copy per packet id (sim_fec.c:104-119)

    for i in range(k):
        if (present[i >> 6] >> (i & 63)) & 1:
            L.flex_fec_receiver_on_segment(r, C.byref(segs[i]), C.byref(lst))
            while lst.size:
                add(list_pop(lst))
    for l, f in enumerate(fecs):
        if (pp >> l) & 1:
            c = libc.malloc(C.sizeof(f))  # the receiver owns it
            C.memmove(c, C.addressof(f), C.sizeof(f))
            add(L.flex_fec_receiver_on_fec(r, c))
    got, keep = [0, 0], {}
    while bag:
        pid = min(bag)
        s = bag.pop(pid)
        pos = pid - base_id
        got[pos >> 6] |= 1 << (pos & 63)
        keep[pos] = s
        L.flex_fec_receiver_on_segment(r, C.byref(s), C.byref(lst))  # cascade
        while lst.size:
            add(list_pop(lst))
    L.flex_fec_receiver_desotry(r)
    return got, [seg_hash(keep[p]) for p in sorted(keep)][:16]


@pytest.mark.parametrize("name", [c["name"] for c in MANIFEST["cases"] if c["kind"] == "erasures"])
def test_flex_receiver_erasure_fixture(flex, oracle1000, name):
    c = CASES[name]
    lib = flex
    shards, hdr, _ = pc.erasure_inputs(oracle1000, c)
    work = make_segments(lib, shards[0], hdr[0])
    snd = lib.lib.flex_fec_sender_create()
    try:
        fecs = sender_group(lib, snd, work, c["protect_fraction"])
    finally:
        lib.lib.flex_fec_sender_destroy(snd)
    assert len(fecs) == c["parities"]
    segs = make_segments(lib, shards[0], hdr[0])  # pristine copies for the receiver
    base_id = segs[0].packet_id
    pats = po.load_erasures(c)
    for p, exp in enumerate(pats):
        got, hashes = run_receiver(lib, segs, fecs, [int(x) for x in exp["present"]], int(exp["parity_present"]),
                                   base_id)
        assert got == [int(x) for x in exp["recovered"]], f"pattern {p}: recovered {got} != {exp['recovered']}"
        assert len(hashes) == min(16, int(exp["n_recovered"]))
        assert hashes == [int(x) for x in exp["hash"][:len(hashes)]], f"pattern {p}: hashes"


def test_flex_sender_random_fixture(flex, oracle1000):
    """64 groups of random k and protect fraction (tests/golden random_k),
    each through one flex_fec_sender_update."""
    c = CASES["random_k"]
    lib = flex
    recs, pays = po.load_parities(c)
    groups = np.fromfile(po.GOLDEN / c["groups_file"], np.uint32).reshape(-1, 3)
    snd = lib.lib.flex_fec_sender_create()
    try:
        for g, (k, pf, n) in enumerate(groups):
            shards, hdr = oracle1000.fill_groups(c["config_id"] * 1000 + g, 1, int(k), c["S"], ragged=True)
            fecs = sender_group(lib, snd, make_segments(lib, shards[0], hdr[0]), int(pf))
            sel = np.nonzero(recs["group"] == g)[0]
            assert len(fecs) == len(sel) == n, f"group {g}"
            for f, ri in zip(fecs, sel):
                r = recs[ri]
                assert (f.row, f.col, f.index, f.count, f.base_id) == (
                    int(r["row"]), int(r["col"]), int(r["index"]), int(r["count"]), int(r["base_id"]))
                L = int(r["fec_data_size"])
                assert f.fec_data_size == L
                assert np.frombuffer(bytes(f.fec_meta), po.HDR_DTYPE)[0].tobytes() == r["meta"].tobytes()
                assert bytes(f.fec_data)[:L] == pays[ri][:L].tobytes()
    finally:
        lib.lib.flex_fec_sender_destroy(snd)

