"""ctypes bindings of the CPU oracle (oracle/rfec_oracle.c) and readers for the
golden fixtures in tests/golden/.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product (razor_amd, librazor_fec.so) never
imports this module.
"""
from __future__ import annotations

import ctypes as C
import json
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent
GOLDEN = ROOT / "tests" / "golden"
LIBDIR = HERE / "lib"
REFDIR = HERE / "_ref"

HDR_DTYPE = np.dtype([("seq", "<u4"), ("fid", "<u4"), ("ts", "<u4"), ("index", "<u2"), ("total", "<u2"),
                      ("ftype", "u1"), ("payload_type", "u1"), ("size", "<u2")])
PARITY_REC = np.dtype([("fec_id", "<u2"), ("row", "u1"), ("col", "u1"), ("index", "u1"), ("status", "i1"),
                       ("count", "<u2"), ("base_id", "<u4"), ("meta", HDR_DTYPE), ("fec_data_size", "<u2"),
                       ("group", "<u2"), ("line", "u1"), ("pad", "u1", (11,))])
ERASURE_REC = np.dtype([("present", "<u8", (2,)), ("parity_present", "<u8"), ("recovered", "<u8", (2,)),
                        ("group", "<u4"), ("n_recovered", "<u4"), ("hash", "<u8", (16,))])
assert PARITY_REC.itemsize == 48 and ERASURE_REC.itemsize == 176

# wire codec (include/razor_fec.h rfec_fec_stamp / rfec_seg_stamp / rfec_wire_rec)
FEC_STAMP = np.dtype([("uid", "<u4"), ("base_id", "<u4"), ("send_ts", "<u4"), ("fec_id", "<u2"), ("count", "<u2"),
                      ("transport_seq", "<u2"), ("row", "u1"), ("col", "u1"), ("index", "u1"), ("reserved", "u1"),
                      ("pad", "u1", (2,))])
SEG_STAMP = np.dtype([("uid", "<u4"), ("fec_id", "<u2"), ("send_ts", "<u2"), ("transport_seq", "<u2"), ("remb", "u1"),
                      ("reserved", "u1")])
WIRE_REC = np.dtype([("status", "i1"), ("ver", "u1"), ("mid", "u1"), ("remb", "u1"), ("uid", "<u4"),
                     ("hdr", HDR_DTYPE), ("base_id", "<u4"), ("send_ts", "<u4"), ("fec_id", "<u2"), ("count", "<u2"),
                     ("transport_seq", "<u2"), ("data_size", "<u2"), ("row", "u1"), ("col", "u1"), ("index", "u1"),
                     ("reserved", "u1", (17,))])
# fixture records (oracle/gen_wire.c)
WIRE_FEC_IN = np.dtype([("uid", "<u4"), ("base_id", "<u4"), ("send_ts", "<u4"), ("fec_id", "<u2"), ("count", "<u2"),
                        ("transport_seq", "<u2"), ("row", "u1"), ("col", "u1"), ("index", "u1"), ("pad0", "u1"),
                        ("meta", HDR_DTYPE), ("fec_data_size", "<u2"), ("dlen", "<u2"), ("pad1", "u1", (2,))])
WIRE_SEG_IN = np.dtype([("uid", "<u4"), ("packet_id", "<u4"), ("fid", "<u4"), ("timestamp", "<u4"), ("index", "<u2"),
                        ("total", "<u2"), ("ftype", "u1"), ("payload_type", "u1"), ("remb", "u1"), ("pad0", "u1"),
                        ("fec_id", "<u2"), ("send_ts", "<u2"), ("transport_seq", "<u2"), ("data_size", "<u2"),
                        ("dlen", "<u2"), ("pad1", "u1", (2,))])
WIRE_PARSE_IN = np.dtype([("len", "<u2"), ("kind", "u1"), ("pad", "u1", (5,)), ("rec", WIRE_REC)])
assert FEC_STAMP.itemsize == 24 and SEG_STAMP.itemsize == 12 and WIRE_REC.itemsize == 64
assert WIRE_FEC_IN.itemsize == 48 and WIRE_SEG_IN.itemsize == 36 and WIRE_PARSE_IN.itemsize == 72
CRC_SEED = 0x0E3DFC0A

# sender staging (include/razor_fec.h rfec_frame / rfec_sender_state / rfec_seg_plan / rfec_group_plan)
FRAME = np.dtype([("data", "<u8"), ("size", "<u4"), ("payload_type", "u1"), ("ftype", "u1"),
                  ("protect_fraction", "u1"), ("reserved", "u1"), ("now_ms", "<i8")])
SENDER_STATE = np.dtype([("packet_id_seed", "<u4"), ("send_id_seed", "<u4"), ("frame_id_seed", "<u4"),
                         ("pad0", "<u4"), ("first_ts", "<i8"), ("fec_ts", "<i8"), ("base_id", "<u4"),
                         ("open_seg", "<i4"), ("fec_id", "<u2"), ("segs_count", "<u2"), ("first", "<i4"),
                         ("transport_seq_seed", "<u4"), ("pad1", "<u4")])
SEG_PLAN = np.dtype([("frame", "<u4"), ("offset", "<u4"), ("packet_id", "<u4"), ("send_id", "<u4"), ("fid", "<u4"),
                     ("timestamp", "<u4"), ("index", "<u2"), ("total", "<u2"), ("data_size", "<u2"),
                     ("fec_id", "<u2"), ("ftype", "u1"), ("payload_type", "u1"), ("reserved", "u1", (2,)),
                     ("group", "<i4")])
GROUP_PLAN = np.dtype([("first_seg", "<i4"), ("count", "<u2"), ("fec_id", "<u2"), ("base_id", "<u4"),
                       ("fec_send_id0", "<u4"), ("fec_ts", "<u4"), ("protect_fraction", "u1"), ("n_lines", "u1"),
                       ("reserved", "u1", (2,))])
assert FRAME.itemsize == 24 and SENDER_STATE.itemsize == 56 and SEG_PLAN.itemsize == 40 and GROUP_PLAN.itemsize == 24
RX_SEG = np.dtype([("hdr", HDR_DTYPE), ("fec_id", "<u2"), ("reserved", "<u2")])
assert RX_SEG.itemsize == 24

SEED = 0x52415A4F52464543


def build_oracle() -> None:
    """Builds oracle/lib/*.so (own C restatement) with gcc if missing."""
    need = [LIBDIR / n for n in ("liboracle.so", "liboracle_v1200.so", "liboracle_O0_v1200.so")]
    srcs = [HERE / "rfec_oracle.c", HERE / "rfec_oracle.h", ROOT / "include" / "razor_fec.h"]
    newest = max(p.stat().st_mtime for p in srcs)
    if all(p.exists() and p.stat().st_mtime >= newest for p in need):
        return
    subprocess.run(["make", "-s", "-C", str(HERE), "oracle"], check=True)


class rfec_line(C.Structure):
    _fields_ = [("first", C.c_uint8), ("stride", C.c_uint8), ("count", C.c_uint8), ("index", C.c_uint8)]


class rfec_plan(C.Structure):
    _fields_ = [("k", C.c_uint16), ("row", C.c_uint8), ("col", C.c_uint8), ("rc", C.c_uint8),
                ("n_lines", C.c_uint8), ("n_row_lines", C.c_uint8), ("reserved", C.c_uint8),
                ("line", rfec_line * 64)]

    def lines(self):
        return [(self.line[i].first, self.line[i].stride, self.line[i].count, self.line[i].index)
                for i in range(self.n_lines)]

    def members(self, l):
        ln = self.line[l]
        return [ln.first + q * ln.stride for q in range(ln.count)]


def _np_ptr(a):
    return a.ctypes.data_as(C.c_void_p)


class Oracle:
    def __init__(self, video_size: int = 1000, opt: str = "O2"):
        build_oracle()
        if video_size == 1000:
            name = "liboracle.so"
        elif opt == "O0":
            name = f"liboracle_O0_v{video_size}.so"
        else:
            name = f"liboracle_v{video_size}.so"
        self.lib = C.CDLL(str(LIBDIR / name))
        L = self.lib
        P = C.c_void_p
        L.oracle_fill_groups.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, P, P]
        L.oracle_fill_stream.argtypes = [C.c_uint64, C.POINTER(C.c_uint64), C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.c_uint32, C.c_uint32, C.c_int, P, P]
        L.oracle_num_packets.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.oracle_plan_from_fraction.argtypes = [C.c_int, C.c_int, C.c_uint, C.POINTER(rfec_plan)]
        L.oracle_plan_matrix.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint, C.POINTER(rfec_plan)]
        L.oracle_encode_batch.argtypes = [C.POINTER(rfec_plan), C.c_uint32, C.c_uint32, C.c_uint32,
                                          P, P, P, P, P, P]
        L.oracle_recover_batch.argtypes = [C.POINTER(rfec_plan), C.c_uint32, C.c_uint32, C.c_uint32,
                                           P, P, P, P, P, P, P, P]
        L.oracle_recover_batch_out.argtypes = [C.POINTER(rfec_plan), C.c_uint32, C.c_uint32, C.c_uint32,
                                               P, P, P, P, P, P, P, P, C.c_uint32, P, P, P]
        L.oracle_generate.argtypes = [P, C.c_int, P, C.c_int]
        L.oracle_recover.argtypes = [P, C.c_int, P, P]
        L.oracle_encode_aos.argtypes = [C.POINTER(rfec_plan), C.c_uint32, P, P]
        L.oracle_encode_aos.restype = C.c_long
        L.oracle_encode_aos_mt.argtypes = [C.POINTER(rfec_plan), C.c_uint32, P, P, C.c_int]
        L.oracle_encode_aos_mt.restype = C.c_long
        L.oracle_recover_aos.argtypes = [C.POINTER(rfec_plan), C.c_uint32, P, P, P, P]
        L.oracle_recover_aos.restype = C.c_long
        L.oracle_recover_aos_mt.argtypes = [C.POINTER(rfec_plan), C.c_uint32, P, P, P, P, C.c_int]
        L.oracle_recover_aos_mt.restype = C.c_long
        L.oracle_crc32.argtypes = [C.c_uint32, P, C.c_size_t]
        L.oracle_crc32.restype = C.c_uint32
        L.oracle_wire_frame_fec_batch.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, P, P, P, P, P, C.c_uint32, P, P]
        L.oracle_wire_frame_seg_batch.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, P, P, P, C.c_uint32, P, P]
        L.oracle_wire_parse_batch.argtypes = [C.c_uint32, C.c_uint32, P, P, C.c_uint32, C.c_uint32, P, P]
        L.oracle_sender_init.argtypes = [P]
        L.oracle_sender_plan.argtypes = [P, P, C.c_uint32, C.c_uint32, P, C.c_uint32, P, P, C.c_uint32, P]
        L.oracle_rx_recover.argtypes = [C.c_uint32, P, P, C.c_uint32, C.c_uint32, P, P, P, C.c_uint32, P, P]
        L.oracle_rx_recover_ev.argtypes = [C.c_uint32, P, P, C.c_uint32, C.c_uint32, P, P, P, C.c_uint32, P, P,
                                           C.c_uint32]
        L.oracle_segment_size.restype = C.c_size_t
        L.oracle_fec_size.restype = C.c_size_t
        self.video_size = L.oracle_sim_video_size()
        self.segment_size = L.oracle_segment_size()
        self.fec_size = L.oracle_fec_size()

    # -- inputs -------------------------------------------------------------
    def fill_groups(self, config_id, groups, k, S, stride=None, ragged=False):
        stride = stride or ((S + 15) // 16) * 16
        shards = np.zeros((groups, k, stride), np.uint8)
        hdr = np.zeros((groups, k), HDR_DTYPE)
        self.lib.oracle_fill_groups(config_id, groups, k, S, stride, int(ragged), _np_ptr(shards), _np_ptr(hdr))
        return shards, hdr

    def fill_stream(self, config_id, k, S, stride=None, ragged=False):
        """Generator of (g0, shards, hdr) pieces of the fill_groups stream."""
        stride = stride or ((S + 15) // 16) * 16
        state = (C.c_uint64 * 2)(0, 0)
        lib = self.lib

        def piece(g0, groups):
            shards = np.empty((groups, k, stride), np.uint8)
            hdr = np.zeros((groups, k), HDR_DTYPE)
            lib.oracle_fill_stream(config_id, state, g0, groups, k, S, stride, int(ragged), _np_ptr(shards),
                                   _np_ptr(hdr))
            return shards, hdr

        return piece

    # -- planner ------------------------------------------------------------
    def num_packets(self, n, pf):
        r, c = C.c_int(), C.c_int()
        rc = self.lib.oracle_num_packets(n, pf, C.byref(r), C.byref(c))
        return rc, r.value, c.value

    def plan_from_fraction(self, k, pf, layers=3):
        p = rfec_plan()
        if self.lib.oracle_plan_from_fraction(k, pf, layers, C.byref(p)) != 0:
            raise ValueError("bad plan")
        return p

    def plan_matrix(self, k, row, col, layers=3):
        p = rfec_plan()
        if self.lib.oracle_plan_matrix(k, row, col, layers, C.byref(p)) != 0:
            raise ValueError("bad plan")
        return p

    # -- batched restatement ------------------------------------------------
    def encode_batch(self, plan, shards, hdr, capacity):
        G, k, stride = shards.shape
        n = plan.n_lines
        parity = np.zeros((G, n, stride), np.uint8)
        meta = np.zeros((G, n), HDR_DTYPE)
        fsize = np.zeros((G, n), np.uint16)
        status = np.zeros((G, n), np.int8)
        self.lib.oracle_encode_batch(C.byref(_as_oracle_plan(plan)), G, stride, capacity, _np_ptr(shards),
                                     _np_ptr(hdr), _np_ptr(parity), _np_ptr(meta), _np_ptr(fsize), _np_ptr(status))
        return parity, meta, fsize, status

    def recover_batch(self, plan, shards, hdr, present, parity, meta, fsize, parity_present, capacity):
        """In place on copies; returns (shards, hdr, recovered)."""
        shards = np.ascontiguousarray(shards).copy()
        hdr = np.ascontiguousarray(hdr).copy()
        G, k, stride = shards.shape
        rec = np.zeros((G, 2), np.uint64)
        self.lib.oracle_recover_batch(C.byref(_as_oracle_plan(plan)), G, stride, capacity, _np_ptr(shards),
                                      _np_ptr(hdr), _np_ptr(np.ascontiguousarray(present, np.uint64)),
                                      _np_ptr(np.ascontiguousarray(parity)), _np_ptr(np.ascontiguousarray(meta)),
                                      _np_ptr(np.ascontiguousarray(fsize, np.uint16)),
                                      _np_ptr(np.ascontiguousarray(parity_present, np.uint64)), _np_ptr(rec))
        return shards, hdr, rec

    def recover_batch_out(self, plan, shards, hdr, present, parity, meta, fsize, parity_present, capacity,
                          per_group):
        """rfec_recover_batch_out's semantics: returns (out_shards [G][E][stride],
        out_hdr [G][E], out_index [G][E], recovered [G][2])."""
        shards = np.ascontiguousarray(shards)
        hdr = np.ascontiguousarray(hdr)
        G, k, stride = shards.shape
        E = per_group
        rec = np.zeros((G, 2), np.uint64)
        o_s = np.zeros((G, E, stride), np.uint8)
        o_h = np.zeros((G, E), HDR_DTYPE)
        o_i = np.zeros((G, E), np.uint8)
        self.lib.oracle_recover_batch_out(C.byref(_as_oracle_plan(plan)), G, stride, capacity, _np_ptr(shards),
                                          _np_ptr(hdr), _np_ptr(np.ascontiguousarray(present, np.uint64)),
                                          _np_ptr(np.ascontiguousarray(parity)), _np_ptr(np.ascontiguousarray(meta)),
                                          _np_ptr(np.ascontiguousarray(fsize, np.uint16)),
                                          _np_ptr(np.ascontiguousarray(parity_present, np.uint64)), _np_ptr(rec), E,
                                          _np_ptr(o_s), _np_ptr(o_h), _np_ptr(o_i))
        return o_s, o_h, o_i, rec

    # -- wire codec ----------------------------------------------------------
    def crc32(self, data: bytes, seed: int = CRC_SEED) -> int:
        b = np.frombuffer(bytes(data), np.uint8)
        return int(self.lib.oracle_crc32(seed, _np_ptr(b), len(b)))

    def frame_fec_batch(self, parity, meta, fsize, status, stamps, capacity, dstride):
        """parity [N][stride] (or [G][n][stride]) -> (dgram [N][dstride], dlen [N])."""
        stride = parity.shape[-1]
        N = parity.size // stride
        dgram = np.zeros((N, dstride), np.uint8)
        dlen = np.zeros(N, np.uint16)
        st = None if status is None else _np_ptr(np.ascontiguousarray(status, np.int8))
        self.lib.oracle_wire_frame_fec_batch(N, stride, capacity, _np_ptr(np.ascontiguousarray(parity)),
                                             _np_ptr(np.ascontiguousarray(meta)),
                                             _np_ptr(np.ascontiguousarray(fsize, np.uint16)), st,
                                             _np_ptr(np.ascontiguousarray(stamps)), dstride, _np_ptr(dgram),
                                             _np_ptr(dlen))
        return dgram, dlen

    def frame_seg_batch(self, shards, hdr, stamps, capacity, dstride):
        stride = shards.shape[-1]
        N = shards.size // stride
        dgram = np.zeros((N, dstride), np.uint8)
        dlen = np.zeros(N, np.uint16)
        self.lib.oracle_wire_frame_seg_batch(N, stride, capacity, _np_ptr(np.ascontiguousarray(shards)),
                                             _np_ptr(np.ascontiguousarray(hdr)), _np_ptr(np.ascontiguousarray(stamps)),
                                             dstride, _np_ptr(dgram), _np_ptr(dlen))
        return dgram, dlen

    def parse_batch(self, dgram, dlen, stride, capacity):
        N, dstride = dgram.shape
        recs = np.zeros(N, WIRE_REC)
        payload = np.zeros((N, stride), np.uint8)
        self.lib.oracle_wire_parse_batch(N, dstride, _np_ptr(np.ascontiguousarray(dgram)),
                                         _np_ptr(np.ascontiguousarray(dlen, np.uint16)), stride, capacity,
                                         _np_ptr(recs), _np_ptr(payload))
        return recs, payload

    # -- sender staging ----------------------------------------------------------
    def sender_init(self):
        st = np.zeros(1, SENDER_STATE)
        self.lib.oracle_sender_init(_np_ptr(st))
        return st

    def sender_plan(self, st, frames, seg_size, max_segs=1 << 16, max_groups=1 << 14):
        segs = np.zeros(max_segs, SEG_PLAN)
        groups = np.zeros(max_groups, GROUP_PLAN)
        ns, ng = C.c_uint32(), C.c_uint32()
        rc = self.lib.oracle_sender_plan(_np_ptr(st), _np_ptr(np.ascontiguousarray(frames)), len(frames), seg_size,
                                         _np_ptr(segs), max_segs, C.byref(ns), _np_ptr(groups), max_groups,
                                         C.byref(ng))
        if rc != 0:
            raise ValueError("sender plan: output arrays too small")
        return segs[:ns.value], groups[:ng.value]

    # -- receiver ingestion ------------------------------------------------------
    def rx_recover(self, recs, payload, capacity, max_ts=0, max_out=1 << 16, evict_every=0):
        """evict_every > 0: sim_fec_evict after every evict_every arrivals."""
        n, stride = payload.shape
        out = np.zeros(max_out, RX_SEG)
        outp = np.zeros((max_out, stride), np.uint8)
        mts, no, dropped = C.c_uint32(max_ts), C.c_uint32(), C.c_uint32()
        rc = self.lib.oracle_rx_recover_ev(n, _np_ptr(np.ascontiguousarray(recs)),
                                           _np_ptr(np.ascontiguousarray(payload)), stride, capacity, C.byref(mts),
                                           _np_ptr(out), _np_ptr(outp), max_out, C.byref(no), C.byref(dropped),
                                           evict_every)
        if rc != 0:
            raise ValueError("rx: output too small")
        return out[:no.value], outp[:no.value], mts.value, dropped.value

    # -- AoS (reference-shaped) path for the CPU baseline ---------------------
    def seg_dtype(self):
        """numpy mirror of sim_segment_t (sim_proto.h:80-99) at this build's SIM_VIDEO_SIZE."""
        return np.dtype({"names": ["packet_id", "fid", "timestamp", "index", "total", "ftype", "payload_type",
                                   "data_size", "data"],
                         "formats": ["<u4", "<u4", "<u4", "<u2", "<u2", "u1", "u1", "<u2", ("u1", self.video_size)],
                         "offsets": [0, 4, 8, 12, 14, 16, 17, 32, 34], "itemsize": self.segment_size})

    def to_aos(self, shards, hdr):
        """sim_segment_t[G*k] (as a structured array) from the device layout."""
        G, k, stride = shards.shape
        seg = np.zeros(G * k, self.seg_dtype())
        h = hdr.reshape(-1)
        for a, b in (("packet_id", "seq"), ("fid", "fid"), ("timestamp", "ts"), ("index", "index"),
                     ("total", "total"), ("ftype", "ftype"), ("payload_type", "payload_type"), ("data_size", "size")):
            seg[a] = h[b]
        n = min(stride, self.video_size)
        seg["data"][:, :n] = shards.reshape(G * k, stride)[:, :n]
        return seg

    def encode_aos(self, plan, groups, seg_bytes, threads=1):
        fec = np.zeros((groups * plan.n_lines, self.fec_size), np.uint8)
        assert seg_bytes.nbytes == groups * plan.k * self.segment_size
        p = _as_oracle_plan(plan)
        if threads > 1:
            n = self.lib.oracle_encode_aos_mt(C.byref(p), groups, _np_ptr(seg_bytes), _np_ptr(fec), threads)
        else:
            n = self.lib.oracle_encode_aos(C.byref(p), groups, _np_ptr(seg_bytes), _np_ptr(fec))
        return n, fec

    def recover_aos(self, plan, groups, seg_bytes, fec_bytes, present, threads=1, out=None):
        out = np.zeros_like(seg_bytes) if out is None else out
        assert seg_bytes.nbytes == groups * plan.k * self.segment_size
        pres = np.ascontiguousarray(present, np.uint64)
        if threads > 1:
            n = self.lib.oracle_recover_aos_mt(C.byref(_as_oracle_plan(plan)), groups, _np_ptr(seg_bytes),
                                               _np_ptr(fec_bytes), _np_ptr(pres), _np_ptr(out), threads)
        else:
            n = self.lib.oracle_recover_aos(C.byref(_as_oracle_plan(plan)), groups, _np_ptr(seg_bytes),
                                            _np_ptr(fec_bytes), _np_ptr(pres), _np_ptr(out))
        return n, out


def _as_oracle_plan(plan) -> rfec_plan:
    if isinstance(plan, rfec_plan):
        return plan
    p = rfec_plan()
    C.memmove(C.byref(p), C.byref(plan), C.sizeof(p))
    return p


# ---------------------------------------------------------------------------
# golden fixtures
# ---------------------------------------------------------------------------
def manifest() -> dict:
    return json.loads((GOLDEN / "manifest.json").read_text())


def case(name: str) -> dict:
    for c in manifest()["cases"]:
        if c["name"] == name:
            return c
    raise KeyError(name)


def load_parities(c: dict):
    """-> (records, payloads[N, S])"""
    raw = np.fromfile(GOLDEN / c["file"], np.uint8)
    S = c["S"]
    rec_bytes = PARITY_REC.itemsize + S
    raw = raw.reshape(-1, rec_bytes)
    recs = raw[:, :PARITY_REC.itemsize].copy().view(PARITY_REC).reshape(-1)
    return recs, raw[:, PARITY_REC.itemsize:].copy()


def load_erasures(c: dict):
    return np.fromfile(GOLDEN / c["file"], ERASURE_REC)


def wire_manifest() -> dict:
    return json.loads((GOLDEN / "wire_manifest.json").read_text())


def _walk(path, rec_dtype, count, tail):
    """Variable-length records: fixed header, then tail(rec) -> [(name, nbytes)] byte fields."""
    raw = np.fromfile(GOLDEN / path, np.uint8)
    out, off = [], 0
    for _ in range(count):
        r = raw[off:off + rec_dtype.itemsize].copy().view(rec_dtype)[0]
        off += rec_dtype.itemsize
        fields = {}
        for name, nb in tail(r):
            fields[name] = raw[off:off + nb].copy()
            off += nb
        out.append((r, fields))
    assert off == len(raw), f"{path}: {len(raw) - off} trailing bytes"
    return out


def load_wire_fec():
    m = wire_manifest()["fec"]
    return _walk(m["file"], WIRE_FEC_IN, m["count"],
                 lambda r: [("payload", int(r["fec_data_size"])), ("dgram", int(r["dlen"]))])


def load_wire_seg():
    m = wire_manifest()["seg"]
    return _walk(m["file"], WIRE_SEG_IN, m["count"],
                 lambda r: [("payload", int(r["data_size"])), ("dgram", int(r["dlen"]))])


def load_wire_parse():
    m = wire_manifest()["parse"]
    return _walk(m["file"], WIRE_PARSE_IN, m["count"],
                 lambda r: [("dgram", int(r["len"])), ("payload", int(r["rec"]["data_size"]))])


def stage_fixture() -> dict:
    return json.loads((GOLDEN / "stage.json").read_text())


def stage_frames(scn, now_ms=1_700_000_000_000):
    """(frames dtype FRAME with data pointers into `blob`, blob) for a stage.json scenario."""
    sizes = [f[0] for f in scn["frames"]]
    st = C.c_uint64(0x5354414745 ^ scn["id"])
    blob = np.zeros(sum(sizes) + 8, np.uint8)
    off = 0
    for s in sizes:
        words = (s + 7) // 8
        v = np.array([_xs_next(st) for _ in range(words)], np.uint64).view(np.uint8)
        blob[off:off + s] = v[:s]
        off += s
    frames = np.zeros(len(sizes), FRAME)
    off = 0
    for i, f in enumerate(scn["frames"]):
        frames[i]["data"] = blob.ctypes.data + off
        frames[i]["size"], frames[i]["ftype"], frames[i]["payload_type"], frames[i]["protect_fraction"] = f
        frames[i]["now_ms"] = now_ms
        off += f[0]
    return frames, blob


def rx_fixture() -> dict:
    return json.loads((GOLDEN / "rx.json").read_text())


def rx_items(oracle, frames, blob, segs, groups, video_size=1000):
    """Parsed-datagram records (WIRE_REC) + payload rows of everything a sender
    plan emits: (seg_rec, seg_pay, par_rec, par_pay, par_group).  Segment
    headers from the plan (pinned by stage.json), timestamps 33 ms per frame as
    gen_rx.c, parities from the oracle encode (pinned by the enc_* fixtures)."""
    stride = (video_size + 15) // 16 * 16
    ns = len(segs)
    seg_pay = np.zeros((ns, stride), np.uint8)
    base = blob.ctypes.data
    for i, s in enumerate(segs):
        off = int(frames["data"][s["frame"]] - base) + int(s["offset"])
        n = int(s["data_size"])
        seg_pay[i, :n] = blob[off:off + n]
    seg_rec = np.zeros(ns, WIRE_REC)
    seg_rec["mid"], seg_rec["ver"] = 0x17, 1
    for a, b in (("seq", "packet_id"), ("fid", "fid"), ("index", "index"), ("total", "total"), ("ftype", "ftype"),
                 ("payload_type", "payload_type"), ("size", "data_size")):
        seg_rec["hdr"][a] = segs[b]
    seg_rec["hdr"]["ts"] = 33 * segs["frame"]  # gen_rx.c: 33 ms per frame
    seg_rec["fec_id"] = segs["fec_id"]
    seg_rec["data_size"] = segs["data_size"]
    seg_rec["remb"] = 0xFF
    par_rec, par_pay, par_group = [], [], []
    for gi, g in enumerate(groups):
        k, pf = int(g["count"]), int(g["protect_fraction"])
        if int(g["first_seg"]) < 0 or k == 0:
            continue
        if k > 255:  # above the 8-bit plan lines: the sender's lines restated here
            for r in _big_group_parities(oracle, seg_rec, seg_pay, g, k, pf):
                par_rec.append(r[0])
                par_pay.append(r[1])
                par_group.append(gi)
            continue
        plan = oracle.plan_from_fraction(k, pf, 3)
        mem = segs[int(g["first_seg"]):int(g["first_seg"]) + k]
        hdr = np.zeros((1, k), HDR_DTYPE)
        hdr[0] = seg_rec["hdr"][int(g["first_seg"]):int(g["first_seg"]) + k]
        par, meta, fs, _ = oracle.encode_batch(plan, seg_pay[int(g["first_seg"]):int(g["first_seg"]) + k][None], hdr,
                                               video_size)
        close_frame = int(mem["frame"][-1])
        for l in range(plan.n_lines):
            r = np.zeros((), WIRE_REC)
            r["mid"], r["ver"] = 0x1C, 1
            r["fec_id"], r["base_id"], r["count"] = g["fec_id"], g["base_id"], k
            r["row"], r["col"], r["index"] = plan.row, plan.col, plan.line[l].index
            r["send_ts"] = 33 * close_frame
            r["hdr"] = meta[0, l]
            r["data_size"] = fs[0, l]
            par_rec.append(r)
            par_pay.append(par[0, l])
            par_group.append(gi)
    return seg_rec, seg_pay, par_rec, par_pay, par_group


def _big_group_parities(oracle, seg_rec, seg_pay, g, k, pf):
    """The parities flex_fec_sender_update emits for a group of k > 255
    segments (flex_fec_sender.c:146-245): the planner's (row, col)
    (oracle_num_packets, :81-135); with col > 1, one parity per row over
    segments [r col, min(k, (r + 1) col)), index r (:157-188), and in matrix
    mode with row > 1 one per column over r col + c < k, index 0x80 | c
    (:199-233); a
    line of fewer than 2 members emits none (flex_fec_xor.c:9-10).  Each
    parity = flex_fec_generate: payload XOR zero-padded to L = max data_size,
    meta = XOR of the 20-byte headers (flex_fec_xor.c:13-50)."""
    rc, row, col = oracle.num_packets(k, pf)
    f0 = int(g["first_seg"])
    hdr32 = seg_rec["hdr"][f0:f0 + k].copy().view(np.uint32).reshape(k, 5)
    pay = seg_pay[f0:f0 + k]
    sizes = seg_rec["data_size"][f0:f0 + k].astype(np.int64)
    lines = [(list(range(r * col, min(k, (r + 1) * col))), r) for r in range(row)] if col > 1 else []
    if col > 1 and row > 1 and rc == 1:
        lines += [([r * col + c for r in range(row) if r * col + c < k], 0x80 | c) for c in range(col)]
    out = []
    for mem, index in lines:
        if len(mem) < 2:
            continue
        L = int(sizes[mem].max())
        pp = np.bitwise_xor.reduce(pay[mem], axis=0)
        pp[L:] = 0
        m = np.bitwise_xor.reduce(hdr32[mem], axis=0)
        r = np.zeros((), WIRE_REC)
        r["mid"], r["ver"] = 0x1C, 1
        r["fec_id"], r["base_id"], r["count"] = g["fec_id"], g["base_id"], k
        r["row"], r["col"], r["index"] = row, col, index
        r["send_ts"] = 33 * int(seg_rec["hdr"]["ts"][f0 + k - 1] // 33)
        r["hdr"] = m.view(r["hdr"].dtype)[0]
        r["data_size"] = L
        out.append((r, pp))
    return out


def _gather_arrivals(arr, items, stride):
    seg_rec, seg_pay, par_rec, par_pay, _ = items
    recs = np.zeros(len(arr), WIRE_REC)
    pay = np.zeros((len(arr), stride), np.uint8)
    for a, (kind, idx) in enumerate(arr):
        if kind == 0:
            recs[a], pay[a] = seg_rec[idx], seg_pay[idx]
        else:
            recs[a], pay[a] = par_rec[idx], par_pay[idx]
    return recs, pay


def _peer_groups(segs, listed):
    """GROUP_PLAN rows for listed [fec_id, base_id, count, protect_fraction]
    groups over the planned segments (their fec_id / group fields set)."""
    groups = np.zeros(len(listed), GROUP_PLAN)
    first = {int(pid): i for i, pid in enumerate(segs["packet_id"])}
    segs["group"] = -1
    for gi, (fec_id, base_id, count, pf) in enumerate(listed):
        f = first[int(base_id)]
        groups[gi]["first_seg"], groups[gi]["count"], groups[gi]["fec_id"] = f, count, fec_id
        groups[gi]["base_id"], groups[gi]["protect_fraction"] = base_id, pf
        segs["fec_id"][f:f + count] = fec_id
        segs["group"][f:f + count] = gi
    return groups


def rx_stream(oracle, scn, video_size=1000):
    """Parsed-datagram records (WIRE_REC) + payload rows, in the arrival order
    of an rx.json scenario."""
    frames, blob = stage_frames(scn)
    st = oracle.sender_init()
    segs, groups = oracle.sender_plan(st, frames, video_size)
    if int(scn.get("flush_at", 100)) != 100:
        # a foreign peer's sender that closes groups later than razor's 100 (gen_rx.c g_flush_at):
        # the segments are split as razor's, the groups are the scenario's
        groups = _peer_groups(segs, scn["groups"])
    assert [(int(g["fec_id"]), int(g["base_id"]), int(g["count"]), int(g["protect_fraction"])) for g in groups] == \
        [tuple(g) for g in scn["groups"]]
    items = rx_items(oracle, frames, blob, segs, groups, video_size)
    assert [(int(items[2][p]["index"])) for p in range(len(items[2]))] == [q[1] for q in scn["parities"]]
    arr = np.array(scn["arrivals"], np.int64).reshape(-1, 2)
    recs, pay = _gather_arrivals(arr, items, (video_size + 15) // 16 * 16)
    return recs, pay, segs, items[1]


def synth_rx_stream(oracle, frames, blob, segs, groups, rng, loss=0.12, window=40, dup=0.04, late=0.0,
                    late_by=1600, video_size=1000):
    """A lossy network over a sender plan: send order = each segment, and a
    group's parities right after the segment that closes it; each datagram is
    lost with `loss`, delayed by up to `window` positions, duplicated with
    `dup`, and a parity is held back `late_by` positions with `late`."""
    items = rx_items(oracle, frames, blob, segs, groups, video_size)
    closes = {}
    for p, gi in enumerate(items[4]):
        g = groups[gi]
        closes.setdefault(int(g["first_seg"]) + int(g["count"]) - 1, []).append(p)
    order = []
    for i in range(len(segs)):
        order.append((0, i))
        order.extend((1, p) for p in closes.get(i, []))
    keys = []
    for pos, item in enumerate(order):
        if rng.random() < loss:
            continue
        key = pos + int(rng.integers(0, window))
        if item[0] == 1 and rng.random() < late:
            key += late_by
        keys.append((key, pos, item))
        if rng.random() < dup:
            keys.append((key + int(rng.integers(1, 3 * window)), pos, item))
    keys.sort(key=lambda t: (t[0], t[1]))
    return _gather_arrivals([t[2] for t in keys], items, (video_size + 15) // 16 * 16)


def _xs_next(st: C.c_uint64) -> int:
    """xorshift64* (test/common_test.c:10-16), Python side for small inputs."""
    x = st.value
    x ^= x >> 12
    x ^= (x << 25) & 0xFFFFFFFFFFFFFFFF
    x ^= x >> 27
    st.value = x
    return (x * 2685821657736338717) & 0xFFFFFFFFFFFFFFFF


def plan_table() -> np.ndarray:
    return np.fromfile(GOLDEN / "plan_table.bin", np.uint8).reshape(256, 256, 3)


def fnv1a(data: bytes, h: int = 0xCBF29CE484222325) -> int:
    for b in data:
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def seg_hash(hdr_rec: np.void, payload: np.ndarray) -> int:
    """Hash used by gen_golden.c: 20-byte header record + data[0:data_size]."""
    rec = np.array([hdr_rec], HDR_DTYPE).tobytes()
    return fnv1a(payload[: int(hdr_rec["size"])].tobytes(), fnv1a(rec))


def ragged_present_bits(k: int, erased) -> np.ndarray:
    p = np.zeros(2, np.uint64)
    for i in range(k):
        if i not in erased:
            p[i >> 6] |= np.uint64(1 << (i & 63))
    return p
