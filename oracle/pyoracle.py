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
        L.oracle_generate.argtypes = [P, C.c_int, P, C.c_int]
        L.oracle_recover.argtypes = [P, C.c_int, P, P]
        L.oracle_encode_aos.argtypes = [C.POINTER(rfec_plan), C.c_uint32, P, P]
        L.oracle_encode_aos.restype = C.c_long
        L.oracle_encode_aos_mt.argtypes = [C.POINTER(rfec_plan), C.c_uint32, P, P, C.c_int]
        L.oracle_encode_aos_mt.restype = C.c_long
        L.oracle_recover_aos.argtypes = [C.POINTER(rfec_plan), C.c_uint32, P, P, P, P]
        L.oracle_recover_aos.restype = C.c_long
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

    def recover_aos(self, plan, groups, seg_bytes, fec_bytes, present):
        out = np.zeros_like(seg_bytes)
        assert seg_bytes.nbytes == groups * plan.k * self.segment_size
        n = self.lib.oracle_recover_aos(C.byref(_as_oracle_plan(plan)), groups, _np_ptr(seg_bytes),
                                        _np_ptr(fec_bytes), _np_ptr(np.ascontiguousarray(present, np.uint64)),
                                        _np_ptr(out))
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
