"""Python view of the C ABI in include/razor_fec.h (ctypes).

The product is librazor_fec.so (HIP kernels + C host layer).  This module only
loads it, mirrors its structs, and passes device pointers / streams through;
it has no compute path of its own.  Loading fails loudly when the library is
missing, and every call checks the C return code.

Reference interface mirrored (yuanrongxi/razor):
  flex_fec_generate / flex_fec_recover      sim_transport/fec/flex_fec_xor.h:7-8
  flex_fec_sender_num_packets (planner)     sim_transport/fec/flex_fec_sender.c:81-135
  row/column parity lines                   sim_transport/fec/flex_fec_sender.c:158-233
"""
from __future__ import annotations

import ctypes as C
import os
import re
from pathlib import Path

import numpy as np

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
LIBDIR = PKG / "lib"
HEADER = ROOT / "include" / "razor_fec.h"
HEADERS = sorted((ROOT / "include").glob("*.h"))

RFEC_MAX_K = 128
RFEC_MAX_LINES = 64
RFEC_LAYER_ROWS = 1
RFEC_LAYER_COLS = 2
RFEC_TUNE_GENERIC = 1
RFEC_TUNE_NO_SERVICE = 1 << 30

# 20-byte header record == sim_fec_meta_t layout (sim_proto.h:145-155)
HDR_DTYPE = np.dtype([("seq", "<u4"), ("fid", "<u4"), ("ts", "<u4"), ("index", "<u2"), ("total", "<u2"),
                      ("ftype", "u1"), ("payload_type", "u1"), ("size", "<u2")])
assert HDR_DTYPE.itemsize == 20

# wire codec records (include/razor_fec.h)
RFEC_WIRE_SEG = 0x17
RFEC_WIRE_FEC = 0x1C
RFEC_WIRE_FEC_OVERHEAD = 49
FEC_STAMP_DTYPE = np.dtype([("uid", "<u4"), ("base_id", "<u4"), ("send_ts", "<u4"), ("fec_id", "<u2"),
                            ("count", "<u2"), ("transport_seq", "<u2"), ("row", "u1"), ("col", "u1"), ("index", "u1"),
                            ("reserved", "u1"), ("pad", "u1", (2,))])
SEG_STAMP_DTYPE = np.dtype([("uid", "<u4"), ("fec_id", "<u2"), ("send_ts", "<u2"), ("transport_seq", "<u2"),
                            ("remb", "u1"), ("reserved", "u1")])
WIRE_REC_DTYPE = np.dtype([("status", "i1"), ("ver", "u1"), ("mid", "u1"), ("remb", "u1"), ("uid", "<u4"),
                           ("hdr", HDR_DTYPE), ("base_id", "<u4"), ("send_ts", "<u4"), ("fec_id", "<u2"),
                           ("count", "<u2"), ("transport_seq", "<u2"), ("data_size", "<u2"), ("row", "u1"),
                           ("col", "u1"), ("index", "u1"), ("reserved", "u1", (17,))])
assert FEC_STAMP_DTYPE.itemsize == 24 and SEG_STAMP_DTYPE.itemsize == 12 and WIRE_REC_DTYPE.itemsize == 64

# sender staging (include/razor_fec.h)
FRAME_DTYPE = np.dtype([("data", "<u8"), ("size", "<u4"), ("payload_type", "u1"), ("ftype", "u1"),
                        ("protect_fraction", "u1"), ("reserved", "u1"), ("now_ms", "<i8")])
SENDER_STATE_DTYPE = np.dtype([("packet_id_seed", "<u4"), ("send_id_seed", "<u4"), ("frame_id_seed", "<u4"),
                               ("pad0", "<u4"), ("first_ts", "<i8"), ("fec_ts", "<i8"), ("base_id", "<u4"),
                               ("open_seg", "<i4"), ("fec_id", "<u2"), ("segs_count", "<u2"), ("first", "<i4"),
                               ("transport_seq_seed", "<u4"), ("pad1", "<u4")])
SEG_PLAN_DTYPE = np.dtype([("frame", "<u4"), ("offset", "<u4"), ("packet_id", "<u4"), ("send_id", "<u4"),
                           ("fid", "<u4"), ("timestamp", "<u4"), ("index", "<u2"), ("total", "<u2"),
                           ("data_size", "<u2"), ("fec_id", "<u2"), ("ftype", "u1"), ("payload_type", "u1"),
                           ("reserved", "u1", (2,)), ("group", "<i4")])
GROUP_PLAN_DTYPE = np.dtype([("first_seg", "<i4"), ("count", "<u2"), ("fec_id", "<u2"), ("base_id", "<u4"),
                             ("fec_send_id0", "<u4"), ("fec_ts", "<u4"), ("protect_fraction", "u1"),
                             ("n_lines", "u1"), ("reserved", "u1", (2,))])
RX_SEG_DTYPE = np.dtype([("hdr", HDR_DTYPE), ("fec_id", "<u2"), ("reserved", "<u2")])
assert RX_SEG_DTYPE.itemsize == 24


class rfec_rx_report(C.Structure):
    _fields_ = [("n_groups", C.c_uint32), ("n_shapes", C.c_uint32), ("n_recovered", C.c_uint32),
                ("n_fec_dropped", C.c_uint32), ("n_unmodelled", C.c_uint32), ("reserved", C.c_uint32),
                ("host_us", C.c_double), ("h2d_us", C.c_double), ("kernel_us", C.c_double),
                ("d2h_us", C.c_double), ("total_us", C.c_double)]


class rfec_send_report(C.Structure):
    _fields_ = [("n_segs", C.c_uint32), ("n_groups", C.c_uint32), ("n_parities", C.c_uint32),
                ("n_shapes", C.c_uint32), ("plan_us", C.c_double), ("stage_us", C.c_double),
                ("h2d_us", C.c_double), ("kernel_us", C.c_double), ("d2h_us", C.c_double),
                ("total_us", C.c_double), ("zero_copy", C.c_uint32), ("reserved", C.c_uint32)]


class rfec_rx_session_info(C.Structure):
    _fields_ = [("max_ts", C.c_uint32), ("open_flexes", C.c_uint32), ("cached_segments", C.c_uint32),
                ("records_held", C.c_uint32), ("rows_held", C.c_uint32), ("pending", C.c_uint32),
                ("threads", C.c_uint32), ("batches_parallel", C.c_uint32), ("batches_serial", C.c_uint32),
                ("batches_rolled_back", C.c_uint32), ("reserved", C.c_uint32), ("split_us", C.c_double),
                ("replay_us", C.c_double), ("verify_us", C.c_double), ("tables_us", C.c_double),
                ("compact_us", C.c_double)]


assert C.sizeof(rfec_rx_session_info) == 88


class rfec_service_info(C.Structure):
    _fields_ = [("jobs", C.c_uint64), ("launches", C.c_uint64), ("stage_host_us", C.c_double),
                ("wait_us", C.c_double), ("dev_stage_us", C.c_double), ("dev_work_us", C.c_double),
                ("dev_release_us", C.c_double), ("request_in_device", C.c_uint32), ("reserved", C.c_uint32)]


class rfec_udp_addr(C.Structure):
    _fields_ = [("ip", C.c_uint32), ("port", C.c_uint16), ("reserved", C.c_uint16)]


class rfec_udp_stats(C.Structure):
    _fields_ = [("datagrams", C.c_uint64), ("bytes", C.c_uint64), ("skipped", C.c_uint64), ("dropped", C.c_uint64),
                ("truncated", C.c_uint64), ("syscalls", C.c_uint64), ("stalls", C.c_uint64)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


RFEC_EAGAIN = -4
RFEC_UDP_SERVER = 1
RFEC_UDP_RECV_BYTES = 1500
RFEC_UDP_MIN_DGRAM = 6
UDP_ADDR_DTYPE = np.dtype([("ip", "<u4"), ("port", "<u2"), ("reserved", "<u2")])


class RfecError(RuntimeError):
    pass


class rfec_line(C.Structure):
    _fields_ = [("first", C.c_uint8), ("stride", C.c_uint8), ("count", C.c_uint8), ("index", C.c_uint8)]


class rfec_plan(C.Structure):
    _fields_ = [("k", C.c_uint16), ("row", C.c_uint8), ("col", C.c_uint8), ("rc", C.c_uint8),
                ("n_lines", C.c_uint8), ("n_row_lines", C.c_uint8), ("reserved", C.c_uint8),
                ("line", rfec_line * RFEC_MAX_LINES)]

    def lines(self):
        return [(self.line[i].first, self.line[i].stride, self.line[i].count, self.line[i].index)
                for i in range(self.n_lines)]

    def members(self, l):
        ln = self.line[l]
        return [ln.first + q * ln.stride for q in range(ln.count)]

    def __repr__(self):
        return (f"rfec_plan(k={self.k}, row={self.row}, col={self.col}, rc={self.rc}, "
                f"n_lines={self.n_lines}, lines={self.lines()})")


class rfec_host_timing(C.Structure):
    _fields_ = [("gather_us", C.c_double), ("h2d_us", C.c_double), ("kernel_us", C.c_double),
                ("d2h_us", C.c_double), ("scatter_us", C.c_double), ("total_us", C.c_double),
                ("zero_copy", C.c_uint32), ("reserved", C.c_uint32)]


RFEC_ABI_VERSION = 7  # include/razor_fec.h


def seg_dtype(video_size: int) -> np.dtype:
    """numpy mirror of sim_segment_t (sim_proto.h:80-99)."""
    size = ((34 + video_size + 3) // 4) * 4
    return np.dtype({"names": ["packet_id", "fid", "timestamp", "index", "total", "ftype", "payload_type",
                               "fec_id", "data_size", "data"],
                     "formats": ["<u4", "<u4", "<u4", "<u2", "<u2", "u1", "u1", "<u2", "<u2", ("u1", video_size)],
                     "offsets": [0, 4, 8, 12, 14, 16, 17, 20, 32, 34], "itemsize": size})


def fec_dtype(video_size: int) -> np.dtype:
    """numpy mirror of sim_fec_t (sim_proto.h:157-174)."""
    size = ((42 + video_size + 3) // 4) * 4
    return np.dtype({"names": ["fec_id", "row", "col", "index", "count", "base_id", "meta", "fec_data_size",
                               "fec_data"],
                     "formats": ["<u2", "u1", "u1", "u1", "<u2", "<u4", HDR_DTYPE, "<u2", ("u1", video_size)],
                     "offsets": [0, 2, 3, 4, 6, 8, 20, 40, 42], "itemsize": size})


def sim_types(video_size: int):
    """ctypes mirrors of sim_segment_t / sim_fec_t (sim_proto.h:80-99, 157-174)."""

    class sim_segment_t(C.Structure):
        _fields_ = [("packet_id", C.c_uint32), ("fid", C.c_uint32), ("timestamp", C.c_uint32),
                    ("index", C.c_uint16), ("total", C.c_uint16), ("ftype", C.c_uint8),
                    ("payload_type", C.c_uint8), ("remb", C.c_uint8), ("fec_id", C.c_uint16),
                    ("send_ts", C.c_uint16), ("transport_seq", C.c_uint16), ("send_id", C.c_uint32),
                    ("data_size", C.c_uint16), ("data", C.c_uint8 * video_size)]

    class sim_fec_meta_t(C.Structure):
        _fields_ = [("seq", C.c_uint32), ("fid", C.c_uint32), ("ts", C.c_uint32), ("index", C.c_uint16),
                    ("total", C.c_uint16), ("ftype", C.c_uint8), ("payload_type", C.c_uint8),
                    ("size", C.c_uint16)]

    class sim_fec_t(C.Structure):
        _fields_ = [("fec_id", C.c_uint16), ("row", C.c_uint8), ("col", C.c_uint8), ("index", C.c_uint8),
                    ("count", C.c_uint16), ("base_id", C.c_uint32), ("send_ts", C.c_uint32),
                    ("transport_seq", C.c_uint16), ("fec_meta", sim_fec_meta_t), ("fec_data_size", C.c_uint16),
                    ("fec_data", C.c_uint8 * video_size)]

    assert C.sizeof(sim_fec_meta_t) == 20
    assert C.sizeof(sim_segment_t) == ((34 + video_size + 3) // 4) * 4
    return sim_segment_t, sim_fec_t


_P = C.c_void_p
_SIGS = {
    "flex_fec_generate": (C.c_int, [_P, C.c_int, _P]),
    "flex_fec_recover": (C.c_int, [_P, C.c_int, _P, _P]),
    "rfec_sim_video_size": (C.c_int, []),
    "rfec_abi_version": (C.c_uint32, []),
    "rfec_num_packets": (C.c_int, [C.c_uint16, C.c_uint8, C.POINTER(C.c_uint8), C.POINTER(C.c_uint8)]),
    "rfec_plan_from_fraction": (C.c_int, [C.c_uint16, C.c_uint8, C.c_uint, C.POINTER(rfec_plan)]),
    "rfec_plan_matrix": (C.c_int, [C.c_uint16, C.c_uint8, C.c_uint8, C.c_uint, C.POINTER(rfec_plan)]),
    "rfec_encode_batch": (C.c_int, [C.POINTER(rfec_plan), C.c_uint32, C.c_uint32, C.c_uint32,
                                    _P, _P, _P, _P, _P, _P, _P]),
    "rfec_recover_workspace_size": (C.c_size_t, [C.POINTER(rfec_plan), C.c_uint32]),
    "rfec_recover_batch": (C.c_int, [C.POINTER(rfec_plan), C.c_uint32, C.c_uint32, C.c_uint32,
                                     _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "rfec_recover_batch_out": (C.c_int, [C.POINTER(rfec_plan), C.c_uint32, C.c_uint32, C.c_uint32,
                                         _P, _P, _P, _P, _P, _P, _P, _P, C.c_uint32, _P, _P, _P, _P, _P]),
    "rfec_packed_stride": (C.c_size_t, [C.POINTER(rfec_plan), C.c_uint32]),
    "rfec_pack_erasures": (C.c_int, [C.POINTER(rfec_plan), C.c_uint32, _P, _P, _P, _P, _P, C.c_uint32, _P, _P]),
    "rfec_recover_packed_out": (C.c_int, [C.POINTER(rfec_plan), C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P, _P,
                                          C.c_uint32, _P, _P, _P, _P]),
    "rfec_zero_tails": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P]),
    "rfec_timing_events": (C.c_int, [_P, _P]),
    "rfec_timing_launches": (C.c_uint32, []),
    "rfec_wire_frame_fec": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P, _P, _P, _P, C.c_uint32, _P,
                                      _P, _P]),
    "rfec_wire_frame_seg": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P, _P, C.c_uint32, _P, _P, _P]),
    "rfec_wire_parse": (C.c_int, [C.c_uint32, C.c_uint32, _P, _P, C.c_uint32, C.c_uint32, _P, _P, _P]),
    "rfec_sender_init": (None, [_P]),
    "rfec_sender_plan": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, _P, C.c_uint32, _P, _P, C.c_uint32, _P]),
    "rfec_host_send_frames": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, _P, C.c_uint32, _P, C.c_uint32,
                                        C.c_uint32, _P, _P, _P, _P, C.c_uint32, C.POINTER(rfec_send_report)]),
    "rfec_rx_recover": (C.c_int, [C.c_uint32, _P, _P, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), _P, _P,
                                  C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(rfec_rx_report), _P]),
    "rfec_set_tuning": (None, [C.c_uint]),
    "rfec_get_tuning": (C.c_uint, []),
    "rfec_service_stop": (C.c_int, []),
    "rfec_service_get_info": (C.c_int, [C.c_void_p]),
    "rfec_last_error": (C.c_char_p, []),
    "rfec_host_encode_groups": (C.c_int, [C.POINTER(rfec_plan), C.c_uint32, _P, _P, C.c_uint16, _P]),
    "rfec_host_recover_groups": (C.c_int, [C.POINTER(rfec_plan), C.c_uint32, _P, _P, C.c_uint32, _P, _P, _P, _P]),
    "rfec_probe_read": (C.c_int, [_P, C.c_size_t, _P, C.c_uint, _P]),
    "rfec_probe_copy": (C.c_int, [_P, _P, C.c_size_t, C.c_uint, _P]),
    "rfec_probe_write": (C.c_int, [_P, C.c_size_t, C.c_uint, _P]),
    "rfec_probe_mix": (C.c_int, [_P, _P, C.c_size_t, C.c_uint, C.c_uint, _P]),
    "rfec_fill_xorshift": (C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P]),
    "rfec_xorshift_jump": (C.c_uint64, [C.c_uint64, C.c_uint64]),
    "rfec_udp_open": (C.c_int, [C.c_char_p, C.c_uint16, C.c_uint, C.c_uint32, C.POINTER(C.c_int),
                                C.POINTER(rfec_udp_addr)]),
    "rfec_udp_close": (None, [C.c_int]),
    "rfec_udp_addr_of": (C.c_int, [C.c_char_p, C.c_uint16, C.POINTER(rfec_udp_addr)]),
    "rfec_udp_send_batch": (C.c_int, [C.c_int, C.POINTER(rfec_udp_addr), C.c_uint32, C.c_uint32, _P, _P, C.c_uint32,
                                      C.POINTER(C.c_uint32), C.POINTER(rfec_udp_stats)]),
    "rfec_udp_recv_batch": (C.c_int, [C.c_int, C.c_uint32, C.c_uint32, _P, _P, _P, C.c_uint32,
                                      C.POINTER(C.c_uint32), C.POINTER(rfec_udp_stats)]),
    "rfec_host_recv_datagrams": (C.c_int, [C.c_uint32, C.c_uint32, _P, _P, C.c_uint32, C.c_uint32,
                                           C.POINTER(C.c_uint32), _P, _P, _P, C.c_uint32, C.POINTER(C.c_uint32),
                                           C.POINTER(rfec_rx_report)]),
    "rfec_pinned_alloc": (_P, [C.c_size_t]),
    "rfec_rx_session_create": (_P, [C.c_uint32, C.c_uint32]),
    "rfec_rx_session_destroy": (None, [_P]),
    "rfec_rx_session_push": (C.c_int, [_P, C.c_uint32, _P, _P, _P, _P, C.c_uint32, C.POINTER(C.c_uint32),
                                       C.POINTER(rfec_rx_report), _P]),
    "rfec_rx_session_push_datagrams": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _P, _P, _P, _P, C.c_uint32,
                                                 C.POINTER(C.c_uint32), C.POINTER(rfec_rx_report)]),
    "rfec_rx_session_push_datagrams_async": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _P, _P, _P, _P, C.c_uint32,
                                                       C.POINTER(C.c_uint32), C.POINTER(rfec_rx_report)]),
    "rfec_rx_session_evict": (C.c_int, [_P, _P]),
    "rfec_rx_session_get_info": (C.c_int, [_P, C.POINTER(rfec_rx_session_info)]),
    "rfec_rx_session_set_threads": (C.c_int, [_P, C.c_uint32]),
    "rfec_pinned_free": (None, [_P]),
}


def header_functions() -> list[str]:
    """Every function declared in include/*.h."""
    text = "\n".join(h.read_text() for h in HEADERS)
    text = re.sub(r"^\s*typedef[^;]*;", "", text, flags=re.M)  # function-pointer typedefs
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b([a-z_][a-z0-9_]*)\s*\(", text, flags=re.M)))


def as_plan(p) -> rfec_plan:
    """Accepts any ctypes struct with rfec_plan's layout (e.g. the oracle's)."""
    if isinstance(p, rfec_plan):
        return p
    if C.sizeof(p) != C.sizeof(rfec_plan):
        raise TypeError("not an rfec_plan")
    q = rfec_plan()
    C.memmove(C.byref(q), C.byref(p), C.sizeof(q))
    return q


class Native:
    """One loaded variant of librazor_fec.so."""

    def __init__(self, video_size: int = 1000, path: str | os.PathLike | None = None):
        name = "librazor_fec.so" if video_size == 1000 else f"librazor_fec_v{video_size}.so"
        self.path = Path(path) if path else LIBDIR / name
        if not self.path.exists():
            raise RfecError(f"{self.path} is missing: build it with `python -m razor_amd.build` "
                            "(there is no fallback path)")
        # One HIP runtime per process: torch bundles its own libamdhip64 (soname
        # libamdhip64.so.7, but its users link it by file name), so it must be
        # loaded before this library, whose libamdhip64.so.7 then resolves to it.
        # Loaded the other way round, the process holds two runtimes and the
        # second one to initialise sees no device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        self.lib = C.CDLL(str(self.path))
        for fn, (res, args) in _SIGS.items():
            try:
                f = getattr(self.lib, fn)
            except AttributeError:
                if path is None:  # the product library exports every symbol
                    raise
                continue  # a test build of the host layer alone (tests/host_stub)
            f.restype = res
            f.argtypes = args
        self.video_size = self.lib.rfec_sim_video_size()
        if self.video_size != video_size:
            raise RfecError(f"{self.path} was built with SIM_VIDEO_SIZE={self.video_size}")
        abi = self.lib.rfec_abi_version() if hasattr(self.lib, "rfec_abi_version") else RFEC_ABI_VERSION
        if abi != RFEC_ABI_VERSION:
            raise RfecError(f"{self.path}: ABI {abi}, these bindings expect {RFEC_ABI_VERSION}")
        self.sim_segment_t, self.sim_fec_t = sim_types(self.video_size)

    # -- planner -------------------------------------------------------------
    def num_packets(self, k: int, protect_fraction: int):
        r, c = C.c_uint8(), C.c_uint8()
        rc = self.lib.rfec_num_packets(k, protect_fraction, C.byref(r), C.byref(c))
        return rc, r.value, c.value

    def plan_from_fraction(self, k: int, protect_fraction: int, layers: int = RFEC_LAYER_ROWS | RFEC_LAYER_COLS):
        p = rfec_plan()
        self._check(self.lib.rfec_plan_from_fraction(k, protect_fraction, layers, C.byref(p)), "plan")
        return p

    def plan_matrix(self, k: int, row: int, col: int, layers: int = RFEC_LAYER_ROWS | RFEC_LAYER_COLS):
        p = rfec_plan()
        self._check(self.lib.rfec_plan_matrix(k, row, col, layers, C.byref(p)), "plan")
        return p

    # -- batched device API (pointers are device addresses as ints) ----------
    def encode_batch(self, plan, groups, stride, capacity, shards, hdr, parity, meta, fec_size, status,
                     stream=None):
        self._check(self.lib.rfec_encode_batch(C.byref(as_plan(plan)), groups, stride, capacity, shards, hdr, parity,
                                               meta, fec_size, status, stream), "rfec_encode_batch")

    def fill_xorshift(self, shards, config_id, g0, groups, k, S, stride, stream=None):
        """SURVEY §8(d) synthetic payloads of groups [g0, g0 + groups) into the
        device slots at `shards` (bench / test inputs; jump-ahead per slot)."""
        self._check(self.lib.rfec_fill_xorshift(shards, config_id, g0, groups, k, S, stride, stream),
                    "rfec_fill_xorshift")

    def workspace_size(self, plan, groups) -> int:
        return self.lib.rfec_recover_workspace_size(C.byref(as_plan(plan)), groups)

    def recover_batch(self, plan, groups, stride, capacity, shards, hdr, present, parity, meta, fec_size,
                      parity_present, recovered, workspace, stream=None):
        self._check(self.lib.rfec_recover_batch(C.byref(as_plan(plan)), groups, stride, capacity, shards, hdr, present,
                                                parity, meta, fec_size, parity_present, recovered, workspace,
                                                stream), "rfec_recover_batch")

    def recover_batch_out(self, plan, groups, stride, capacity, shards, hdr, present, parity, meta, fec_size,
                          parity_present, recovered, per_group, out_shards, out_hdr, out_index, workspace,
                          stream=None):
        self._check(self.lib.rfec_recover_batch_out(C.byref(as_plan(plan)), groups, stride, capacity, shards, hdr,
                                                    present, parity, meta, fec_size, parity_present, recovered,
                                                    per_group, out_shards, out_hdr, out_index, workspace, stream),
                    "rfec_recover_batch_out")

    def packed_stride(self, plan, per_group) -> int:
        """rfec_packed_stride: bytes per group record (0: not a packed layout)."""
        return self.lib.rfec_packed_stride(C.byref(as_plan(plan)), per_group)

    def pack_erasures(self, plan, groups, hdr, present, meta, fec_size, parity_present, per_group, packed,
                      stream=None):
        self._check(self.lib.rfec_pack_erasures(C.byref(as_plan(plan)), groups, hdr, present, meta, fec_size,
                                                parity_present, per_group, packed, stream), "rfec_pack_erasures")

    def recover_packed_out(self, plan, groups, stride, capacity, shards, parity, packed, recovered, per_group,
                           out_shards, out_hdr, out_index, stream=None):
        self._check(self.lib.rfec_recover_packed_out(C.byref(as_plan(plan)), groups, stride, capacity, shards, parity,
                                                     packed, recovered, per_group, out_shards, out_hdr, out_index,
                                                     stream), "rfec_recover_packed_out")

    def host_encode_groups(self, plan, groups, seg_ptrs, fec_ptrs, fec_id0=1):
        """seg_ptrs / fec_ptrs: host addresses (uint64 numpy arrays) of the
        sim_segment_t / sim_fec_t structs; returns the per-stage timing (us)."""
        t = rfec_host_timing()
        seg_ptrs = np.ascontiguousarray(seg_ptrs, np.uint64)
        fec_ptrs = np.ascontiguousarray(fec_ptrs, np.uint64)
        self._check(self.lib.rfec_host_encode_groups(C.byref(as_plan(plan)), groups, seg_ptrs.ctypes.data,
                                                     fec_ptrs.ctypes.data, fec_id0, C.addressof(t)),
                    "rfec_host_encode_groups")
        return {f: getattr(t, f) for f, _ in rfec_host_timing._fields_}

    def host_recover_groups(self, plan, groups, seg_ptrs, fec_ptrs, per_group, out_ptrs):
        """rfec_host_recover_groups: seg_ptrs [G*k] / fec_ptrs [G*n] host addresses of
        the received sim_segment_t / sim_fec_t (0 = lost), out_ptrs [G*per_group] the
        out_seg structs; returns (out_index [G][per_group] u8, recovered [G][2] u64,
        per-stage timing in us)."""
        t = rfec_host_timing()
        seg_ptrs = np.ascontiguousarray(seg_ptrs, np.uint64)
        fec_ptrs = np.ascontiguousarray(fec_ptrs, np.uint64)
        out_ptrs = np.ascontiguousarray(out_ptrs, np.uint64)
        oi = np.zeros((groups, per_group), np.uint8)
        rec = np.zeros((groups, 2), np.uint64)
        self._check(self.lib.rfec_host_recover_groups(C.byref(as_plan(plan)), groups, seg_ptrs.ctypes.data,
                                                      fec_ptrs.ctypes.data, per_group, out_ptrs.ctypes.data,
                                                      oi.ctypes.data, rec.ctypes.data, C.addressof(t)),
                    "rfec_host_recover_groups")
        return oi, rec, {f: getattr(t, f) for f, _ in rfec_host_timing._fields_}

    def timing_events(self, start, stop):
        """The next kernel this thread launches records its own start / stop on
        these hipEvent_t handles (rfec_timing_events)."""
        self.lib.rfec_timing_events(start, stop)

    def timing_launches(self) -> int:
        return int(self.lib.rfec_timing_launches())

    def zero_tails(self, groups, k, stride, shards, hdr, stream=None):
        self._check(self.lib.rfec_zero_tails(groups, k, stride, shards, hdr, stream), "rfec_zero_tails")

    # -- wire codec (device pointers) -------------------------------------------
    def wire_frame_fec(self, count, stride, capacity, parity, meta, fec_size, status, stamps, dstride, dgram, dlen,
                       stream=None, order=None):
        self._check(self.lib.rfec_wire_frame_fec(count, stride, capacity, parity, meta, fec_size, status, stamps,
                                                 order, dstride, dgram, dlen, stream), "rfec_wire_frame_fec")

    def wire_frame_seg(self, count, stride, capacity, shards, hdr, stamps, dstride, dgram, dlen, stream=None,
                       order=None):
        self._check(self.lib.rfec_wire_frame_seg(count, stride, capacity, shards, hdr, stamps, order, dstride, dgram,
                                                 dlen, stream), "rfec_wire_frame_seg")

    def wire_parse(self, n, dstride, dgram, dlen, stride, capacity, recs, payload, stream=None):
        self._check(self.lib.rfec_wire_parse(n, dstride, dgram, dlen, stride, capacity, recs, payload, stream),
                    "rfec_wire_parse")

    # -- sender staging (host memory) -------------------------------------------
    def sender_init(self):
        st = np.zeros(1, SENDER_STATE_DTYPE)
        self.lib.rfec_sender_init(st.ctypes.data)
        return st

    def sender_plan(self, st, frames, seg_size, max_segs=1 << 16, max_groups=1 << 14):
        segs = np.zeros(max_segs, SEG_PLAN_DTYPE)
        groups = np.zeros(max_groups, GROUP_PLAN_DTYPE)
        ns, ng = C.c_uint32(), C.c_uint32()
        self._check(self.lib.rfec_sender_plan(st.ctypes.data, np.ascontiguousarray(frames).ctypes.data, len(frames),
                                              seg_size, segs.ctypes.data, max_segs, C.byref(ns), groups.ctypes.data,
                                              max_groups, C.byref(ng)), "rfec_sender_plan")
        return segs[:ns.value], groups[:ng.value]

    def send_frames(self, st, frames, uid, dstride, max_segs=1 << 16, max_groups=1 << 14, max_parities=1 << 17,
                    bufs=None):
        """Frames -> (segs, groups, seg datagrams, seg lengths, fec datagrams, fec lengths, report).
        bufs: optional (sdg, sdl, fdg, fdl) output arrays to reuse (e.g. views of
        pinned memory from pinned_array), sized for max_segs / max_parities."""
        segs = np.zeros(max_segs, SEG_PLAN_DTYPE)
        groups = np.zeros(max_groups, GROUP_PLAN_DTYPE)
        if bufs is None:
            sdg = np.zeros((max_segs, dstride), np.uint8)
            sdl = np.zeros(max_segs, np.uint16)
            fdg = np.zeros((max_parities, dstride), np.uint8)
            fdl = np.zeros(max_parities, np.uint16)
        else:
            sdg, sdl, fdg, fdl = bufs
            assert sdg.shape[0] >= max_segs and fdg.shape[0] >= max_parities and sdg.shape[1] == dstride
        rep = rfec_send_report()
        self._check(self.lib.rfec_host_send_frames(st.ctypes.data, np.ascontiguousarray(frames).ctypes.data,
                                                   len(frames), uid, segs.ctypes.data, max_segs, groups.ctypes.data,
                                                   max_groups, dstride, sdg.ctypes.data, sdl.ctypes.data,
                                                   fdg.ctypes.data, fdl.ctypes.data, max_parities, C.byref(rep)),
                    "rfec_host_send_frames")
        ns, ng, npar = rep.n_segs, rep.n_groups, rep.n_parities
        return segs[:ns], groups[:ng], sdg[:ns], sdl[:ns], fdg[:npar], fdl[:npar], rep

    # -- receiver ingestion ---------------------------------------------------------
    def rx_recover(self, n, recs, payload, stride, capacity, max_ts=0, max_out=1 << 16, stream=None):
        """recs / payload: device pointers (rfec_wire_parse output, arrival order).
        Returns (segments, payload rows, max_ts, report), segments ascending packet_id."""
        out = np.zeros(max_out, RX_SEG_DTYPE)
        outp = np.zeros((max_out, stride), np.uint8)
        mts, nout, rep = C.c_uint32(max_ts), C.c_uint32(), rfec_rx_report()
        self._check(self.lib.rfec_rx_recover(n, recs, payload, stride, capacity, C.byref(mts), out.ctypes.data,
                                             outp.ctypes.data, max_out, C.byref(nout), C.byref(rep), stream),
                    "rfec_rx_recover")
        return out[:nout.value], outp[:nout.value], mts.value, rep

    def host_recv_datagrams(self, n, dstride, dgram, dlen, stride, capacity, max_ts=0, max_out=1 << 16,
                            want_recs=False):
        """dgram / dlen: HOST addresses of n received datagram slots.  Returns
        (segments, payload rows, max_ts, report, recs or None)."""
        out = np.zeros(max_out, RX_SEG_DTYPE)
        outp = np.zeros((max_out, stride), np.uint8)
        recs = np.zeros(n, WIRE_REC_DTYPE) if want_recs else None
        mts, nout, rep = C.c_uint32(max_ts), C.c_uint32(), rfec_rx_report()
        self._check(self.lib.rfec_host_recv_datagrams(n, dstride, dgram, dlen, stride, capacity, C.byref(mts),
                                                      None if recs is None else recs.ctypes.data, out.ctypes.data,
                                                      outp.ctypes.data, max_out, C.byref(nout), C.byref(rep)),
                    "rfec_host_recv_datagrams")
        return out[:nout.value], outp[:nout.value], mts.value, rep, recs

    def pinned_array(self, shape, dtype):
        """A numpy array over rfec_pinned_alloc memory (freed with the array's keeper: keep `.base` alive)."""
        dt = np.dtype(dtype)
        n = int(np.prod(shape)) * dt.itemsize
        p = self.lib.rfec_pinned_alloc(max(n, 1))
        if not p:
            raise RfecError(f"rfec_pinned_alloc({n}) failed: {self.last_error()}")
        keeper = _Pinned(self, p, n)
        arr = np.frombuffer((C.c_uint8 * n).from_address(p), dtype=dt).reshape(shape)
        keeper.arr = arr
        return arr, keeper

    def rx_session(self, stride, capacity, threads=0):
        """threads: control-plane shards (0: the library's default, RFEC_RX_THREADS or 8; 1: serial)."""
        return RxSession(self, stride, capacity, threads)

    # -- batched UDP I/O (host memory) -------------------------------------------
    def udp_open(self, ip="127.0.0.1", port=0, flags=RFEC_UDP_SERVER, buf_bytes=0):
        """Returns (fd, bound rfec_udp_addr)."""
        fd, a = C.c_int(-1), rfec_udp_addr()
        self._check(self.lib.rfec_udp_open(ip.encode() if ip else None, port, flags, buf_bytes, C.byref(fd),
                                           C.byref(a)), "rfec_udp_open")
        return fd.value, a

    def udp_close(self, fd):
        self.lib.rfec_udp_close(fd)

    def udp_addr(self, ip, port):
        a = rfec_udp_addr()
        self._check(self.lib.rfec_udp_addr_of(ip.encode(), port, C.byref(a)), "rfec_udp_addr_of")
        return a

    def udp_send(self, fd, peer, n, dstride, dgram, dlen, wait_ms=100, stats=None):
        """dgram / dlen: host addresses.  Returns (rc, slots consumed); rc is
        0 or RFEC_EAGAIN, other errors raise."""
        done = C.c_uint32()
        rc = self.lib.rfec_udp_send_batch(fd, C.byref(peer), n, dstride, dgram, dlen, wait_ms, C.byref(done),
                                          None if stats is None else C.byref(stats))
        if rc not in (0, RFEC_EAGAIN):
            self._check(rc, "rfec_udp_send_batch")
        return rc, done.value

    def udp_recv(self, fd, max_n, dstride, dgram, dlen, wait_ms=5, stats=None, src=None):
        """dgram / dlen / src (UDP_ADDR_DTYPE array or None): host addresses.
        Returns the number of datagrams stored."""
        n = C.c_uint32()
        self._check(self.lib.rfec_udp_recv_batch(fd, max_n, dstride, dgram, dlen,
                                                 None if src is None else src.ctypes.data, wait_ms, C.byref(n),
                                                 None if stats is None else C.byref(stats)), "rfec_udp_recv_batch")
        return n.value

    def set_tuning(self, flags: int):
        self.lib.rfec_set_tuning(flags)

    def get_tuning(self) -> int:
        return self.lib.rfec_get_tuning()

    # -- drop-in symbols --------------------------------------------------------
    def flex_fec_generate(self, segs, fec) -> int:
        arr = (C.c_void_p * max(1, len(segs)))(*[C.addressof(s) for s in segs])
        return self.lib.flex_fec_generate(arr, len(segs), C.byref(fec))

    def flex_fec_recover(self, segs, fec, out_seg, count=None) -> int:
        arr = (C.c_void_p * max(1, len(segs)))(*[C.addressof(s) for s in segs])
        n = len(segs) if count is None else count
        return self.lib.flex_fec_recover(arr, n, C.byref(fec), C.byref(out_seg))

    def last_error(self) -> str:
        v = self.lib.rfec_last_error()
        return v.decode() if v else ""

    def _check(self, rc, what):
        if rc != 0:
            raise RfecError(f"{what} failed ({rc}): {self.last_error()}")


class _Pinned:
    def __init__(self, native, p, n):
        self.native, self.p, self.n = native, p, n

    def __del__(self):
        try:
            self.native.lib.rfec_pinned_free(self.p)
        except Exception:
            pass


class RxSession:
    """rfec_rx_session: receiver-side FEC state kept across batches."""

    def __init__(self, native: Native, stride: int, capacity: int, threads: int = 0):
        self.n, self.stride = native, stride
        self.h = native.lib.rfec_rx_session_create(stride, capacity)
        if not self.h:
            raise RfecError(f"rfec_rx_session_create failed: {native.last_error()}")
        if threads:
            native._check(native.lib.rfec_rx_session_set_threads(self.h, threads), "rfec_rx_session_set_threads")

    def push(self, n, recs, payload, max_out=1 << 16, stream=None):
        """recs / payload: DEVICE addresses.  Returns (segments, payload rows, report)."""
        out = np.zeros(max_out, RX_SEG_DTYPE)
        outp = np.zeros((max_out, self.stride), np.uint8)
        nout, rep = C.c_uint32(), rfec_rx_report()
        self.n._check(self.n.lib.rfec_rx_session_push(self.h, n, recs, payload, out.ctypes.data, outp.ctypes.data,
                                                      max_out, C.byref(nout), C.byref(rep), stream),
                      "rfec_rx_session_push")
        return out[:nout.value], outp[:nout.value], rep

    def push_datagrams(self, n, dstride, dgram, dlen, max_out=1 << 16, want_recs=False, pinned_out=False):
        """dgram / dlen: HOST addresses of n datagram slots.  pinned_out: the
        payload output in pinned memory (the library gathers into it directly)."""
        out = np.zeros(max_out, RX_SEG_DTYPE)
        keep = None
        if pinned_out:
            outp, keep = self.n.pinned_array((max_out, self.stride), np.uint8)
        else:
            outp = np.zeros((max_out, self.stride), np.uint8)
        recs = np.zeros(n, WIRE_REC_DTYPE) if want_recs else None
        nout, rep = C.c_uint32(), rfec_rx_report()
        self.n._check(self.n.lib.rfec_rx_session_push_datagrams(
            self.h, n, dstride, dgram, dlen, None if recs is None else recs.ctypes.data, out.ctypes.data,
            outp.ctypes.data, max_out, C.byref(nout), C.byref(rep)), "rfec_rx_session_push_datagrams")
        rows = outp[:nout.value].copy() if keep is not None else outp[:nout.value]
        return out[:nout.value], rows, rep, recs

    def push_datagrams_async(self, n, dstride, dgram, dlen, max_out=1 << 16, want_recs=False, pinned_out=False):
        """The pipelined push: starts these n datagrams (n = 0: flush) and returns
        the PREVIOUS batch's (segments, payload rows, report, its records).  The
        slots at dgram / dlen must stay unchanged until the next call."""
        out = np.zeros(max_out, RX_SEG_DTYPE)
        keep = None
        if pinned_out:
            outp, keep = self.n.pinned_array((max_out, self.stride), np.uint8)
        else:
            outp = np.zeros((max_out, self.stride), np.uint8)
        prev = self.info()["pending"]  # the batch this call ingests
        recs = np.zeros(prev, WIRE_REC_DTYPE) if want_recs else None
        nout, rep = C.c_uint32(), rfec_rx_report()
        self.n._check(self.n.lib.rfec_rx_session_push_datagrams_async(
            self.h, n, dstride, dgram, dlen, None if recs is None or prev == 0 else recs.ctypes.data,
            out.ctypes.data, outp.ctypes.data, max_out, C.byref(nout), C.byref(rep)),
            "rfec_rx_session_push_datagrams_async")
        rows = outp[:nout.value].copy() if keep is not None else outp[:nout.value]
        return out[:nout.value], rows, rep, recs

    def evict(self, stream=None):
        self.n._check(self.n.lib.rfec_rx_session_evict(self.h, stream), "rfec_rx_session_evict")

    def info(self):
        i = rfec_rx_session_info()
        self.n._check(self.n.lib.rfec_rx_session_get_info(self.h, C.byref(i)), "rfec_rx_session_get_info")
        return {f: getattr(i, f) for f, _ in i._fields_}

    def close(self):
        if self.h:
            self.n.lib.rfec_rx_session_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_CACHE: dict[int, Native] = {}


def native(video_size: int = 1000) -> Native:
    if video_size not in _CACHE:
        _CACHE[video_size] = Native(video_size)
    return _CACHE[video_size]


# ---------------------------------------------------------------------------
# torch helpers: a device-resident batch in the layout of include/razor_fec.h
# ---------------------------------------------------------------------------
def _ptr(t):
    return None if t is None else t.data_ptr()


class DeviceBatch:
    """G groups of k segments in HBM (torch tensors as the allocator only)."""

    def __init__(self, plan, groups: int, payload: int, device, stride: int | None = None):
        import torch

        self.plan, self.groups, self.capacity = plan, groups, payload
        self.stride = stride or ((payload + 15) // 16) * 16
        self.k, self.n = plan.k, plan.n_lines
        dev = torch.device(device)
        u8 = torch.uint8
        self.shards = torch.zeros((groups, self.k, self.stride), dtype=u8, device=dev)
        self.hdr = torch.zeros((groups, self.k, 20), dtype=u8, device=dev)
        self.parity = torch.zeros((groups, max(1, self.n), self.stride), dtype=u8, device=dev)
        self.meta = torch.zeros((groups, max(1, self.n), 20), dtype=u8, device=dev)
        self.fec_size = torch.zeros((groups, max(1, self.n)), dtype=torch.int16, device=dev)
        self.status = torch.zeros((groups, max(1, self.n)), dtype=torch.int8, device=dev)
        self.present = torch.zeros((groups, 2), dtype=torch.int64, device=dev)
        self.parity_present = torch.zeros((groups,), dtype=torch.int64, device=dev)
        self.recovered = torch.zeros((groups, 2), dtype=torch.int64, device=dev)
        ws = (groups * ((2 + 2 * self.n + 15) // 16 * 16) + 15) // 16 * 16 + 16 + 4 * groups  # rfec_recover_workspace_size()
        self.workspace = torch.zeros((max(16, ws),), dtype=u8, device=dev)

    def encode(self, lib: Native, stream=None):
        lib.encode_batch(self.plan, self.groups, self.stride, self.capacity, _ptr(self.shards), _ptr(self.hdr),
                         _ptr(self.parity), _ptr(self.meta), _ptr(self.fec_size), _ptr(self.status), stream)

    def recover(self, lib: Native, stream=None):
        lib.recover_batch(self.plan, self.groups, self.stride, self.capacity, _ptr(self.shards), _ptr(self.hdr),
                          _ptr(self.present), _ptr(self.parity), _ptr(self.meta), _ptr(self.fec_size),
                          _ptr(self.parity_present), _ptr(self.recovered), _ptr(self.workspace), stream)

