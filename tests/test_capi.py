"""CPU: the C ABI library loads, exports every symbol include/*.h
declares, and its host-side planner matches the reference (no GPU compute)."""
import ctypes as C
import subprocess
import sys

import numpy as np
import pytest

import pyoracle as po
from razor_amd.fec import header_functions


def test_header_symbols_exported(product, product1200):
    fns = header_functions()
    assert "flex_fec_generate" in fns and "rfec_encode_batch" in fns and "flex_fec_sender_update" in fns
    for lib in (product, product1200):
        for f in fns:
            assert hasattr(lib.lib, f), f"{lib.path.name} does not export {f}"


def test_variants(product, product1200):
    assert product.video_size == 1000 and C.sizeof(product.sim_segment_t) == 1036
    assert product1200.video_size == 1200 and C.sizeof(product1200.sim_segment_t) == 1236
    assert C.sizeof(product.sim_fec_t) == 1044 and C.sizeof(product1200.sim_fec_t) == 1244


def test_planner_table(product):
    """rfec_num_packets == flex_fec_sender_num_packets for n<256, pf<256."""
    t = po.plan_table()
    for n in range(256):
        for pf in range(256):
            assert product.num_packets(n, pf) == tuple(int(x) for x in t[n, pf]), (n, pf)


def test_plan_lines_match_oracle(product, oracle1000):
    for k in range(1, 129):
        for pf in range(0, 256, 3):
            for layers in (1, 2, 3):
                a = product.plan_from_fraction(k, pf, layers)
                b = oracle1000.plan_from_fraction(k, pf, layers)
                assert (a.k, a.row, a.col, a.rc, a.n_lines, a.n_row_lines) == \
                       (b.k, b.row, b.col, b.rc, b.n_lines, b.n_row_lines), (k, pf, layers)
                assert a.lines() == b.lines(), (k, pf, layers)


def test_plan_counts_match_reference_emissions(product):
    """Parities per group in the reference sender fixtures == plan lines."""
    m = po.manifest()
    for c in m["cases"]:
        if c["kind"] == "sender" or (c["kind"] == "sender_large" and c["k"] <= 255):
            p = product.plan_from_fraction(c["k"], c["protect_fraction"])
            assert p.n_lines * c["groups"] == c["parities"], c["name"]
        if c["kind"] == "sender_random":
            groups = np.fromfile(po.GOLDEN / c["groups_file"], np.uint32).reshape(-1, 3)
            for k, pf, n in groups:
                assert product.plan_from_fraction(int(k), int(pf)).n_lines == n


def test_argument_validation(product):
    from razor_amd.fec import RfecError
    plan = product.plan_from_fraction(10, 80, 1)
    with pytest.raises(RfecError):  # stride not a multiple of 16
        product.encode_batch(plan, 4, 1000, 1000, 1, 1, 1, 1, 1, None)
    with pytest.raises(RfecError):  # capacity > stride
        product.encode_batch(plan, 4, 1200, 1201, 1, 1, 1, 1, 1, None)
    with pytest.raises(RfecError):  # NULL buffers
        product.encode_batch(plan, 4, 1200, 1200, None, None, None, None, None, None)
    with pytest.raises(RfecError):
        product.plan_from_fraction(0, 80)
    with pytest.raises(RfecError):
        product.plan_from_fraction(256, 80)  # above RFEC_MAX_K_ENCODE
    with pytest.raises(RfecError):
        product.plan_matrix(10, 2, 4)  # 2x4 does not cover 10
    for row, col in ((64, 2), (2, 64)):  # 66 lines: above RFEC_MAX_LINES (the plan holds 64)
        with pytest.raises(RfecError):
            product.plan_matrix(128, row, col)
    assert product.plan_matrix(124, 62, 2).n_lines == 64
    bad = product.plan_from_fraction(10, 80, 1)
    bad.line[0].count = 20  # member beyond k
    with pytest.raises(RfecError):
        product.encode_batch(bad, 4, 1200, 1200, 1, 1, 1, 1, 1, None)
    assert product.workspace_size(plan, 100) == 100 * 64  # per group: schedule record + task words (16 + 4*10 -> 64 B)
    with pytest.raises(RfecError):  # workspace not 16-byte aligned (checked before any launch)
        product.recover_batch(plan, 4, 1200, 1200, 16, 16, 16, 16, 16, 16, 16, 16, 24, None)
    with pytest.raises(RfecError):  # groups * k beyond 32 bits
        product.zero_tails(1 << 30, 8, 1200, 1, 1, None)


def test_packed_records_geometry(product, oracle1000):
    """rfec_packed_stride and the packed entry points' checks (no launch): row
    layouts of rows <= 4 and k <= 64 only; the host packer (parity_cases) has
    the same stride."""
    from razor_amd.fec import RfecError
    from parity_cases import pack_erasures_np
    c5 = product.plan_matrix(32, 8, 4, 1)
    assert product.packed_stride(c5, 2) == 192  # 16 + 2 x 84 -> 3 x 64 B
    assert product.packed_stride(product.plan_matrix(10, 3, 4, 1), 2) == 192
    assert product.packed_stride(product.plan_matrix(12, 6, 2, 1), 5) == 256  # 16 + 5 x 44 = 236
    assert product.packed_stride(c5, 32) == (16 + 32 * 84 + 63) // 64 * 64
    assert product.packed_stride(c5, 0) == 0 and product.packed_stride(c5, 33) == 0
    assert product.packed_stride(product.plan_matrix(10, 3, 4, 3), 2) == 0  # rows + columns
    assert product.packed_stride(product.plan_matrix(16, 2, 8, 1), 2) == 0  # rows of 8
    assert product.packed_stride(product.plan_matrix(96, 24, 4, 1), 2) == 0  # k > 64
    G, k, col, E = 3, 10, 4, 2
    hdr = np.zeros((G, k), po.HDR_DTYPE)
    meta = np.zeros((G, 3), po.HDR_DTYPE)
    rec = pack_erasures_np(k, col, hdr, np.zeros((G, 2), np.uint64), meta, np.zeros((G, 3), np.uint16),
                           np.zeros(G, np.uint64), E)
    assert rec.shape == (G, product.packed_stride(product.plan_matrix(10, 3, 4, 1), E))
    full = product.plan_matrix(10, 3, 4, 3)
    with pytest.raises(RfecError):  # not a row layout
        product.recover_packed_out(full, 4, 1200, 1200, 16, 16, 16, 16, 2, 16, 16, 16)
    with pytest.raises(RfecError):  # per_group 0
        product.recover_packed_out(c5, 4, 256, 256, 16, 16, 16, 16, 0, 16, 16, 16)
    with pytest.raises(RfecError):  # records not 16-byte aligned
        product.recover_packed_out(c5, 4, 256, 256, 16, 16, 24, 16, 2, 16, 16, 16)
    with pytest.raises(RfecError):  # NULL buffers
        product.recover_packed_out(c5, 4, 256, 256, None, None, 16, None, 2, None, None, None)
    with pytest.raises(RfecError):
        product.pack_erasures(c5, 4, None, None, None, None, None, 2, 16)
    with pytest.raises(RfecError):  # groups x slots beyond 32 bits
        product.pack_erasures(c5, 1 << 30, 16, 16, 16, 16, 16, 32, 16)


def test_packed_records_layout():
    """The host restatement of the packed erasure records (what the GPU tests
    compare rfec_pack_erasures against) follows razor_fec.h's layout: k = 8 in
    rows of 4, segments 1 and 6 lost, two slots."""
    from parity_cases import pack_erasures_np
    k, col, E = 8, 4, 2
    hdr = np.zeros((1, k), po.HDR_DTYPE)
    hdr["seq"] = np.arange(100, 100 + k)
    meta = np.zeros((1, 2), po.HDR_DTYPE)
    meta["seq"] = [7, 9]
    fs = np.array([[300, 400]], np.uint16)
    present = np.array([[0xFF & ~(1 << 1) & ~(1 << 6), 0]], np.uint64)
    pp = np.array([3], np.uint64)
    rec = pack_erasures_np(k, col, hdr, present, meta, fs, pp, E)
    assert rec.shape == (1, 192)  # 16 + 2 x (24 + 3 x 20) = 184 -> 192
    u64 = rec[0, :16].view(np.uint64)
    assert u64[0] == present[0, 0] and u64[1] == 3
    for e, (row, members) in enumerate(((0, (0, 2, 3)), (1, (4, 5, 7)))):
        o = 16 + e * 84
        assert rec[0, o:o + 20].view(po.HDR_DTYPE)[0]["seq"] == meta[0, row]["seq"]
        assert rec[0, o + 20:o + 22].view(np.uint16)[0] == fs[0, row] and not rec[0, o + 22:o + 24].any()
        seqs = [int(rec[0, o + 24 + 20 * q:o + 44 + 20 * q].view(po.HDR_DTYPE)[0]["seq"]) for q in range(3)]
        assert seqs == [100 + i for i in members]
    assert not rec[0, 184:].any()


def test_dropin_fails_loudly_without_gpu():
    """No CPU path: without a HIP device the drop-in symbols print and return -1."""
    code = r'''
import ctypes as C, sys
sys.path.insert(0, ".")
from razor_amd.fec import native
lib = native(1000)
a, b = lib.sim_segment_t(), lib.sim_segment_t()
a.data_size = b.data_size = 10
f = lib.sim_fec_t()
print("RC", lib.flex_fec_generate([a, b], f))
'''
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       cwd=str(po.ROOT))
    assert "RC -1" in r.stdout, r.stdout + r.stderr
    assert "razor_fec" in r.stderr


def test_sender_plan_product(product):
    """rfec_sender_plan (host C, no GPU needed) reproduces the reference flex
    sender's grouping and stamps (tests/golden/stage.json)."""
    import stage_cases as sc

    sc.check_plan(product.sender_plan, product.sender_init)
