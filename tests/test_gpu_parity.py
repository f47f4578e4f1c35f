"""GPU: the HIP path (librazor_fec.so through its C ABI) against the golden
fixtures of the compiled reference and against the oracle, bit-exact."""
import ctypes as C
import json

import numpy as np
import pytest

import parity_cases as pc
import pyoracle as po

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

MANIFEST = po.manifest()
CASES = {c["name"]: c for c in MANIFEST["cases"]}
TUNINGS = {"default": 0, "generic": 1}  # RFEC_TUNE_GENERIC: the plan-driven kernels as the cross-check


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")
    from gpu_engine import GpuEngine
    return GpuEngine


@pytest.mark.parametrize("tuning", list(TUNINGS))
@pytest.mark.parametrize("name", [c["name"] for c in MANIFEST["cases"]
                                  if c["kind"] == "sender" or (c["kind"] == "sender_large" and c["k"] <= 255)])
def test_sender_fixture_gpu(gpu, oracle1000, name, tuning):
    pc.check_sender_case(gpu(tuning=TUNINGS[tuning]), oracle1000, CASES[name])


def test_sender_random_fixture_gpu(gpu, oracle1000):
    pc.check_sender_random_case(gpu(), oracle1000, CASES["random_k"])


@pytest.mark.parametrize("tuning", list(TUNINGS))
@pytest.mark.parametrize("name", [c["name"] for c in MANIFEST["cases"] if c["kind"] == "rows"])
def test_rows_fixture_gpu(gpu, oracle1000, oracle1200, name, tuning):
    c = CASES[name]
    o = oracle1200 if c["S"] > 1000 else oracle1000
    pc.check_rows_case(gpu(tuning=TUNINGS[tuning]), o, c, capacity=max(c["S"], 1000))


@pytest.mark.parametrize("output", ["in_place", "dense"])
@pytest.mark.parametrize("tuning", list(TUNINGS))
@pytest.mark.parametrize("name", [c["name"] for c in MANIFEST["cases"] if c["kind"] == "erasures"])
def test_erasure_fixture_gpu(gpu, oracle1000, name, tuning, output):
    """The reference receiver's verdicts and segment hashes (era_*.bin) through
    rfec_recover_batch (in place) and rfec_recover_batch_out (a slot per
    segment, scattered back): every plan, the full 3x4 plan's cascades too."""
    eng = gpu(tuning=TUNINGS[tuning])
    pc.check_erasure_case(eng if output == "in_place" else pc.DenseAsInPlace(eng), oracle1000, CASES[name])


@pytest.mark.parametrize("tuning", list(TUNINGS))
@pytest.mark.parametrize("name", [c["name"] for c in MANIFEST["cases"] if c["kind"] == "erasures" and c["rows_only"]])
def test_erasure_fixture_rows_plan_gpu(gpu, oracle1000, name, tuning):
    """Row-parity-only fixtures against the row-layer plan (pairwise disjoint
    lines: the fused one-launch decode applies where rows have <= 4 members)."""
    pc.check_erasure_case(gpu(tuning=TUNINGS[tuning]), oracle1000, CASES[name], layers=1)


def test_single_cases_dropin_gpu(product):
    """flex_fec_generate / flex_fec_recover (drop-in symbols) on the GPU vs the
    reference's single-call outputs, including failures and in-place padding."""
    from test_oracle_golden import run_single_cases

    seg_t, fec_t = product.sim_segment_t, product.sim_fec_t
    run_single_cases(lambda s, f: product.flex_fec_generate(s, f),
                     lambda s, f, o: product.flex_fec_recover(s, f, o), seg_t, fec_t, 1000)


def test_dropin_1200(product1200, oracle1200):
    """The SIM_VIDEO_SIZE=1200 variant: a 1200-B row through the drop-in symbols."""
    lib, o = product1200, oracle1200
    shards, hdr = o.fill_groups(101, 1, 4, 1200, ragged=True)
    segs = []
    for i in range(4):
        s = lib.sim_segment_t()
        h = hdr[0, i]
        s.packet_id, s.fid, s.timestamp = int(h["seq"]), int(h["fid"]), int(h["ts"])
        s.index, s.total, s.ftype, s.payload_type = int(h["index"]), int(h["total"]), int(h["ftype"]), 0
        s.data_size = int(h["size"])
        C.memmove(C.addressof(s) + 34, shards[0, i].tobytes(), 1200)
        segs.append(s)
    fec = lib.sim_fec_t()
    assert lib.flex_fec_generate(segs, fec) == 0
    parity, meta, fsize, _ = o.encode_batch(o.plan_matrix(4, 1, 4, 1), shards, hdr, 1200)
    L = int(fsize[0, 0])
    assert fec.fec_data_size == L
    assert bytes(fec.fec_data)[:L] == parity[0, 0, :L].tobytes()
    out = lib.sim_segment_t()
    assert lib.flex_fec_recover(segs[1:], fec, out) == 0
    assert out.data_size == hdr[0, 0]["size"] and out.packet_id == hdr[0, 0]["seq"]
    assert bytes(out.data)[:out.data_size] == shards[0, 0, :out.data_size].tobytes()


# ---- full-size properties ---------------------------------------------------
def _device_batch(G, k, S, seed, device="cuda:0"):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    shards = torch.randint(0, 256, (G, k, S), dtype=torch.uint8, device=device, generator=g)
    hdr = np.zeros((G, k), po.HDR_DTYPE)
    gi = np.arange(G, dtype=np.uint32)[:, None]
    ii = np.arange(k, dtype=np.uint32)[None, :]
    hdr["seq"] = 1 + gi * k + ii
    hdr["fid"] = 1 + gi
    hdr["ts"] = 33 * gi
    hdr["index"] = ii
    hdr["total"] = k
    hdr["ftype"] = (gi % 60 == 0)
    hdr["size"] = S
    d_hdr = torch.from_numpy(hdr.view(np.uint8).reshape(G, k, 20).copy()).to(device)
    return shards, hdr, d_hdr


def _run_encode(lib, plan, G, S, shards, d_hdr, tuning=0):
    n = plan.n_lines
    dev = shards.device
    par = torch.empty((G, n, S), dtype=torch.uint8, device=dev)
    meta = torch.empty((G, n, 20), dtype=torch.uint8, device=dev)
    fs = torch.empty((G, n), dtype=torch.int16, device=dev)
    st = torch.empty((G, n), dtype=torch.int8, device=dev)
    lib.set_tuning(tuning)
    try:
        lib.encode_batch(plan, G, S, S, shards.data_ptr(), d_hdr.data_ptr(), par.data_ptr(), meta.data_ptr(),
                         fs.data_ptr(), st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    finally:
        lib.set_tuning(0)
    torch.cuda.synchronize()
    return par, meta, fs, st


@pytest.mark.parametrize("layers", [1, 3])
def test_full_size_k10_roundtrip(product, oracle1200, layers):
    """Config 2/3 shape (G=65536, k=10, 1200 B): fast == generic kernel bit for
    bit, a sample equals the oracle, and 2 erasures per group round-trip."""
    lib, o = product, oracle1200
    G, k, S = 65536, 10, 1200
    plan = lib.plan_from_fraction(k, 80, layers)
    shards, hdr, d_hdr = _device_batch(G, k, S, 1234)
    par, meta, fs, st = _run_encode(lib, plan, G, S, shards, d_hdr)
    for tuning in (1,):
        par2, meta2, fs2, st2 = _run_encode(lib, plan, G, S, shards, d_hdr, tuning=tuning)
        assert torch.equal(par, par2) and torch.equal(meta, meta2) and torch.equal(fs, fs2), tuning
        del par2, meta2, fs2, st2
    assert int(st.abs().sum()) == 0
    # oracle on a sample of groups
    idx = np.r_[0:8, G // 2:G // 2 + 8, G - 8:G]
    sh_h = shards[idx].cpu().numpy()
    p_o, m_o, f_o, s_o = o.encode_batch(o.plan_from_fraction(k, 80, layers), sh_h, hdr[idx], 1200)
    assert np.array_equal(par[idx].cpu().numpy(), p_o)
    assert np.array_equal(meta[idx].cpu().numpy().view(po.HDR_DTYPE).reshape(len(idx), -1), m_o)
    assert np.array_equal(fs[idx].cpu().numpy().view(np.uint16), f_o)
    # erasures: 2 per group; rows only -> distinct rows (all recoverable)
    rng = np.random.default_rng(7)
    if layers == 1:
        rows = [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]
        pairs = [(a, b) for r1 in range(3) for r2 in range(r1 + 1, 3) for a in rows[r1] for b in rows[r2]]
        assert len(pairs) == 32
    else:
        pairs = [(a, b) for a in range(k) for b in range(a + 1, k)]
        assert len(pairs) == 45
    choice = rng.integers(0, len(pairs), G)
    er = np.array(pairs)[choice]
    present = np.full((G, 2), 0, np.uint64)
    present[:, 0] = np.uint64((1 << k) - 1) & ~((np.uint64(1) << er[:, 0].astype(np.uint64)) |
                                               (np.uint64(1) << er[:, 1].astype(np.uint64)))
    gi = torch.arange(G, device=shards.device)
    d_pres = torch.from_numpy(present.view(np.int64)).to(shards.device)
    d_pp = torch.full((G,), (1 << plan.n_lines) - 1, dtype=torch.int64, device=shards.device)
    ws = torch.empty((lib.workspace_size(plan, G),), dtype=torch.uint8, device=shards.device)
    exp = ((1 << er[:, 0]) | (1 << er[:, 1])).astype(np.int64)
    # default (fused one-launch decode for the disjoint row layer), forced peel + replay
    for dec_tuning in (0, 1):
        rx = shards.clone()
        rx_hdr = d_hdr.clone()
        for c in range(2):
            e = torch.from_numpy(er[:, c]).to(rx.device)
            rx[gi, e] = 0xA5
            rx_hdr[gi, e] = 0
        rec = torch.empty((G, 2), dtype=torch.int64, device=rx.device)
        lib.set_tuning(dec_tuning)
        try:
            lib.recover_batch(plan, G, S, S, rx.data_ptr(), rx_hdr.data_ptr(), d_pres.data_ptr(), par.data_ptr(),
                              meta.data_ptr(), fs.data_ptr(), d_pp.data_ptr(), rec.data_ptr(), ws.data_ptr(),
                              torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
        finally:
            lib.set_tuning(0)
        assert torch.equal(rx, shards), dec_tuning
        assert torch.equal(rx_hdr, d_hdr), dec_tuning
        assert np.array_equal(rec[:, 0].cpu().numpy(), exp), dec_tuning


def test_full_size_k32_s256(product, oracle1000):
    """Config 5 shape: k=32, 8 rows of 4, 256-B packets, G=65536."""
    lib, o = product, oracle1000
    G, k, S = 65536, 32, 256
    plan = lib.plan_matrix(k, 8, 4, 1)
    assert plan.n_lines == 8
    shards, hdr, d_hdr = _device_batch(G, k, S, 99)
    par, meta, fs, st = _run_encode(lib, plan, G, S, shards, d_hdr)
    for tuning in (1,):
        par2, meta2, fs2, _ = _run_encode(lib, plan, G, S, shards, d_hdr, tuning=tuning)
        assert torch.equal(par, par2) and torch.equal(meta, meta2) and torch.equal(fs, fs2), tuning
    idx = np.r_[0:4, G - 4:G]
    p_o, m_o, f_o, _ = o.encode_batch(o.plan_matrix(k, 8, 4, 1), shards[idx].cpu().numpy(), hdr[idx], 256)
    assert np.array_equal(par[idx].cpu().numpy(), p_o)
    assert np.array_equal(meta[idx].cpu().numpy().view(po.HDR_DTYPE).reshape(len(idx), -1), m_o)
    # decode: up to one erasure in each of 3 random rows per group (row decode kernel, vector masks
    # at 16 chunks per slot), some rows with their parity lost as well
    rng = np.random.default_rng(11)
    er_rows = np.stack([rng.permutation(8)[:3] for _ in range(G)])
    er = er_rows * 4 + rng.integers(0, 4, (G, 3))
    er[G // 3:G // 2, 2] = er[G // 3:G // 2, 1]  # some groups with 2 erasures only
    present = np.uint64((1 << k) - 1) & ~np.bitwise_or.reduce(np.uint64(1) << er.astype(np.uint64), axis=1)
    pp = np.full(G, 0xFF, np.uint64)
    pp[::5] &= ~(np.uint64(1) << er_rows[::5, 0].astype(np.uint64))  # parity of the first erased row lost
    exp = present.copy()
    gi = torch.arange(G, device=shards.device)
    for dec_tuning in (0, 1):
        rx = shards.clone()
        rx_hdr = d_hdr.clone()
        for c in range(3):
            e = torch.from_numpy(er[:, c]).to(rx.device)
            rx[gi, e] = 0x5A
            rx_hdr[gi, e] = 0
        d_pres = torch.from_numpy(np.stack([present, np.zeros(G, np.uint64)], 1).view(np.int64)).to(rx.device)
        d_pp = torch.from_numpy(pp.view(np.int64)).to(rx.device)
        ws = torch.empty((lib.workspace_size(plan, G),), dtype=torch.uint8, device=rx.device)
        rec = torch.empty((G, 2), dtype=torch.int64, device=rx.device)
        lib.set_tuning(dec_tuning)
        try:
            lib.recover_batch(plan, G, S, S, rx.data_ptr(), rx_hdr.data_ptr(), d_pres.data_ptr(), par.data_ptr(),
                              meta.data_ptr(), fs.data_ptr(), d_pp.data_ptr(), rec.data_ptr(), ws.data_ptr(),
                              torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
        finally:
            lib.set_tuning(0)
        got = rec[:, 0].cpu().numpy().view(np.uint64)
        lost_par = np.zeros(G, np.uint64)
        lost_par[::5] = np.uint64(1) << er[::5, 0].astype(np.uint64)
        want = ~present & np.uint64((1 << k) - 1) & ~lost_par
        assert np.array_equal(got, want), dec_tuning
        ok = torch.from_numpy(((exp | got) == np.uint64((1 << k) - 1))).to(rx.device)
        assert ok.sum().item() == G - len(range(0, G, 5)), dec_tuning
        assert torch.equal(rx[ok], shards[ok]) and torch.equal(rx_hdr[ok], d_hdr[ok]), dec_tuning


def test_zero_tails(product):
    lib = product
    G, k, S = 37, 5, 1200
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, (G, k, S), dtype=np.uint8)
    hdr = np.zeros((G, k), po.HDR_DTYPE)
    hdr["size"] = rng.integers(0, S + 1, (G, k))
    hdr["size"][0, 0] = 0
    hdr["size"][0, 1] = S
    hdr["size"][0, 2] = 17
    d = torch.from_numpy(data.copy()).cuda()
    dh = torch.from_numpy(hdr.view(np.uint8).reshape(-1).copy()).cuda()
    lib.zero_tails(G, k, S, d.data_ptr(), dh.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    exp = data.copy()
    for g in range(G):
        for i in range(k):
            exp[g, i, hdr["size"][g, i]:] = 0
    assert np.array_equal(d.cpu().numpy(), exp)


def test_empty_and_degenerate(product):
    lib = product
    s = torch.cuda.current_stream().cuda_stream
    plan = lib.plan_from_fraction(10, 80, 1)
    # zero groups: a no-op that returns OK
    lib.encode_batch(plan, 0, 1200, 1200, None, None, None, None, None, None, s)
    # a plan with no lines (pf = 0 -> col = 0)
    p0 = lib.plan_from_fraction(10, 0, 3)
    assert p0.n_lines == 0
    d = torch.zeros(16, dtype=torch.uint8, device="cuda")
    lib.encode_batch(p0, 4, 16, 16, d.data_ptr(), d.data_ptr(), d.data_ptr(), d.data_ptr(), d.data_ptr(), None, s)
    torch.cuda.synchronize()


@pytest.mark.parametrize("layers", [1, 3])
def test_encode_large_stride_small_capacity(product1200, oracle1200, layers):
    """A legal batch whose slot stride is far larger than its capacity (16-B
    payloads in 40 MiB slots): the fused encodes address a wave's groups through
    one buffer descriptor whose range is ~2 GiB, and one wave here spans all 8
    groups (2.9 GB of offsets), so launch_encode must take the generic kernel.
    Parities / meta / sizes equal the oracle's on the compact layout."""
    lib, o = product1200, oracle1200
    G, k, cap, stride = 8, 10, 16, 40 << 20
    sh_c, hdr = o.fill_groups(307, G, k, cap, ragged=True)
    plan = o.plan_from_fraction(k, 80, layers)
    n = plan.n_lines
    par_c, meta_c, fs_c, st_c = o.encode_batch(plan, sh_c, hdr, cap)
    sh = torch.zeros((G, k, stride), dtype=torch.uint8, device="cuda")
    sh[:, :, :16] = torch.from_numpy(sh_c).cuda()
    dh = torch.from_numpy(hdr.view(np.uint8).reshape(-1).copy()).cuda()
    par = torch.full((G, n, stride), 0x5A, dtype=torch.uint8, device="cuda")
    meta = torch.empty((G, n, 20), dtype=torch.uint8, device="cuda")
    fs = torch.empty((G, n), dtype=torch.int16, device="cuda")
    st = torch.empty((G, n), dtype=torch.int8, device="cuda")
    lib.encode_batch(plan, G, stride, cap, sh.data_ptr(), dh.data_ptr(), par.data_ptr(), meta.data_ptr(),
                     fs.data_ptr(), st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(par[:, :, :16].cpu().numpy(), par_c[:, :, :16])
    assert np.array_equal(meta.cpu().numpy().reshape(-1), meta_c.view(np.uint8).reshape(-1))
    assert np.array_equal(fs.cpu().numpy().view(np.uint16), fs_c)
    assert np.array_equal(st.cpu().numpy(), st_c)
    del sh, par
    torch.cuda.empty_cache()


def test_capacity_status(product):
    """status -1 where a line's fec_data_size exceeds capacity (flex_fec_xor.c:27-28)."""
    lib = product
    plan = lib.plan_matrix(4, 2, 2, 1)
    G, k, S = 3, 4, 64
    hdr = np.zeros((G, k), po.HDR_DTYPE)
    hdr["size"] = 10
    hdr["size"][1, 2] = 60  # group 1, row 1 over capacity 48
    sh = torch.zeros((G, k, S), dtype=torch.uint8, device="cuda")
    dh = torch.from_numpy(hdr.view(np.uint8).reshape(-1).copy()).cuda()
    par = torch.empty((G, 2, S), dtype=torch.uint8, device="cuda")
    meta = torch.empty((G, 2, 20), dtype=torch.uint8, device="cuda")
    fs = torch.empty((G, 2), dtype=torch.int16, device="cuda")
    st = torch.empty((G, 2), dtype=torch.int8, device="cuda")
    lib.encode_batch(plan, G, S, 48, sh.data_ptr(), dh.data_ptr(), par.data_ptr(), meta.data_ptr(), fs.data_ptr(),
                     st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    exp = np.zeros((G, 2), np.int8)
    exp[1, 1] = -1
    assert np.array_equal(st.cpu().numpy(), exp)
    assert fs.cpu().numpy()[1, 1] == 60


def _host_arrays(lib, n, dtype, mem, fill=0):
    """n structs of `dtype` in pageable numpy memory, or in an rfec_pinned_alloc
    block (the zero-copy path); `fill` pre-sets every byte (stale contents a
    caller's buffers may hold)."""
    if mem == "pinned":
        a, keep = lib.pinned_array((n,), dtype)
    else:
        a, keep = np.zeros(n, dtype), None
    a.view(np.uint8)[...] = fill
    return a, keep


def _ptrs(a):
    return a.ctypes.data + np.arange(a.shape[0], dtype=np.uint64) * a.dtype.itemsize


def _host_segs(lib, o, seed, G, k, S, mem):
    from razor_amd.fec import seg_dtype

    shards, hdr = o.fill_groups(seed, G, k, S, ragged=True)
    segs, keep = _host_arrays(lib, G * k, seg_dtype(1200), mem)
    h = hdr.reshape(-1)
    for a, b in (("seq", "packet_id"), ("fid", "fid"), ("ts", "timestamp"), ("index", "index"),
                 ("total", "total"), ("ftype", "ftype"), ("payload_type", "payload_type"), ("size", "data_size")):
        segs[b] = h[a]
    segs["data"] = shards.reshape(G * k, S)
    return shards, hdr, segs, keep


def _fields_equal(got, want, size_field, data_field):
    """Every named field equal, the payload compared up to its size field
    (bytes past it are unspecified in the reference's structs)."""
    for f in got.dtype.names:
        if f != data_field:
            assert np.array_equal(got[f], want[f]), f
    for j in range(got.shape[0]):
        L = int(want[size_field][j])
        L = 0 if L == 0xFFFF else L
        assert np.array_equal(got[data_field][j, :L], want[data_field][j, :L]), j


@pytest.mark.parametrize("mem", ["pageable", "pinned"])
def test_host_encode_groups(product1200, oracle1200, mem):
    """rfec_host_encode_groups (host AoS in, host sim_fec_t out) vs the oracle's
    reference-shaped AoS path (flex_fec_generate per line + sender stamps).
    "pinned": segments and parities in rfec_pinned_alloc memory, so the device
    gathers and scatters the structs itself (timing.zero_copy); its output
    equals the staged path's field for field and zero past fec_data_size; a
    line whose flex_fec_generate fails (oversize data_size) gets 0xFFFF."""
    from razor_amd.fec import fec_dtype

    lib, o = product1200, oracle1200
    G, k, S = 37, 10, 1200
    shards, hdr, segs, ks = _host_segs(lib, o, 202, G, k, S, mem)
    plan = o.plan_from_fraction(k, 80, 3)  # full 3x4 plan: 7 parities
    n = plan.n_lines
    fecs, kf = _host_arrays(lib, G * n, fec_dtype(1200), mem, fill=0xA5)
    t = lib.host_encode_groups(plan, G, _ptrs(segs), _ptrs(fecs), fec_id0=1)
    assert t["total_us"] > 0 and t["zero_copy"] == (mem == "pinned")
    nref, ref = o.encode_aos(plan, G, o.to_aos(shards, hdr))
    assert nref == G * n
    ref = ref.view(fec_dtype(1200)).reshape(-1)
    for f in ("fec_id", "row", "col", "index", "count", "base_id", "fec_data_size"):
        assert np.array_equal(fecs[f], ref[f]), f
    assert np.array_equal(fecs["meta"], ref["meta"])
    for j in range(G * n):
        L = int(ref["fec_data_size"][j])
        assert np.array_equal(fecs["fec_data"][j, :L], ref["fec_data"][j, :L])
    if mem != "pinned":
        return
    for j in range(G * n):
        assert not fecs["fec_data"][j, int(fecs["fec_data_size"][j]):].any(), j
    # against the staged path, fec_id0 wrapping past 65535 and failing lines
    segs["data_size"][3 * k + 2] = 1300  # > SIM_VIDEO_SIZE: its row and column lines fail
    stale = np.zeros(G * n, fec_dtype(1200))
    stale.view(np.uint8)[...] = 0x5A
    fecs.view(np.uint8)[...] = 0x5A
    t = lib.host_encode_groups(plan, G, _ptrs(segs), _ptrs(fecs), fec_id0=65520)
    assert t["zero_copy"] == 1
    pg = np.zeros(G * k, segs.dtype)
    pg[...] = segs
    t = lib.host_encode_groups(plan, G, _ptrs(pg), _ptrs(stale), fec_id0=65520)
    assert t["zero_copy"] == 0
    assert (stale["fec_data_size"] == 0xFFFF).sum() >= 2
    assert stale["fec_id"].min() >= 1 and stale["fec_id"].max() == 65535
    _fields_equal(fecs, stale, "fec_data_size", "fec_data")


def test_host_zero_copy_eligibility(product1200, oracle1200, monkeypatch):
    """The zero-copy form runs only when every struct pointer of an array lies
    in ONE rfec_pinned_alloc block and RFEC_HOST_ZEROCOPY is not "0"; segments
    split over two pinned blocks, or the variable set, take the staged form --
    same parities either way (and the oracle's)."""
    from razor_amd.fec import fec_dtype, seg_dtype

    lib, o = product1200, oracle1200
    G, k, S = 64, 10, 1200
    shards, hdr, segs, ks = _host_segs(lib, o, 204, G, k, S, "pinned")
    plan = o.plan_from_fraction(k, 80, 3)
    n = plan.n_lines
    nref, ref = o.encode_aos(plan, G, o.to_aos(shards, hdr))
    ref = ref.view(fec_dtype(1200)).reshape(-1)

    def run(sp, expect_zc):
        fecs, kf = _host_arrays(lib, G * n, fec_dtype(1200), "pinned", fill=0x33)
        t = lib.host_encode_groups(plan, G, sp, _ptrs(fecs), fec_id0=1)
        assert t["zero_copy"] == expect_zc
        _fields_equal(fecs, ref, "fec_data_size", "fec_data")

    run(_ptrs(segs), 1)
    half, kh = _host_arrays(lib, G * k // 2, seg_dtype(1200), "pinned")
    half[...] = segs[G * k // 2:]
    split = _ptrs(segs).copy()
    split[G * k // 2:] = _ptrs(half)
    run(split, 0)  # two blocks: staged
    monkeypatch.setenv("RFEC_HOST_ZEROCOPY", "0")
    run(_ptrs(segs), 0)


@pytest.mark.parametrize("mem", ["pageable", "pinned"])
@pytest.mark.parametrize("k,layers,G", [(10, 1, 301), (10, 3, 301), (10, 3, 4500), (128, 1, 3000)])
def test_host_recover_groups(product1200, oracle1200, k, layers, G, mem):
    """rfec_host_recover_groups (host AoS in, flex_fec_recover-style out_seg
    out): groups encoded by rfec_host_encode_groups (checked above), 1-3
    segments and 0-2 parities of each lost; out_index / recovered masks equal
    the oracle's rfec_recover_batch_out restatement, every recovered out_seg
    equals the lost segment (header fields, data_size, data, zero past it)
    and carries the group's fec_id.  4,500 groups: three double-buffered
    chunks of packed received rows (2,048, 2,048, 404).  k = 128 with a
    64-line plan (64 rows of 2): chunks sized by bytes (~1,400 groups of
    ~470 KB device staging each), not by the group count alone.  "pinned":
    every struct in rfec_pinned_alloc memory (the zero-copy path, with some
    out pointers NULL), output equal to the staged path's field for field,
    out structs not recovered into left as they were."""
    from razor_amd.fec import fec_dtype, seg_dtype

    lib, o = product1200, oracle1200
    S, E = 1200, 3
    shards, hdr, segs, ks = _host_segs(lib, o, 203, G, k, S, mem)
    plan = o.plan_from_fraction(k, 80, layers) if k <= 10 else o.plan_matrix(k, 64, 2, layers)
    assert plan.n_lines == ({1: 3, 3: 7}[layers] if k == 10 else 64)
    n = plan.n_lines
    fecs, kf = _host_arrays(lib, G * n, fec_dtype(1200), mem)
    sp, fp = _ptrs(segs), _ptrs(fecs)
    lib.host_encode_groups(plan, G, sp, fp, fec_id0=1)
    rng = np.random.default_rng(layers)
    present = np.zeros((G, 2), np.uint64)
    ppm = np.zeros(G, np.uint64)
    sp_rx, fp_rx = sp.copy(), fp.copy()
    for g in range(G):
        lost = rng.choice(k, int(rng.integers(1, 4)), replace=False)
        sp_rx[g * k + lost] = 0
        pm = sum(1 << i for i in range(k) if i not in lost)
        present[g, 0], present[g, 1] = pm & (2**64 - 1), pm >> 64
        plost = rng.choice(n, int(rng.integers(0, 3)), replace=False)
        fp_rx[g * n + plost] = 0
        ppm[g] = sum(1 << l for l in range(n) if l not in plost)
    out, ko = _host_arrays(lib, G * E, seg_dtype(1200), mem, fill=0xA5 if mem == "pinned" else 0)
    op = _ptrs(out)
    if mem == "pinned":
        op[::7] = 0  # out_seg NULL: skipped
    oi, rec, t = lib.host_recover_groups(plan, G, sp_rx, fp_rx, E, op)
    assert t["total_us"] > 0 and t["zero_copy"] == (mem == "pinned")
    # the oracle on the same received set (lost members' slots / headers zero)
    rx_sh = shards.copy()
    rx_h = hdr.copy()
    for g in range(G):
        for i in range(k):
            if not (int(present[g, i >> 6]) >> (i & 63)) & 1:
                rx_sh[g, i] = 0
                rx_h[g, i] = 0
    par = fecs["fec_data"].reshape(G, n, S)
    meta = np.ascontiguousarray(fecs["meta"].reshape(G, n))
    fsz = fecs["fec_data_size"].reshape(G, n)
    _, _, o_i, o_rec = o.recover_batch_out(plan, rx_sh, rx_h, present, par, meta, fsz, ppm, 1200, E)
    assert np.array_equal(oi, o_i) and np.array_equal(rec, o_rec)
    assert (oi != 0xFF).sum() > G // 4  # a good share came back (rows only: many groups lose 2 in a row)
    for g in range(G):
        for e in range(E):
            i = int(oi[g, e])
            if i == 0xFF or op[g * E + e] == 0:
                continue
            got, want = out[g * E + e], segs[g * k + i]
            for f in ("packet_id", "fid", "timestamp", "index", "total", "ftype", "payload_type", "data_size"):
                assert got[f] == want[f], (g, e, f)
            nb = int(want["data_size"])
            assert np.array_equal(got["data"][:nb], want["data"][:nb]) and not got["data"][nb:].any()
            assert got["fec_id"] == fecs["fec_id"][g * n]
    if mem != "pinned":
        return
    # the staged path on pageable copies of the same structs and stale out contents
    pseg = np.zeros(G * k, segs.dtype)
    pseg[...] = segs
    pfec = np.zeros(G * n, fecs.dtype)
    pfec[...] = fecs
    pout = np.zeros(G * E, out.dtype)
    pout.view(np.uint8)[...] = 0xA5
    pop = _ptrs(pout)
    pop[::7] = 0
    psp = np.where(sp_rx == 0, 0, _ptrs(pseg))
    pfp = np.where(fp_rx == 0, 0, _ptrs(pfec))
    oi2, rec2, t2 = lib.host_recover_groups(plan, G, psp, pfp, E, pop)
    assert t2["zero_copy"] == 0
    assert np.array_equal(oi2, oi) and np.array_equal(rec2, rec)
    _fields_equal(out, pout, "data_size", "data")
    untouched = (oi.reshape(-1) == 0xFF) | (op == 0)
    assert (out.view(np.uint8).reshape(G * E, -1)[untouched] == 0xA5).all()


def test_host_recover_groups_rejections_zero_copy(product1200, oracle1200):
    """The zero-copy recover on the sender's 3 x 4 plan sends whole only the
    lines the dense cascade decode reads, as headers the rest of the lines
    holding an erased member, and nothing of the others (rfec_hostmem.c
    zc_lines_read).  With header rejections (a parity whose fec_data_size is
    below its members' sizes: the exact peel bans the line and recovers
    through another, whose members may have crossed as headers only) the
    out_index / recovered masks / out_seg structs equal the staged path's on
    pageable copies of the same structs, field for field."""
    from razor_amd.fec import fec_dtype, seg_dtype

    lib, o = product1200, oracle1200
    G, k, S, E = 3000, 10, 1200, 3
    shards, hdr, segs, ks = _host_segs(lib, o, 205, G, k, S, "pinned")
    plan = o.plan_from_fraction(k, 80, 3)
    n = plan.n_lines
    fecs, kf = _host_arrays(lib, G * n, fec_dtype(1200), "pinned")
    sp, fp = _ptrs(segs), _ptrs(fecs)
    lib.host_encode_groups(plan, G, sp, fp, fec_id0=1)
    rng = np.random.default_rng(11)
    sp_rx, fp_rx = sp.copy(), fp.copy()
    for g in range(G):
        lost = rng.choice(k, int(rng.integers(1, 4)), replace=False)
        sp_rx[g * k + lost] = 0
        fp_rx[g * n + rng.choice(n, int(rng.integers(0, 2)), replace=False)] = 0
    bad = rng.choice(G * n, G // 3, replace=False)  # their lines fail the size check when they fire
    fecs["fec_data_size"][bad] = 600
    out, ko = _host_arrays(lib, G * E, seg_dtype(1200), "pinned", fill=0xA5)
    oi, rec, t = lib.host_recover_groups(plan, G, sp_rx, fp_rx, E, _ptrs(out))
    assert t["zero_copy"] == 1
    pseg = np.zeros(G * k, segs.dtype)
    pseg[...] = segs
    pfec = np.zeros(G * n, fecs.dtype)
    pfec[...] = fecs
    pout = np.zeros(G * E, out.dtype)
    pout.view(np.uint8)[...] = 0xA5
    oi2, rec2, t2 = lib.host_recover_groups(plan, G, np.where(sp_rx == 0, 0, _ptrs(pseg)),
                                            np.where(fp_rx == 0, 0, _ptrs(pfec)), E, _ptrs(pout))
    assert t2["zero_copy"] == 0
    assert np.array_equal(oi2, oi) and np.array_equal(rec2, rec)
    _fields_equal(out, pout, "data_size", "data")
    # the header checks changed the peel in a good share of the groups
    mask_only = np.array([bin(int(r)).count("1") for r in rec[:, 0]])
    assert (oi != 0xFF).sum() > G // 2 and mask_only.sum() > 0


def _gapped(lib, n, dtype, gap, fill, canary):
    """n structs of `dtype` in ONE rfec_pinned_alloc block, `gap` canary bytes
    after each (the last struct ends exactly at the block's end): returns the
    block's bytes, the structs' addresses and a structured view per struct."""
    isz = np.dtype(dtype).itemsize
    step = isz + gap
    raw, keep = lib.pinned_array((n * step - gap,), np.uint8)
    raw[...] = canary
    for i in range(n):
        raw[i * step:i * step + isz] = fill
    ptrs = raw.ctypes.data + np.arange(n, dtype=np.uint64) * step
    return raw, keep, ptrs, step, isz


def _gaps_intact(raw, n, step, isz, canary):
    g = np.ones(raw.shape[0], bool)
    for i in range(n):
        g[i * step:i * step + isz] = False
    return (raw[g] == canary).all()


def test_host_zero_copy_1000_struct_bounds(product, oracle1000):
    """The zero-copy kernels at SIM_VIDEO_SIZE 1000 (librazor_fec.so): the
    data runs 1,000 bytes = 62.5 chunks, so a struct's last 16-byte chunk
    reaches past sizeof(sim_fec_t) = 1,044 / sizeof(sim_segment_t) = 1,036.
    Structs placed with 16-byte canary gaps between them (and the last one
    ending at the pinned block's end): encode parities and recovered out_seg
    equal the oracle's, and no byte outside a written struct changes."""
    from razor_amd.fec import fec_dtype, seg_dtype

    lib, o = product, oracle1000
    G, k, S, E, CAN = 29, 10, 1000, 3, 0xC3
    shards, hdr = o.fill_groups(301, G, k, S, ragged=True)
    sdt, fdt = seg_dtype(1000), fec_dtype(1000)
    assert sdt.itemsize == 1036 and fdt.itemsize == 1044
    plan = o.plan_from_fraction(k, 80, 3)
    n = plan.n_lines
    aos = o.to_aos(shards, hdr)
    sraw, ks, sp, sstep, ssz = _gapped(lib, G * k, sdt, 16, 0, CAN)
    for i in range(G * k):
        sraw[i * sstep:i * sstep + ssz] = aos[i:i + 1].view(np.uint8)
    fraw, kf, fp, fstep, fsz = _gapped(lib, G * n, fdt, 16, 0xA5, CAN)
    t = lib.host_encode_groups(plan, G, sp, fp, fec_id0=1)
    assert t["zero_copy"] == 1
    assert _gaps_intact(fraw, G * n, fstep, fsz, CAN)
    assert _gaps_intact(sraw, G * k, sstep, ssz, CAN)
    nref, ref = o.encode_aos(plan, G, aos)
    ref = ref.view(fdt).reshape(-1)
    got = np.stack([fraw[i * fstep:i * fstep + fsz] for i in range(G * n)]).reshape(-1).view(fdt)
    for f in ("fec_id", "row", "col", "index", "count", "base_id", "fec_data_size", "meta"):
        assert np.array_equal(got[f], ref[f]), f
    for j in range(G * n):
        L = int(ref["fec_data_size"][j])
        assert np.array_equal(got["fec_data"][j, :L], ref["fec_data"][j, :L]), j
        assert not got["fec_data"][j, L:].any(), j
    # receive: 1-3 segments and 0-1 parities lost per group, out_seg structs gapped too
    rng = np.random.default_rng(11)
    present = np.zeros((G, 2), np.uint64)
    ppm = np.zeros(G, np.uint64)
    sp_rx, fp_rx = sp.copy(), fp.copy()
    for g in range(G):
        lost = rng.choice(k, int(rng.integers(1, 4)), replace=False)
        sp_rx[g * k + lost] = 0
        present[g, 0] = sum(1 << i for i in range(k) if i not in lost)
        plost = rng.choice(n, int(rng.integers(0, 2)), replace=False)
        fp_rx[g * n + plost] = 0
        ppm[g] = sum(1 << l for l in range(n) if l not in plost)
    oraw, ko, op, ostep, osz = _gapped(lib, G * E, sdt, 16, 0xA5, CAN)
    oi, rec, t = lib.host_recover_groups(plan, G, sp_rx, fp_rx, E, op)
    assert t["zero_copy"] == 1
    assert _gaps_intact(oraw, G * E, ostep, osz, CAN)
    rx_sh, rx_h = shards.copy(), hdr.copy()
    for g in range(G):
        for i in range(k):
            if not (int(present[g, 0]) >> i) & 1:
                rx_sh[g, i] = 0
                rx_h[g, i] = 0
    par = got["fec_data"].reshape(G, n, S)
    par = np.pad(par, ((0, 0), (0, 0), (0, shards.shape[2] - S)))
    meta = np.ascontiguousarray(got["meta"].reshape(G, n))
    _, _, o_i, o_rec = o.recover_batch_out(plan, rx_sh, rx_h, present, par, meta,
                                           got["fec_data_size"].reshape(G, n), ppm, S, E)
    assert np.array_equal(oi, o_i) and np.array_equal(rec, o_rec)
    assert (oi != 0xFF).sum() > G // 2
    for g in range(G):
        for e in range(E):
            i = int(oi[g, e])
            blk = oraw[(g * E + e) * ostep:(g * E + e) * ostep + osz]
            if i == 0xFF:
                assert (blk == 0xA5).all(), (g, e)
                continue
            got_s, want = blk.view(sdt)[0], aos[g * k + i]
            for f in ("packet_id", "fid", "timestamp", "index", "total", "ftype", "payload_type", "data_size"):
                assert got_s[f] == want[f], (g, e, f)
            nb = int(want["data_size"])
            assert np.array_equal(got_s["data"][:nb], want["data"][:nb]) and not got_s["data"][nb:].any()


def test_host_zero_copy_unaligned_takes_staged(product1200, oracle1200):
    """A struct pointer that is not 4-byte aligned inside a pinned block: the
    zero-copy kernels move dwords and use the low pointer bits as flags, so
    the batch takes the staged form (timing.zero_copy = 0), same parities."""
    from razor_amd.fec import fec_dtype, seg_dtype

    lib, o = product1200, oracle1200
    G, k, S = 8, 10, 1200
    shards, hdr = o.fill_groups(305, G, k, S, ragged=True)
    aos = o.to_aos(shards, hdr)
    sdt, fdt = seg_dtype(1200), fec_dtype(1200)
    raw, keep = lib.pinned_array((G * k * sdt.itemsize + 8,), np.uint8)
    raw[2:2 + aos.nbytes] = aos.view(np.uint8)
    sp = raw.ctypes.data + 2 + np.arange(G * k, dtype=np.uint64) * sdt.itemsize
    plan = o.plan_from_fraction(k, 80, 3)
    fecs, kf = _host_arrays(lib, G * plan.n_lines, fdt, "pinned")
    t = lib.host_encode_groups(plan, G, sp, _ptrs(fecs), fec_id0=1)
    assert t["zero_copy"] == 0
    _, ref = o.encode_aos(plan, G, aos)
    _fields_equal(fecs, ref.view(fdt).reshape(-1), "fec_data_size", "fec_data")


@pytest.mark.parametrize("name", ["c2_k10_rows_S1200_G65536", "c3_k10_full_S1200_G65536",
                                  "c4_k10_rows_S1200_G1048576", "c5_k32_rows4_S256_G65536",
                                  "k10_full_ragged_S1000_G65536"])
def test_full_size_digest_gpu(gpu, oracle1000, name):
    """Every group of a BASELINE-sized batch bit-exact vs the reference: the
    SHA-256 of the HIP encode's outputs equals the digest oracle/gen_full.c took
    of the reference's flex_fec_generate over the same PRNG inputs (config 4:
    1,048,576 groups, encoded in 65,536-group launches)."""
    import full_digest as fd

    c = fd.cases()[name]
    assert fd.digest(gpu().encode, oracle1000, c, chunk=65536) == c["sha256"]


def _w(a, g):
    """A [G][2] u64 mask array's row g as one int (bit i = segment i, k <= 128)."""
    return int(a[g, 0]) | int(a[g, 1]) << 64


def _mask_peel(plan, k, present, pp):
    """Recovered mask of the canonical peel over the masks alone (no header checks)."""
    have = int(present)
    rec = 0
    progress = True
    while progress:
        progress = False
        for l in range(plan.n_lines):
            if not (int(pp) >> l) & 1:
                continue
            mem = plan.members(l)
            miss = [i for i in mem if not (have >> i) & 1]
            if len(miss) == 1 and len(miss) < len(mem):
                have |= 1 << miss[0]
                rec |= 1 << miss[0]
                progress = True
    return rec


@pytest.mark.parametrize("tuning", list(TUNINGS))
def test_cascade_header_rejections_gpu(gpu, oracle1000, tuning):
    """Full 3x4 plan groups whose headers make the exact peel reject lines the
    masks alone would fire (fec_data_size above capacity, a member larger than
    fec_data_size): the one-launch cascade decode replays those groups' exact
    schedules in its fix-up pass and must equal the oracle, recovered masks,
    headers and data.  The workspace starts as random bytes."""
    o = oracle1000
    k, G, S = 10, 1024, 1000
    plan = o.plan_from_fraction(k, 80, 3)
    assert plan.n_lines == 7
    rng = np.random.default_rng(77)
    shards, hdr = o.fill_groups(9, G, k, S, ragged=True)
    cap = min(o.video_size, shards.shape[-1])
    parity, meta, fsize, _ = o.encode_batch(plan, shards, hdr, cap)
    present = np.zeros((G, 2), np.uint64)
    pp = np.full(G, (1 << plan.n_lines) - 1, np.uint64)
    shards_rx, hdr_rx, fsize_rx = shards.copy(), hdr.copy(), fsize.copy()
    for g in range(G):
        m = (1 << k) - 1
        for i in rng.choice(k, int(rng.integers(1, 5)), replace=False):
            m &= ~(1 << int(i))
            shards_rx[g, i] = 0xA5
            hdr_rx[g, i] = np.zeros((), po.HDR_DTYPE)
        present[g, 0] = m
        if rng.random() < 0.2:
            pp[g] &= ~np.uint64(1 << int(rng.integers(plan.n_lines)))
        r = rng.random()
        if r < 0.25:
            fsize_rx[g, rng.integers(plan.n_lines)] = cap + 1
        elif r < 0.5:
            l = int(rng.integers(plan.n_lines))
            fsize_rx[g, l] = max(1, int(fsize_rx[g, l]) - 7)
        elif r < 0.7:
            i = int(rng.integers(k))
            if (m >> i) & 1:
                hdr_rx[g, i]["size"] = min(cap, int(hdr_rx[g, i]["size"]) + 50)
    e_s, e_h, e_rec = o.recover_batch(plan, shards_rx, hdr_rx, present, parity, meta, fsize_rx, pp, cap)
    rejected = sum(int(e_rec[g, 0]) != _mask_peel(plan, k, present[g, 0], pp[g]) for g in range(G))
    assert rejected >= 20, f"only {rejected} groups where the header checks change the peel"
    eng = gpu(tuning=TUNINGS[tuning], random_workspace=True)
    out_s, out_h, rec = eng.recover(plan, shards_rx, hdr_rx, present, parity, meta, fsize_rx, pp, cap)
    assert np.array_equal(rec, e_rec)
    for g in range(G):
        for i in range(k):
            if (int(rec[g, 0]) >> i) & 1:
                assert out_h[g, i] == e_h[g, i], f"group {g} segment {i}: header"
                L = int(e_h[g, i]["size"])
                assert np.array_equal(out_s[g, i, :L], e_s[g, i, :L]), f"group {g} segment {i}: data"


@pytest.mark.parametrize("k", [36, 64])
def test_cascade_long_schedules_gpu(gpu, oracle1000, k):
    """Schedules longer than the payload lanes' 7 replayed steps: the sender's
    full 6x6 / 8x8 plans (one-launch cascade decode) with 8-12 erasures per
    group, lost parities, header rejections (fec_data_size above capacity or
    short, a member above fec_data_size) and a workspace of random bytes.  The
    groups of > 7 steps go through the fix-up pass; masks, headers and data
    must equal the oracle (the > 7-step path had no targeted case)."""
    o = oracle1000
    plan = o.plan_from_fraction(k, 80, 3)
    assert plan.n_lines == (12 if k == 36 else 16)
    G, S = 768, 256
    rng = np.random.default_rng(4242 + k)
    shards, hdr = o.fill_groups(40 + k, G, k, S, ragged=True)
    cap = S
    parity, meta, fsize, _ = o.encode_batch(plan, shards, hdr, cap)
    present = np.zeros((G, 2), np.uint64)
    pp = np.full(G, (1 << plan.n_lines) - 1, np.uint64)
    rx, rh, fs_rx = shards.copy(), hdr.copy(), fsize.copy()
    for g in range(G):
        m = (1 << k) - 1
        for i in rng.choice(k, int(rng.integers(8, 13)), replace=False):
            m &= ~(1 << int(i))
            rx[g, i] = 0xA5
            rh[g, i] = np.zeros((), po.HDR_DTYPE)
        present[g, 0] = m
        if rng.random() < 0.15:
            pp[g] &= ~np.uint64(1 << int(rng.integers(plan.n_lines)))
        r = rng.random()
        if r < 0.1:
            fs_rx[g, rng.integers(plan.n_lines)] = cap + 1
        elif r < 0.2:
            l = int(rng.integers(plan.n_lines))
            fs_rx[g, l] = max(1, int(fs_rx[g, l]) - 5)
        elif r < 0.3:
            i = int(rng.integers(k))
            if (m >> i) & 1:
                rh[g, i]["size"] = min(cap, int(rh[g, i]["size"]) + 9)
    steps = [bin(_mask_peel(plan, k, present[g, 0], pp[g])).count("1") for g in range(G)]
    assert sum(s > 7 for s in steps) >= G // 8, "too few groups with > 7 peel steps"
    e_s, e_h, e_rec = o.recover_batch(plan, rx, rh, present, parity, meta, fs_rx, pp, cap)
    rejected = sum(int(e_rec[g, 0]) != _mask_peel(plan, k, present[g, 0], pp[g]) for g in range(G))
    assert rejected >= 10, f"only {rejected} groups where the header checks change the peel"
    out_s, out_h, rec = gpu(random_workspace=True).recover(plan, rx, rh, present, parity, meta, fs_rx, pp, cap)
    assert np.array_equal(rec, e_rec)
    for g in range(G):
        for i in range(k):
            if (int(rec[g, 0]) >> i) & 1:
                assert out_h[g, i] == e_h[g, i], f"group {g} segment {i}: header"
                L = int(e_h[g, i]["size"])
                assert np.array_equal(out_s[g, i, :L], e_s[g, i, :L]), f"group {g} segment {i}: data"


@pytest.mark.parametrize("k", [6, 7, 9, 11, 12, 13, 15, 16])
@pytest.mark.parametrize("tuning", list(TUNINGS))
def test_full_plan_shapes_gpu(gpu, oracle1000, k, tuning):
    """The sender's full plans of k = 6..15 (3 or 4 columns, 5-8 lines: the
    one-launch cascade decode by default, peel + replay as the A/B) against
    the oracle: 1-5 erasures and lost parities per group, ragged sizes,
    recovered masks, headers and data bit-exact."""
    o = oracle1000
    plan = o.plan_from_fraction(k, 80, 3)
    G = 512
    rng = np.random.default_rng(100 + k)
    shards, hdr = o.fill_groups(20 + k, G, k, 1000, ragged=True)
    parity, meta, fsize, _ = o.encode_batch(plan, shards, hdr, 1000)
    present = np.zeros((G, 2), np.uint64)
    pp = np.full(G, (1 << plan.n_lines) - 1, np.uint64)
    rx, rh = shards.copy(), hdr.copy()
    for g in range(G):
        m = (1 << k) - 1
        for i in rng.choice(k, int(rng.integers(1, 6)), replace=False):
            m &= ~(1 << int(i))
            rx[g, i] = 0xA5
            rh[g, i] = np.zeros((), po.HDR_DTYPE)
        present[g, 0] = m
        if rng.random() < 0.25:
            pp[g] &= ~np.uint64(1 << int(rng.integers(plan.n_lines)))
    e_s, e_h, e_rec = o.recover_batch(plan, rx, rh, present, parity, meta, fsize, pp, 1000)
    out_s, out_h, rec = gpu(tuning=TUNINGS[tuning]).recover(plan, rx, rh, present, parity, meta, fsize, pp, 1000)
    assert np.array_equal(rec, e_rec)
    assert int(sum(bin(int(x)).count("1") for x in rec[:, 0])) > G // 2
    for g in range(G):
        for i in range(k):
            if (int(rec[g, 0]) >> i) & 1:
                assert out_h[g, i] == hdr[g, i] and out_h[g, i] == e_h[g, i]
                assert np.array_equal(out_s[g, i], shards[g, i]), f"k={k} group {g} segment {i}"


@pytest.mark.parametrize("k,col,S", [(10, 4, 64), (32, 4, 256), (12, 2, 16), (16, 8, 128), (10, 4, 1000),
                                     (96, 4, 512), (20, 3, 256), (24, 4, 1000), (13, 2, 1000)])
@pytest.mark.parametrize("tuning", list(TUNINGS))
def test_disjoint_decode_header_rejections_gpu(gpu, oracle1000, k, col, S, tuning):
    """Row plans (disjoint lines: the fused decodes) with up to 6 erasures per
    group, lost parities and corrupted headers (fec_data_size above capacity or
    below a member's size, a member's data_size above fec_data_size): recovered
    masks, headers and data equal the oracle's, under every fused form: the
    flat (group, chunk) lanes (default below 64 chunks per slot), the
    output-mapped (group, line, chunk) lanes (row kernel at k = 10 / 32,
    plan-driven otherwise), header blocks spread over the grid or at its head."""
    o = oracle1000
    rows = (k + col - 1) // col
    plan = o.plan_matrix(k, rows, col, 1)
    G = 700
    rng = np.random.default_rng(k * 1000 + S)
    shards, hdr = o.fill_groups(31, G, k, S, ragged=True)
    cap = min(o.video_size, S)
    parity, meta, fsize, _ = o.encode_batch(plan, shards, hdr, cap)
    present = np.zeros((G, 2), np.uint64)
    pp = np.full(G, (1 << plan.n_lines) - 1, np.uint64)
    rx, rh, fs_rx = shards.copy(), hdr.copy(), fsize.copy()
    for g in range(G):
        m = (1 << k) - 1
        for i in rng.choice(k, int(rng.integers(0, 7)), replace=False):
            m &= ~(1 << int(i))
            rx[g, i] = 0xA5
            rh[g, i] = np.zeros((), po.HDR_DTYPE)
        present[g, 0], present[g, 1] = m & (2**64 - 1), m >> 64
        if rng.random() < 0.2:
            pp[g] &= ~np.uint64(1 << int(rng.integers(plan.n_lines)))
        r = rng.random()
        if r < 0.15:
            fs_rx[g, rng.integers(plan.n_lines)] = cap + 1
        elif r < 0.3:
            l = int(rng.integers(plan.n_lines))
            fs_rx[g, l] = max(1, int(fs_rx[g, l]) - 3)
        elif r < 0.45:
            i = int(rng.integers(k))
            if (m >> i) & 1:
                rh[g, i]["size"] = min(cap, int(rh[g, i]["size"]) + 5)
    e_s, e_h, e_rec = o.recover_batch(plan, rx, rh, present, parity, meta, fs_rx, pp, cap)
    out_s, out_h, rec = gpu(tuning=TUNINGS[tuning]).recover(plan, rx, rh, present, parity, meta, fs_rx, pp, cap)
    assert np.array_equal(rec, e_rec)
    assert sum(bin(_w(rec, g)).count("1") for g in range(G)) > G // 4
    for g in range(G):
        for i in range(k):
            if (_w(rec, g) >> i) & 1:
                assert out_h[g, i] == e_h[g, i], f"group {g} segment {i}: header"
                L = int(e_h[g, i]["size"])
                assert np.array_equal(out_s[g, i, :L], e_s[g, i, :L]), f"group {g} segment {i}: data"
            elif (_w(present, g) >> i) & 1:
                assert out_h[g, i] == rh[g, i] and np.array_equal(out_s[g, i], rx[g, i])


@pytest.mark.parametrize("k,col,S", [(10, 4, 1200), (32, 4, 256), (12, 2, 16), (16, 8, 128), (10, 4, 64),
                                     (96, 4, 512), (20, 3, 256), (24, 4, 1200), (20, 3, 1200), (64, 4, 1024)])
@pytest.mark.parametrize("tuning", list(TUNINGS))
def test_dense_output_decode_gpu(gpu, oracle1000, oracle1200, k, col, S, tuning):
    """rfec_recover_batch_out (recovered segments into a dense output, as
    flex_fec_recover's caller-allocated out_seg): row plans with up to 6
    erasures per group, lost parities and header rejections.  Out slot e of a
    group holds its e-th erased segment: index, header and bytes equal the
    oracle's in-place recovery, 0xFF where it was not recovered; erased
    segments beyond per_group are left out of the recovered mask; the inputs
    stay untouched (checked in recover_out)."""
    o = oracle1200 if S > 1000 else oracle1000
    rows = (k + col - 1) // col
    plan = o.plan_matrix(k, rows, col, 1)
    G = 600
    rng = np.random.default_rng(k * 77 + S)
    shards, hdr = o.fill_groups(51, G, k, S, ragged=True)
    cap = min(o.video_size, S)
    parity, meta, fsize, _ = o.encode_batch(plan, shards, hdr, cap)
    present = np.zeros((G, 2), np.uint64)
    pp = np.full(G, (1 << plan.n_lines) - 1, np.uint64)
    rx, rh, fs_rx = shards.copy(), hdr.copy(), fsize.copy()
    for g in range(G):
        m = (1 << k) - 1
        for i in rng.choice(k, int(rng.integers(0, 7)), replace=False):
            m &= ~(1 << int(i))
            rx[g, i] = 0xA5
            rh[g, i] = np.zeros((), po.HDR_DTYPE)
        present[g, 0], present[g, 1] = m & (2**64 - 1), m >> 64
        if rng.random() < 0.2:
            pp[g] &= ~np.uint64(1 << int(rng.integers(plan.n_lines)))
        r = rng.random()
        if r < 0.15:
            fs_rx[g, rng.integers(plan.n_lines)] = cap + 1
        elif r < 0.3:
            l = int(rng.integers(plan.n_lines))
            fs_rx[g, l] = max(1, int(fs_rx[g, l]) - 3)
        elif r < 0.45:
            i = int(rng.integers(k))
            if (m >> i) & 1:
                rh[g, i]["size"] = min(cap, int(rh[g, i]["size"]) + 5)
    e_s, e_h, e_rec = o.recover_batch(plan, rx, rh, present, parity, meta, fs_rx, pp, cap)
    for E in (1, 2, 3):
        out_s, out_h, out_i, rec = gpu(tuning=TUNINGS[tuning]).recover_out(plan, rx, rh, present, parity, meta,
                                                                           fs_rx, pp, cap, E)
        n_rec = 0
        for g in range(G):
            missing = [i for i in range(k) if not (_w(present, g) >> i) & 1]
            want_mask = 0
            for e in range(E):
                if e >= len(missing) or not (_w(e_rec, g) >> missing[e]) & 1:
                    assert out_i[g, e] == 0xFF, (g, e)
                    continue
                i = missing[e]
                want_mask |= 1 << i
                n_rec += 1
                assert out_i[g, e] == i, (g, e)
                assert out_h[g, e] == e_h[g, i], f"group {g} out {e}: header"
                L = int(e_h[g, i]["size"])
                assert np.array_equal(out_s[g, e, :L], e_s[g, i, :L]), f"group {g} out {e}: data"
            assert _w(rec, g) == want_mask, g
        assert n_rec > G // 4


@pytest.mark.parametrize("k,col,S", [(10, 4, 1200), (32, 4, 256), (12, 2, 16), (10, 4, 64), (20, 3, 256),
                                     (24, 4, 1200), (64, 4, 1024), (11, 4, 100), (9, 3, 1000)])
def test_packed_decode_gpu(gpu, oracle1000, oracle1200, k, col, S):
    """rfec_pack_erasures + rfec_recover_packed_out (packed erasure records) vs
    rfec_recover_batch_out on the same batch (itself pinned to the oracle by
    test_dense_output_decode_gpu): out_index, recovered, the recovered headers
    and every written payload chunk bit-exact, with up to 6 erasures per group,
    lost parities and header rejections.  The device-built records equal the
    host restatement's byte for byte, and records written by the host (a
    receiver filling them as segments arrive) decode the same."""
    o = oracle1200 if S > 1000 else oracle1000
    plan = o.plan_matrix(k, (k + col - 1) // col, col, 1)
    G = 500
    rng = np.random.default_rng(k * 91 + S)
    shards, hdr = o.fill_groups(53, G, k, S, ragged=True)
    cap = min(o.video_size, S)
    cd16 = (cap + 15) // 16 * 16
    parity, meta, fsize, _ = o.encode_batch(plan, shards, hdr, cap)
    present = np.zeros((G, 2), np.uint64)
    pp = np.full(G, (1 << plan.n_lines) - 1, np.uint64)
    rx, rh, fs_rx = shards.copy(), hdr.copy(), fsize.copy()
    for g in range(G):
        m = (1 << k) - 1
        for i in rng.choice(k, int(rng.integers(0, 7)), replace=False):
            m &= ~(1 << int(i))
            rx[g, i] = 0xA5
            rh[g, i] = np.zeros((), po.HDR_DTYPE)
        present[g, 0] = m
        if rng.random() < 0.2:
            pp[g] &= ~np.uint64(1 << int(rng.integers(plan.n_lines)))
        r = rng.random()
        if r < 0.15:
            fs_rx[g, rng.integers(plan.n_lines)] = cap + 1
        elif r < 0.3:
            l = int(rng.integers(plan.n_lines))
            fs_rx[g, l] = max(1, int(fs_rx[g, l]) - 3)
        elif r < 0.45:
            i = int(rng.integers(k))
            if (m >> i) & 1:
                rh[g, i]["size"] = min(cap, int(rh[g, i]["size"]) + 5)
    eng = gpu()
    for E in sorted({1, 2, 3, k}):
        w_s, w_h, w_i, w_rec = eng.recover_out(plan, rx, rh, present, parity, meta, fs_rx, pp, cap, E)
        host_pk = pc.pack_erasures_np(k, col, rh, present, meta, fs_rx, pp, E)
        for packed in (None, host_pk):
            g_s, g_h, g_i, g_rec, pk = eng.recover_packed(plan, rx, rh, present, parity, meta, fs_rx, pp, cap, E,
                                                           packed=packed)
            assert np.array_equal(pk, host_pk), f"E={E}: packed records"
            assert np.array_equal(g_i, w_i), f"E={E}: out_index"
            assert np.array_equal(g_rec, w_rec), f"E={E}: recovered"
            sel = w_i != 0xFF
            assert sel.sum() > G // 4 or E == 1
            assert np.array_equal(g_h[sel], w_h[sel]), f"E={E}: recovered headers"
            assert np.array_equal(g_s[sel][:, :cd16], w_s[sel][:, :cd16]), f"E={E}: payloads"


@pytest.mark.parametrize("name,layers", [("k10_rows_le3", 1), ("k10_rows_ragged_le4", 1), ("k16_rows_random", 1),
                                         ("k5_strip_le3", 3)])
def test_erasure_fixture_packed_gpu(gpu, oracle1000, name, layers):
    """The reference receiver's verdicts and segment hashes (era_*.bin) through
    the packed erasure records (a slot per segment, scattered back), for the
    fixtures whose plan is a row layout."""
    pc.check_erasure_case(pc.PackedAsInPlace(gpu()), oracle1000, CASES[name], layers=layers)


def _lossy_rx(o, plan, k, G, S, rng, n_erase, p_lost_parity=0.2, corrupt=0.45):
    """A received batch: n_erase(rng) erasures per group, a lost parity with
    probability p_lost_parity, and (probability `corrupt`) header corruptions
    that make the exact peel reject lines: fec_data_size above capacity or
    below a member's size, a member's data_size above fec_data_size."""
    shards, hdr = o.fill_groups(71 + k, G, k, S, ragged=True)
    cap = min(o.video_size, S)
    parity, meta, fsize, _ = o.encode_batch(plan, shards, hdr, cap)
    present = np.zeros((G, 2), np.uint64)
    pp = np.full(G, (1 << plan.n_lines) - 1, np.uint64)
    rx, rh, fs_rx = shards.copy(), hdr.copy(), fsize.copy()
    for g in range(G):
        m = (1 << k) - 1
        for i in rng.choice(k, int(n_erase(rng)), replace=False):
            m &= ~(1 << int(i))
            rx[g, i] = 0xA5
            rh[g, i] = np.zeros((), po.HDR_DTYPE)
        present[g, 0], present[g, 1] = m & (2**64 - 1), m >> 64
        if rng.random() < p_lost_parity:
            pp[g] &= ~np.uint64(1 << int(rng.integers(plan.n_lines)))
        r = rng.random() / corrupt if corrupt else 1.0
        if r < 1 / 3:
            fs_rx[g, rng.integers(plan.n_lines)] = cap + 1
        elif r < 2 / 3:
            l = int(rng.integers(plan.n_lines))
            fs_rx[g, l] = max(1, int(fs_rx[g, l]) - 3)
        elif r < 1:
            i = int(rng.integers(k))
            if (m >> i) & 1:
                rh[g, i]["size"] = min(cap, int(rh[g, i]["size"]) + 5)
    return shards, hdr, rx, rh, present, parity, meta, fs_rx, pp, cap


def _check_dense(got, exp, G, E, where):
    o_s, o_h, o_i, rec = got
    e_s, e_h, e_i, e_rec = exp
    assert np.array_equal(rec, e_rec), f"{where}: recovered masks"
    assert np.array_equal(o_i, e_i), f"{where}: out_index"
    n = 0
    for g in range(G):
        for e in range(E):
            if e_i[g, e] == 0xFF:
                continue
            n += 1
            assert o_h[g, e] == e_h[g, e], f"{where}: group {g} out {e}: header"
            L = int(e_h[g, e]["size"])
            assert np.array_equal(o_s[g, e, :L], e_s[g, e, :L]), f"{where}: group {g} out {e}: data"
    return n


# the dense cascade decode of the sender's matrix plans: the kernel compiled for the shape (default), the
# plan-driven cascade kernel (RFEC_TUNE_PLAN_CASCADE) and the LDS peel + replay (RFEC_TUNE_GENERIC)
CASC_TUNINGS = {"default": 0, "plan_cascade": 1 << 2, "generic": 1}


@pytest.mark.parametrize("k", list(range(6, 17)))
@pytest.mark.parametrize("tuning", list(CASC_TUNINGS))
def test_dense_output_cascade_gpu(gpu, oracle1000, k, tuning):
    """rfec_recover_batch_out over the sender's full plans (rows + columns,
    recoveries cascade): 1-6 erasures per group, lost parities and header
    rejections, E = 1..4 output slots and E = k; out slots, headers, indices and
    recovered masks equal the oracle's dense restatement (only erased segments
    of rank < E recoverable; E >= the erasure count gives the in-place peel).
    Default: the one-launch cascade decode compiled for the plan's shape
    (k_decode_matrix_dense<k, col>, k = 6..16); plan_cascade: the plan-driven
    one-launch cascade decode; generic: the LDS peel + replay into the dense
    output."""
    o = oracle1000
    plan = o.plan_from_fraction(k, 80, 3)
    G, S = 500, 1000 if k <= 10 else 256
    rng = np.random.default_rng(500 + k)
    _, _, rx, rh, present, parity, meta, fs, pp, cap = _lossy_rx(o, plan, k, G, S, rng,
                                                                 lambda r: r.integers(1, 7))
    e_s, e_h, e_rec = o.recover_batch(plan, rx, rh, present, parity, meta, fs, pp, cap)
    for E in (1, 2, 3, 4, k):
        exp = o.recover_batch_out(plan, rx, rh, present, parity, meta, fs, pp, cap, E)
        got = gpu(tuning=CASC_TUNINGS[tuning]).recover_out(plan, rx, rh, present, parity, meta, fs, pp, cap, E)
        n = _check_dense(got, exp, G, E, f"k={k} E={E}")
        assert n > G // 3, (E, n)
        if E == k:  # every erased segment has a slot: the in-place peel's result
            assert np.array_equal(exp[3], e_rec)


@pytest.mark.parametrize("k", [36, 64])
def test_dense_output_long_schedules_gpu(gpu, oracle1000, k):
    """Full plans with more than 8 lines (generic peel + replay into the dense
    output): 8-12 erasures, cascades that read recovered segments back from
    their out slots."""
    o = oracle1000
    plan = o.plan_from_fraction(k, 80, 3)
    G, S = 300, 256
    rng = np.random.default_rng(900 + k)
    _, _, rx, rh, present, parity, meta, fs, pp, cap = _lossy_rx(o, plan, k, G, S, rng,
                                                                 lambda r: r.integers(8, 13), corrupt=0.3)
    for E in (3, 12):
        exp = o.recover_batch_out(plan, rx, rh, present, parity, meta, fs, pp, cap, E)
        got = gpu().recover_out(plan, rx, rh, present, parity, meta, fs, pp, cap, E)
        assert _check_dense(got, exp, G, E, f"k={k} E={E}") > G


@pytest.mark.parametrize("k,col,S", [(12, 4, 1200), (24, 4, 1200), (12, 2, 16), (16, 8, 128), (20, 3, 256),
                                     (96, 4, 512), (50, 16, 1000), (7, 7, 1000), (100, 20, 64)])
@pytest.mark.parametrize("tuning", list(TUNINGS))
def test_row_plan_encode_gpu(gpu, oracle1000, oracle1200, k, col, S, tuning):
    """Row layouts other than the compiled k = 10 / 32 ones (strip-mode plans,
    flex_fec_sender.c:112-132) through the run-time-k output-mapped encode
    (rows of up to 16 members; wider rows take the plan-driven kernel):
    parity bytes, meta records, sizes and status equal the oracle's on ragged
    segments."""
    o = oracle1200 if S > 1000 else oracle1000
    rows = (k + col - 1) // col
    plan = o.plan_matrix(k, rows, col, 1)
    G = 300
    shards, hdr = o.fill_groups(61 + k, G, k, S, ragged=True)
    cap = min(o.video_size, S)
    e_p, e_m, e_f, e_s = o.encode_batch(plan, shards, hdr, cap)
    p, m, f, s = gpu(tuning=TUNINGS[tuning]).encode(plan, shards, hdr, cap)
    assert np.array_equal(s, e_s) and np.array_equal(f, e_f)
    ok = e_s == 0
    assert np.array_equal(m[ok], e_m[ok])
    for g in range(G):
        for l in range(plan.n_lines):
            if ok[g, l]:
                L = int(e_f[g, l])
                assert np.array_equal(p[g, l, :L], e_p[g, l, :L]), f"group {g} line {l}"
