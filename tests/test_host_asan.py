"""Host control plane under AddressSanitizer + UBSan, on the CPU.

The C host layer (razor_amd/build.py HOST_SRC: rfec_host.c, rfec_dropin.c,
rfec_hostmem.c, rfec_sender.c, rfec_rx.c) is compiled together with
tests/host_stub/stub_hip.c (a
host-memory stand-in for the HIP runtime and the kernel launches; test
infrastructure only, it does no FEC arithmetic) and driven through the same
ctypes view the GPU tests use.  What is checked here is the host side alone:

  * rfec_rx_recover's arrival-order control plane (sim_fec.c:104-241,
    flex_fec_receiver.c:208-280, sim_receiver.c:780-827) delivers the same
    packets (headers, fec_id), max_ts and dropped-parity count as the
    reference receiver / the oracle on the tests/golden/rx.json streams and on
    synthetic lossy, reordered, duplicated streams;
  * rfec_host_send_frames plans the same segments and groups as the oracle
    sender (pinned to the reference flex sender by stage.json);
  * argument checks and the error paths;
  * and none of it trips a sanitizer.

The payload bytes are not checked here (the stub computes none); the GPU
suite (test_receiver.py, test_sender.py) checks them bit-exact.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from razor_amd.build import HOST_SRC  # noqa: E402  (the C host layer's translation units)

ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def _libasan():
    r = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if r.returncode == 0 and os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def stub_lib(tmp_path_factory):
    if _libasan() is None:
        pytest.skip("libasan not available")
    if not (ROCM / "include" / "hip" / "hip_runtime_api.h").exists():
        pytest.skip("HIP headers not available")
    out = tmp_path_factory.mktemp("hoststub") / "librazor_fec_hoststub.so"
    inc = [f"-I{ROCM / 'include'}", f"-I{ROOT / 'include'}", f"-I{ROOT / 'razor_amd' / 'csrc'}"]
    cmd = ["gcc", "-std=c99", "-O1", "-g", "-fPIC", "-shared", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-DSIM_VIDEO_SIZE=1000",
           "-D__HIP_PLATFORM_AMD__", *inc, *(str(ROOT / "razor_amd" / "csrc" / f) for f in HOST_SRC),
           str(ROOT / "razor_amd" / "csrc" / "rfec_net.c"), str(ROOT / "tests" / "host_stub" / "stub_hip.c"), "-o", str(out), "-lpthread", "-lm"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


CHILD = r"""
import sys
import numpy as np
sys.path[:0] = [{root!r}, {root!r} + "/oracle", {root!r} + "/tests"]
import pyoracle as po
from razor_amd.fec import Native, RfecError, WIRE_REC_DTYPE, RFEC_WIRE_SEG, RFEC_WIRE_FEC

lib = Native(1000, path={lib!r})
o = po.Oracle(1000)
STRIDE = 1008

def rx(recs, pay, max_ts=0, max_out=1 << 16):
    recs = np.ascontiguousarray(recs)
    pay = np.ascontiguousarray(pay)
    return lib.rx_recover(len(recs), recs.ctypes.data, pay.ctypes.data, pay.shape[1], 1000, max_ts, max_out)

def check(recs, pay, max_ts=0):
    out, _, mts, rep = rx(recs, pay, max_ts)
    eo, _, emts, edrop = o.rx_recover(recs, pay, 1000, max_ts, max_out=1 << 17)
    idx = np.argsort(eo["hdr"]["seq"], kind="stable")
    assert len(out) == len(eo), (len(out), len(eo))
    assert np.array_equal(out["hdr"], eo["hdr"][idx])
    assert np.array_equal(out["fec_id"], eo["fec_id"][idx])
    assert mts == emts and rep.n_fec_dropped == edrop and rep.n_unmodelled == 0, (mts, emts, rep.n_fec_dropped, edrop)
    return len(out)

# 1. the reference receiver's own streams
fx = po.rx_fixture()
for scn in [s for s in fx["scenarios"] if not s["evict_every"]]:  # one-call ingestion: no heartbeat
    recs, pay, _, _ = po.rx_stream(o, scn)
    out, _, mts, rep = rx(recs, pay)
    assert len(out) == len(scn["recovered"]), scn["name"]
    assert sorted(int(s) for s in out["hdr"]["seq"]) == sorted(r[0] for r in scn["recovered"])
    assert mts == scn["max_ts"]
    check(recs, pay)
print("fixtures ok", len(fx["scenarios"]))

# 2. synthetic streams: oracle sender plan, parities' headers from the oracle
#    encode, arrival order shuffled with loss / duplicates / late parities
def stream(seed, frames_n, ks, pfs, loss, window, dup, late):
    rng = np.random.default_rng(seed)
    sizes = rng.choice(ks, frames_n) * 1000 - rng.integers(0, 900, frames_n)
    blob = rng.integers(0, 256, int(sizes.sum()) + 8, dtype=np.uint8)
    frames = np.zeros(frames_n, po.FRAME)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    frames["data"] = blob.ctypes.data + offs.astype(np.uint64)
    frames["size"] = sizes
    frames["payload_type"] = 96
    frames["ftype"] = np.arange(frames_n) % 50 == 0
    frames["protect_fraction"] = rng.choice(pfs, frames_n)
    frames["now_ms"] = 1_700_000_000_000 + np.arange(frames_n) * 33
    st = o.sender_init()
    segs, groups = o.sender_plan(st, frames, 1000, max_segs=frames_n * 12 + 64, max_groups=frames_n + 64)
    return po.synth_rx_stream(o, frames, blob, segs, groups, rng, loss=loss, window=window, dup=dup, late=late)

total = 0
for seed, args in enumerate([(600, (10,), (80,), 0.12, 40, 0.04, 0.0),
                             (500, (1, 3, 10, 24), (20, 50, 80, 100), 0.15, 80, 0.04, 0.0),
                             (400, (10,), (80,), 0.1, 40, 0.04, 0.25),
                             (300, (6, 10), (100,), 0.35, 200, 0.2, 0.0),
                             (3000, (10,), (80,), 0.12, 40, 0.04, 0.0)]):  # > 2048 flexes left open
    recs, pay = stream(seed, *args)
    total += check(recs, pay)
assert total > 100, total
print("synthetic ok", total)

# 2b. a peer's geometries razor's sender never emits (columns c >= col, rows
#     past row * col): modelled like the reference receiver, none unmodelled
import rx_cases as rc0
npeer = 0
for seed in range(3):
    recs, pay = rc0.peer_stream(o, np.random.default_rng(40 + seed))
    npeer += check(recs, pay)
assert npeer > 300, npeer
print("peer geometry ok", npeer)

# 2c. a peer's flex of <= 128 segments with more than 64 lines (a huge shape:
#     line jobs, not the batched peel), and the same counts with a device plan
nhuge = 0
for k, row, col in [(128, 64, 2), (128, 2, 64), (100, 50, 2)]:
    recs, pay = rc0.single_group_stream(o, k, 80, {{0, 1, 3, 2 * col + 1, 7 * col, k - 2}}, seed=k + row,
                                        shape=(row, col))
    nhuge += check(recs, pay)
assert nhuge >= 12, nhuge
print("huge small-count ok", nhuge)

# 3. across calls: max_ts carries in, old parities are dropped
recs, pay = stream(9, 200, (10,), (80,), 0.1, 10, 0.0, 0.0)
_, _, m1, _ = rx(recs, pay)
_, _, m2, rep = rx(recs, pay, m1 + 10_000)
assert m2 == m1 + 10_000 and rep.n_fec_dropped > 0

# 4. edges
out, _, mts, rep = lib.rx_recover(0, 0, 0, STRIDE, 1000, 77, 4)
assert len(out) == 0 and mts == 77
bad = np.zeros(8, WIRE_REC_DTYPE)
bad["status"] = -1
out, _, mts, rep = rx(bad, np.zeros((8, STRIDE), np.uint8), 5)
assert len(out) == 0 and mts == 5 and rep.n_groups == 0
out, _, _, _ = rx(recs, pay)
for args in [(len(out) - 1,), ()]:
    try:
        if args:
            rx(recs, pay, 0, args[0])
        else:
            lib.rx_recover(len(recs), recs.ctypes.data, pay.ctypes.data, 1000, 1000, 0, 16)
        raise AssertionError("expected RfecError")
    except RfecError:
        pass
print("edges ok")

# 5. sender staging: plan == oracle plan; the stub frames nothing, so only the
#    host side (plan, staging layout, report) runs
for seed in range(3):
    rng = np.random.default_rng(100 + seed)
    n = 300
    sizes = rng.choice((1, 3, 10, 24), n) * 1000 - rng.integers(0, 900, n)
    blob = rng.integers(0, 256, int(sizes.sum()) + 8, dtype=np.uint8)
    frames = np.zeros(n, po.FRAME)
    frames["data"] = blob.ctypes.data + np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    frames["size"] = sizes
    frames["payload_type"] = 96
    frames["protect_fraction"] = rng.choice((0, 20, 80, 100), n)
    frames["now_ms"] = 1_700_000_000_000 + np.arange(n) * 33
    segs, groups, _, _, _, _, rep = lib.send_frames(lib.sender_init(), frames, 7, 1056, max_segs=n * 25,
                                                    max_groups=n + 64, max_parities=n * 40)
    es, eg = o.sender_plan(o.sender_init(), frames, 1000, max_segs=n * 25, max_groups=n + 64)
    assert np.array_equal(segs, es) and np.array_equal(groups, eg)
print("sender ok")

# 6b. receiver sessions: the fixtures pushed in batches (with the reference's
#     evictions between them), split-invariance on a synthetic stream
import rx_cases as rc
def by_seq(rows):
    return sorted(rows, key=lambda r: r[0])
for scn in fx["scenarios"]:
    recs, pay, _, _ = po.rx_stream(o, scn)
    E = scn["evict_every"]
    sess = lib.rx_session(pay.shape[1], 1000)
    rng = np.random.default_rng(len(scn["name"]))
    a, rows = 0, []
    while a < len(recs):
        b = min(len(recs), a + (E if E else int(rng.integers(1, 700))))
        out, _, rep = sess.push(b - a, recs[a:b].ctypes.data, np.ascontiguousarray(pay[a:b]).ctypes.data)
        rows += [tuple(int(v) for v in (h["seq"], h["fid"], h["ts"], h["index"], h["total"], h["ftype"],
                                         h["payload_type"], h["size"])) + (int(f),) for h, f in zip(out["hdr"], out["fec_id"])]
        if E and b - a == E:
            sess.evict()
        a = b
    want = [tuple(r[:9]) for r in rc.expected(scn)]
    assert by_seq(rows) == by_seq(want), scn["name"]
    info = sess.info()
    assert info["max_ts"] == scn["max_ts"], scn["name"]
    if E:
        assert (info["open_flexes"], info["cached_segments"]) == (scn["flexes_left"], scn["cache_left"]), (scn["name"], info)
    sess.close()
print("sessions ok")

# 6. batched UDP I/O over loopback (rfec_net.c): slots out, slots in, the
#    reference's length rules, more than one sendmmsg / recvmmsg batch
from razor_amd.fec import RFEC_UDP_SERVER, rfec_udp_stats
rxfd, rxa = lib.udp_open("127.0.0.1", 0, RFEC_UDP_SERVER, 4 << 20)
txfd, _ = lib.udp_open("127.0.0.1", 0, RFEC_UDP_SERVER, 4 << 20)
rng = np.random.default_rng(6)
D = 1504
lens = rng.integers(0, 1500, 1500).astype(np.uint16)
dg = rng.integers(0, 256, (1500, D), dtype=np.uint8)
got = np.zeros((1500, 512), np.uint8)
gl = np.zeros(1500, np.uint16)
st = rfec_udp_stats()
n_in, off = 0, 0
while off < 1500:
    rc, done = lib.udp_send(txfd, rxa, min(200, 1500 - off), D, dg[off:].ctypes.data, lens[off:].ctypes.data, 100)
    off += done
    n_in += lib.udp_recv(rxfd, 1500 - n_in, 512, got[n_in:].ctypes.data, gl[n_in:].ctypes.data, 20, st)
for _ in range(20):
    n_in += lib.udp_recv(rxfd, 1500 - n_in, 512, got[n_in:].ctypes.data, gl[n_in:].ctypes.data, 20, st)
keep = lens >= 6
assert n_in == keep.sum(), (n_in, keep.sum())
assert np.array_equal(gl[:n_in], np.minimum(lens[keep], 512))
assert st.truncated == (lens[keep] > 512).sum() and st.dropped == ((lens > 0) & ~keep).sum()
lib.udp_close(rxfd)
lib.udp_close(txfd)
print("udp ok")

# 7. host-memory batches (rfec_hostmem.c), staged and zero-copy: the pinned-block
#    registry, the pointer / mask tables with the header-only marks, the chunk
#    and slot arithmetic, the host gathers / scatters, up to the launches the
#    stub refuses (the error comes back cleanly)
from razor_amd.fec import seg_dtype, fec_dtype
plan = lib.plan_from_fraction(10, 80, 3)
G, k, n, E = 2600, 10, plan.n_lines, 3
keep = []
def arr(cnt, dt, mem):
    if mem == "pageable":
        return np.zeros(cnt, dt)
    a, kp = lib.pinned_array((cnt,), dt)
    a.view(np.uint8)[...] = 0
    keep.append(kp)
    return a
ptrs = lambda a: a.ctypes.data + np.arange(a.shape[0], dtype=np.uint64) * a.dtype.itemsize
for mem in ("pinned", "pageable"):
    segs, fecs, out = arr(G * k, seg_dtype(1000), mem), arr(G * n, fec_dtype(1000), mem), arr(G * E, seg_dtype(1000), mem)
    segs["data_size"] = 1000
    sp, fp, op = ptrs(segs), ptrs(fecs), ptrs(out)
    for call in (lambda: lib.host_encode_groups(plan, G, sp, fp),
                 lambda: lib.host_recover_groups(plan, G, np.where(np.arange(G * k) % 7 == 0, 0, sp), fp, E, op)):
        try:  # (the stub refuses the recover and the zero-copy launches: an error is the expected outcome)
            call()
        except RfecError:
            pass
print("hostmem ok")

# 8. packed erasure records (rfec_host.c): the stride and argument checks, up to
#    the launches the stub refuses
c5 = lib.plan_matrix(32, 8, 4, 1)
assert lib.packed_stride(c5, 2) == 192 and lib.packed_stride(lib.plan_matrix(10, 3, 4, 3), 2) == 0
for call in (lambda: lib.pack_erasures(c5, 4, 16, 16, 16, 16, 16, 2, 16),
             lambda: lib.recover_packed_out(c5, 4, 256, 256, 16, 16, 16, 16, 2, 16, 16, 16),
             lambda: lib.recover_packed_out(lib.plan_matrix(10, 3, 4, 3), 4, 1200, 1200, 16, 16, 16, 16, 2, 16, 16,
                                            16)):
    try:
        call()
    except RfecError:
        pass
print("packed ok")
"""


def test_host_control_plane_under_asan(stub_lib, tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD.format(root=str(ROOT), lib=str(stub_lib)))
    env = dict(os.environ)
    env["LD_PRELOAD"] = _libasan()
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:halt_on_error=1:exitcode=66"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-8000:]
    assert "sender ok" in r.stdout and "udp ok" in r.stdout and "hostmem ok" in r.stdout and "packed ok" in r.stdout
