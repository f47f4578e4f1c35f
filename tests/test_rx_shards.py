"""CPU: the receiver session's sharded control plane (rfec_rx.c, the
fec_id-partitioned replay) against the oracle's event-by-event receiver
(oracle_rx_recover, pinned to the reference's sim_fec.c / flex receiver by
tests/golden/rx.json) -- delivered headers, fec_id, max_ts, dropped parities
-- on every path a batch can take:

  * parallel: every packet id under one fec_id, no parity near the 3 s drop;
  * in arrival order over the shards: a parity of the batch could meet the
    drop through an earlier segment timestamp (sim_fec.c:148);
  * rolled back: a recovery raises max_ts past a later parity's limit while
    the shards run in parallel -- undone (the journal) and replayed in order;
  * merged: a packet id under two fec_ids (the partition does not hold) --
    rolled back, the shards merged into one serial state for good;
  * evictions between batches (sim_fec_evict over the union of the shards).

The C host layer is built with tests/host_stub/stub_hip.c (host stand-in for
the HIP runtime; no payload arithmetic: the GPU suite checks bytes,
tests/test_receiver.py)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from razor_amd.build import HOST_SRC  # noqa: E402

import pyoracle as po  # noqa: E402
from rx_cases import c3_groups, c3_metas, c3_records, c3_shuffle  # noqa: E402

ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
CAP = 16


@pytest.fixture(scope="module")
def stub(tmp_path_factory):
    if not (ROCM / "include" / "hip" / "hip_runtime_api.h").exists():
        pytest.skip("HIP headers not available")
    out = tmp_path_factory.mktemp("rxshards") / "librazor_fec_rxshards.so"
    inc = [f"-I{ROCM / 'include'}", f"-I{ROOT / 'include'}", f"-I{ROOT / 'razor_amd' / 'csrc'}"]
    cmd = ["gcc", "-std=c99", "-O1", "-g", "-fPIC", "-shared", "-DSIM_VIDEO_SIZE=1200", "-D__HIP_PLATFORM_AMD__", *inc,
           *(str(ROOT / "razor_amd" / "csrc" / f) for f in HOST_SRC), str(ROOT / "razor_amd" / "csrc" / "rfec_net.c"),
           str(ROOT / "tests" / "host_stub" / "stub_hip.c"), "-o", str(out), "-lpthread", "-lm"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    from razor_amd.fec import Native
    return Native(1200, path=str(out))


@pytest.fixture(scope="module")
def oracle():
    return po.Oracle(1200)


def push_all(lib, recs, batch, threads, evict_every=0):
    """The stream in batches through a fresh session; evictions after every
    `evict_every` records (batches end there).  Returns (delivered sorted by
    packet id, max_ts, dropped, session info)."""
    from razor_amd.fec import RX_SEG_DTYPE, rfec_rx_report
    sess = lib.rx_session(CAP, CAP, threads)
    pay = np.zeros((len(recs), CAP), np.uint8)
    recs = np.ascontiguousarray(recs)
    max_out = 4 * max(batch, evict_every or 0) + 64
    out = np.zeros(max_out, RX_SEG_DTYPE)
    outp = np.zeros((max_out, CAP), np.uint8)
    nout, rep = C.c_uint32(), rfec_rx_report()
    got, dropped, a = [], 0, 0
    while a < len(recs):
        b = min(len(recs), a + batch)
        if evict_every:
            b = min(b, (a // evict_every + 1) * evict_every)
        lib._check(lib.lib.rfec_rx_session_push(sess.h, b - a, recs.ctypes.data + a * 64, pay.ctypes.data + a * CAP,
                                                out.ctypes.data, outp.ctypes.data, max_out, C.byref(nout),
                                                C.byref(rep), None), "push")
        got.append(out[:nout.value].copy())
        dropped += rep.n_fec_dropped
        assert rep.n_unmodelled == 0
        if evict_every and b % evict_every == 0:
            sess.evict()
        a = b
    info = sess.info()
    sess.close()
    got = np.concatenate(got) if got else np.zeros(0, RX_SEG_DTYPE)
    return got[np.argsort(got["hdr"]["seq"], kind="stable")], info["max_ts"], dropped, info


def expect(oracle, recs, evict_every=0):
    eo, _, mts, drop = oracle.rx_recover(np.ascontiguousarray(recs), np.zeros((len(recs), CAP), np.uint8), CAP,
                                         max_out=1 << 20, evict_every=evict_every)
    return eo[np.argsort(eo["hdr"]["seq"], kind="stable")], mts, drop


def same(got, want):
    g, mts, drop, _ = got
    e, emts, edrop = want
    assert len(g) == len(e)
    assert np.array_equal(g["hdr"], e["hdr"]) and np.array_equal(g["fec_id"], e["fec_id"])
    assert (mts, drop) == (emts, edrop)


@pytest.mark.parametrize("threads", [2, 3, 8])
@pytest.mark.parametrize("batch", [97, 1024])
def test_parallel_equals_serial(stub, oracle, threads, batch):
    """A conforming c3 stream (5 % loss, reordering, duplicates): every batch
    replays in parallel, deliveries = the oracle's = the serial session's."""
    recs = c3_records(1500, 0.05, 32, seed=threads + batch)
    want = expect(oracle, recs)
    got = push_all(stub, recs, batch, threads)
    same(got, want)
    info = got[3]
    assert info["threads"] == threads and info["batches_parallel"] > 0
    assert info["batches_serial"] == info["batches_rolled_back"] == 0
    same(push_all(stub, recs, batch, 1), want)


def test_parity_near_drop_replays_in_order(stub, oracle):
    """Parities arriving 3+ s behind the newest segment (sim_fec.c:148 drops
    them): those batches replay in arrival order over the shards, the rest in
    parallel; the drops match."""
    seg, fec = c3_groups(1200, cap=CAP)
    fec["send_ts"][600:700] -= 5000  # (their send_ts only: metas unchanged)
    recs = c3_shuffle(seg, fec, 0.05, 32, seed=3)
    want = expect(oracle, recs)
    assert want[2] > 0
    got = push_all(stub, recs, 256, 8)
    same(got, want)
    assert got[3]["batches_serial"] > 0 and got[3]["batches_parallel"] > 0 and got[3]["threads"] == 8


def test_recovery_raising_max_ts_rolls_back(stub, oracle):
    """A lost segment whose timestamp is far ahead (group 300's member 1 at
    10^6 ms): its recovery raises max_ts mid-batch, so later parities of the
    same batch are dropped in the reference.  The parallel replay sees it,
    rolls every shard back to the batch's start and replays it in order."""
    seg, fec = c3_groups(900, cap=CAP)
    seg["hdr"]["ts"][300, 1] = 1_000_000
    c3_metas(seg, fec)
    recs = c3_shuffle(seg, fec, 0.0, 8, seed=5, dup=0.0)
    recs = recs[~((recs["mid"] == seg["mid"][0, 0]) & (recs["hdr"]["seq"] == seg["hdr"]["seq"][300, 1]))]
    want = expect(oracle, recs)
    assert want[1] == 1_000_000 and want[2] > 0
    got = push_all(stub, recs, 4096, 8)
    same(got, want)
    assert got[3]["batches_rolled_back"] >= 1 and got[3]["threads"] == 8


def test_packet_id_under_two_fec_ids_merges(stub, oracle):
    """A segment of group 400 re-sent under group 401's fec_id (a packet id
    under two fec_ids: the partition no longer holds) -- the batch is rolled
    back and the shards merged into one serial state; deliveries still equal
    the reference's."""
    seg, fec = c3_groups(1000, cap=CAP)
    recs = c3_shuffle(seg, fec, 0.05, 32, seed=7)
    stray = seg[400, 3].copy()
    stray["fec_id"] = seg["fec_id"][401, 0]
    at = int(np.nonzero((recs["mid"] == seg["mid"][0, 0]) & (recs["hdr"]["seq"] >= seg["hdr"]["seq"][405, 0]))[0][0])
    recs = np.concatenate([recs[:at], [stray], recs[at:]])
    want = expect(oracle, recs)
    got = push_all(stub, recs, 512, 8)
    same(got, want)
    assert got[3]["threads"] == 1 and got[3]["batches_rolled_back"] >= 1 and got[3]["batches_parallel"] > 0


@pytest.mark.parametrize("threads", [1, 8])
def test_evictions_between_batches(stub, oracle, threads):
    """sim_fec_evict between batches (every 700 records): flexes in fec_id
    order and cached segments in packet-id order over the union of the
    shards, as the oracle's evictions on the whole stream."""
    recs = c3_records(1500, 0.08, 48, seed=11)
    want = expect(oracle, recs, evict_every=700)
    got = push_all(stub, recs, 256, threads, evict_every=700)
    same(got, want)


def test_set_threads_rules(stub):
    """Shards are chosen before the first push (1..64)."""
    from razor_amd.fec import RfecError
    sess = stub.rx_session(CAP, CAP, 5)
    assert sess.info()["threads"] == 5
    for bad in (0, 65):
        with pytest.raises(RfecError):
            stub._check(stub.lib.rfec_rx_session_set_threads(sess.h, bad), "set_threads")
    recs = np.ascontiguousarray(c3_records(20, 0.0, 4))
    pay = np.zeros((len(recs), CAP), np.uint8)
    sess.push(len(recs), recs.ctypes.data, pay.ctypes.data)
    with pytest.raises(RfecError):
        stub._check(stub.lib.rfec_rx_session_set_threads(sess.h, 2), "set_threads")
    sess.close()
