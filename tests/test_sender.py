"""Sender staging end to end on the GPU: frames in host memory ->
rfec_host_send_frames -> SIM_SEG / SIM_FEC datagrams in host memory, checked
against what the reference flex sender emitted for the same frames
(tests/golden/stage.json, oracle/gen_stage.c) and against the oracle's wire
parser."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import pyoracle as po
import stage_cases as sc

UID = 0x1234ABCD
DSTRIDE = 1056  # >= 1000 + 49


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")
    from razor_amd.fec import native
    return native(1000)


def _fnv(b: bytes) -> int:
    h = 0xCBF29CE484222325
    for x in b:
        h ^= x
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _check_scenario(lib, oracle, scn, splits, zero_copy=False):
    frames, blob = po.stage_frames(scn)
    keep = []
    if zero_copy:  # frames and datagram outputs in rfec_pinned_alloc blocks: the device reads / writes them
        pb, k = lib.pinned_array(blob.shape, np.uint8)
        pb[...] = blob
        frames["data"] = frames["data"] - np.uint64(blob.ctypes.data) + np.uint64(pb.ctypes.data)
        blob = pb
        keep.append(k)
    st = lib.sender_init()
    segs, groups, sdg, sdl, fdg, fdl = [], [], [], [], [], []
    seg_base = 0
    for lo, hi in zip(splits[:-1], splits[1:]):
        bufs, kw = None, {}
        if zero_copy:
            ms = 64 * (hi - lo) + 256
            mp = 2 * ms
            out = [lib.pinned_array(shape, dt) for shape, dt in (((ms, DSTRIDE), np.uint8), ((ms,), np.uint16),
                                                                 ((mp, DSTRIDE), np.uint8), ((mp,), np.uint16))]
            keep += [o[1] for o in out]
            bufs = tuple(o[0] for o in out)
            kw = dict(max_segs=ms, max_parities=mp, bufs=bufs)
        s, g, a, al, b, bl, rep = lib.send_frames(st, frames[lo:hi], UID, DSTRIDE, **kw)
        if zero_copy:
            assert rep.zero_copy == 3 or (rep.n_segs == 0 and rep.zero_copy & 2), rep.zero_copy
            a, al, b, bl = a.copy(), al.copy(), b.copy(), bl.copy()
        s = s.copy()
        s["frame"] += lo
        g = g.copy()
        g["first_seg"] += seg_base
        seg_base += len(s)
        for lst, v in ((segs, s), (groups, g), (sdg, a), (sdl, al), (fdg, b), (fdl, bl)):
            lst.append(v)
    segs, groups = np.concatenate(segs), np.concatenate(groups)
    sdg, sdl, fdg, fdl = np.concatenate(sdg), np.concatenate(sdl), np.concatenate(fdg), np.concatenate(fdl)
    exp = np.array(scn["segments"], np.int64)
    for j, k in enumerate(sc.SEG_FIELDS[:-1]):
        assert np.array_equal(segs[k].astype(np.int64), exp[:, j]), (scn["name"], k)
    # SIM_SEG datagrams: header fields and payload = the frame bytes
    recs, pay = oracle.parse_batch(sdg, sdl, 1008, 1000)
    assert (recs["status"] == 0).all() and (recs["mid"] == 0x17).all() and (recs["uid"] == UID).all()
    assert np.array_equal(recs["hdr"]["seq"], segs["packet_id"]) and np.array_equal(recs["fec_id"], segs["fec_id"])
    assert np.array_equal(recs["data_size"], segs["data_size"]) and (recs["remb"] == 0xFF).all()  # remb 1 on the wire
    base = blob.ctypes.data
    for i in range(len(segs)):
        off = int(frames["data"][segs["frame"][i]] - base) + int(segs["offset"][i])
        n = int(segs["data_size"][i])
        assert np.array_equal(pay[i, :n], blob[off:off + n]), (scn["name"], i)
    # SIM_FEC datagrams, group by group: what the reference sender emitted
    frecs, fpay = oracle.parse_batch(fdg, fdl, 1008, 1000)
    assert (frecs["status"] == 0).all() and (frecs["mid"] == 0x1C).all()
    p = 0
    assert len(groups) == len(scn["groups"])
    for g, eg in zip(groups, scn["groups"]):
        for par in eg["parities"]:
            r = frecs[p]
            got = [int(r["index"]), int(r["row"]), int(r["col"]), int(r["count"]), int(r["hdr"]["seq"]),
                   int(r["hdr"]["fid"]), int(r["hdr"]["ts"]), int(r["hdr"]["index"]), int(r["hdr"]["total"]),
                   int(r["hdr"]["ftype"]), int(r["hdr"]["payload_type"]), int(r["hdr"]["size"]),
                   int(r["data_size"])]
            assert got == par[:13], (scn["name"], p)
            assert int(r["fec_id"]) == eg["fec_id"] and int(r["base_id"]) == eg["base_id"]
            assert f"{_fnv(fpay[p, :int(r['data_size'])].tobytes()):016x}" == par[13], (scn["name"], p)
            p += 1
    assert p == len(frecs)
    # transport_seq: creation order, each group's parities right after its last segment
    order = []
    gi = 0
    for i in range(len(segs)):
        order.append(("s", i))
        while gi < len(groups) and groups["first_seg"][gi] + groups["count"][gi] - 1 == i:
            order.extend(("f", q) for q in range(int(groups["n_lines"][gi])))
            gi += 1
    ts = np.zeros(len(order), np.int64)
    fcur = 0
    for t, (kind, i) in enumerate(order):
        if kind == "s":
            ts[t] = recs["transport_seq"][i]
        else:
            ts[t] = frecs["transport_seq"][fcur]
            fcur += 1
    assert np.array_equal(ts, np.arange(len(order)) & 0xFFFF)


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", [False, True])
@pytest.mark.parametrize("name", ["steady_k10_pf80", "mixed", "fractions"])
def test_send_frames_gpu(lib, oracle1000, name, zero_copy):
    """zero_copy: the frames and the datagram outputs in pinned blocks (the
    device gathers the segments out of the frames at their byte offsets and
    frames straight into the outputs)."""
    scn = {s["name"]: s for s in po.stage_fixture()["scenarios"]}[name]
    _check_scenario(lib, oracle1000, scn, [0, len(scn["frames"])], zero_copy)


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", [False, True])
@pytest.mark.parametrize("name", ["mixed", "fractions"])
def test_send_frames_split_calls_gpu(lib, oracle1000, name, zero_copy):
    """The same frames over several calls: open groups are carried across
    (zero copy: the carried segments from the pinned staging, the rows of
    their datagrams past the caller's output not written)."""
    scn = {s["name"]: s for s in po.stage_fixture()["scenarios"]}[name]
    n = len(scn["frames"])
    _check_scenario(lib, oracle1000, scn, [0, 1, 2, 5, n // 2, n // 2 + 1, n], zero_copy)
