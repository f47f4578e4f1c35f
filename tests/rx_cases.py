"""Receiver-ingestion checks: the recovered segments against the reference's
sim_fec.c + flex receiver on the lossy streams of tests/golden/rx.json."""
from __future__ import annotations

import numpy as np

import pyoracle as po


def expected(scn):
    rec = scn["recovered"]
    return [(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7], r[8], r[9]) for r in rec]


def got_rows(out, pay):
    rows = []
    for o, p in zip(out, pay):
        h = o["hdr"]
        n = int(h["size"])
        rows.append((int(h["seq"]), int(h["fid"]), int(h["ts"]), int(h["index"]), int(h["total"]), int(h["ftype"]),
                     int(h["payload_type"]), n, int(o["fec_id"]), f"{po.fnv1a(p[:n].tobytes()):016x}"))
        assert not p[n:].any()
    return rows


def _peer_plan(k, row, col, xcols):
    """The lines the reference receiver walks for a (count = k, row, col) flex
    (flex_fec_receiver.c:118-126 rows of col, :175-183 columns of row, both
    cut at count): every row, the columns c < col, and the extra columns
    `xcols` (c >= col); lines of fewer than 2 members dropped."""
    p = po.rfec_plan()
    p.k, p.row, p.col, p.rc = k, row, col, 1
    lines = []
    r = 0
    while r * col < k:
        n = min(col, k - r * col)
        if n >= 2:
            lines.append((r * col, 1, n, r))
        r += 1
    for c in list(range(col)) + sorted(xcols):
        n = 0
        while n < row and n * col + c < k:
            n += 1
        if n >= 2:
            lines.append((c, col, n, 0x80 | c))
    assert len(lines) <= 64
    for i, (f, s, n, idx) in enumerate(lines):
        p.line[i].first, p.line[i].stride, p.line[i].count, p.line[i].index = f, s, n, idx
    p.n_lines = len(lines)
    p.n_row_lines = sum(1 for ln in lines if ln[3] < 0x80)
    return p


def peer_stream(oracle, rng, n_groups=90, video_size=1000):
    """Parsed-datagram records + payload rows of FEC groups in geometries
    razor's own sender never emits but a peer may: parities of columns
    c >= col, and row * col < count (members past the matrix, reachable by
    rows only).  Per group its datagrams arrive shuffled, 15% of the segments
    and 10% of the parities lost."""
    stride = (video_size + 15) // 16 * 16
    recs, pays = [], []
    pid, ts = 1, 0
    for g in range(n_groups):
        kind = g % 3
        if kind == 0:  # extra columns
            col = int(rng.integers(3, 7))
            k = int(rng.integers(col + 2, 40))
            row = -(-k // col)
            xc = [c for c in range(col, min(k, 100)) if rng.random() < 0.3][:12]
        elif kind == 1:  # rows past the matrix
            col = int(rng.integers(2, 6))
            row = int(rng.integers(1, 4))
            k = row * col + int(rng.integers(1, 2 * col + 1))
            xc = [c for c in range(col, min(k, 100)) if rng.random() < 0.2][:6]
        else:  # razor's own geometry
            col = int(rng.integers(3, 6))
            k = int(rng.integers(6, 30))
            row = -(-k // col)
            xc = []
        plan = _peer_plan(k, row, col, xc)
        hdr = np.zeros((1, k), po.HDR_DTYPE)
        hdr["seq"] = pid + np.arange(k)
        hdr["fid"] = 1 + g
        hdr["ts"] = ts
        hdr["index"] = np.arange(k)
        hdr["total"] = k
        hdr["payload_type"] = 96
        hdr["size"] = rng.integers(1, video_size + 1, k)
        sh = np.zeros((1, k, stride), np.uint8)
        for i in range(k):
            sh[0, i, :int(hdr["size"][0, i])] = rng.integers(0, 256, int(hdr["size"][0, i]), dtype=np.uint8)
        par, meta, fs, st = oracle.encode_batch(plan, sh, hdr, video_size)
        items = []
        for i in range(k):
            if rng.random() < 0.15:
                continue
            r = np.zeros((), po.WIRE_REC)
            r["mid"], r["ver"], r["remb"] = 0x17, 1, 0xFF
            r["hdr"] = hdr[0, i]
            r["fec_id"], r["data_size"] = 1 + g, hdr["size"][0, i]
            items.append((r, sh[0, i]))
        for l in range(plan.n_lines):
            if rng.random() < 0.10 or st[0, l] != 0:
                continue
            r = np.zeros((), po.WIRE_REC)
            r["mid"], r["ver"] = 0x1C, 1
            r["fec_id"], r["base_id"], r["count"] = 1 + g, pid, k
            r["row"], r["col"], r["index"] = row, col, plan.line[l].index
            r["send_ts"] = ts
            r["hdr"] = meta[0, l]
            r["data_size"] = fs[0, l]
            items.append((r, par[0, l]))
        for j in rng.permutation(len(items)):
            recs.append(items[j][0])
            pays.append(items[j][1])
        pid += k
        ts += 33
    return np.array(recs, po.WIRE_REC), np.array(pays, np.uint8)


def matrix_parities(seg, pay, fec_id, base_id, k, row, col):
    """A foreign peer's flex of `row` rows x `col` columns (not razor's
    planner): one parity per row over [r col, min(k, (r + 1) col)), index r,
    and one per column over r col + c < k, index 0x80 | c
    (flex_fec_sender.c:157-233 with the peer's row / col), each one
    flex_fec_generate (flex_fec_xor.c:13-50): payloads XORed zero-padded to
    L = max data_size, meta = XOR of the 20-byte headers."""
    hdr32 = seg["hdr"][:k].copy().view(np.uint32).reshape(k, 5)
    sizes = seg["data_size"][:k].astype(np.int64)
    lines = [(list(range(r * col, min(k, (r + 1) * col))), r) for r in range(row)]
    lines += [([r * col + c for r in range(row) if r * col + c < k], 0x80 | c) for c in range(col)]
    out = []
    for mem, index in lines:
        if len(mem) < 2:
            continue
        L = int(sizes[mem].max())
        pp = np.bitwise_xor.reduce(pay[mem], axis=0)
        pp[L:] = 0
        r = np.zeros((), po.WIRE_REC)
        r["mid"], r["ver"] = 0x1C, 1
        r["fec_id"], r["base_id"], r["count"] = fec_id, base_id, k
        r["row"], r["col"], r["index"] = row, col, index
        r["send_ts"] = int(seg["hdr"]["ts"][k - 1])
        r["hdr"] = np.bitwise_xor.reduce(hdr32[mem], axis=0).view(r["hdr"].dtype)[0]
        r["data_size"] = L
        out.append((r, pp))
    return out


def single_group_stream(oracle, k, pf, erase, tamper=None, seed=0, video_size=1000, shape=None):
    """One flex of k segments (packet ids 1..k, ragged sizes) and every parity
    the reference sender emits for it (k <= 255: the oracle's plan + encode;
    above: pyoracle's restatement of flex_fec_sender_update), arriving after
    the segments not in `erase`.  tamper = (parity index, data_size): that
    parity's fec_data_size is cut below a member's size, so flex_fec_recover
    rejects its line (flex_fec_xor.c:88-89).  shape = (row, col): a peer's
    matrix flex of that shape instead of the sender's plan for pf.  Returns
    (recs, pay)."""
    rng = np.random.default_rng(seed)
    stride = (video_size + 15) // 16 * 16
    sizes = rng.integers(video_size // 2, video_size + 1, k)
    pay = np.zeros((k, stride), np.uint8)
    for i in range(k):
        pay[i, :sizes[i]] = rng.integers(0, 256, sizes[i], dtype=np.uint8)
    seg = np.zeros(k, po.WIRE_REC)
    seg["mid"], seg["ver"], seg["remb"] = 0x17, 1, 0xFF
    seg["hdr"]["seq"] = 1 + np.arange(k)
    seg["hdr"]["fid"] = 1 + np.arange(k) // 10
    seg["hdr"]["ts"] = 33 * (np.arange(k) // 10)
    seg["hdr"]["index"] = np.arange(k) % 10
    seg["hdr"]["total"] = 10
    seg["hdr"]["payload_type"] = 96
    seg["hdr"]["size"] = sizes
    seg["data_size"] = sizes
    seg["fec_id"] = 7
    g = np.zeros((), po.GROUP_PLAN)
    g["first_seg"], g["count"], g["fec_id"], g["base_id"], g["protect_fraction"] = 0, k, 7, 1, pf
    if shape is not None:
        pars = matrix_parities(seg, pay, 7, 1, k, *shape)
    elif k > 255:
        pars = po._big_group_parities(oracle, seg, pay, g, k, pf)
    else:
        plan = oracle.plan_from_fraction(k, pf, 3)
        hdr = np.zeros((1, k), po.HDR_DTYPE)
        hdr[0] = seg["hdr"]
        par, meta, fs, _ = oracle.encode_batch(plan, pay[None], hdr, video_size)
        pars = []
        for l in range(plan.n_lines):
            r = np.zeros((), po.WIRE_REC)
            r["mid"], r["ver"] = 0x1C, 1
            r["fec_id"], r["base_id"], r["count"] = 7, 1, k
            r["row"], r["col"], r["index"] = plan.row, plan.col, plan.line[l].index
            r["send_ts"] = int(seg["hdr"]["ts"][-1])
            r["hdr"], r["data_size"] = meta[0, l], fs[0, l]
            pars.append((r, par[0, l]))
    recs, rows = [], []
    for i in range(k):
        if i not in erase:
            recs.append(seg[i])
            rows.append(pay[i])
    for r, p in pars:
        if tamper is not None and int(r["index"]) == tamper[0]:
            r = r.copy()
            r["data_size"] = tamper[1]
        recs.append(r)
        rows.append(p)
    return np.array(recs, po.WIRE_REC), np.array(rows, np.uint8)


C3_LINES = [(0, 1, 4, 0), (4, 1, 4, 1), (8, 1, 2, 2), (0, 4, 3, 0x80), (1, 4, 3, 0x81), (2, 4, 2, 0x82),
            (3, 4, 2, 0x83)]  # the sender's 3 x 4 plan at k = 10: rows, then columns (first, stride, count, index)


def c3_groups(G, k=10, cap=16):
    """Parsed-datagram records of G groups of the sender's 3 x 4 plan, in
    order: segments [G][k] (packet ids 1 + g k + i, timestamp 33 g, data_size
    cap) and parities [G][7] (send_ts 33 g, meta = XOR of the members'
    headers).  Headers only: for the control plane (tests/test_rx_shards.py,
    tools/rx_host_bench.py)."""
    from razor_amd.fec import RFEC_WIRE_FEC, RFEC_WIRE_SEG, WIRE_REC_DTYPE
    seg = np.zeros((G, k), WIRE_REC_DTYPE)
    seg["mid"], seg["ver"], seg["remb"] = RFEC_WIRE_SEG, 1, 0xFF
    g = np.arange(G)[:, None]
    i = np.arange(k)[None, :]
    seg["hdr"]["seq"] = 1 + g * k + i
    seg["hdr"]["fid"] = 1 + g
    seg["hdr"]["ts"] = 33 * g
    seg["hdr"]["index"] = i
    seg["hdr"]["total"] = k
    seg["hdr"]["payload_type"] = 96
    seg["hdr"]["size"] = cap
    seg["data_size"] = cap
    seg["fec_id"] = (np.arange(G)[:, None] % 65535 + 1) * np.ones((1, k), np.int64)
    fec = np.zeros((G, len(C3_LINES)), WIRE_REC_DTYPE)
    fec["mid"], fec["ver"] = RFEC_WIRE_FEC, 1
    fec["fec_id"] = seg["fec_id"][:, :1]
    fec["base_id"] = seg["hdr"]["seq"][:, :1]
    fec["count"], fec["row"], fec["col"] = k, 3, 4
    fec["send_ts"] = 33 * g
    fec["data_size"] = cap
    c3_metas(seg, fec)
    return seg, fec


def c3_metas(seg, fec):
    """fec[:, l].hdr = XOR of line l's members' headers (flex_fec_xor.c:13-44)."""
    from razor_amd.fec import HDR_DTYPE
    G, k = seg.shape
    hv = seg["hdr"].copy().view(np.uint32).reshape(G, k, 5)
    for l, (first, stride, cnt, idx) in enumerate(C3_LINES):
        x = np.bitwise_xor.reduce(hv[:, first:first + stride * cnt:stride], axis=1)
        fec["hdr"][:, l] = x.view(HDR_DTYPE).reshape(G)
        fec["index"][:, l] = idx


def c3_shuffle(seg, fec, loss, window, seed=1, dup=0.02):
    """The arrival order: each group's parities after its last segment,
    independent loss, reordering within `window` arrivals, `dup` duplicates
    (arriving up to 3 windows late)."""
    rng = np.random.default_rng(seed)
    G, k = seg.shape
    nl = fec.shape[1]
    g = np.arange(G)[:, None]
    recs = np.concatenate([seg, fec], axis=1).reshape(-1)
    pos = (np.concatenate([np.broadcast_to(np.arange(k, dtype=np.float64), (G, k)),
                           np.broadcast_to(k - 1 + (np.arange(nl) + 1) / (nl + 1), (G, nl))], axis=1)
           + g * (k + 1)).reshape(-1)
    keep = rng.random(len(recs)) >= loss
    recs, pos = recs[keep], pos[keep]
    d = rng.random(len(recs)) < dup
    key = np.concatenate([pos + rng.integers(0, window, len(pos)),
                          pos[d] + rng.integers(window, 3 * window, int(d.sum()))])
    recs = np.concatenate([recs, recs[d]])
    return recs[np.argsort(key, kind="stable")]


def c3_records(G, loss, window, seed=1, k=10, cap=16):
    """c3_groups shuffled by c3_shuffle: a lossy, reordered c3 stream with duplicates."""
    seg, fec = c3_groups(G, k, cap)
    return c3_shuffle(seg, fec, loss, window, seed)
