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
