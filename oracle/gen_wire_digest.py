"""Writes tests/golden/wire_c3_digest.json: the SHA-256 of the oracle's
datagrams for the first 4,096 groups of bench.py's c3 workload -- the
SURVEY §8(d) stream of config 2 (k = 10, 1,200-B payloads, the row layer of
the 3 x 4 plan), its parities from the oracle's encode, framed as SIM_FEC and
SIM_SEG (oracle_wire_frame_*_batch, the restatement of sim_proto.c:40-97 /
sim_proto.inl:83-307, pinned to the reference's own datagrams by
tests/golden/wire_*.bin) with bench.wire_stamps' fields, into 1,280-B slots.
bench.py's `wire` sub-object compares the device framing's digest with it.

Test infrastructure (imports the oracle); run in the container:
    python oracle/gen_wire_digest.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]

import bench  # noqa: E402
from pyoracle import Oracle  # noqa: E402

G, K, S, PF = 4096, 10, 1200, 80


def digests():
    o = Oracle(1200)
    shards, hdr = o.fill_groups(bench.CONFIGS["c3"]["config_id"], G, K, S)
    assert np.array_equal(hdr.view(np.uint8), bench.make_headers(G, K, S, 0).view(np.uint8)), "headers"
    plan = o.plan_from_fraction(K, PF, 1)
    n = plan.n_lines
    parity, meta, fsize, status = o.encode_batch(plan, shards, hdr, S)
    fst, sst = bench.wire_stamps(hdr, plan, n)
    D = bench.WIRE_DSTRIDE
    dg_f, dl_f = o.frame_fec_batch(parity, meta, fsize, status, fst, S, D)
    dg_s, dl_s = o.frame_seg_batch(shards, hdr, sst, S, D)
    out = {"groups": G, "k": K, "payload": S, "payload_stride": shards.shape[2], "dstride": D, "config_id": 2,
           "fec_datagrams": int(G * n), "seg_datagrams": int(G * K),
           "fec_sha256": bench.wire_digest(dg_f, dl_f), "seg_sha256": bench.wire_digest(dg_s, dl_s),
           "generator": "oracle/gen_wire_digest.py"}
    return out


def main():
    out = digests()
    (ROOT / "tests" / "golden" / "wire_c3_digest.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
