"""Full-size digests (tests/golden/full_hashes.json, written by
oracle/gen_full.c from the reference's flex_fec_generate): regenerate a
BASELINE.json-sized batch from the PRNG spec piece by piece, run an engine
over each piece, and SHA-256 the outputs group by group in the order
    parity [n][stride] | meta [n] (20 B) | fec_data_size [n] (u16 LE)."""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

import numpy as np

import pyoracle as po

GOLDEN = Path(__file__).resolve().parent / "golden"


def cases():
    return {c["name"]: c for c in json.loads((GOLDEN / "full_hashes.json").read_text())["cases"]}


def case_plan(oracle, c):
    if c["plan"] == "matrix":
        return oracle.plan_matrix(c["k"], c["row"], c["col"], c["layers"])
    return oracle.plan_from_fraction(c["k"], c["pf"], c["layers"])


def group_records(parity, meta, fsize):
    """[G][n*stride + 20n + 2n] bytes: the digest's per-group record."""
    G = parity.shape[0]
    return np.concatenate([parity.reshape(G, -1), np.ascontiguousarray(meta).view(np.uint8).reshape(G, -1),
                           np.ascontiguousarray(fsize).astype("<u2").view(np.uint8).reshape(G, -1)], axis=1)


def digest(engine_encode, oracle, c, chunk=65536):
    """engine_encode(plan, shards, hdr, capacity) -> (parity, meta, fsize, status)."""
    plan = case_plan(oracle, c)
    assert plan.n_lines == c["n_lines"]
    piece = oracle.fill_stream(c["config_id"], c["k"], c["S"], c["stride"], ragged=bool(c["ragged"]))
    h = hashlib.sha256()
    for g0 in range(0, c["groups"], chunk):
        ng = min(chunk, c["groups"] - g0)
        shards, hdr = piece(g0, ng)
        parity, meta, fsize, status = engine_encode(plan, shards, hdr, c["S"])
        assert int(np.count_nonzero(status)) == 0
        h.update(group_records(parity, meta, fsize).tobytes())
        del shards, hdr, parity, meta, fsize
    return h.hexdigest()
