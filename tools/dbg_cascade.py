"""Lab: one cascade-decode call on the inputs of a GPU test, against a chosen
library build (e.g. an A/B build from tools/build_ab.sh), serialised.
Usage: python tools/dbg_cascade.py LIB [k] [G] [mode]   (mode: in_place | dense)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))
import numpy as np
import torch

import pyoracle as po
from gpu_engine import GpuEngine
from razor_amd.fec import Native

lib_path = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
G = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
mode = sys.argv[4] if len(sys.argv) > 4 else "in_place"
o = po.Oracle(1000)
plan = o.plan_from_fraction(k, 80, 3)
rng = np.random.default_rng(77)
S = 1000
shards, hdr = o.fill_groups(9, G, k, S, ragged=True)
cap = min(o.video_size, shards.shape[-1])
parity, meta, fsize, _ = o.encode_batch(plan, shards, hdr, cap)
present = np.zeros((G, 2), np.uint64)
pp = np.full(G, (1 << plan.n_lines) - 1, np.uint64)
rx, rh, fs = shards.copy(), hdr.copy(), fsize.copy()
for g in range(G):
    m = (1 << k) - 1
    for i in rng.choice(k, int(rng.integers(1, 5)), replace=False):
        m &= ~(1 << int(i))
        rx[g, i] = 0xA5
        rh[g, i] = np.zeros((), po.HDR_DTYPE)
    present[g, 0] = m
    if rng.random() < 0.2:
        pp[g] &= ~np.uint64(1 << int(rng.integers(plan.n_lines)))
    r = rng.random()
    if r < 0.25:
        fs[g, rng.integers(plan.n_lines)] = cap + 1
    elif r < 0.5:
        l = int(rng.integers(plan.n_lines))
        fs[g, l] = max(1, int(fs[g, l]) - 7)
    elif r < 0.7:
        i = int(rng.integers(k))
        if (m >> i) & 1:
            rh[g, i]["size"] = min(cap, int(rh[g, i]["size"]) + 50)
eng = GpuEngine(1000, "cuda:0")
eng.lib = Native(1000, lib_path)
print("groups", G, "k", k, "stride", rx.shape[-1], "mode", mode, flush=True)
if mode == "dense":
    got = eng.recover_out(plan, rx, rh, present, parity, meta, fs, pp, cap, 4)
    exp = o.recover_batch_out(plan, rx, rh, present, parity, meta, fs, pp, cap, 4)
    print("recovered equal:", np.array_equal(got[3], exp[3]), "index equal:", np.array_equal(got[2], exp[2]))
else:
    s_, h_, rec = eng.recover(plan, rx, rh, present, parity, meta, fs, pp, cap)
    e_s, e_h, e_rec = o.recover_batch(plan, rx, rh, present, parity, meta, fs, pp, cap)
    print("recovered equal:", np.array_equal(rec, e_rec))
