"""Benchmark: device-resident flex-FEC encode + decode on MI355X.

Workload (BASELINE.json configs[2], the metric's config, at N = 1): G = 65,536
FEC groups of k = 10 segments of 1,200 bytes; the r = 3 row parities of the
reference's 3x4 plan (rows {4,4,2}, flex_fec_sender.c:166-188); 2 erasures
per group drawn from the 32 distinct-row pairs, recovered by peeling
(flex_fec_receiver.c:105-150).  Payloads are the SURVEY §8(d) xorshift64*
stream (config id 2, so the parity equals the reference digest c2 of
tests/golden/full_hashes.json), generated on the device, resident in HBM
before timing.

One step = encode one buffer set, then recover the set encoded one step
earlier (receiver order: its parity arrived over the network, so it is not
in the 256 MB MALL), over >= 2 disjoint buffer sets rotated per step.

Multi-GPU: one process per GPU; the driver starts them with torchrun,
`bench.py --gpus N` alone starts them itself.  FEC groups are independent, so
the default at every N is weak scaling of config 3: rank r runs groups
[r * 65,536, (r + 1) * 65,536) of the same stream -- the N = 1 workload per GPU,
so value(N) / (N * value(1)) is a scaling efficiency.  `--config c4` is
BASELINE.json configs[3] at any N (N = 1 included): 1,048,576 groups split
into contiguous slices (razor_amd/dist.py), strong scaling.  No data-path
collective; the control plane (barrier, max-over-ranks time, byte sum) is a
CPU gloo group, so no RCCL is brought up and several ranks may share one GPU.
Every rank checks its slice against the reference's digest of exactly those
groups (tests/golden/full_hashes.json: c2 / the weak chunks, the c4 slices).

Timing: `value` is the wall clock of the K timed steps (barrier + device
synchronize on both sides, max over ranks).  The roofline's launch duration
is each kernel's own start / stop, HIP events bound to the launch itself
(rfec_timing_events -> hipExtLaunchKernel, on the launch stream), which is
what rocprofv3 reports per kernel; no event marker sits between the launches
then.  `--timing bracket` records stream events around each call instead
(the window then also holds the command processor's dispatch gap, 3-4 µs per
launch).  Either kind is recorded on every 8th timed step only: an event pair
around a launch adds ~4.6 µs of dispatch gap to its step (tools/gap_probe.py:
0.2888 ms per c3 step without events, 0.2981 with the kernels' own events on
every step), which would otherwise be charged to `value`.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from razor_amd.dist import StepWindow, device_identity, gather_objects, shard_groups  # noqa: E402
from razor_amd.fec import FEC_STAMP_DTYPE, HDR_DTYPE, SEG_STAMP_DTYPE, Native, native  # noqa: E402

METRIC = "FEC encode+decode GiB/s (device-resident), 1200B pkts k=10/r=3; % HBM peak"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
GOLDEN = ROOT / "tests" / "golden" / "full_hashes.json"

# name -> (k, S, plan, total groups, config id of the input stream, golden digest case)
CONFIGS = {
    "c3": dict(k=10, S=1200, plan="rows", groups=65536, config_id=2, golden="c2_k10_rows_S1200_G65536",
               weak_golden="c3_weak_k10_rows_S1200_G524288",
               desc="BASELINE configs[2]: encode + decode, k=10 r=3, 1200 B, 2 erasures/group"),
    "c3full": dict(k=10, S=1200, plan="full", groups=65536, config_id=3, golden="c3_k10_full_S1200_G65536",
                   desc="configs[2] variant: the reference sender's full 3x4 plan (7 parities)"),
    "c4": dict(k=10, S=1200, plan="rows", groups=1048576, config_id=4, golden="c4_k10_rows_S1200_G1048576",
               desc="BASELINE configs[3]: 1M groups split over the GPUs, k=10 r=3, 1200 B"),
    "c5": dict(k=32, S=256, plan="col4", groups=65536, config_id=5, golden="c5_k32_rows4_S256_G65536",
               desc="BASELINE configs[4]: k=32 r=8 (8 rows of 4), 256 B"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_headers(G, k, S, group0):
    """SURVEY §8(d) headers: contiguous packet ids (sim_sender.c:338)."""
    hdr = np.zeros((G, k), HDR_DTYPE)
    gi = (np.arange(G, dtype=np.uint64) + group0)[:, None]
    ii = np.arange(k, dtype=np.uint64)[None, :]
    hdr["seq"] = (1 + gi * k + ii).astype(np.uint32)
    hdr["fid"] = (1 + gi).astype(np.uint32)
    hdr["ts"] = (33 * gi).astype(np.uint32)
    hdr["index"] = ii
    hdr["total"] = k
    hdr["ftype"] = (gi % 60 == 0)
    hdr["size"] = S
    return hdr


WIRE_DSTRIDE = 1280  # datagram slots of 10 x 128 B: whole-line stores
WIRE_GOLDEN = ROOT / "tests" / "golden" / "wire_c3_digest.json"


def wire_stamps(hdr, plan, n):
    """The sender's fields around the FEC of the c3 workload's datagrams
    (sim_sender.c:103-122 / sim_proto.inl:83-307): parities get uid, fec_id
    (+1 per group, 0 skipped), base_id, count, row, col, index, send_ts and a
    running transport_seq; segments uid, fec_id, send_ts, transport_seq."""
    G, k = hdr.shape
    fid = (np.arange(G) % 65535 + 1).astype(np.uint16)
    f = np.zeros((G, n), FEC_STAMP_DTYPE)
    f["uid"] = 0x52415A4F
    f["fec_id"] = fid[:, None]
    f["base_id"] = hdr["seq"][:, :1]
    f["count"] = k
    f["row"], f["col"] = plan.row, plan.col
    f["index"] = [plan.line[l].index for l in range(n)]
    f["send_ts"] = hdr["ts"][:, :1]
    f["transport_seq"] = (np.arange(G * n) & 0xFFFF).reshape(G, n)
    s = np.zeros((G, k), SEG_STAMP_DTYPE)
    s["uid"] = 0x52415A4F
    s["fec_id"] = fid[:, None]
    s["send_ts"] = hdr["ts"] & 0xFFFF
    s["transport_seq"] = (np.arange(G * k) & 0xFFFF).reshape(G, k)
    s["remb"] = 0xFF
    return f.reshape(-1), s.reshape(-1)


def wire_digest(dg, dl):
    """SHA-256 of datagrams (host arrays [N][dstride], lengths [N]): the
    lengths, then each datagram's bytes in order."""
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(dl, np.uint16).tobytes())
    h.update(dg[np.arange(dg.shape[1])[None, :] < dl.astype(np.int64)[:, None]].tobytes())
    return h.hexdigest()


def distinct_row_pairs(plan):
    rows = [plan.members(l) for l in range(plan.n_lines)]
    return [(a, b) for r1 in range(len(rows)) for r2 in range(r1 + 1, len(rows)) for a in rows[r1] for b in rows[r2]]


def peel_bytes(plan, k, erased, S):
    """Algorithmic decode bytes of one erasure set under the canonical peel
    (lines in plan order, repeated to a fixpoint, as the oracle and the
    device decoders run it): each fired line reads its other members and its
    parity and writes the missing member, (count + 1) * S.  None when the
    set is not recoverable."""
    have = set(range(k)) - set(erased)
    total, progress = 0, True
    while progress:
        progress = False
        for l in range(plan.n_lines):
            mem = plan.members(l)
            miss = [i for i in mem if i not in have]
            if len(miss) == 1:
                have.add(miss[0])
                total += (len(mem) + 1) * S
                progress = True
    return total if len(have) == k else None


class Workload:
    def __init__(self, lib, G, k, S, pf, device, group0, seed, stride=None, col=0, full_plan=False, config_id=2,
                 in_place=False, launch_groups=0):
        self.lib, self.G, self.k, self.S = lib, G, k, S
        self.launch_groups = launch_groups
        self.stride = stride or (S + 15) // 16 * 16  # slot width in HBM (>= S, multiple of 16)
        if col:  # explicit rows of `col` (config 5: k = 32 as 8 rows of 4)
            self.plan = lib.plan_matrix(k, (k + col - 1) // col, col, 1)
        elif full_plan:  # the reference sender's whole plan: rows and columns (3x4 -> 7 parities at k = 10)
            self.plan = lib.plan_from_fraction(k, pf, 3)
        else:
            self.plan = lib.plan_from_fraction(k, pf, 1)  # row layer: r = 3 at k = 10
        self.n = self.plan.n_lines
        dev = device
        st = torch.cuda.current_stream(dev).cuda_stream
        # SURVEY §8(d) payloads: xorshift64* stream of `config_id`, groups [group0, group0 + G)
        self.shards = torch.empty((G, k, self.stride), dtype=torch.uint8, device=dev)
        lib.fill_xorshift(self.shards.data_ptr(), config_id, group0, G, k, S, self.stride, st)
        self.hdr_np = make_headers(G, k, S, group0)
        self.hdr = torch.from_numpy(self.hdr_np.view(np.uint8).reshape(G, k, 20).copy()).to(dev)
        self.parity = torch.empty((G, self.n, self.stride), dtype=torch.uint8, device=dev)
        self.meta = torch.empty((G, self.n, 20), dtype=torch.uint8, device=dev)
        self.fsize = torch.empty((G, self.n), dtype=torch.int16, device=dev)
        self.status = torch.empty((G, self.n), dtype=torch.int8, device=dev)
        # receive side: the same groups with 2 erasures each (rows only: in distinct rows; full plan: any pair)
        if full_plan:
            pairs = np.array([(a, b) for a in range(k) for b in range(a + 1, k)
                              if peel_bytes(self.plan, k, (a, b), S) is not None])
        else:
            pairs = np.array(distinct_row_pairs(self.plan))
        rng = np.random.default_rng(seed)
        pick = rng.integers(0, len(pairs), G)
        self.erased = pairs[pick]
        present = np.zeros((G, 2), np.uint64)
        full = np.uint64((1 << k) - 1)
        present[:, 0] = full & ~((np.uint64(1) << self.erased[:, 0].astype(np.uint64)) |
                                 (np.uint64(1) << self.erased[:, 1].astype(np.uint64)))
        self.present_np = present
        self.present = torch.from_numpy(present.view(np.int64)).to(dev)
        self.parity_present = torch.full((G,), (1 << self.n) - 1, dtype=torch.int64, device=dev)
        self.rx = self.shards.clone()
        self.rx_hdr = self.hdr.clone()
        gi = torch.arange(G, device=dev)
        for c in range(2):
            e = torch.from_numpy(self.erased[:, c]).to(dev)
            self.rx[gi, e] = 0xA5
            self.rx_hdr[gi, e] = 0
        self.recovered = torch.empty((G, 2), dtype=torch.int64, device=dev)
        # recovered segments: into a dense output [G][2] (rfec_recover_batch_out, as flex_fec_recover's
        # caller-allocated out_seg), or in place (rfec_recover_batch, --in-place)
        self.dense = not in_place
        if self.dense:
            self.out_shards = torch.empty((G, 2, self.stride), dtype=torch.uint8, device=dev)
            self.out_hdr = torch.empty((G, 2, 20), dtype=torch.uint8, device=dev)
            self.out_index = torch.empty((G, 2), dtype=torch.uint8, device=dev)
        self.ws = torch.empty((lib.workspace_size(self.plan, launch_groups or G),), dtype=torch.uint8, device=dev)
        # packed erasure records (rfec_recover_packed_out), for row layouts: see use_packed
        self.packed = False
        self.pks = lib.packed_stride(self.plan, 2) if self.dense else 0
        self.packed_rec = None
        # algorithmic payload bytes (headers excluded): encode reads k*S, writes r*S
        self.enc_bytes = G * (k + self.n) * S
        # decode: per recovered segment read its line's other members + the parity, write 1
        pair_bytes = np.array([peel_bytes(self.plan, k, tuple(p), S) for p in pairs.tolist()], np.int64)
        self.dec_bytes = int(pair_bytes[pick].sum())

    def use_packed(self, on):
        """Decode from packed erasure records (rfec_pack_erasures' layout: per
        group the masks, then per output slot its row's meta, fec_data_size
        and other members' records) instead of the batch layout's header
        arrays.  The records are built once the parity exists (prepare(), before
        timing: a receiver writes them as segments arrive, as the batch layout's
        arrays are written).  The outputs are poisoned so verify() sees this
        path's results."""
        assert not on or self.pks, "packed records need a dense row-layout decode"
        self.packed = on
        if on and self.packed_rec is None:
            self.packed_rec = torch.empty((self.G, self.pks), dtype=torch.uint8, device=self.shards.device)
        if on:
            for t in (self.out_shards, self.out_hdr, self.out_index, self.recovered):
                t.view(torch.uint8).fill_(0xEE)

    def prepare(self, stream):
        """Untimed, after the priming encode: the packed records from this set's
        received headers, masks and the encode's meta / fec_data_size."""
        if self.packed:
            self.lib.pack_erasures(self.plan, self.G, self.rx_hdr.data_ptr(), self.present.data_ptr(),
                                   self.meta.data_ptr(), self.fsize.data_ptr(), self.parity_present.data_ptr(), 2,
                                   self.packed_rec.data_ptr(), stream)

    def _chunks(self):
        """(first group, groups) of each launch: the whole batch, or launches of
        `self.launch_groups` groups (the c4 sub-object: every launch the size of
        the headline's, so per-kernel rocprofv3 averages stay comparable)."""
        c = self.launch_groups or self.G
        return [(g0, min(c, self.G - g0)) for g0 in range(0, self.G, c)]

    def encode(self, stream):
        k, n, st = self.k, self.n, self.stride
        for g0, g in self._chunks():
            self.lib.encode_batch(self.plan, g, st, self.S, self.shards.data_ptr() + g0 * k * st,
                                  self.hdr.data_ptr() + g0 * k * 20, self.parity.data_ptr() + g0 * n * st,
                                  self.meta.data_ptr() + g0 * n * 20, self.fsize.data_ptr() + g0 * n * 2,
                                  self.status.data_ptr() + g0 * n, stream)

    def decode(self, stream):
        k, n, st = self.k, self.n, self.stride
        for g0, g in self._chunks():
            if self.packed:
                self.lib.recover_packed_out(self.plan, g, st, self.S, self.rx.data_ptr() + g0 * k * st,
                                            self.parity.data_ptr() + g0 * n * st,
                                            self.packed_rec.data_ptr() + g0 * self.pks,
                                            self.recovered.data_ptr() + g0 * 16, 2,
                                            self.out_shards.data_ptr() + g0 * 2 * st,
                                            self.out_hdr.data_ptr() + g0 * 40, self.out_index.data_ptr() + g0 * 2,
                                            stream)
            elif self.dense:
                self.lib.recover_batch_out(self.plan, g, st, self.S, self.rx.data_ptr() + g0 * k * st,
                                           self.rx_hdr.data_ptr() + g0 * k * 20, self.present.data_ptr() + g0 * 16,
                                           self.parity.data_ptr() + g0 * n * st, self.meta.data_ptr() + g0 * n * 20,
                                           self.fsize.data_ptr() + g0 * n * 2, self.parity_present.data_ptr() + g0 * 8,
                                           self.recovered.data_ptr() + g0 * 16, 2,
                                           self.out_shards.data_ptr() + g0 * 2 * st, self.out_hdr.data_ptr() + g0 * 40,
                                           self.out_index.data_ptr() + g0 * 2, self.ws.data_ptr(), stream)
            else:
                self.lib.recover_batch(self.plan, g, st, self.S, self.rx.data_ptr() + g0 * k * st,
                                       self.rx_hdr.data_ptr() + g0 * k * 20, self.present.data_ptr() + g0 * 16,
                                       self.parity.data_ptr() + g0 * n * st, self.meta.data_ptr() + g0 * n * 20,
                                       self.fsize.data_ptr() + g0 * n * 2, self.parity_present.data_ptr() + g0 * 8,
                                       self.recovered.data_ptr() + g0 * 16, self.ws.data_ptr(), stream)

    def verify(self):
        """Whole-batch checks after the timed steps (not timed): every parity
        line equals a torch XOR of its members (payload and 20-B meta record),
        and every erased segment came back bit-exact."""
        S = self.S
        ok = True
        hdr32 = self.hdr.view(torch.int32).reshape(self.G, self.k, 5)
        meta32 = self.meta.view(torch.int32).reshape(self.G, self.n, 5)
        for l in range(self.n):
            mem = self.plan.members(l)
            ref = self.shards[:, mem[0], :S].clone()
            href = hdr32[:, mem[0]].clone()
            for i in mem[1:]:
                ref ^= self.shards[:, i, :S]
                href ^= hdr32[:, i]
            ok = ok and torch.equal(self.parity[:, l, :S], ref) and torch.equal(meta32[:, l], href)
        if self.dense:  # out slot e = the e-th erased segment in index order; the received set untouched
            gi = torch.arange(self.G, device=self.shards.device)
            for e in range(2):
                idx = torch.from_numpy(np.sort(self.erased, axis=1)[:, e].astype(np.int64)).to(self.shards.device)
                ok = ok and torch.equal(self.out_shards[:, e, :S], self.shards[gi, idx, :S])
                ok = ok and torch.equal(self.out_hdr[:, e], self.hdr[gi, idx])
                ok = ok and torch.equal(self.out_index[:, e].long(), idx)
        else:
            ok = ok and torch.equal(self.rx[:, :, :S], self.shards[:, :, :S]) and torch.equal(self.rx_hdr, self.hdr)
        exp = ((1 << self.erased[:, 0]) | (1 << self.erased[:, 1])).astype(np.int64)
        ok = ok and np.array_equal(self.recovered[:, 0].cpu().numpy(), exp)
        ok = ok and int(self.status.abs().sum()) == 0
        return bool(ok)

    def digest(self, chunk=65536):
        """SHA-256 of the encode outputs group by group, parity[n][S] |
        meta[n] (20 B) | fec_data_size[n] (u16 LE): the record
        oracle/gen_full.c digests from the reference's flex_fec_generate."""
        h = hashlib.sha256()
        for g0 in range(0, self.G, chunk):
            g1 = min(self.G, g0 + chunk)
            n = g1 - g0
            rec = torch.cat([self.parity[g0:g1, :, :self.S].reshape(n, -1), self.meta[g0:g1].reshape(n, -1),
                             self.fsize[g0:g1].view(torch.uint8).reshape(n, -1)], dim=1)
            h.update(rec.cpu().numpy().tobytes())
        return h.hexdigest()


def copy_ceiling(lib, device, nbytes=1 << 30, reps=10):
    """Measured HBM copy rate (read + write bytes / time, GB/s) of the
    library's streaming copy probe (rfec_probe_copy: one 16-B vector per lane,
    non-temporal loads and stores), on torch's current stream."""
    a = torch.empty(nbytes, dtype=torch.uint8, device=device)
    b = torch.empty_like(a)
    st = torch.cuda.current_stream(device).cuda_stream

    def run():
        rc = lib.lib.rfec_probe_copy(a.data_ptr(), b.data_ptr(), nbytes, 1, st)
        if rc:
            raise RuntimeError(f"rfec_probe_copy failed: {rc}")

    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(device)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize(device)
    t = e0.elapsed_time(e1) / 1e3 / reps
    del a, b
    return 2 * nbytes / t / 1e9


def mix_ceiling(lib, device, r, w, stream_bytes, reps=10):
    """Measured HBM rate (GB/s, read + write bytes / time) of the library's
    r : w streaming probe (rfec_probe_mix: r read streams XORed into w write
    streams, one 16-B vector per lane, non-temporal) over the encode's own
    byte volume, two rotated buffer sets: the ceiling of the encode's read /
    write mix (writes cost HBM more than reads: 10 : 3 streams at ~0.77 of
    8 TB/s, 10 : 7 at ~0.71)."""
    st = torch.cuda.current_stream(device).cuda_stream
    sets = [(torch.empty(r * stream_bytes, dtype=torch.uint8, device=device),
             torch.empty(w * stream_bytes, dtype=torch.uint8, device=device)) for _ in range(2)]

    def run(i):
        a, b = sets[i % 2]
        rc = lib.lib.rfec_probe_mix(a.data_ptr(), b.data_ptr(), stream_bytes, r, w, st)
        if rc:
            raise RuntimeError(f"rfec_probe_mix {r}:{w} failed: {rc}")

    for i in range(4):
        run(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(device)
    e0.record()
    for i in range(reps):
        run(i)
    e1.record()
    torch.cuda.synchronize(device)
    t = e0.elapsed_time(e1) / 1e3 / reps
    del sets
    return (r + w) * stream_bytes / t / 1e9


def encode_mix(w):
    """(reads, writes, stream bytes) of the probe with the encode's byte mix, or None."""
    lines = [w.plan.line[l].count for l in range(w.n)]
    if w.k == 10 and w.n in (3, 7):  # rows {4,4,2} (10 : 3), the full 3 x 4 plan (10 : 7)
        return 10, w.n, w.G * w.S
    if len(set(lines)) == 1 and lines[0] == 4 and w.k == 4 * w.n:  # rows of 4 (c5: 4 : 1)
        return 4, 1, w.G * w.n * w.S
    return None


def host_cores():
    """(cores this process may run on, os.cpu_count()): the affinity set,
    capped by a cgroup v2 CPU quota when one is set."""
    n = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = n
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            avail = min(avail, max(1, math.ceil(int(q) / int(period))))
    except (OSError, ValueError):
        pass
    return avail, n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(w: Workload, seconds: float):
    """The oracle's reference-shaped path (flex_fec_generate per line,
    flex_fec_recover per erasure, over AoS sim_segment_t) on a
    bounded sample of the same groups (the device-generated xorshift64*
    payloads): (i) 1 core at the reference's own flags (-O0), (ii) 1 core at
    -O2, (iii) every available core at -O2 with a pthread group split."""
    sys.path.insert(0, str(ROOT / "oracle"))
    from pyoracle import Oracle

    sample = min(w.G, 16384)
    shards = w.shards[:sample, :, :w.S].cpu().numpy()
    hdr = w.hdr_np[:sample]
    present = w.present_np[:sample]
    cores, nproc = host_cores()
    out = {}
    legs = (("O2_1core", "O2", 1, seconds), ("O0_1core", "O0", 1, seconds / 4),
            (f"O2_{cores}threads", "O2", cores, seconds / 4))
    for label, opt, threads, budget in legs:
        o = Oracle(1200, opt)
        segs = o.to_aos(shards, hdr)
        rec_out = np.zeros_like(segs)
        t_enc = t_dec = 0.0
        reps = 0
        while t_enc + t_dec < budget or reps == 0:
            t0 = time.perf_counter()
            n, fec = o.encode_aos(w.plan, sample, segs, threads=threads)
            t1 = time.perf_counter()
            nrec, _ = o.recover_aos(w.plan, sample, segs, fec, present, threads=threads, out=rec_out)
            t2 = time.perf_counter()
            assert n == sample * w.n and nrec == 2 * sample
            t_enc += t1 - t0
            t_dec += t2 - t1
            reps += 1
        enc_b = sample * (w.k + w.n) * w.S * reps
        dec_b = w.dec_bytes * sample / w.G * reps
        out[label] = {"gibps": (enc_b + dec_b) / (t_enc + t_dec) / 2**30, "encode_gibps": enc_b / t_enc / 2**30,
                      "decode_gibps": dec_b / t_dec / 2**30, "reps": reps, "seconds": t_enc + t_dec,
                      "threads": threads}
    main = out["O2_1core"]
    allc = out[f"O2_{cores}threads"]
    return {"value": round(main["gibps"], 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{sample} groups x {main['reps']} passes ({main['seconds']:.1f} s) of the same workload "
                      f"(k={w.k}, {w.n} parities, {w.S} B, 2 erasures/group, the device's xorshift64* payloads), "
                      f"oracle/rfec_oracle.c at -O2 over AoS sim_segment_t, one thread",
            "cpu": cpu_model(), "nproc": nproc, "cores_available": cores,
            "encode_gibps": round(main["encode_gibps"], 4), "decode_gibps": round(main["decode_gibps"], 4),
            "reference_flags_O0_1core_gibps": round(out["O0_1core"]["gibps"], 4),
            "all_cores_O2_gibps": round(allc["gibps"], 4),
            "all_cores_O2_encode_gibps": round(allc["encode_gibps"], 4),
            "all_cores_O2_decode_gibps": round(allc["decode_gibps"], 4),
            "all_cores_threads": cores}


def load_traffic(workload_name, kind):
    """HBM bytes per encode / decode launch from the committed rocprofv3 PMC
    summary (tools/pmc_traffic.py), or None."""
    p = ROOT / "profiles" / "traffic.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        e = d.get(workload_name)
        return None if e is None else e.get(f"{kind}_hbm_bytes_per_launch")
    except (ValueError, OSError):
        return None


def golden_digest(case, world, rank, chunk=0):
    """The reference's digest of this rank's groups (tests/golden/full_hashes.json):
    the whole case at world 1; the strong-scaling slice [G r / N, G (r + 1) / N)
    ("slices"); with `chunk`, the weak-scaling slice [r chunk, (r + 1) chunk)
    ("chunks")."""
    try:
        cases = {c["name"]: c for c in json.loads(GOLDEN.read_text())["cases"]}
    except (OSError, ValueError):
        return None
    c = cases.get(case)
    if c is None:
        return None
    if chunk:
        ch = c.get("chunks", [])
        return ch[rank] if c.get("chunk") == chunk and rank < len(ch) else None
    if world == 1:
        return c["sha256"]
    return c.get("slices", {}).get(str(world), [None] * world)[rank]


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


TIMING_OWN = ("the kernel's own start / stop: HIP events bound to the launch (rfec_timing_events -> "
              "hipExtLaunchKernel) on the launch stream, mean over every 8th timed step (events on every step "
              "would add ~4.6 us of dispatch gap per launch to the timed region)")
TIMING_BRACKET = ("HIP events recorded on the launch stream before and after the call on every 8th timed step "
                  "(holds the dispatch gap; --timing bracket, or a call that launches more than one kernel)")


# Kernel windows are recorded on every TIMING_EVERY-th timed step only: an
# event pair around a launch (hipExtLaunchKernel's or the stream's) costs the
# step ~4.6 us of dispatch gap (tools/gap_probe.py: 0.2888 ms per step with no
# events, 0.2981 with the kernels' own events on every step, 0.3035 with
# stream events); the windows are still those of launches inside the timed
# region.
TIMING_EVERY = 8
SUB_EVERY = TIMING_EVERY  # the c5 / c3full sub-objects (80 steps: 10 samples)


def time_steps(lib, sets, steps, warmup, stream, dist, timing, hot, every=TIMING_EVERY):
    """Primes every set's parity, runs `warmup` untimed steps, then times
    `steps` steps (encode one set, decode the set encoded one step earlier, or
    the same set when `hot` or one set) between a barrier + device
    synchronize on both sides (razor_amd/dist.StepWindow).  Returns (the job's
    wall seconds: max over ranks of t1 - min over ranks of t0, CLOCK_MONOTONIC;
    encode / decode launch seconds of the sampled steps (every TIMING_EVERY-th,
    from the first); whether each is the kernel's own window; the window's
    per-rank readings and skews)."""
    nset = len(sets)
    sp = stream.cuda_stream
    device = stream.device

    def dec_set(i):
        return sets[i % nset] if hot else sets[(i - 1) % nset]

    for ws in sets:  # every set holds its parity before the first (cold) decode
        ws.encode(sp)
    for ws in sets:
        ws.prepare(sp)
    for i in range(warmup):
        sets[i % nset].encode(sp)
        dec_set(i).decode(sp)
    ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)) for _ in range(steps)]
    # the kernels' own start / stop (rfec_timing_events -> hipExtLaunchKernel on the launch stream):
    # the roofline's launch duration, without the dispatch gap the stream-event bracket also holds
    kev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)) for _ in range(steps)]
    for q in kev:
        for e in q:
            e.record(stream)  # creates the event (torch allocates it at its first record)
    # does each call launch exactly one kernel (then its own window is its launch duration)?
    lib.timing_events(kev[0][0].cuda_event, kev[0][1].cuda_event)
    sets[0].encode(sp)
    n_enc = lib.timing_launches()
    lib.timing_events(kev[0][2].cuda_event, kev[0][3].cuda_event)
    dec_set(1).decode(sp)
    n_dec = lib.timing_launches()
    own_enc = timing == "own" and n_enc == 1
    own_dec = timing == "own" and n_dec == 1
    torch.cuda.synchronize(device)
    win = StepWindow(dist, lambda: torch.cuda.synchronize(device))
    win.start()  # barrier, synchronize, t0 (CLOCK_MONOTONIC)
    for i in range(steps):
        # sampled steps: the kernels' own events where a call is one launch (no marker between launches),
        # else a bracket
        smp = i % every == 0
        ka, kb, kc, kd = kev[i]
        a, b, c, d = ev[i]
        if smp and own_enc:
            lib.timing_events(ka.cuda_event, kb.cuda_event)
        elif smp:
            a.record(stream)
        sets[(warmup + i) % nset].encode(sp)
        if smp and not own_enc:
            b.record(stream)
        if smp and own_dec:
            lib.timing_events(kc.cuda_event, kd.cuda_event)
        elif smp:
            c.record(stream)
        dec_set(warmup + i).decode(sp)
        if smp and not own_dec:
            d.record(stream)
    win.stop()  # synchronize, t1, barrier
    sampled = list(zip(kev, ev))[::every]
    t_enc = np.array([(q if own_enc else e)[0].elapsed_time((q if own_enc else e)[1]) for q, e in sampled]) / 1e3
    t_dec = np.array([(q if own_dec else e)[2].elapsed_time((q if own_dec else e)[3]) for q, e in sampled]) / 1e3
    window = win.reduce()  # every rank's (t0, t1): the job's window is max(t1) - min(t0)
    return window["elapsed_s"], t_enc, t_dec, own_enc, own_dec, window


def c4_strong(lib, device, stream, dist, world, rank, pf, steps, warmup, verify):
    """BASELINE configs[3] beside the weak-scaling headline: the 1,048,576
    groups of config 4 split into contiguous slices over the ranks
    (razor_amd/dist.shard_groups; all of them on one GPU at N = 1), `steps`
    timed encode + decode steps over two buffer sets, the decode on the set
    encoded one step earlier (the headline's discipline), each direction
    as launches of 65,536 groups (the headline's launch size: the kernels'
    rocprofv3 averages over a whole bench run stay those of one size).  Every rank
    checks its slice against the reference's digest of exactly those groups
    (full_hashes.json: the whole case at N = 1, "slices" at N = 2 / 4 / 8).
    Returns the sub-object on rank 0 (None elsewhere); value = all ranks'
    bytes / max-over-ranks time, so value(N) / value(1) is the strong-scaling
    speedup."""
    cfg = CONFIGS["c4"]
    total = cfg["groups"]
    group0, my = shard_groups(total, world, rank)
    sets = [Workload(lib, my, cfg["k"], cfg["S"], pf, device, group0, seed=3000 + rank, config_id=cfg["config_id"],
                     launch_groups=CONFIGS["c3"]["groups"]) for _ in range(2)]
    w = sets[0]
    elapsed, t_enc, t_dec, own_enc, own_dec, _ = time_steps(lib, sets, steps, warmup, stream, dist, "own", False)
    verified = digest_ok = None
    if verify:
        verified = all(ws.verify() for ws in sets)
        want = golden_digest(cfg["golden"], world, rank)
        if want is not None:
            digest_ok = w.digest() == want
            verified = verified and digest_ok
    per_rank = torch.tensor([w.G, w.enc_bytes + w.dec_bytes, float(t_enc.mean()) * 1e6, float(t_dec.mean()) * 1e6,
                             -1 if verified is None else int(verified), -1 if digest_ok is None else int(digest_ok)],
                            dtype=torch.float64)
    rows = [per_rank]
    if dist:
        rows = [torch.zeros_like(per_rank) for _ in range(world)]
        dist.all_gather(rows, per_rank)
    del w, sets
    torch.cuda.empty_cache()
    if rank != 0:
        return None
    step_bytes = sum(float(r[1]) for r in rows)
    enc_b = rows[0][0].item() * (cfg["k"] + 3) * cfg["S"]
    flags = [(int(r[4]), int(r[5])) for r in rows]
    return {"workload": f"c4: k10_r3_S1200_G{total} split into {world} contiguous slice(s) "
                        f"[r*{total}/{world}, (r+1)*{total}/{world})",
            "scaling": "strong", "value": round(step_bytes * steps / elapsed / 2**30, 3), "unit": "GiB/s",
            "steps": steps, "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 4),
            "buffer_sets": 2, "decode_order": "cold (the set encoded one step earlier), as the headline",
            "groups_per_rank": [int(r[0]) for r in rows],
            "launch_groups": CONFIGS["c3"]["groups"],
            "encode_us_per_rank": [round(float(r[2]), 2) for r in rows],
            "decode_us_per_rank": [round(float(r[3]), 2) for r in rows],
            "rank0_encode_frac_of_peak": round(enc_b / (float(rows[0][2]) * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
            "timing": ("per step and direction: " + (TIMING_OWN if own_enc and own_dec else TIMING_BRACKET)),
            "verified": None if not verify else all(f[0] == 1 for f in flags),
            "verified_vs_reference_digest": None if not verify else (
                False if any(f[1] == 0 for f in flags) else (True if all(f[1] == 1 for f in flags) else None))}


def wire_sub(lib, w, device, reps=10):
    """§8(f1) on the default line: the c3 workload's datagrams -- its 196,608
    parities as SIM_FEC (rfec_wire_frame_fec) and 655,360 segments as SIM_SEG
    (rfec_wire_frame_seg), into 1,280-B slots -- and both parsed back
    (rfec_wire_parse), each kernel timed by its own start / stop events over
    `reps` launches.  Algorithmic bytes per datagram (tools/wire_bench.py):
    frame read payload + header + stamp, write the datagram + its length;
    parse read datagram + length, write the 64-B record + the payload slot.
    Checked: parse(frame(x)) = x on every datagram, and the datagrams of the
    first 4,096 groups against the oracle's bytes for the same groups
    (tests/golden/wire_c3_digest.json, made by oracle/gen_wire_digest.py)."""
    G, k, n, S, P = w.G, w.k, w.n, w.S, w.stride
    NF, NS, D = G * n, G * k, WIRE_DSTRIDE
    st = torch.cuda.current_stream(device)
    sp = st.cuda_stream
    fst, sst = wire_stamps(w.hdr_np, w.plan, n)
    d_fst = torch.from_numpy(fst.view(np.uint8).copy()).to(device)
    d_sst = torch.from_numpy(sst.view(np.uint8).copy()).to(device)
    dg_f = torch.empty((NF, D), dtype=torch.uint8, device=device)
    dl_f = torch.empty((NF,), dtype=torch.int16, device=device)
    dg_s = torch.empty((NS, D), dtype=torch.uint8, device=device)
    dl_s = torch.empty((NS,), dtype=torch.int16, device=device)
    rec_f = torch.empty((NF, 64), dtype=torch.uint8, device=device)
    pay_f = torch.empty((NF, P), dtype=torch.uint8, device=device)
    rec_s = torch.empty((NS, 64), dtype=torch.uint8, device=device)
    pay_s = torch.empty((NS, P), dtype=torch.uint8, device=device)
    calls = {
        "frame_fec": lambda: lib.wire_frame_fec(NF, P, S, w.parity.data_ptr(), w.meta.data_ptr(), w.fsize.data_ptr(),
                                                w.status.data_ptr(), d_fst.data_ptr(), D, dg_f.data_ptr(),
                                                dl_f.data_ptr(), sp),
        "frame_seg": lambda: lib.wire_frame_seg(NS, P, S, w.shards.data_ptr(), w.hdr.data_ptr(), d_sst.data_ptr(), D,
                                                dg_s.data_ptr(), dl_s.data_ptr(), sp),
        "parse_fec": lambda: lib.wire_parse(NF, D, dg_f.data_ptr(), dl_f.data_ptr(), P, S, rec_f.data_ptr(),
                                            pay_f.data_ptr(), sp),
        "parse_seg": lambda: lib.wire_parse(NS, D, dg_s.data_ptr(), dl_s.data_ptr(), P, S, rec_s.data_ptr(),
                                            pay_s.data_ptr(), sp)}
    for f in calls.values():
        f()
    torch.cuda.synchronize(device)
    lf = dl_f.cpu().numpy().view(np.uint16).astype(np.int64)
    ls = dl_s.cpu().numpy().view(np.uint16).astype(np.int64)
    alg = {"frame_fec": int(NF * (S + 20 + 24 + 2) + lf.sum() + 2 * NF),
           "frame_seg": int(NS * (S + 20 + 12) + ls.sum() + 2 * NS),
           "parse_fec": int(lf.sum() + 2 * NF + NF * (64 + S)),
           "parse_seg": int(ls.sum() + 2 * NS + NS * (64 + S))}
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps * 4)]
    for a, b in ev:
        a.record(st)
        b.record(st)
    torch.cuda.synchronize(device)
    kern = {}
    for i, (name, f) in enumerate(calls.items()):
        for r in range(reps):
            a, b = ev[i * reps + r]
            lib.timing_events(a.cuda_event, b.cuda_event)
            f()
        torch.cuda.synchronize(device)
        t = np.array([a.elapsed_time(b) * 1e-3 for a, b in ev[i * reps:(i + 1) * reps]])
        kern[name] = {"launch_us": round(float(t.mean()) * 1e6, 2), "launch_us_median": round(float(np.median(t)) * 1e6, 2),
                      "algorithmic_bytes": alg[name], "GBps": round(alg[name] / t.mean() / 1e9, 1),
                      "frac": round(alg[name] / t.mean() / 1e9 / HBM_PEAK_GBPS, 4)}
    kern["frame_fec"]["kernel"] = kern["frame_seg"]["kernel"] = "k_frame_{fec,seg}_q (quarter-wave, slice-by-16 CRC)"
    kern["parse_fec"]["kernel"] = kern["parse_seg"]["kernel"] = "k_parse_q (quarter-wave, CRC by row)"
    # parse(frame(x)) = x: payload bytes, zero slot tails, OK records with the input headers
    ok = bool(torch.equal(pay_f.view(NF, P)[:, :S], w.parity.view(NF, P)[:, :S]) and
              torch.equal(pay_s.view(NS, P)[:, :S], w.shards.view(NS, P)[:, :S]))
    ok = ok and (S == P or not (bool(pay_f[:, S:].any()) or bool(pay_s[:, S:].any())))
    ok = ok and bool((rec_f[:, 0] == 0).all()) and bool((rec_s[:, 0] == 0).all())
    ok = ok and torch.equal(rec_s[:, 8:28], w.hdr.view(NS, 20)) and torch.equal(rec_f[:, 8:28], w.meta.view(NF, 20))
    digest_ok = None
    if WIRE_GOLDEN.exists():
        gold = json.loads(WIRE_GOLDEN.read_text())
        g = gold["groups"]
        if gold["dstride"] == D and gold["payload_stride"] == P and g <= G:
            got_f = wire_digest(dg_f[:g * n].cpu().numpy(), lf[:g * n])
            got_s = wire_digest(dg_s[:g * k].cpu().numpy(), ls[:g * k])
            digest_ok = got_f == gold["fec_sha256"] and got_s == gold["seg_sha256"]
    res = {"workload": f"c3 datagrams: {NF} SIM_FEC + {NS} SIM_SEG of {S} B in {D}-B slots, parsed back",
           "kernels": kern, "reps": reps, "timing": TIMING_OWN.split(" (")[0],
           "verified_round_trip": ok, "verified_vs_oracle_digest": digest_ok,
           "digest_scope": "the datagrams of groups [0, 4,096) (both kinds) = the oracle's framing of the same "
                           "groups (pinned to the reference's datagrams at S <= 1,000: tests/golden/wire_*.bin)"}
    del dg_f, dg_s, rec_f, rec_s, pay_f, pay_s
    torch.cuda.empty_cache()
    return res


def kernel_desc(w, k, S, full_plan):
    """(encode kernel, decode kernels) the library launches for this workload
    (rfec_launch_encode / rfec_launch_recover_out dispatch, rfec_kernels.hip)."""
    lines = [w.plan.line[l].count for l in range(w.n)]
    rows_layout = not full_plan and len(set(lines[:-1])) <= 1
    if rows_layout and (k, lines[0]) in ((10, 4), (32, 4)):
        enc_kernel = f"k_encode_out<{k},{lines[0]}>"
    elif rows_layout and lines[0] <= 16:
        enc_kernel = "k_encode_out_rt (run-time k, col)"
    elif full_plan:
        enc_kernel = f"k_encode_matrix_out<{k},{w.plan.col}>"
    else:
        enc_kernel = "k_encode (plan-driven)"
    cd = (S + 15) // 16
    if w.packed:
        kt = f"{k},{lines[0]}" if (k, lines[0]) in ((10, 4), (32, 4)) else "0,4 (run-time k, col)"
        return enc_kernel, (f"k_decode_rows<{kt}> packed (rfec_recover_packed_out: one lane per (group, output "
                            "slot, chunk); header lanes per (group, output slot) on the packed erasure records, "
                            "spread)"), lines, rows_layout
    per = ("one lane per (group, output slot, chunk)" if w.dense and 2 <= len(lines)
           else "one lane per (group, line, chunk)")
    if full_plan:
        dense_k = (f"k_decode_matrix_dense<{k},{w.plan.col}>" if 6 <= k <= 16 and w.plan.col == (3 if k <= 9 else 4)
                   else "k_decode_cascade_dense")
        dec_kernels = (f"{dense_k} (one launch: checker blocks spread over the payload lanes, one "
                       "lane per (group, output slot, chunk))" if w.dense else
                       "k_cascade_check + k_decode_cascade (one lane per (group, schedule step, chunk))")
    elif rows_layout and (k, lines[0]) in ((10, 4), (32, 4)) and (cd >= 64 or (w.dense and 2 <= len(lines)
                                                                              and cd >= 16)):
        dec_kernels = f"k_decode_rows<{k},{lines[0]}> ({per}; header blocks spread)"
    elif cd >= 64:
        dec_kernels = f"k_decode_out ({per}; header blocks spread)"
    else:
        dec_kernels = "k_decode_disjoint (one lane per (group, chunk), every fired line; header blocks spread)"
    return enc_kernel, dec_kernels, lines, rows_layout


def config_sub(lib, name, device, stream, dist, world, rank, pf, steps, warmup, verify):
    """A BASELINE configuration beside the c3 headline on the driver's default
    line (c5 = configs[4]; c3full = configs[2] under the sender's whole 3 x 4
    plan, the plan it really emits under loss): every rank runs the config's
    65,536 groups on its own slice of the config's stream (groups
    [r * 65,536, (r + 1) * 65,536), weak, as the headline), `steps` timed
    encode + decode steps over two buffer sets with the headline's timing
    discipline.  Every rank checks its outputs (torch XOR of every line, every
    erased segment back bit-exact); rank 0's groups are the reference's
    full-size digest case (full_hashes.json).  Returns the sub-object on rank
    0 (None elsewhere)."""
    cfg = CONFIGS[name]
    k, S, G = cfg["k"], cfg["S"], cfg["groups"]
    col = int(cfg["plan"][3:]) if cfg["plan"].startswith("col") else 0
    full_plan = cfg["plan"] == "full"
    sets = [Workload(lib, G, k, S, pf, device, rank * G, seed=2000 + 17 * rank, col=col, full_plan=full_plan,
                     config_id=cfg["config_id"]) for _ in range(2)]
    w = sets[0]
    # (kernel windows on every SUB_EVERY-th step: 10 samples of the default 80 steps)
    elapsed, t_enc, t_dec, own_enc, own_dec, _ = time_steps(lib, sets, steps, warmup, stream, dist, "own", False,
                                                         SUB_EVERY)
    verified = digest_ok = None
    if verify:
        verified = all(ws.verify() for ws in sets)
        if rank == 0:
            want = golden_digest(cfg["golden"], 1, 0)
            digest_ok = None if want is None else w.digest() == want
            verified = verified and digest_ok is not False
    # row layouts: the same steps again with the decode on packed erasure records (rfec_recover_packed_out)
    t_pk, pk_ok = 0.0, -1
    if w.pks:
        for ws in sets:
            ws.use_packed(True)
        _, _, t_dec_pk, _, own_pk, _ = time_steps(lib, sets, steps, warmup, stream, dist, "own", False, SUB_EVERY)
        t_pk = float(t_dec_pk.mean()) * 1e6 if own_pk else -1.0
        # the records' producer here: rfec_pack_erasures (k_pack_rows) from the batch layout, outside the
        # decode's time; timed the same way so the line shows what the records cost to build
        pev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in pev:
            a.record(stream)
            b.record(stream)
        for a, b in pev:
            lib.timing_events(a.cuda_event, b.cuda_event)
            w.prepare(stream.cuda_stream)
        torch.cuda.synchronize(device)
        t_pack = float(np.mean([a.elapsed_time(b) for a, b in pev])) * 1e3
        if verify:
            pk_ok = int(all(ws.verify() for ws in sets))
            verified = verified and bool(pk_ok)
        pk_kernels = kernel_desc(w, k, S, full_plan)[1]
        for ws in sets:
            ws.use_packed(False)
    else:
        t_pack = -1.0
    per_rank = torch.tensor([w.enc_bytes + w.dec_bytes, float(t_enc.mean()) * 1e6, float(t_dec.mean()) * 1e6,
                             -1 if verified is None else int(verified), t_pk, pk_ok, t_pack], dtype=torch.float64)
    rows = [per_rank]
    if dist:
        rows = [torch.zeros_like(per_rank) for _ in range(world)]
        dist.all_gather(rows, per_rank)
    res = None
    if rank == 0:
        enc_kernel, dec_kernels, lines, _ = kernel_desc(w, k, S, full_plan)
        mix = encode_mix(w)
        mix_gbps = mix_ceiling(lib, device, *mix) if mix else None
        enc_us, dec_us = float(rows[0][1]), float(rows[0][2])
        ach = w.enc_bytes / (enc_us * 1e-6) / 1e9
        wn = f"k{k}_r{w.n}_S{S}_G{G}"
        res = {"workload": f"{name}: {wn}" + (f" per GPU x {world} (weak)" if world > 1 else ""),
               "desc": cfg["desc"], "scaling": "weak",
               "value": round(sum(float(r[0]) for r in rows) * steps / elapsed / 2**30, 3), "unit": "GiB/s",
               "steps": steps, "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 4),
               "buffer_sets": 2, "decode_order": "cold (the set encoded one step earlier), as the headline",
               "plan_lines": lines, "bytes_per_step_per_gpu": {"encode": w.enc_bytes, "decode": w.dec_bytes},
               "encode": {"kernel": enc_kernel, "launch_us": round(enc_us, 2),
                          "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": load_traffic(wn, "encode"),
                          "mix_ceiling": None if not mix else {
                              "probe": f"rfec_probe_mix {mix[0]} reads : {mix[1]} writes, {mix[2]} B per stream",
                              "GBps": round(mix_gbps, 1), "frac_of_peak": round(mix_gbps / HBM_PEAK_GBPS, 4),
                              "kernel_vs_ceiling": round(ach / mix_gbps, 4)}},
               "decode": {"kernels": dec_kernels, "launch_us": round(dec_us, 2),
                          "frac": round(w.dec_bytes / (dec_us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
                          "traffic": load_traffic(wn, "decode")},
               "decode_packed": None if not w.pks else {
                   "kernels": pk_kernels, "input": "packed erasure records (rfec_pack_erasures layout, "
                   f"{w.pks} B per group), built before timing; the same steps and outputs",
                   "launch_us": round(float(rows[0][4]), 2) if float(rows[0][4]) > 0 else None,
                   "frac": round(w.dec_bytes / (float(rows[0][4]) * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)
                   if float(rows[0][4]) > 0 else None,
                   "traffic": load_traffic(wn + "+packed", "decode"),
                   "launch_us_per_rank": [round(float(r[4]), 2) for r in rows],
                   "verified": None if not verify else all(int(r[5]) == 1 for r in rows),
                   "producer": {"call": "rfec_pack_erasures (kernel k_pack_rows) from the batch layout's headers, "
                                        "masks and the encode's meta, before the timed steps (not in launch_us)",
                                "launch_us": round(float(rows[0][6]), 2),
                                "frac_with_pack": round(w.dec_bytes / ((float(rows[0][4]) + float(rows[0][6])) * 1e-6)
                                                        / 1e9 / HBM_PEAK_GBPS, 4) if float(rows[0][4]) > 0 else None}},
               "encode_us_per_rank": [round(float(r[1]), 2) for r in rows],
               "decode_us_per_rank": [round(float(r[2]), 2) for r in rows],
               "timing": "per launch: " + (TIMING_OWN if own_enc and own_dec else TIMING_BRACKET),
               "verified": None if not verify else all(int(r[3]) == 1 for r in rows),
               "verified_vs_reference_digest": digest_ok,
               "digest_scope": "rank 0's groups [0, 65,536) = the reference's full-size digest case "
                               f"{cfg['golden']}; the other ranks' groups are checked by the torch XOR checks"}
    del w, sets
    torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=list(CONFIGS),
                    help="c3 (default): weak scaling, 65,536 groups per GPU; c4: 1M groups split over the GPUs")
    ap.add_argument("--groups", type=int, default=0, help="custom: groups per GPU (weak scaling)")
    ap.add_argument("--total-groups", type=int, default=0, help="custom: split this many groups over the GPUs")
    ap.add_argument("--k", type=int, default=0)
    ap.add_argument("--payload", type=int, default=0)
    ap.add_argument("--stride", type=int, default=0, help="HBM slot width (default: payload rounded to 16)")
    ap.add_argument("--protect-fraction", type=int, default=80)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--tuning", type=int, default=0)
    ap.add_argument("--lib", default="", help="A/B only: another build of librazor_fec.so")
    ap.add_argument("--timing", choices=("own", "bracket"), default="own",
                    help="roofline launch duration: the kernel's own start/stop events (hipExtLaunchKernel) or "
                         "stream events around the call")
    ap.add_argument("--sets", type=int, default=2, help="disjoint buffer sets rotated per step (MALL-proof timing)")
    ap.add_argument("--col", type=int, default=0, help="custom: rows of COL segments")
    ap.add_argument("--full-plan", action="store_true", help="custom: rows + columns of the reference plan")
    ap.add_argument("--in-place", action="store_true",
                    help="decode into the received shards (rfec_recover_batch) instead of a dense output")
    ap.add_argument("--packed-decode", action="store_true",
                    help="dense row-layout decodes from packed erasure records (rfec_recover_packed_out)")
    ap.add_argument("--hot-decode", action="store_true",
                    help="decode the set encoded in the same step (its parity still MALL-resident)")
    ap.add_argument("--c4-steps", type=int, default=10,
                    help="timed steps of the c4_strong sub-object (config c3 only; 0 = skip it)")
    ap.add_argument("--no-wire", action="store_true", help="skip the wire sub-object (§8(f1) kernels)")
    ap.add_argument("--sub-steps", type=int, default=80,
                    help="timed steps of the c5 / c3full sub-objects (config c3 only; 0 = skip them)")
    args = ap.parse_args()

    # --gpus N without a launcher: start N ranks under torchrun as a child
    # process (nothing here has touched the GPU yet), exit with its code
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(Path(__file__).resolve())]
        raise SystemExit(subprocess.call(cmd + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")  # control plane only: barrier, max time, byte sum
    ndev = torch.cuda.device_count()
    if ndev < 1 or not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    torch.cuda.set_device(local % ndev)
    device = torch.device("cuda", local % ndev)

    lib = Native(1000, args.lib) if args.lib else native(1000)
    lib.set_tuning(args.tuning)
    custom = args.groups or args.total_groups or args.k or args.payload or args.col or args.full_plan
    cfg_name = args.config
    cfg = dict(CONFIGS[cfg_name])
    if args.full_plan:
        cfg.update(plan="full", config_id=3)
    if args.col:
        cfg.update(plan=f"col{args.col}")
    if args.k:
        cfg["k"] = args.k
    if args.payload:
        cfg["S"] = args.payload
    if custom:
        cfg.update(golden=None, desc="custom")
        cfg_name = "custom"
    k, S = cfg["k"], cfg["S"]
    if args.groups:
        group0, my_groups, total, scaling = rank * args.groups, args.groups, args.groups * world, "weak"
    else:
        total = args.total_groups or cfg["groups"]
        if cfg_name == "c4" or args.total_groups:
            group0, my_groups = shard_groups(total, world, rank)
            scaling = "strong"
        else:  # per-GPU config (c3 / c3full / c5): every rank runs the whole config on its own groups
            group0, my_groups, scaling = rank * total, total, "weak"
            total *= world
    col = int(cfg["plan"][3:]) if cfg["plan"].startswith("col") else 0
    full_plan = cfg["plan"] == "full"
    sets = [Workload(lib, my_groups, k, S, args.protect_fraction, device, group0, seed=1000 + rank,
                     stride=args.stride or None, col=col, full_plan=full_plan, config_id=cfg["config_id"],
                     in_place=args.in_place)
            for _ in range(max(1, args.sets))]
    if args.packed_decode:
        if not sets[0].pks:
            raise SystemExit("bench.py: --packed-decode needs a dense decode of a row layout (rows of <= 4, k <= 64)")
        for ws in sets:
            ws.use_packed(True)
    w = sets[0]
    nset = len(sets)
    stream = torch.cuda.current_stream(device)
    sp = stream.cuda_stream
    torch.cuda.synchronize(device)

    elapsed, t_enc, t_dec, own_enc, own_dec, window = time_steps(lib, sets, args.steps, args.warmup, stream, dist,
                                                                 args.timing, args.hot_decode)
    ranks = gather_objects(dist, dict(rank=rank, local_rank=local, **device_identity(device)))

    verified, digest_ok = None, None
    if not args.no_verify:
        verified = all(ws.verify() for ws in sets)
        # the reference's digest of exactly these groups, where the golden file holds one
        want = None
        if cfg["golden"] and scaling == "strong":
            want = golden_digest(cfg["golden"], world, rank)
        elif cfg["golden"] and group0 == 0:
            want = golden_digest(cfg["golden"], 1, 0)
        elif cfg.get("weak_golden"):  # weak scaling: this rank's chunk of the stream
            want = golden_digest(cfg["weak_golden"], world, rank, chunk=w.G)
        if want is not None:
            digest_ok = w.digest() == want
            verified = verified and digest_ok
    if dist:
        # verified: every rank's checks held; digest: True only when every rank had a reference digest for
        # its groups and matched it, False when any rank mismatched, None when some rank had none
        vt = torch.tensor([1 if verified in (None, True) else 0, 0 if digest_ok is False else 1,
                           1 if digest_ok is True else 0], dtype=torch.int32)
        dist.all_reduce(vt, op=dist.ReduceOp.MIN)
        verified = None if args.no_verify else bool(vt[0].item())
        digest_ok = None if args.no_verify else (False if not vt[1].item() else (True if vt[2].item() else None))

    # BASELINE configs[3] beside the weak headline (default run only): the 1M-group strong split
    c4 = None
    if cfg_name == "c3" and args.c4_steps > 0 and not args.lib:
        log("c4 strong split ...")
        c4 = c4_strong(lib, device, stream, dist, world, rank, args.protect_fraction, args.c4_steps, 2,
                       not args.no_verify)
        if c4 and c4["verified"] is False:
            verified = False
    # BASELINE configs[4] (c5) and the sender's full plan (c3full) on the same line (default run only)
    subs = {}
    if cfg_name == "c3" and args.sub_steps > 0 and not args.lib:
        for sub in ("c5", "c3full"):
            log(f"{sub} ...")
            subs[sub] = config_sub(lib, sub, device, stream, dist, world, rank, args.protect_fraction,
                                   args.sub_steps, 2, not args.no_verify)
            if subs[sub] and subs[sub]["verified"] is False:
                verified = False

    # whole-job bytes: every rank's slice (equal slices up to one group)
    nb = torch.tensor([w.enc_bytes + w.dec_bytes, w.G], dtype=torch.float64)
    if dist:
        dist.all_reduce(nb, op=dist.ReduceOp.SUM)
    step_bytes = float(nb[0].item())
    value = step_bytes * args.steps / elapsed / 2**30
    enc_mean = float(t_enc.mean())
    dec_mean = float(t_dec.mean())
    achieved = w.enc_bytes / enc_mean / 1e9
    res = None
    if rank == 0:
        ceiling = copy_ceiling(lib, device)
        mix = encode_mix(w)
        mix_gbps = mix_ceiling(lib, device, *mix) if mix else None
        workload_name = f"k{k}_r{w.n}_S{S}_G{w.G}"
        enc_kernel, dec_kernels, lines, _ = kernel_desc(w, k, S, full_plan)
        if full_plan:
            plan_desc = (f"full reference plan {w.plan.row}x{w.plan.col}: {w.plan.n_row_lines} rows + "
                         f"{w.n - w.plan.n_row_lines} columns, line sizes {lines}")
            pairs_desc = "uniform over all recoverable pairs (peeling, with cascades)"
        else:
            plan_desc = ("row layer of the reference 3x4 plan, rows {4,4,2}" if (k, col) == (10, 0)
                         else f"rows of sizes {lines}")
            pairs_desc = f"uniform over the {len(distinct_row_pairs(w.plan))} distinct-row pairs"
        traffic = load_traffic(workload_name, "encode")
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": (f"synthetic: SURVEY §8(d) xorshift64* payloads (config id {cfg['config_id']}, generated on the "
                     f"device by jump-ahead), sequential headers; resident in HBM before timing"),
            "config": {"workload": f"{cfg_name}: {workload_name}" + (
                           (f" (rank 0's slice of {total})" if scaling == "strong" else
                            f" per GPU x {world} (weak scaling: rank r runs groups [r*{w.G}, (r+1)*{w.G}))")
                           if world > 1 else ""),
                       "scaling_rule": ("weak: every GPU runs the N = 1 workload on its own groups, value = all "
                                        "ranks' bytes / max-over-ranks time" if scaling == "weak" else
                                        "strong: the config's groups split over the GPUs (--config c4 at N = 1 "
                                        "runs all of them on one GPU)"),
                       "config": cfg_name, "desc": cfg["desc"], "groups_per_gpu": w.G, "total_groups": total,
                       "k": k, "r": w.n, "payload_bytes": S, "plan": plan_desc,
                       "erasures_per_group": 2, "erasure_pairs": pairs_desc,
                       "parallelism": f"batch split over {world} GPU(s) (contiguous group slices), no collective; "
                                      f"control plane on a CPU gloo group" if world > 1 else "1 GPU",
                       "buffer_sets": nset,
                       "decode_order": "hot (same step's set)" if args.hot_decode or nset == 1 else
                                       "cold (the set encoded one step earlier)",
                       "bytes_per_step_per_gpu": {"encode": w.enc_bytes, "decode": w.dec_bytes},
                       "algorithmic_bytes": "payload bytes read + written (20-B headers excluded)"},
            "roofline": {"bound": "hbm", "kernel": enc_kernel, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "launch_us": round(enc_mean * 1e6, 2),
                         "launch_us_median": round(float(np.median(t_enc)) * 1e6, 2),
                         "timing": TIMING_OWN if own_enc else TIMING_BRACKET,
                         "algorithmic_bytes_per_launch": w.enc_bytes,
                         "mix_ceiling": None if not mix else {
                             "probe": f"rfec_probe_mix {mix[0]} reads : {mix[1]} writes, {mix[2]} B per stream "
                                      f"(the encode's byte mix and volume, contiguous streams)",
                             "GBps": round(mix_gbps, 1), "frac_of_peak": round(mix_gbps / HBM_PEAK_GBPS, 4),
                             "kernel_vs_ceiling": round(achieved / mix_gbps, 4)}},
            "encode_gibps": round(w.enc_bytes / enc_mean / 2**30, 2),
            # source bytes k*S*G over the encode time, and that as a fraction of the peak
            "encode_source_gibps": round(w.G * w.k * w.S / enc_mean / 2**30, 2),
            "encode_read_only_frac": round(w.G * w.k * w.S / enc_mean / 1e9 / HBM_PEAK_GBPS, 4),
            "decode_gibps": round(w.dec_bytes / dec_mean / 2**30, 2),
            "decode_output": ("dense: rfec_recover_batch_out, recovered segments to [G][2] slots (flex_fec_recover's "
                              "out_seg); the received shards read only" if w.dense else "in place: rfec_recover_batch")
            + ("; header input: packed erasure records (rfec_recover_packed_out)" if w.packed else ""),
            "decode_roofline": {"achieved": round(w.dec_bytes / dec_mean / 1e9, 1), "frac":
                                round(w.dec_bytes / dec_mean / 1e9 / HBM_PEAK_GBPS, 4),
                                "launch_us": round(dec_mean * 1e6, 2),
                                "launch_us_median": round(float(np.median(t_dec)) * 1e6, 2),
                                "timing": TIMING_OWN if own_dec else TIMING_BRACKET,
                                "traffic": load_traffic(workload_name + ("+packed" if w.packed else ""), "decode"),
                                "kernels": dec_kernels,
                                "parity_operand": "cold: written one step (>= 1.7 GB of traffic) before"
                                if not (args.hot_decode or nset == 1) else "hot: written by this step's encode"},
            "copy_ceiling_GBps": round(ceiling, 1),  # rfec_probe_copy, read + write bytes
            "timing_window": {"rule": "value = all ranks' bytes x steps / (max over ranks of t1 - min over ranks "
                                      "of t0); t0 after the opening barrier + synchronize, t1 after the closing "
                                      "synchronize (before the closing barrier), CLOCK_MONOTONIC",
                              **{kk: window[kk] for kk in ("start_skew_us", "stop_skew_us", "t0_us", "t1_us",
                                                            "clock")},
                              "rank_elapsed_max_ms": round(window["rank_elapsed_max_s"] * 1e3, 4)},
            "ranks": ranks,
            "distinct_devices": len({r["pci_bus_id"] for r in ranks}),
            "verified": verified,
            "verified_vs_reference_digest": digest_ok,
            "tuning": args.tuning,
        }
        if cfg_name == "c3" and not args.no_wire and not args.lib:
            log("wire ...")
            res["wire"] = wire_sub(lib, w, device)
            if res["wire"]["verified_round_trip"] is False or res["wire"]["verified_vs_oracle_digest"] is False:
                verified = res["verified"] = False
        if c4 is not None:
            res["c4_strong"] = c4
        for sub, d in subs.items():
            if d is not None:
                res[sub] = d
        if world == 1 and not args.no_cpu:
            log("cpu baseline ...")
            res["cpu_baseline"] = cpu_baseline(w, args.cpu_seconds)
        print(json.dumps(res), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if verified is False:
        raise SystemExit("verification failed")


if __name__ == "__main__":
    main()
