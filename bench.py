"""Benchmark: device-resident flex-FEC encode + decode on MI355X.

Workload (BASELINE.json configs[2], the metric's config): per GPU, G = 65,536
FEC groups of k = 10 segments of 1,200 bytes; the r = 3 row parities of the
reference's 3x4 plan (rows {4,4,2}, flex_fec_sender.c:166-188); 2 erasures
per group drawn from the 32 distinct-row pairs, recovered by peeling
(flex_fec_receiver.c:105-150).  One step = encode every group, then recover
every erased segment.  Inputs are synthetic, resident in HBM before timing.

Multi-GPU: one process per GPU (torchrun); groups are independent, so each
rank encodes/decodes its own slice of the batch with no data-path collective
(weak scaling); a barrier + max-over-ranks time bracket the timed steps.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from razor_amd.dist import shard_groups  # noqa: E402
from razor_amd.fec import HDR_DTYPE, native  # noqa: E402

METRIC = "FEC encode+decode GiB/s (device-resident), 1200B pkts k=10/r=3; % HBM peak"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_headers(G, k, S, group0):
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
    def __init__(self, lib, G, k, S, pf, device, group0, seed, stride=None, col=0, full_plan=False):
        self.lib, self.G, self.k, self.S = lib, G, k, S
        self.stride = stride or (S + 15) // 16 * 16  # slot width in HBM (>= S, multiple of 16)
        if col:  # explicit rows of `col` (config 5: k = 32 as 8 rows of 4)
            self.plan = lib.plan_matrix(k, (k + col - 1) // col, col, 1)
        elif full_plan:  # the reference sender's whole plan: rows and columns (3x4 -> 7 parities at k = 10)
            self.plan = lib.plan_from_fraction(k, pf, 3)
        else:
            self.plan = lib.plan_from_fraction(k, pf, 1)  # row layer: r = 3 at k = 10
        self.n = self.plan.n_lines
        dev = device
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed)
        if self.stride == S:
            self.shards = torch.randint(0, 256, (G, k, S), dtype=torch.uint8, device=dev, generator=gen)
        else:
            self.shards = torch.zeros((G, k, self.stride), dtype=torch.uint8, device=dev)
            self.shards[:, :, :S] = torch.randint(0, 256, (G, k, S), dtype=torch.uint8, device=dev, generator=gen)
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
        self.erased = pairs[rng.integers(0, len(pairs), G)]
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
        self.ws = torch.empty((lib.workspace_size(self.plan, G),), dtype=torch.uint8, device=dev)
        # algorithmic payload bytes (headers excluded): encode reads k*S, writes r*S
        self.enc_bytes = G * (k + self.n) * S
        # decode: per recovered segment read its line's other members + the parity, write 1
        pair_bytes = {tuple(p): peel_bytes(self.plan, k, tuple(p), S) for p in pairs.tolist()}
        self.dec_bytes = int(sum(pair_bytes[(int(a), int(b))] for a, b in self.erased))

    def encode(self, stream):
        self.lib.encode_batch(self.plan, self.G, self.stride, self.S, self.shards.data_ptr(), self.hdr.data_ptr(),
                              self.parity.data_ptr(), self.meta.data_ptr(), self.fsize.data_ptr(),
                              self.status.data_ptr(), stream)

    def decode(self, stream):
        self.lib.recover_batch(self.plan, self.G, self.stride, self.S, self.rx.data_ptr(), self.rx_hdr.data_ptr(),
                               self.present.data_ptr(), self.parity.data_ptr(), self.meta.data_ptr(),
                               self.fsize.data_ptr(), self.parity_present.data_ptr(), self.recovered.data_ptr(),
                               self.ws.data_ptr(), stream)

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
        ok = ok and torch.equal(self.rx[:, :, :S], self.shards[:, :, :S]) and torch.equal(self.rx_hdr, self.hdr)
        exp = ((1 << self.erased[:, 0]) | (1 << self.erased[:, 1])).astype(np.int64)
        ok = ok and np.array_equal(self.recovered[:, 0].cpu().numpy(), exp)
        ok = ok and int(self.status.abs().sum()) == 0
        return bool(ok)


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


def cpu_baseline(w: Workload, seconds: float):
    """The oracle's reference-shaped path (flex_fec_generate per line, flex_fec_recover
    per erasure, over AoS sim_segment_t) on a bounded sample of the same groups."""
    sys.path.insert(0, str(ROOT / "oracle"))
    from pyoracle import Oracle

    sample = min(w.G, 4096)
    shards = w.shards[:sample, :, :w.S].cpu().numpy()
    hdr = w.hdr_np[:sample]
    present = w.present_np[:sample]
    out = {}
    for label, opt, threads in (("O2_1core", "O2", 1), ("O0_1core", "O0", 1), ("O2_16threads", "O2", 16)):
        o = Oracle(1200, opt)
        segs = o.to_aos(shards, hdr)
        budget = seconds if label == "O2_1core" else seconds / 4
        t_enc = t_dec = 0.0
        reps = 0
        fec = None
        while t_enc + t_dec < budget or reps == 0:
            t0 = time.perf_counter()
            n, fec = o.encode_aos(w.plan, sample, segs, threads=threads)
            t1 = time.perf_counter()
            if threads == 1:
                nrec, _ = o.recover_aos(w.plan, sample, segs, fec, present)
                assert nrec == 2 * sample
            t2 = time.perf_counter()
            t_enc += t1 - t0
            t_dec += t2 - t1
            reps += 1
        enc_b = sample * (w.k + w.n) * w.S * reps
        dec_b = w.dec_bytes * sample / w.G * reps
        if threads == 1:
            out[label] = {"gibps": (enc_b + dec_b) / (t_enc + t_dec) / 2**30,
                          "encode_gibps": enc_b / t_enc / 2**30, "decode_gibps": dec_b / t_dec / 2**30,
                          "reps": reps, "seconds": t_enc + t_dec}
        else:
            out[label] = {"encode_gibps": enc_b / t_enc / 2**30, "reps": reps, "seconds": t_enc}
    main = out["O2_1core"]
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(main["gibps"], 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{sample} groups x {reps_str(main)} of the same workload (k=10, rows {{4,4,2}}, 1200 B, "
                      f"2 erasures/group), oracle/rfec_oracle.c at -O2 over AoS sim_segment_t, one thread",
            "cpu": cpu, "encode_gibps": round(main["encode_gibps"], 4), "decode_gibps": round(main["decode_gibps"], 4),
            "reference_flags_O0_1core_gibps": round(out["O0_1core"]["gibps"], 4),
            "O2_16threads_encode_gibps": round(out["O2_16threads"]["encode_gibps"], 4)}


def reps_str(d):
    return f"{d['reps']} passes ({d['seconds']:.1f} s)"


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--groups", type=int, default=65536, help="groups per GPU (weak scaling)")
    ap.add_argument("--total-groups", type=int, default=0,
                    help="split this many groups over the GPUs instead (strong scaling, e.g. 1048576)")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--payload", type=int, default=1200)
    ap.add_argument("--stride", type=int, default=0, help="HBM slot width (default: payload rounded to 16)")
    ap.add_argument("--protect-fraction", type=int, default=80)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--tuning", type=int, default=0)
    ap.add_argument("--sets", type=int, default=2, help="disjoint buffer sets rotated per step (MALL-proof timing)")
    ap.add_argument("--col", type=int, default=0, help="rows of COL segments (config 5: --k 32 --payload 256 --col 4)")
    ap.add_argument("--full-plan", action="store_true", help="rows + columns of the reference plan (config 3 variant)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=device)

    lib = native(1000)
    lib.set_tuning(args.tuning)
    if args.total_groups:
        group0, my_groups = shard_groups(args.total_groups, world, rank)
        scaling = "strong"
    else:
        group0, my_groups = rank * args.groups, args.groups
        scaling = "weak"
    # rotate over disjoint buffer sets (same inputs), so that the
    # 256 MB MALL never holds a step's operands from the previous step
    sets = [Workload(lib, my_groups, args.k, args.payload, args.protect_fraction, device, group0, seed=1000 + rank,
                     stride=args.stride or None, col=args.col, full_plan=args.full_plan)
            for _ in range(max(1, args.sets))]
    w = sets[0]
    stream = torch.cuda.current_stream(device)
    sp = stream.cuda_stream
    torch.cuda.synchronize(device)

    for i in range(args.warmup):
        sets[i % len(sets)].encode(sp)
        sets[i % len(sets)].decode(sp)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        a, b, c = ev[i]
        ws = sets[i % len(sets)]
        a.record(stream)
        ws.encode(sp)
        b.record(stream)
        ws.decode(sp)
        c.record(stream)
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    t_enc = np.array([a.elapsed_time(b) for a, b, _ in ev]) / 1e3
    t_dec = np.array([b.elapsed_time(c) for _, b, c in ev]) / 1e3
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    verified = None if args.no_verify else all(ws.verify() for ws in sets)
    if dist:
        vt = torch.tensor([1 if verified in (None, True) else 0], dtype=torch.int32, device=device)
        dist.all_reduce(vt, op=dist.ReduceOp.MIN)
        verified = None if args.no_verify else bool(vt.item())

    # whole-job bytes: every rank's slice (equal slices up to one group)
    nb = torch.tensor([w.enc_bytes + w.dec_bytes], dtype=torch.float64, device=device)
    if dist:
        dist.all_reduce(nb, op=dist.ReduceOp.SUM)
    step_bytes = float(nb.item())
    value = step_bytes * args.steps / elapsed / 2**30
    enc_mean = float(t_enc.mean())
    dec_mean = float(t_dec.mean())
    achieved = w.enc_bytes / enc_mean / 1e9
    res = None
    if rank == 0:
        ceiling = copy_ceiling(lib, device)
        workload_name = f"k{args.k}_r{w.n}_S{args.payload}_G{w.G}"
        lines = [w.plan.line[l].count for l in range(w.n)]
        rows_layout = not args.full_plan and len(set(lines[:-1])) <= 1
        enc_kernel = (f"k_encode_rows<{args.k},{lines[0]}>" if rows_layout and (args.k, lines[0]) in ((10, 4), (32, 4))
                      else "k_encode (plan-driven)")
        dec_kernels = ("k_peel_lds + k_recover_flat (cascading peel: schedule, then replay)" if args.full_plan
                       else "k_decode_disjoint (peel headers + payload, one launch)")
        if args.full_plan:
            plan_desc = f"full reference plan {w.plan.row}x{w.plan.col}: {w.plan.n_row_lines} rows + {w.n - w.plan.n_row_lines} columns, line sizes {lines}"
            pairs_desc = "uniform over all recoverable pairs (peeling, with cascades)"
        else:
            plan_desc = ("row layer of the reference 3x4 plan, rows {4,4,2}" if (args.k, args.col) == (10, 0)
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
            "data": "synthetic (torch.randint payloads, sequential headers), resident in HBM before timing",
            "config": {"workload": workload_name, "groups_per_gpu": w.G,
                       "total_groups": args.total_groups or args.groups * world, "k": args.k, "r": w.n,
                       "payload_bytes": args.payload, "plan": plan_desc,
                       "erasures_per_group": 2, "erasure_pairs": pairs_desc,
                       "parallelism": f"batch split over {world} GPU(s), no collective",
                       "buffer_sets": len(sets),
                       "bytes_per_step_per_gpu": {"encode": w.enc_bytes, "decode": w.dec_bytes},
                       "algorithmic_bytes": "payload bytes read + written (20-B headers excluded)"},
            "roofline": {"bound": "hbm", "kernel": enc_kernel, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "launch_us": round(enc_mean * 1e6, 2),
                         "launch_us_median": round(float(np.median(t_enc)) * 1e6, 2),
                         "algorithmic_bytes_per_launch": w.enc_bytes},
            "encode_gibps": round(w.enc_bytes / enc_mean / 2**30, 2),
            # source bytes k*S*G over the encode time, and that as a fraction of the peak
            "encode_source_gibps": round(w.G * w.k * w.S / enc_mean / 2**30, 2),
            "encode_read_only_frac": round(w.G * w.k * w.S / enc_mean / 1e9 / HBM_PEAK_GBPS, 4),
            "decode_gibps": round(w.dec_bytes / dec_mean / 2**30, 2),
            "decode_roofline": {"achieved": round(w.dec_bytes / dec_mean / 1e9, 1), "frac":
                                round(w.dec_bytes / dec_mean / 1e9 / HBM_PEAK_GBPS, 4),
                                "launch_us": round(dec_mean * 1e6, 2),
                                "launch_us_median": round(float(np.median(t_dec)) * 1e6, 2),
                                "traffic": load_traffic(workload_name, "decode"),
                                "kernels": dec_kernels},
            "copy_ceiling_GBps": round(ceiling, 1),  # rfec_probe_copy, read + write bytes
            "verified": verified,
            "tuning": args.tuning,
        }
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
