"""GPU, two ranks on the one leased GPU (CPU gloo control plane, no RCCL):
the config-4 batch split (razor_amd/dist.py) through librazor_fec.so itself.

Each rank generates its contiguous slice of the 1,048,576-group config-4
stream on the device (jump-ahead, no outputs before its slice), encodes it
with the product library in 65,536-group launches and digests its outputs;
each slice digest must equal the one oracle/gen_full.c took of the
reference's flex_fec_generate over the same groups
(tests/golden/full_hashes.json, c4 "slices").  Groups are independent
(flex_fec_sender.c:146-245, sim_fec.c:152-166), so the split needs no
data-path collective.  Then bench.py --gpus 2 end to end."""
import hashlib
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden" / "full_hashes.json"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _c4():
    return {c["name"]: c for c in json.loads(GOLDEN.read_text())["cases"]}["c4_k10_rows_S1200_G1048576"]


def _worker(rank, world, port, outdir):
    sys.path[:0] = [str(ROOT)]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from bench import make_headers
    from razor_amd.dist import shard_groups
    from razor_amd.fec import native

    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = _c4()
    lib = native(1000)
    dev = torch.device("cuda", 0)  # both ranks on the one leased GPU
    torch.cuda.set_device(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    k, S, total = c["k"], c["S"], c["groups"]
    plan = lib.plan_from_fraction(k, c["pf"], c["layers"])
    assert plan.n_lines == c["n_lines"]
    lo, n = shard_groups(total, world, rank)
    chunk = 65536
    shards = torch.empty((chunk, k, S), dtype=torch.uint8, device=dev)
    par = torch.empty((chunk, plan.n_lines, S), dtype=torch.uint8, device=dev)
    meta = torch.empty((chunk, plan.n_lines, 20), dtype=torch.uint8, device=dev)
    fs = torch.empty((chunk, plan.n_lines), dtype=torch.int16, device=dev)
    status = torch.empty((chunk, plan.n_lines), dtype=torch.int8, device=dev)
    h = hashlib.sha256()
    bad = 0
    for g in range(lo, lo + n, chunk):
        m = min(chunk, lo + n - g)
        lib.fill_xorshift(shards.data_ptr(), c["config_id"], g, m, k, S, S, st)
        hdr = make_headers(m, k, S, g)
        d_hdr = torch.from_numpy(hdr.view(np.uint8).reshape(m, k, 20).copy()).to(dev)
        lib.encode_batch(plan, m, S, S, shards.data_ptr(), d_hdr.data_ptr(), par.data_ptr(), meta.data_ptr(),
                         fs.data_ptr(), status.data_ptr(), st)
        torch.cuda.synchronize(dev)
        bad += int(status[:m].abs().sum())
        rec = torch.cat([par[:m].reshape(m, -1), meta[:m].reshape(m, -1), fs[:m].view(torch.uint8).reshape(m, -1)],
                        dim=1)
        h.update(rec.cpu().numpy().tobytes())
    res = [None] * world
    dist.all_gather_object(res, {"lo": lo, "n": n, "digest": h.hexdigest(), "bad": bad})
    if rank == 0:
        Path(outdir, "result.json").write_text(json.dumps(res))
    dist.barrier()
    dist.destroy_process_group()


def test_c4_split_two_ranks_one_gpu(tmp_path):
    import torch.multiprocessing as mp

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = json.loads((tmp_path / "result.json").read_text())
    c = _c4()
    lo = 0
    for r, s in enumerate(res):
        assert s["lo"] == lo and s["bad"] == 0  # contiguous, no gap, no overlap
        lo += s["n"]
        assert s["digest"] == c["slices"][str(world)][r], f"rank {r} slice differs from the reference"
    assert lo == c["groups"]


def _bench(*args, timeout=600):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_two_ranks_one_gpu():
    """bench.py --gpus 2 starts its own two ranks (torchrun, gloo control
    plane) on the one GPU: one JSON line, weak scaling of config 3 (the N = 1
    workload on each rank's own 65,536 groups), every rank's groups equal to
    the reference digest of exactly those groups."""
    d = _bench("--gpus", "2", "--steps", "3", "--warmup", "1", "--no-cpu", "--sets", "2", "--c4-steps", "2")
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["config"]["config"] == "c3" and d["config"]["groups_per_gpu"] == 65536
    assert d["config"]["total_groups"] == 2 * 65536
    assert d["config"]["workload"].startswith("c3: k10_r3_S1200_G65536 per GPU x 2")
    assert d["verified"] is True and d["verified_vs_reference_digest"] is True
    assert d["value"] > 0
    _check_window(d, 2)
    # one kernel per call: the roofline takes each kernel's own start / stop events
    for key in ("roofline", "decode_roofline"):
        assert d[key]["timing"].startswith("the kernel's own") and d[key]["launch_us"] > 0
    _check_c4_strong(d["c4_strong"], 2)


def _check_c4_strong(c4, n):
    """The driver's default line carries BASELINE configs[3] too: the 1M
    groups split over the n ranks, each slice equal to the reference's."""
    assert c4["scaling"] == "strong" and c4["workload"].startswith("c4: k10_r3_S1200_G1048576")
    assert c4["groups_per_rank"] == [1048576 // n] * n
    assert c4["verified"] is True and c4["verified_vs_reference_digest"] is True
    assert c4["value"] > 0 and len(c4["encode_us_per_rank"]) == n and c4["launch_groups"] == 65536
    assert all(t > 0 for t in c4["encode_us_per_rank"] + c4["decode_us_per_rank"])


def _check_subs(d, n):
    """The default line carries BASELINE configs[4] (c5) and the sender's full
    3 x 4 plan (c3full) too: driver-timed, each rank on its own 65,536 groups,
    rank 0's outputs equal to the reference's full-size digest."""
    for name, enc, lines in (("c5", "k_encode_out<32,4>", [4] * 8),
                             ("c3full", "k_encode_matrix_out<10,4>", [4, 4, 2, 3, 3, 2, 2])):
        c = d[name]
        assert c["workload"].startswith(f"{name}: ") and c["scaling"] == "weak"
        assert c["plan_lines"] == lines and c["encode"]["kernel"] == enc
        assert c["verified"] is True and c["verified_vs_reference_digest"] is True
        assert c["value"] > 0 and len(c["encode_us_per_rank"]) == n
        assert all(t > 0 for t in c["encode_us_per_rank"] + c["decode_us_per_rank"])
        assert 0 < c["encode"]["frac"] < 1 and 0 < c["decode"]["frac"] < 1
        assert c["encode"]["mix_ceiling"]["kernel_vs_ceiling"] > 0
    assert d["c3full"]["decode"]["kernels"].startswith("k_decode_matrix_dense<10,4>")
    # c5 (a row layout) also decodes from packed erasure records; c3full has none
    pk = d["c5"]["decode_packed"]
    assert pk["verified"] is True and pk["kernels"].startswith("k_decode_rows<32,4> packed")
    assert len(pk["launch_us_per_rank"]) == n and all(t > 0 for t in pk["launch_us_per_rank"])
    assert d["c3full"]["decode_packed"] is None
    assert d["c5"]["encode"]["mix_ceiling"]["probe"].startswith("rfec_probe_mix 4 reads : 1 writes")
    assert d["c3full"]["encode"]["mix_ceiling"]["probe"].startswith("rfec_probe_mix 10 reads : 7 writes")


@pytest.mark.timeout(600)
def test_bench_one_gpu_c4_strong():
    """The default N = 1 line: weak c3 as `value`, plus the c4_strong object
    over all 1,048,576 groups on the one GPU (the N = 1 point of the strong
    curve), bit-exact against the reference's c4 digest, and the c5 / c3full
    objects."""
    d = _bench("--gpus", "1", "--steps", "3", "--warmup", "1", "--no-cpu", "--c4-steps", "2", "--sub-steps", "3")
    assert d["n_gpus"] == 1 and d["scaling"] == "weak" and d["config"]["config"] == "c3"
    assert d["verified_vs_reference_digest"] is True
    _check_c4_strong(d["c4_strong"], 1)
    _check_subs(d, 1)
    assert d["roofline"]["mix_ceiling"]["probe"].startswith("rfec_probe_mix 10 reads : 3 writes")
    # §8(f1) on the line: the c3 workload's datagrams framed and parsed back, the first 4,096 groups'
    # datagrams equal to the oracle's (tests/golden/wire_c3_digest.json)
    wire = d["wire"]
    assert wire["verified_round_trip"] is True and wire["verified_vs_oracle_digest"] is True
    assert set(wire["kernels"]) == {"frame_fec", "frame_seg", "parse_fec", "parse_seg"}
    assert all(0 < v["frac"] < 1 and v["launch_us"] > 0 for v in wire["kernels"].values())
    _check_window(d, 1)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("n", [4, 8])
def test_bench_n_ranks_one_gpu(n):
    """The driver's N = 4 / N = 8 launch path before an 8-GPU node runs it:
    bench.py --gpus n starts n ranks under torchrun on the one leased GPU
    (LOCAL_RANK % device_count), one JSON line; every rank's weak c3 chunk
    equals the reference digest of exactly its 65,536 groups (full_hashes.json
    c3_weak chunks[0..n)), c4_strong's slices equal the reference's n-way
    slice digests, groups_per_rank = 1,048,576 / n each.  Groups are
    independent (sim_fec.c:152-166): no data-path collective."""
    d = _bench("--gpus", str(n), "--steps", "2", "--warmup", "1", "--no-cpu", "--c4-steps", "2", "--sub-steps", "2",
               timeout=840)
    assert d["n_gpus"] == n and d["scaling"] == "weak"
    assert d["config"]["total_groups"] == n * 65536
    assert d["config"]["workload"].startswith(f"c3: k10_r3_S1200_G65536 per GPU x {n}")
    assert d["verified"] is True and d["verified_vs_reference_digest"] is True
    _check_window(d, n)
    _check_c4_strong(d["c4_strong"], n)
    _check_subs(d, n)


def _check_window(d, n):
    """The line's clock (razor_amd/dist.StepWindow): every rank's CLOCK_MONOTONIC
    t0 / t1, ms_per_step = (max t1 - min t0) / steps, the start skew, and every
    rank's physical device (here all share the one leased GPU)."""
    w = d["timing_window"]
    assert len(w["t0_us"]) == len(w["t1_us"]) == n and min(w["t0_us"]) == 0
    assert w["start_skew_us"] == max(w["t0_us"]) and w["start_skew_us"] >= 0 and w["stop_skew_us"] >= 0
    assert abs(max(w["t1_us"]) / 1e3 / d["steps"] - d["ms_per_step"]) < 1e-3
    assert w["rank_elapsed_max_ms"] <= max(w["t1_us"]) / 1e3 + 1e-3  # (rounded to 0.1 us and 0.01 us)
    assert [r["rank"] for r in d["ranks"]] == list(range(n))
    for r in d["ranks"]:
        assert len(r["pci_bus_id"].split(":")) == 3 and r["name"]
    assert d["distinct_devices"] == 1


@pytest.mark.timeout(900)
def test_bench_c4_strong_scaling_lines():
    """--config c4 at N = 1 and N = 2 (two ranks on the one GPU): both lines
    name config 4 over the same 1,048,576 groups (strong scaling), so their
    ratio is an efficiency of the same workload; N = 2 checks each rank's
    slice against the reference's slice digest."""
    one = _bench("--gpus", "1", "--config", "c4", "--steps", "3", "--warmup", "1", "--no-cpu", "--sets", "1",
                 "--no-verify")
    two = _bench("--gpus", "2", "--config", "c4", "--steps", "3", "--warmup", "1", "--no-cpu", "--sets", "1")
    for d, n in ((one, 1), (two, 2)):
        assert d["n_gpus"] == n and d["scaling"] == "strong"
        assert d["config"]["config"] == "c4" and d["config"]["total_groups"] == 1048576
        assert d["config"]["workload"].startswith("c4: k10_r3_S1200_G")
        assert d["value"] > 0
    assert one["config"]["groups_per_gpu"] == 1048576 and two["config"]["groups_per_gpu"] == 524288
    assert two["verified"] is True and two["verified_vs_reference_digest"] is True
