"""GPU: the drop-in's resident service (razor_amd/csrc/rfec_service.hip) is
taken off the device by rfec_service_stop and launched again by the next
drop-in call, whose output is still the reference sender's
(tests/golden/enc_k10_pf80_S1000.bin).  A module of its own, so the service
counters are not shared with test_flex_dropin's module-scoped modes."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import pyoracle as po
from test_flex_dropin import CASES, _svc_stats, bar_host_mapped, bind_flex, make_segments, sender_group

pytestmark = pytest.mark.gpu


def test_service_stop_and_relaunch(product, oracle1000):
    """rfec_service_stop takes the resident workgroup off the device; the next
    drop-in call launches it again and its output is still the reference's."""
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")
    lib = bind_flex(product)
    L = lib.lib
    L.rfec_set_tuning(0)
    c = CASES["k10_pf80_S1000"]
    shards, hdr = oracle1000.fill_groups(c["config_id"], c["groups"], c["k"], c["S"], ragged=c["ragged"])
    recs, pays = po.load_parities(c)
    snd = L.flex_fec_sender_create()
    try:
        for g in range(3):
            before = _svc_stats(L)
            assert L.rfec_service_stop() == 0
            fecs = sender_group(lib, snd, make_segments(lib, shards[g], hdr[g]), c["protect_fraction"])
            after = _svc_stats(L)
            assert after[0] == before[0] + 1 and after[1] == before[1] + 1, (before, after)
            sel = np.nonzero(recs["group"] == g)[0]
            assert len(fecs) == len(sel)
            for f, ri in zip(fecs, sel):
                n = int(recs[ri]["fec_data_size"])
                assert f.fec_data_size == n and bytes(f.fec_data)[:n] == pays[ri][:n].tobytes()
    finally:
        L.flex_fec_sender_destroy(snd)
        assert L.rfec_service_stop() == 0


_HOL_SCRIPT = r"""
import json, sys, time
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import torch
import pyoracle as po
from razor_amd.fec import native
from test_flex_dropin import CASES, bind_flex, make_segments, sender_group

lib = bind_flex(native(1000))
L = lib.lib
c = CASES["k10_pf80_S1000"]
shards, hdr = po.Oracle(1000).fill_groups(c["config_id"], 1, c["k"], c["S"], ragged=c["ragged"])
snd = L.flex_fec_sender_create()
dev = torch.device("cuda", 0)
x = torch.ones(1 << 20, device=dev)
streams = [torch.cuda.Stream(dev) for _ in range(8)]
for s in streams:  # warm every stream up before the service is resident
    with torch.cuda.stream(s):
        x.mul_(1.0)
    s.synchronize()
t_call = time.perf_counter()
sender_group(lib, snd, make_segments(lib, shards[0], hdr[0]), c["protect_fraction"])
waits = []
for s in streams + [torch.cuda.current_stream(dev)]:
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        x.mul_(1.0)
    s.synchronize()
    waits.append(time.perf_counter() - t0)
t0 = time.perf_counter()
torch.cuda.synchronize()
sync = time.perf_counter() - t0
L.flex_fec_sender_destroy(snd)
assert L.rfec_service_stop() == 0
print(json.dumps({"stream_waits_s": waits, "device_sync_s": sync, "since_call_s": time.perf_counter() - t_call}))
"""


@pytest.mark.parametrize("life_us", [1_500_000, None])
def test_service_does_not_hold_other_streams(tmp_path, life_us):
    """While the resident service runs, kernels on other streams (8 torch
    streams and the current one: more than the GPU_MAX_HW_QUEUES = 4 hardware
    queues they share) still finish at once -- the service's stream is a
    non-blocking one of the highest priority, i.e. a hardware queue of its
    own (a normal-priority stream shared a queue with one torch stream, a
    CU-masked one blocked the legacy default stream: 1.5 s waits).
    A device-wide synchronize does
    wait for it: with a 1.5-s lifetime it takes about that long, with the
    default lifetime (4 ms) a few ms at most."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ)
    env.pop("RFEC_SERVICE", None)
    if life_us:
        env.update(RFEC_SERVICE_LIFE_US=str(life_us), RFEC_SERVICE_IDLE_US=str(life_us))
    else:
        env.pop("RFEC_SERVICE_LIFE_US", None)
        env.pop("RFEC_SERVICE_IDLE_US", None)
    r = subprocess.run([sys.executable, "-c", _HOL_SCRIPT, str(root), str(root / "tests"),
                        ], capture_output=True, text=True, timeout=120, env=env,
                       cwd=str(root / "oracle"))
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert max(d["stream_waits_s"]) < 0.1, d
    if life_us:
        assert 0.5 < d["since_call_s"] < 5.0, d  # the service really was resident meanwhile
    else:
        assert d["device_sync_s"] < 0.05, d


@pytest.mark.parametrize("stage", ["default", "host"])
def test_group_dropin_request_side(stage):
    """tools/dropin_group_bench.c (built with the library): 300 group-level
    sender updates and receiver recoveries through the service, their outputs
    equal to the line-level drop-in's, with the request side (doorbell, job,
    staged segments) in host-mapped device memory (default, where the host maps
    it) or in pinned host memory (RFEC_SERVICE_STAGE=host)."""
    import json
    import os
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parent.parent / "razor_amd" / "lib" / "fec_dropin_group_bench"
    assert exe.exists(), "razor_amd/lib/fec_dropin_group_bench not built"
    env = dict(os.environ)
    env.pop("RFEC_SERVICE", None)
    if stage == "host":
        env["RFEC_SERVICE_STAGE"] = "host"
    else:
        env.pop("RFEC_SERVICE_STAGE", None)
    r = subprocess.run([str(exe), "300"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout)
    assert d["outputs_equal"] is True
    svc = d["service_sender"]
    assert svc["jobs"] >= 300
    if stage == "host":
        assert svc["request_in_device"] == 0
    elif not bar_host_mapped():
        pytest.skip("device memory is not host-mapped here (small BAR): the request side stays in pinned memory")
    else:
        assert svc["request_in_device"] == 1
