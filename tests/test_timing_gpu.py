"""rfec_timing_events (include/razor_fec.h): the next kernel a thread launches
through the library records its own start / stop on the caller's events; the
setting is consumed by that launch and rfec_timing_launches counts the
kernels since.  bench.py's roofline durations rest on this."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from razor_amd.fec import HDR_DTYPE, native

pytestmark = pytest.mark.gpu


def _events(n):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
    s = torch.cuda.current_stream()
    for e in ev:
        e.record(s)  # torch creates an event at its first record
    torch.cuda.synchronize()
    return ev


def test_timing_events_time_one_launch(oracle1200):
    o = oracle1200
    lib = native(1000)
    G, k, S = 4096, 10, 1008  # video size 1000: slots of 1,008 bytes
    plan = o.plan_from_fraction(k, 80, 1)
    n = plan.n_lines
    dev = torch.device("cuda:0")
    sh = torch.randint(0, 256, (G * k * S,), dtype=torch.uint8, device=dev)
    h = np.zeros(G * k, HDR_DTYPE)
    h["size"] = 1000
    hdr = torch.from_numpy(h.view(np.uint8).copy()).to(dev)
    par = torch.empty((G * n * S,), dtype=torch.uint8, device=dev)
    meta = torch.empty((G * n * 20,), dtype=torch.uint8, device=dev)
    fs = torch.empty((G * n,), dtype=torch.int16, device=dev)
    st = torch.empty((G * n,), dtype=torch.int8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def encode():
        lib.encode_batch(plan, G, S, 1000, sh.data_ptr(), hdr.data_ptr(), par.data_ptr(), meta.data_ptr(),
                         fs.data_ptr(), st.data_ptr(), stream)

    a, b, c, d = _events(4)
    stamp = c.elapsed_time(d)
    lib.timing_events(a.cuda_event, b.cuda_event)
    encode()
    assert lib.timing_launches() == 1
    encode()  # not timed: the setting was consumed by the first launch
    assert lib.timing_launches() == 2
    torch.cuda.synchronize()
    t = a.elapsed_time(b)
    assert 0 < t < 50.0, t  # ms: one 4,096-group encode takes tens of microseconds
    assert c.elapsed_time(d) == stamp  # untouched events keep their stamps
    # a bracket around the call holds the kernel's own window
    e, f = _events(2)
    lib.timing_events(a.cuda_event, b.cuda_event)
    e.record()
    encode()
    f.record()
    torch.cuda.synchronize()
    assert a.elapsed_time(b) <= e.elapsed_time(f) + 1e-3
    assert np.isfinite(a.elapsed_time(b))
