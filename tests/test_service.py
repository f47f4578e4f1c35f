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
from test_flex_dropin import CASES, _svc_stats, bind_flex, make_segments, sender_group

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
