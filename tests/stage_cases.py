"""Sender staging checks shared by the oracle and the product host code:
rfec_sender_plan against what the reference flex sender did on the scripted
frame sequences of tests/golden/stage.json (oracle/gen_stage.c)."""
from __future__ import annotations

import numpy as np

import pyoracle as po

SEG_FIELDS = ("packet_id", "send_id", "fid", "index", "total", "data_size", "fec_id", "group")


def check_plan(plan_fn, init_fn):
    """plan_fn(state, frames, seg_size) -> (segs, groups); init_fn() -> state."""
    fx = po.stage_fixture()
    for scn in fx["scenarios"]:
        frames, blob = po.stage_frames(scn)
        st = init_fn()
        segs, groups = plan_fn(st, frames, scn["seg_size"])
        exp = np.array(scn["segments"], np.int64)
        assert len(segs) == len(exp), scn["name"]
        for j, k in enumerate(SEG_FIELDS):
            got = segs[k].astype(np.int64)
            bad = np.nonzero(got != exp[:, j])[0]
            assert len(bad) == 0, f"{scn['name']}: segment {bad[0]} {k} {got[bad[0]]} != reference {exp[bad[0], j]}"
        # offsets are the running sum of data sizes within each frame (sim_sender.c:363-364)
        for f in range(len(frames)):
            sel = segs["frame"] == f
            assert np.array_equal(segs["offset"][sel], np.r_[0, np.cumsum(segs["data_size"][sel])[:-1]])
            assert segs["data_size"][sel].sum() == frames["size"][f]
        assert len(groups) == len(scn["groups"]), scn["name"]
        for g, eg in zip(groups, scn["groups"]):
            assert (int(g["fec_id"]), int(g["base_id"]), int(g["count"]), int(g["first_seg"]),
                    int(g["fec_send_id0"]), int(g["n_lines"])) == (eg["fec_id"], eg["base_id"], eg["count"],
                                                                  eg["first_seg"], eg["send_id0"],
                                                                  len(eg["parities"])), scn["name"]
        assert int(st["fec_id"][0]) == scn["open_fec_id"] and int(st["segs_count"][0]) == scn["open_count"]
