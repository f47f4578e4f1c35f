"""The drop-in boundary end to end.

GPU: tests/dropin/fec_test_harness.c (own code: the reference's six FEC tests,
sim_test/fec_test/test_func.c:8-334, replayed call for call through
librazor_fec.so's flex_fec_generate / flex_fec_recover and its group-level
flex_fec_sender_* / flex_fec_receiver_*) prints exactly what the reference
build printed (tests/golden/ref_fec_test_stdout.txt, made by `make -C oracle
golden`).  Nothing built from reference sources goes to the GPU box.

CPU (container-side, when /root/reference is present): the reference's
sender, receiver and tests link unchanged against librazor_fec.so in place of
flex_fec_xor.c (`make dropin`), and the reference's tests with librazor_fec.so
in place of flex_fec_xor.c, flex_fec_sender.c and flex_fec_receiver.c
(`make dropin_flex`).  A link check only: running them needs the GPU.
"""
import os
import subprocess
from pathlib import Path

import pytest

import pyoracle as po

ROOT = Path(__file__).resolve().parent.parent
HARNESS = ROOT / "razor_amd" / "lib" / "fec_test_harness"
REFERENCE = Path("/root/reference")


# the resident service (default: its request side in host-mapped device
# memory where the host maps it), the same with the request side in pinned host
# memory, with four workgroups on column shares (the others leave on `quit`),
# with a relaunch before every call (a 1 us idle window races the workgroup's
# exit against the next post), and kernel launches per call
SERVICE_ENVS = {"service": {}, "service_host_staged": {"RFEC_SERVICE_STAGE": "host"},
                "service_4_workgroups": {"RFEC_SERVICE_GROUPS": "4"},
                "service_4_workgroups_relaunch": {"RFEC_SERVICE_GROUPS": "4", "RFEC_SERVICE_IDLE_US": "1"},
                "service_relaunch": {"RFEC_SERVICE_IDLE_US": "1"}, "launch": {"RFEC_SERVICE": "0"}}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", list(SERVICE_ENVS))
def test_reference_tests_through_dropin_symbols(mode):
    assert HARNESS.exists(), "razor_amd/lib/fec_test_harness not built (python -m razor_amd.build)"
    env = dict(os.environ, **SERVICE_ENVS[mode])
    r = subprocess.run([str(HARNESS)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout == (po.GOLDEN / "ref_fec_test_stdout.txt").read_text()


def test_reference_callers_link_against_dropin():
    if not REFERENCE.is_dir():
        pytest.skip("/root/reference absent (the link check is container-side)")
    r = subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), f"R={REFERENCE}", "dropin", "dropin_flex"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    for exe in ("fec_test_on_razor", "fec_test_on_razor_flex"):
        nm = subprocess.run(["nm", "-D", "--undefined-only", str(po.REFDIR / exe)], capture_output=True, text=True)
        undef = {ln.split()[-1] for ln in nm.stdout.splitlines() if ln.strip()}
        assert {"flex_fec_generate", "flex_fec_recover"} <= undef, exe
        if exe.endswith("_flex"):  # the group-level symbols come from librazor_fec.so too
            assert {"flex_fec_sender_update", "flex_fec_receiver_on_segment", "flex_fec_receiver_on_fec"} <= undef
        ldd = subprocess.run(["ldd", str(po.REFDIR / exe)], capture_output=True, text=True).stdout
        assert str(ROOT / "razor_amd" / "lib" / "librazor_fec.so") in str(Path(ldd.split("librazor_fec.so => ")[1]
                                                                                   .split()[0]).resolve())
